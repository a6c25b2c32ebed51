"""ISTD evaluation metrics on the GPU (src/eval.py:41-139).

``all_metrics(dir1, dir2, size=None, maskdir=None)`` keeps the reference's signature and result
keys (rmse, mae, rmse_non, mae_non, rmse_all, mae_all, and psnr / ssim without a mask dir); the
per-pixel work -- rgb2lab of both images, the masked LAB error sums, the squared error behind
PSNR and SSIM -- runs in ``stc_istd_errors`` / ``stc_istd_ssim`` (csrc/istd_metrics.hip).  Files
are read as RGB uint8 (skimage.io.imread's order) with PIL; the host only decodes PNGs and adds
up the per-image sums.  Pairs must have the same size and ``size`` must be None (the reference's
resize branch, skimage.transform.resize, is not restated).
"""
import math
import os

import numpy as np
import torch

from ._lib import check, lib, ptr, stream


def _dev_u8(a, device):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint8)).to(device)


def istd_errors(img1, img2, mask=None):
    """Per-pair sums [B, 7] fp64: {sum |dLab|_2, sum |dLab|_1, count} over shadow pixels, the same
    over non-shadow pixels, and sum (v1 - v2)^2 (v = u / 255).  img1, img2: uint8 CUDA tensors
    [B, H, W, 3] (RGB); mask: uint8 [B, H, W] or None (every pixel counts as shadow)."""
    if not (img1.is_cuda and img2.is_cuda):
        raise RuntimeError("stcgan_amd.metrics: CUDA (HIP) tensors only")
    B, H, W, C = img1.shape
    assert C == 3 and img2.shape == img1.shape and img1.dtype == torch.uint8 and img2.dtype == torch.uint8
    a, b = img1.contiguous(), img2.contiguous()
    m = None
    if mask is not None:
        assert mask.shape == (B, H, W) and mask.dtype == torch.uint8
        m = mask.contiguous()
    out = torch.empty((B, 7), dtype=torch.float64, device=a.device)
    nbytes = lib().stc_istd_errors_workspace(B, H, W)
    ws = torch.empty(max(int(nbytes), 8), dtype=torch.uint8, device=a.device)
    check(lib().stc_istd_errors(ptr(a), ptr(b), ptr(m), B, H, W, ptr(out), ptr(ws), int(nbytes), stream()),
          "stc_istd_errors")
    return out


def istd_ssim(img1, img2):
    """SSIM per pair [B] fp64 (skimage 0.17 structural_similarity, multichannel, float32 inputs)."""
    if not (img1.is_cuda and img2.is_cuda):
        raise RuntimeError("stcgan_amd.metrics: CUDA (HIP) tensors only")
    B, H, W, C = img1.shape
    assert C == 3 and img2.shape == img1.shape
    a, b = img1.contiguous(), img2.contiguous()
    out = torch.empty((B,), dtype=torch.float64, device=a.device)
    nbytes = lib().stc_istd_errors_workspace(B, H, W)
    ws = torch.empty(max(int(nbytes), 8), dtype=torch.uint8, device=a.device)
    check(lib().stc_istd_ssim(ptr(a), ptr(b), B, H, W, ptr(out), ptr(ws), int(nbytes), stream()), "stc_istd_ssim")
    return out


def psnr_from_sse(sse, H, W):
    """skimage 0.17 peak_signal_noise_ratio for float images in [0, 1] (data_range 1)."""
    mse = sse / (3.0 * H * W)
    return math.inf if mse == 0 else 10.0 * math.log10(1.0 / mse)


def all_metrics(dir1, dir2, size=None, maskdir=None, device="cuda"):
    """src/eval.py:41-115 over the files of dir1 (same names in dir2 / maskdir)."""
    from PIL import Image
    if size is not None:
        raise NotImplementedError("stcgan_amd.metrics: the resize branch (size != None) is not restated")
    sums = np.zeros(7)
    psnrs, ssims = [], []
    for f in sorted(os.listdir(dir1)):
        a = np.asarray(Image.open(os.path.join(dir1, f)).convert("RGB"))
        b = np.asarray(Image.open(os.path.join(dir2, f)).convert("RGB"))
        if a.shape != b.shape:
            raise NotImplementedError(f"stcgan_amd.metrics: {f}: sizes differ ({a.shape} vs {b.shape})")
        m = None
        if maskdir is not None:
            m = _dev_u8(np.asarray(Image.open(os.path.join(maskdir, f)).convert("L"))[None], device)
        A, Bt = _dev_u8(a[None], device), _dev_u8(b[None], device)
        s = istd_errors(A, Bt, m)[0].cpu().numpy()
        sums += s
        if maskdir is None:
            psnrs.append(psnr_from_sse(float(s[6]), a.shape[0], a.shape[1]))
            ssims.append(float(istd_ssim(A, Bt)[0]))
    rs, ms, ns, rn, mn, nn = sums[:6]
    res = {"rmse": rs / ns if ns else float("nan"), "mae": ms / ns if ns else float("nan"),
           "rmse_non": rn / nn if nn else float("nan"), "mae_non": mn / nn if nn else float("nan"),
           "rmse_all": (rn + rs) / (nn + ns), "mae_all": (mn + ms) / (nn + ns)}
    if maskdir is None:
        res["psnr"] = float(np.mean(psnrs))
        res["ssim"] = float(np.mean(ssims))
    return res
