"""ISTD evaluation metrics on the GPU (src/eval.py:41-139).

``all_metrics(dir1, dir2, size=None, maskdir=None)`` keeps the reference's signature and result
keys (rmse, mae, rmse_non, mae_non, rmse_all, mae_all, and psnr / ssim without a mask dir); the
per-pixel work -- rgb2lab of both images, the masked LAB error sums, the squared error behind
PSNR and SSIM -- runs in ``stc_istd_errors`` / ``stc_istd_ssim`` (csrc/istd_metrics.hip).  Files
are read as RGB uint8 (skimage.io.imread's order) with PIL; the host only decodes PNGs and adds
up the per-image sums.  Every resize branch of eval.py:64-81 runs on the GPU too
(``stc_image_resize_f64``: skimage transform.resize, mode "edge", order 1, with the mask's default
anti-aliasing): img2 follows img1's shape, the mask img1's size, and with ``size`` all three are
resized to size x size; types follow the reference (img2 and the mask are float64 after their
resize, img1 stays img_as_float32 unless ``size`` resizes it).
"""
import math
import os

import numpy as np
import torch

from ._lib import check, lib, ptr, stream


def _dev_u8(a, device):
    return torch.from_numpy(np.array(a, dtype=np.uint8, copy=True)).to(device)


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


IMG_U8F32, IMG_U8F64, IMG_F64 = 0, 1, 2


def resize_f64(img, kind, out_hw, anti_alias=False):
    """skimage transform.resize(img, out_hw, mode="edge") on the GPU -> float64 CUDA tensor
    [OH, OW(, C)]; img: uint8 (kind IMG_U8F32 / IMG_U8F64) or float64 CUDA tensor [H, W(, C)]."""
    two_d = img.dim() == 2
    x = img.contiguous()
    H, W = x.shape[:2]
    C = 1 if two_d else x.shape[2]
    OH, OW = out_hw
    out = torch.empty((OH, OW) if two_d else (OH, OW, C), dtype=torch.float64, device=x.device)
    nbytes = lib().stc_image_resize_workspace(H, W, C)
    ws = torch.empty(int(nbytes), dtype=torch.uint8, device=x.device)
    check(lib().stc_image_resize_f64(ptr(x), kind, H, W, C, OH, OW, int(anti_alias), ptr(out), ptr(ws), int(nbytes),
                                     stream()), "stc_image_resize_f64")
    return out


def istd_errors_typed(img1, kind1, img2, kind2, mask=None):
    """[7] float64 sums (as istd_errors) of one pair of typed images [H, W, 3]; mask float64 [H, W]
    (shadow = value > 0.5) or None."""
    H, W = img1.shape[:2]
    out = torch.empty(7, dtype=torch.float64, device=img1.device)
    nbytes = lib().stc_istd_typed_workspace(H, W)
    ws = torch.empty(int(nbytes), dtype=torch.uint8, device=img1.device)
    check(lib().stc_istd_errors_ex(ptr(img1.contiguous()), kind1, ptr(img2.contiguous()), kind2,
                                   ptr(None if mask is None else mask.contiguous()), H, W, ptr(out), ptr(ws),
                                   int(nbytes), stream()), "stc_istd_errors_ex")
    return out


def istd_ssim_typed(img1, kind1, img2, kind2):
    H, W = img1.shape[:2]
    out = torch.empty(1, dtype=torch.float64, device=img1.device)
    nbytes = lib().stc_istd_typed_workspace(H, W)
    ws = torch.empty(int(nbytes), dtype=torch.uint8, device=img1.device)
    check(lib().stc_istd_ssim_ex(ptr(img1.contiguous()), kind1, ptr(img2.contiguous()), kind2, H, W, ptr(out),
                                 ptr(ws), int(nbytes), stream()), "stc_istd_ssim_ex")
    return out


def _read_rgb(path):
    from PIL import Image
    return np.asarray(Image.open(path).convert("RGB"))


def _read_gray(path):
    """io.imread(path, as_gray=True) of a single-channel PNG: the uint8 plane as stored."""
    from PIL import Image
    im = Image.open(path)
    if im.mode not in ("L", "P", "1"):
        raise NotImplementedError(f"stcgan_amd.metrics: {path}: masks are single-channel PNGs ({im.mode})")
    return np.asarray(im.convert("L"))


def pair_sums(a_u8, b_u8, m_u8=None, size=None, device="cuda"):
    """One iteration of eval.py's loop (:62-107) on uint8 arrays: returns (sums [7] over the compared
    images, sse of the PSNR pair, ssim or None)."""
    A, Bt = _dev_u8(a_u8, device), _dev_u8(b_u8, device)
    H, W = a_u8.shape[:2]
    img2 = resize_f64(Bt, IMG_U8F32, (H, W))                      # float64, img1's shape
    mask = resize_f64(_dev_u8(m_u8, device), IMG_U8F64, (H, W), anti_alias=True) if m_u8 is not None else None
    if size is not None:
        i1 = resize_f64(A, IMG_U8F32, (size, size))
        i2 = resize_f64(img2, IMG_F64, (size, size))
        mk = resize_f64(mask, IMG_F64, (size, size), anti_alias=True) if mask is not None else None
        s = istd_errors_typed(i1, IMG_F64, i2, IMG_F64, mk)
    else:
        s = istd_errors_typed(A, IMG_U8F32, img2, IMG_F64, mask)
    s = s.cpu().numpy()
    sse, ss = None, None
    if m_u8 is None:
        sse = float(istd_errors_typed(A, IMG_U8F32, img2, IMG_F64, None)[6]) if size is not None else float(s[6])
        ss = float(istd_ssim_typed(A, IMG_U8F32, img2, IMG_F64)[0]) if H >= 7 and W >= 7 else float("nan")
    return s, sse, ss


def all_metrics(dir1, dir2, size=None, maskdir=None, device="cuda"):
    """src/eval.py:41-115 over the files of dir1 (same names in dir2 / maskdir), every resize branch
    included."""
    sums = np.zeros(7)
    psnrs, ssims = [], []
    for f in sorted(os.listdir(dir1)):
        a = _read_rgb(os.path.join(dir1, f))
        b = _read_rgb(os.path.join(dir2, f))
        m = _read_gray(os.path.join(maskdir, f)) if maskdir is not None else None
        s, sse, ss = pair_sums(a, b, m, size, device)
        sums += s
        if maskdir is None:
            psnrs.append(psnr_from_sse(sse, a.shape[0], a.shape[1]))
            ssims.append(ss)
    rs, ms, ns, rn, mn, nn = sums[:6]
    res = {"rmse": rs / ns if ns else float("nan"), "mae": ms / ns if ns else float("nan"),
           "rmse_non": rn / nn if nn else float("nan"), "mae_non": mn / nn if nn else float("nan"),
           "rmse_all": (rn + rs) / (nn + ns), "mae_all": (mn + ms) / (nn + ns)}
    if maskdir is None:
        res["psnr"] = float(np.mean(psnrs))
        res["ssim"] = float(np.mean(ssims))
    return res
