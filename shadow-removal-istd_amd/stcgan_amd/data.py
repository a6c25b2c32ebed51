"""Training-batch preparation on the GPU (STCGAN/dataset.py:89-147 and
STCGAN/transform.py:103-156).

The reference's ``ISTDDataset.__getitem__`` reads each image with cv2 (BGR), converts it with
``uint2float`` (u / 255), normalises ``(v - 0.5) * 2`` (the intent of dataset.py:122-124, which
references undefined names and raises NameError as written), then applies the transforms of
``transform.transforms(...)`` to (img, mask, target) with shared random draws.  Here the decoded
uint8 batch goes to the device once and ``stc_prepare_batch`` does normalisation, the horizontal
flip and the (zero-padded) random crop in one pass.  The random parameters are drawn on the host
in the reference's order per sample: ``np.random.rand() > flip_prob`` (no flip), then
``randint(0, rows - crop_rows)`` and ``randint(0, cols - crop_cols)``.  Resize is restated for
shrinking (cv.INTER_AREA, ``resize_area``); RandomScale / RandomRotate are not
(``NotImplementedError``).
"""
import numpy as np
import torch

from ._lib import check, lib, ptr, stream


def augment_params(n, H, W, flip_prob=None, crop_size=None, rng=np.random):
    """Per-sample {flip, row_offset, col_offset} and the crop geometry (pad_h, pad_w, OH, OW)."""
    if crop_size is None:
        OH, OW = H, W
    elif isinstance(crop_size, (int, np.integer)):
        OH, OW = int(crop_size), int(crop_size)
    else:
        OH, OW = (int(v) for v in crop_size)
    pad_h, pad_w = (max(OH - H, 0), max(OW - W, 0)) if (OH > H or OW > W) else (0, 0)
    rows, cols = H + 2 * pad_h, W + 2 * pad_w
    params = np.zeros((n, 3), np.int32)
    for i in range(n):
        if flip_prob is not None:
            params[i, 0] = 0 if rng.rand() > flip_prob else 1
        if crop_size is not None:
            params[i, 1] = rng.randint(low=0, high=rows - OH)
            params[i, 2] = rng.randint(low=0, high=cols - OW)
    return params, (pad_h, pad_w, OH, OW)


def resize_area(images_u8, size):
    """Resize (transform.py:159-181) of the normalised images when they shrink in both dimensions
    (cv.INTER_AREA): uint8 [B, H, W, C] -> fp32 NHWC [B, rows, cols, C]."""
    if images_u8.dim() == 3:
        images_u8 = images_u8.unsqueeze(-1)
    src = images_u8.contiguous()
    B, H, W, C = src.shape
    rows, cols = (size, size) if isinstance(size, (int, np.integer)) else size
    if not (rows < H and cols < W):
        raise NotImplementedError("stcgan_amd.data: Resize is restated for shrinking (INTER_AREA) only")
    out = torch.empty((B, rows, cols, C), dtype=torch.float32, device=src.device)
    check(lib().stc_resize_area(ptr(src), B, H, W, C, rows, cols, ptr(out), stream()), "stc_resize_area")
    return out


def prepare(images, params, geom):
    """[B, H, W, C] CUDA tensor -> fp32 [B, C, OH, OW] = crop(flip(v)), v = (u / 255 - 0.5) * 2 for a
    uint8 source, or the fp32 source as is (already normalised, e.g. by resize_area)."""
    if not images.is_cuda:
        raise RuntimeError("stcgan_amd.data: CUDA (HIP) tensors only")
    if images.dim() == 3:
        images = images.unsqueeze(-1)
    src = images.contiguous()
    B, H, W, C = src.shape
    pad_h, pad_w, OH, OW = geom
    p = torch.as_tensor(np.ascontiguousarray(params, np.int32)).to(src.device)
    out = torch.empty((B, C, OH, OW), dtype=torch.float32, device=src.device)
    if src.dtype == torch.uint8:
        check(lib().stc_prepare_batch(ptr(src), B, H, W, C, ptr(p), pad_h, pad_w, OH, OW, ptr(out), stream()),
              "stc_prepare_batch")
    elif src.dtype == torch.float32:
        check(lib().stc_prepare_batch_f32(ptr(src), B, H, W, C, ptr(p), pad_h, pad_w, OH, OW, ptr(out), stream()),
              "stc_prepare_batch_f32")
    else:
        raise TypeError(f"stcgan_amd.data: uint8 or fp32 images, got {src.dtype}")
    return out


def prepare_samples(tensors, flip_prob=None, crop_size=None, rng=np.random, resize=None, scale=None, angle=None):
    """(img, mask, target, ...) uint8 batches sharing one draw per sample -> fp32 NCHW batches."""
    if scale is not None or angle is not None:
        raise NotImplementedError("stcgan_amd.data: RandomScale / RandomRotate are not restated")
    if resize is not None:
        tensors = [resize_area(t, resize) for t in tensors]
    B, H, W = tensors[0].shape[:3]
    params, geom = augment_params(B, H, W, flip_prob, crop_size, rng)
    return [prepare(t, params, geom) for t in tensors], params
