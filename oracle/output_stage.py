"""CPU oracle of the STCGAN.infer() output stage -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker; the product path (stc_infer_output) never calls it.

Restates, in numpy float32 (every product and sum rounded separately, no fused multiply-add):
  * ``x * 0.5 + 0.5``                         -- STCGAN/stcgan.py:355-357
  * ``cv.resize(v, (OW, OH), INTER_LINEAR)``  -- STCGAN/stcgan.py:367-368,373-374: OpenCV's generic
    float32 INTER_LINEAR (resizeGeneric_ / HResizeLinear / VResizeLinear): column coefficients from
    ``float((dx + 0.5) * scale_x - 0.5)`` (double, rounded to float), index clamp with weight 0 at
    both edges, single-term horizontal pass past the right edge, rows clamped to [0, H-1] with the
    unclamped weights; an exact 2x2 downscale is rerouted by cv::resize to INTER_AREA (block mean)
  * ``(r * 255).astype(np.uint8)``            -- STCGAN/utils.py:63-65 (float2uint, truncation)

PARITY UNPINNED against OpenCV itself: cv2 is not importable in this container, so
this restatement of its published algorithm is checked only by the hand-derived cases in
tests/test_output_stage_cpu.py (identity size, constant images, exact interpolation points).  A
build of OpenCV that contracts ``S0*b0 + S1*b1`` into an FMA can differ by one float ulp before
truncation (then, rarely, by 1 in a uint8).
"""
import numpy as np

F32 = np.float32


def _axis_coeffs(dsize, ssize):
    """(s, two, a0, a1) per output index along one axis (resizeGeneric_ xofs/alpha setup)."""
    scale = 1.0 / (float(dsize) / float(ssize))
    d = np.arange(dsize, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(F32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(F32)).astype(F32)
    two = (s + 1) < ssize
    lo = s < 0
    f[lo] = 0
    s[lo] = 0
    hi = s >= ssize - 1
    f[hi] = 0
    s[hi] = ssize - 1
    a0 = (F32(1) - f).astype(F32)
    return s, two, a0, f


def resize_linear(img, oh, ow):
    """cv.resize(img, (ow, oh), interpolation=cv.INTER_LINEAR) for a float32 HxW or HxWxC image."""
    img = np.asarray(img, dtype=F32)
    h, w = img.shape[:2]
    squeeze = img.ndim == 2
    if squeeze:
        img = img[:, :, None]
    if (h, w) == (oh, ow):
        out = img.copy()
    elif h == 2 * oh and w == 2 * ow:  # cv::resize: INTER_LINEAR at an exact 2x2 downscale -> INTER_AREA
        s = img[0::2, 0::2] + img[0::2, 1::2]
        s = (s + img[1::2, 0::2]).astype(F32)
        s = (s + img[1::2, 1::2]).astype(F32)
        out = (s * F32(0.25)).astype(F32)
    else:
        sx, two, a0, a1 = _axis_coeffs(ow, w)
        sx1 = np.where(two, sx + 1, sx)
        # horizontal pass over every source row
        left = (img[:, sx] * a0[None, :, None]).astype(F32)
        right = (img[:, sx1] * a1[None, :, None]).astype(F32)
        hrow = np.where(two[None, :, None], (left + right).astype(F32), left)
        # vertical pass
        scale_y = 1.0 / (float(oh) / float(h))
        dy = np.arange(oh, dtype=np.float64)
        fy = ((dy + 0.5) * scale_y - 0.5).astype(F32)
        sy = np.floor(fy).astype(np.int64)
        fy = (fy - sy.astype(F32)).astype(F32)
        b0 = (F32(1) - fy).astype(F32)
        y0 = np.clip(sy, 0, h - 1)
        y1 = np.clip(sy + 1, 0, h - 1)
        out = ((hrow[y0] * b0[:, None, None]).astype(F32) + (hrow[y1] * fy[:, None, None]).astype(F32)).astype(F32)
    return out[:, :, 0] if squeeze else out


def float2uint(array):
    """STCGAN/utils.py:63-65."""
    return (array * F32(255)).astype(F32).astype(np.uint8)


def infer_output(net_out, oh=192, ow=256):
    """Generator output [B, C, H, W] (numpy/torch fp32) -> uint8 [B, oh, ow, C], the images
    STCGAN.infer hands to cv.imwrite (stcgan.py:355-377)."""
    x = np.asarray(net_out, dtype=F32)
    v = (x * F32(0.5) + F32(0.5)).astype(F32)
    outs = []
    for b in range(v.shape[0]):
        r = resize_linear(v[b].transpose(1, 2, 0), oh, ow)
        if r.ndim == 2:
            r = r[:, :, None]
        outs.append(float2uint(r))
    return np.stack(outs, 0) if outs else np.zeros((0, oh, ow, x.shape[1]), np.uint8)
