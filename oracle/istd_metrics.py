"""CPU oracle of the ISTD evaluation metrics -- TEST INFRASTRUCTURE ONLY.

Only tests/ (and smoke()/bench.py's cpu_baseline leg) may import this module, as the checker; the
product path (stc_istd_errors / stc_istd_ssim) never calls it.

Restates src/eval.py:41-139 with scikit-image 0.17.2's algorithms (the version the reference pins,
requirements.txt) in numpy / scipy:
  * util.img_as_float32(u8)           -> u * float32(1/255) in float32
  * color.rgb2lab (D65, 2 degrees)    -> float32: sRGB gamma, xyz = rgb @ M.T, / white point,
                                         cube root / linear segment, L a b
  * RMSE / MAE (eval.py:124-131)      -> per-pixel |dLab|_2 and sum |dLab| summed over the mask
  * img_as_bool(mask / 255)           -> mask >= 128
  * metrics.peak_signal_noise_ratio   -> data_range 1 (float image with min >= 0), mse in float64
  * metrics.structural_similarity(multichannel=True) -> win 7, uniform filter (scipy.ndimage,
                                         float64), sample covariance, data_range 2 (float dtype
                                         range), K1 0.01, K2 0.03, 3-pixel crop, mean over channels

The resize branches of all_metrics (eval.py:64-81) -- img2 resized to img1's shape, the mask
resized to img1's size, and with ``size`` every image resized to size x size -- follow
skimage 0.17 transform.resize(..., mode="edge"): order-1 (bilinear) _warp_fast in float64 with
the metric transform col_in = s*(c + 0.5) - 0.5 (s = in/out), edge-clamped taps, and for the
mask (anti_aliasing left at its default, True for a non-bool image) a scipy.ndimage
gaussian_filter (sigma = max(0, (s - 1) / 2) per axis, mode 'nearest', truncate 4) first.
Types follow the reference: img2 is float64 after its resize even at equal size; rgb2lab keeps
an image's dtype for the sRGB gamma and computes in float64 from the matrix product on
(skimage's xyz_from_rgb is a float64 array); img_as_bool of a float mask is ``> 0.5``.

PARITY UNPINNED against scikit-image itself: skimage is not importable in this container
(SURVEY.md §8c); the restatement is checked by the known-answer cases in
tests/test_istd_metrics_cpu.py (rgb2lab of white / black / primaries, identical images, a
direct-window SSIM loop, resize identities and hand-derived bilinear points).
"""
import math

import numpy as np

F32 = np.float32
XYZ_FROM_RGB = np.array([[0.412453, 0.357580, 0.180423],
                         [0.212671, 0.715160, 0.072169],
                         [0.019334, 0.119193, 0.950227]])
WHITE_D65 = np.array([0.95047, 1.0, 1.08883])


def img_as_float32(u8):
    return np.asarray(u8, np.uint8).astype(F32) * F32(1.0 / 255.0)


def rgb2lab(rgb):
    """skimage 0.17.2 color.rgb2lab: the sRGB gamma in the image's float dtype (float32 for an
    img_as_float32 image, float64 for a resized one), then ``arr @ xyz_from_rgb.T`` with the float64
    matrix -- float64 from there on (colorconv.rgb2xyz / xyz2lab)."""
    rgb = np.asarray(rgb)
    dt = rgb.dtype.type if rgb.dtype in (np.float32, np.float64) else np.float64
    arr = np.array(rgb, dtype=dt, copy=True)
    m = arr > 0.04045
    arr[m] = np.power((arr[m] + dt(0.055)) / dt(1.055), dt(2.4))
    arr[~m] /= dt(12.92)
    xyz = arr @ XYZ_FROM_RGB.T           # float64 result (float64 matrix)
    arr = xyz / WHITE_D65
    m = arr > 0.008856
    arr[m] = np.cbrt(arr[m])
    arr[~m] = 7.787 * arr[~m] + 16.0 / 116.0
    x, y, z = arr[..., 0], arr[..., 1], arr[..., 2]
    L = 116.0 * y - 16.0
    a = 500.0 * (x - y)
    b = 200.0 * (y - z)
    return np.stack([L, a, b], axis=-1)


def img_as_float64(u8):
    """util.img_as_float of a uint8 image: u * (1/255) in float64."""
    return np.asarray(u8, np.uint8).astype(np.float64) * (1.0 / 255.0)


def resize(img, out_hw, anti_aliasing=False):
    """skimage 0.17 transform.resize(img, out_hw, mode="edge", anti_aliasing=...) of a float image
    [H, W] or [H, W, C] -> float64 (order 1: _warp_fast bilinear; edge mode; clip to the input's
    range, a no-op for the convex bilinear weights up to one float64 ulp, not applied here)."""
    from scipy.ndimage import gaussian_filter
    img = np.asarray(img)
    H, W = img.shape[:2]
    OH, OW = out_hw
    fy, fx = H / OH, W / OW
    x = img.astype(np.float64)
    if anti_aliasing:
        sig = [max(0.0, (fy - 1) / 2), max(0.0, (fx - 1) / 2)] + [0.0] * (x.ndim - 2)
        if any(v > 0 for v in sig):
            x = gaussian_filter(x, sig, mode="nearest")
    r = np.arange(OH, dtype=np.float64) * fy + (0.5 * fy - 0.5)
    c = np.arange(OW, dtype=np.float64) * fx + (0.5 * fx - 0.5)
    r0, c0 = np.floor(r).astype(np.int64), np.floor(c).astype(np.int64)
    r1, c1 = np.ceil(r).astype(np.int64), np.ceil(c).astype(np.int64)
    dr, dc = r - r0, c - c0
    r0, r1 = np.clip(r0, 0, H - 1), np.clip(r1, 0, H - 1)
    c0, c1 = np.clip(c0, 0, W - 1), np.clip(c1, 0, W - 1)
    ex = (slice(None),) + (None,) * (x.ndim - 2)
    tl, tr = x[r0][:, c0], x[r0][:, c1]
    bl, br = x[r1][:, c0], x[r1][:, c1]
    dcb = dc[None, :][(slice(None), slice(None)) + (None,) * (x.ndim - 2)]
    drb = dr[ex][:, None] if x.ndim == 2 else dr[:, None, None]
    top = (1 - dcb) * tl + dcb * tr
    bottom = (1 - dcb) * bl + dcb * br
    return (1 - drb) * top + drb * bottom


def istd_sums(img1_u8, img2_u8, mask_u8=None):
    """[7] float64: {sum RMSE-term, sum MAE-term, count} over shadow, the same over non-shadow,
    sum of squared float differences -- the quantities eval.py:87-104 / 134 accumulate, for a
    same-size pair (img2 float64 after its identity resize, the mask u / 255 > 0.5)."""
    v1 = img_as_float32(img1_u8)
    v2 = img_as_float32(img2_u8).astype(np.float64)
    mask = None if mask_u8 is None else img_as_float64(mask_u8) > 0.5
    return istd_sums_f(v1, v2, mask)


def istd_sums_f(v1, v2, mask=None):
    """istd_sums over float images (float32 or float64) and a bool mask (None: all shadow)."""
    l1, l2 = rgb2lab(v1), rgb2lab(v2)
    d = l1 - l2
    e2 = np.sqrt(np.sum(d * d, axis=-1))
    e1 = np.sum(np.abs(d), axis=-1)
    sh = np.ones(e2.shape, bool) if mask is None else np.asarray(mask, bool)
    q = np.asarray(v1).astype(np.float64) - np.asarray(v2).astype(np.float64)
    return np.array([e2[sh].sum(), e1[sh].sum(), sh.sum(), e2[~sh].sum(), e1[~sh].sum(), (~sh).sum(),
                     np.sum(q * q)])


def psnr(img1_u8, img2_u8):
    return psnr_f(img_as_float32(img1_u8), img_as_float32(img2_u8))


def psnr_f(v1, v2):
    """peak_signal_noise_ratio(img1 float32, img2): data_range 1 (img1 >= 0), mse in float64."""
    q = np.asarray(v1).astype(np.float64) - np.asarray(v2).astype(np.float64)
    mse = np.mean(q * q)
    return math.inf if mse == 0 else 10.0 * math.log10(1.0 / mse)


def ssim(img1_u8, img2_u8, win=7):
    return ssim_f(img_as_float32(img1_u8), img_as_float32(img2_u8), win)


def ssim_f(v1, v2, win=7):
    """skimage 0.17.2 structural_similarity(X, Y, multichannel=True), X float32 (data_range 2)."""
    from scipy.ndimage import uniform_filter
    X, Y = np.asarray(v1).astype(np.float64), np.asarray(v2).astype(np.float64)
    R = 2.0  # dtype_range[float32] = (-1, 1)
    C1, C2 = (0.01 * R) ** 2, (0.03 * R) ** 2
    NP = win * win
    cov_norm = NP / (NP - 1.0)
    pad = (win - 1) // 2
    vals = []
    for c in range(X.shape[-1]):
        x, y = X[..., c], Y[..., c]
        ux, uy = uniform_filter(x, win), uniform_filter(y, win)
        uxx, uyy, uxy = uniform_filter(x * x, win), uniform_filter(y * y, win), uniform_filter(x * y, win)
        vx, vy, vxy = cov_norm * (uxx - ux * ux), cov_norm * (uyy - uy * uy), cov_norm * (uxy - ux * uy)
        S = ((2 * ux * uy + C1) * (2 * vxy + C2)) / ((ux * ux + uy * uy + C1) * (vx + vy + C2))
        vals.append(S[pad:-pad, pad:-pad].mean())
    return float(np.mean(vals))


def all_metrics_arrays(pairs, size=None):
    """src/eval.py:41-115 over in-memory (img1 u8 RGB, img2 u8 RGB, mask u8 or None) triples, with
    every resize branch (img2 -> img1's shape, mask -> img1's size, and size x size when given)."""
    rm, ma, rn, mn, px, pn, ps, ss = [], [], [], [], [], [], [], []
    has_mask = pairs[0][2] is not None
    for a, b, m in pairs:
        img1 = img_as_float32(a)
        img2 = resize(img_as_float32(b), img1.shape[:2], anti_aliasing=False)
        mask = resize(img_as_float64(m), img1.shape[:2], anti_aliasing=True) if m is not None else \
            np.ones(img1.shape[:2], bool)
        if size is not None:
            i1 = resize(img1, (size, size))
            i2 = resize(img2, (size, size))
            mk = (resize(mask.astype(np.float64), (size, size), anti_aliasing=mask.dtype != bool) > 0.5) \
                if m is not None else resize(mask, (size, size)) > 0.5
        else:
            i1, i2 = img1, img2
            mk = mask > 0.5 if mask.dtype != bool else mask
        s = istd_sums_f(i1, i2, mk)
        rm.append(s[0]); ma.append(s[1]); px.append(s[2]); rn.append(s[3]); mn.append(s[4]); pn.append(s[5])
        if not has_mask:
            ps.append(psnr_f(img1, img2))
            ss.append(ssim_f(img1, img2))
    res = {"rmse": np.sum(rm) / np.sum(px), "mae": np.sum(ma) / np.sum(px),
           "rmse_non": np.sum(rn) / np.sum(pn), "mae_non": np.sum(mn) / np.sum(pn),
           "rmse_all": (np.sum(rn) + np.sum(rm)) / (np.sum(pn) + np.sum(px)),
           "mae_all": (np.sum(mn) + np.sum(ma)) / (np.sum(pn) + np.sum(px))}
    if not has_mask:
        res["psnr"] = float(np.mean(ps))
        res["ssim"] = float(np.mean(ss))
    return res
