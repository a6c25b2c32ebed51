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

PARITY UNPINNED against scikit-image itself: skimage is not importable in this container
(SURVEY.md §8c); the restatement is checked by the known-answer cases in
tests/test_istd_metrics_cpu.py (rgb2lab of white / black / primaries, identical images, a
direct-window SSIM loop).
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
    """skimage 0.17.2 color.rgb2lab for a float32 [..., 3] image (float32 arithmetic)."""
    arr = np.array(rgb, dtype=F32, copy=True)
    m = arr > 0.04045
    arr[m] = np.power((arr[m] + F32(0.055)) / F32(1.055), F32(2.4))
    arr[~m] /= F32(12.92)
    xyz = arr @ XYZ_FROM_RGB.T.astype(F32)
    arr = xyz / WHITE_D65.astype(F32)
    m = arr > 0.008856
    arr[m] = np.cbrt(arr[m])
    arr[~m] = F32(7.787) * arr[~m] + F32(16.0 / 116.0)
    x, y, z = arr[..., 0], arr[..., 1], arr[..., 2]
    L = F32(116.0) * y - F32(16.0)
    a = F32(500.0) * (x - y)
    b = F32(200.0) * (y - z)
    return np.stack([L, a, b], axis=-1).astype(F32)


def istd_sums(img1_u8, img2_u8, mask_u8=None):
    """[7] float64: {sum RMSE-term, sum MAE-term, count} over shadow, the same over non-shadow,
    sum of squared float differences -- the quantities eval.py:87-104 / 134 accumulate."""
    v1, v2 = img_as_float32(img1_u8), img_as_float32(img2_u8)
    l1, l2 = rgb2lab(v1).astype(np.float64), rgb2lab(v2).astype(np.float64)
    d = l1 - l2
    e2 = np.sqrt(np.sum(d * d, axis=-1))
    e1 = np.sum(np.abs(d), axis=-1)
    sh = np.ones(e2.shape, bool) if mask_u8 is None else (np.asarray(mask_u8) >= 128)
    q = v1.astype(np.float64) - v2.astype(np.float64)
    return np.array([e2[sh].sum(), e1[sh].sum(), sh.sum(), e2[~sh].sum(), e1[~sh].sum(), (~sh).sum(),
                     np.sum(q * q)])


def psnr(img1_u8, img2_u8):
    v1, v2 = img_as_float32(img1_u8), img_as_float32(img2_u8)
    mse = np.mean((v1 - v2) ** 2, dtype=np.float64)
    return math.inf if mse == 0 else 10.0 * math.log10(1.0 / mse)


def ssim(img1_u8, img2_u8, win=7):
    """skimage 0.17.2 structural_similarity(X, Y, multichannel=True) on float32 images."""
    from scipy.ndimage import uniform_filter
    X, Y = img_as_float32(img1_u8).astype(np.float64), img_as_float32(img2_u8).astype(np.float64)
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
