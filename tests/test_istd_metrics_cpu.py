"""CPU known-answer checks of the ISTD-metrics oracle (oracle/istd_metrics.py; src/eval.py:41-139
with scikit-image 0.17.2 semantics).  skimage is absent here: these cases pin the restatement
(parity vs skimage itself unpinned, see the oracle's header)."""
import math

import numpy as np

from oracle import istd_metrics as M


def test_rgb2lab_known_points():
    px = np.array([[[255, 255, 255], [0, 0, 0], [255, 0, 0], [128, 128, 128]]], np.uint8)
    lab = M.rgb2lab(M.img_as_float32(px))[0]
    # skimage's matrix rows do not sum exactly to the D65 white point: white is (100, -0.0024, 0.0046)
    np.testing.assert_allclose(lab[0], [100.0, -0.0024, 0.0046], atol=3e-4)
    np.testing.assert_allclose(lab[1], [0.0, 0.0, 0.0], atol=1e-6)
    np.testing.assert_allclose(lab[2], [53.24, 80.09, 67.20], atol=0.02)   # sRGB red, D65
    assert abs(lab[3][0] - 53.59) < 0.02 and abs(lab[3][1]) < 3e-3 and abs(lab[3][2]) < 6e-3


def test_identical_images():
    """The same file as img1 and img2: img2 is float64 after its (identity) resize, so its sRGB gamma
    runs in float64 while img1's runs in float32 -- the LAB errors are float32 rounding, not zero
    (as in the reference); the float images themselves are equal (PSNR inf, SSIM 1)."""
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (16, 20, 3), dtype=np.uint8)
    s = M.istd_sums(a, a)
    assert s[2] == 320 and s[5] == 0 and s[6] == 0
    assert 0 < s[0] / 320 < 1e-4 and 0 < s[1] / 320 < 1e-4
    v = M.img_as_float32(a)
    np.testing.assert_array_equal(M.istd_sums_f(v, v)[:2], [0, 0])  # same dtype on both sides: exact
    assert M.psnr(a, a) == math.inf
    assert abs(M.ssim(a, a) - 1.0) < 1e-12


def test_resize_identity_and_bilinear_points():
    """skimage resize (order 1, edge): equal shape is the identity; 2x upsampling samples at
    (c + 0.5) / 2 - 0.5 with edge clamping; the result matches a direct per-pixel loop."""
    rng = np.random.default_rng(3)
    x = rng.random((5, 7, 3))
    np.testing.assert_array_equal(M.resize(x, (5, 7)), x)
    up = M.resize(x[..., 0], (10, 14))
    assert up[0, 0] == x[0, 0, 0]                      # (-0.25, -0.25) clamps to pixel (0, 0)
    assert abs(up[1, 1] - (0.75 * (0.75 * x[0, 0, 0] + 0.25 * x[0, 1, 0])
                           + 0.25 * (0.75 * x[1, 0, 0] + 0.25 * x[1, 1, 0]))) < 1e-15
    out = M.resize(x, (3, 4))
    fy, fx = 5 / 3, 7 / 4
    for r in range(3):
        for c in range(4):
            rr, cc = fy * r + (0.5 * fy - 0.5), fx * c + (0.5 * fx - 0.5)
            r0, c0 = int(np.floor(rr)), int(np.floor(cc))
            r1, c1 = int(np.ceil(rr)), int(np.ceil(cc))
            dr, dc = rr - r0, cc - c0
            g = lambda i, j: x[min(max(i, 0), 4), min(max(j, 0), 6)]  # noqa: E731
            want = (1 - dr) * ((1 - dc) * g(r0, c0) + dc * g(r0, c1)) + dr * ((1 - dc) * g(r1, c0) + dc * g(r1, c1))
            np.testing.assert_allclose(out[r, c], want, rtol=0, atol=1e-15)


def test_all_metrics_arrays_branches():
    """eval.py's branches on arrays: sizes differ (img2 and the mask follow img1), size given, and the
    no-mask PSNR / SSIM; equal-size pairs reduce to istd_sums."""
    rng = np.random.default_rng(4)
    a = rng.integers(0, 256, (24, 32, 3), dtype=np.uint8)
    b = rng.integers(0, 256, (24, 32, 3), dtype=np.uint8)
    m = ((rng.random((24, 32)) < 0.4) * 255).astype(np.uint8)
    r = M.all_metrics_arrays([(a, b, m)])
    s = M.istd_sums(a, b, m)
    assert abs(r["rmse"] - s[0] / s[2]) < 1e-12 * r["rmse"]
    big = np.repeat(np.repeat(b, 2, 0), 2, 1)
    mbig = np.repeat(np.repeat(m, 2, 0), 2, 1)
    r2 = M.all_metrics_arrays([(a, big, mbig)])      # 2x downscale of img2 / mask (mask anti-aliased)
    assert np.isfinite(r2["rmse"]) and np.isfinite(r2["mae_non"])
    r3 = M.all_metrics_arrays([(a, b, None)], size=16)
    assert math.isnan(r3["rmse_non"]) and np.isfinite(r3["psnr"]) and 0 < r3["ssim"] <= 1


def test_mask_split_and_psnr():
    a = np.zeros((4, 4, 3), np.uint8)
    b = np.full((4, 4, 3), 51, np.uint8)          # v = 0.2 everywhere
    mask = np.zeros((4, 4), np.uint8)
    mask[:2] = 255
    mask[2, 0] = 128                              # 128/255 >= 0.5: shadow
    mask[2, 1] = 127                              # 127/255 < 0.5: not
    s = M.istd_sums(a, b, mask)
    assert s[2] == 9 and s[5] == 7
    assert abs(s[0] / 9 - s[3] / 7) < 1e-9        # the same per-pixel error everywhere
    assert abs(M.psnr(a, b) - 10 * math.log10(1 / (np.float32(51) * np.float32(1 / 255)) ** 2)) < 1e-4


def test_ssim_matches_direct_windows():
    rng = np.random.default_rng(1)
    a = rng.integers(0, 256, (12, 15, 3), dtype=np.uint8)
    b = np.clip(a.astype(int) + rng.integers(-40, 41, a.shape), 0, 255).astype(np.uint8)
    X, Y = M.img_as_float32(a).astype(np.float64), M.img_as_float32(b).astype(np.float64)
    C1, C2, cn = (0.02) ** 2, (0.06) ** 2, 49 / 48
    vals = []
    for c in range(3):
        acc = []
        for y in range(3, 12 - 3):
            for x in range(3, 15 - 3):
                wx, wy = X[y - 3:y + 4, x - 3:x + 4, c], Y[y - 3:y + 4, x - 3:x + 4, c]
                ux, uy = wx.mean(), wy.mean()
                vx, vy = cn * ((wx * wx).mean() - ux * ux), cn * ((wy * wy).mean() - uy * uy)
                vxy = cn * ((wx * wy).mean() - ux * uy)
                acc.append((2 * ux * uy + C1) * (2 * vxy + C2) / ((ux * ux + uy * uy + C1) * (vx + vy + C2)))
        vals.append(np.mean(acc))
    assert abs(M.ssim(a, b) - np.mean(vals)) < 1e-12
