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
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (16, 20, 3), dtype=np.uint8)
    s = M.istd_sums(a, a)
    np.testing.assert_array_equal(s, [0, 0, 320, 0, 0, 0, 0])
    assert M.psnr(a, a) == math.inf
    assert abs(M.ssim(a, a) - 1.0) < 1e-12


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
