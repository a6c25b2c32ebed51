"""GPU parity of the ISTD metrics (stc_istd_errors / stc_istd_ssim) with the CPU oracle
(oracle/istd_metrics.py) on random and structured uint8 pairs, with and without masks, and
all_metrics() end to end over PNG directories, including every resize branch of eval.py.
Tolerances: LAB sums rtol 1e-5 for the all-fp32 stc_istd_errors (the oracle keeps skimage's float64
stages), 1e-6 for the typed path (powf ulps of img1's float32 gamma); squared error, SSIM and the
resized images 1e-9 / 1e-12 (fp64)."""
import math

import numpy as np
import pytest
import torch

from oracle import istd_metrics as M
from stcgan_amd import metrics

pytestmark = pytest.mark.gpu


def _pair(seed, B, H, W):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 256, (B, H, W, 3), dtype=np.uint8)
    b = np.clip(a.astype(int) + rng.integers(-60, 61, a.shape), 0, 255).astype(np.uint8)
    m = (rng.random((B, H, W)) < 0.3).astype(np.uint8) * 255
    return a, b, m


@pytest.mark.parametrize("B,H,W,masked", [(2, 256, 256, True), (2, 256, 256, False), (1, 480, 640, True),
                                          (3, 7, 9, True), (1, 1, 1, False)])
def test_istd_errors_vs_oracle(B, H, W, masked):
    a, b, m = _pair(B * 100 + H, B, H, W)
    got = metrics.istd_errors(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda(),
                              torch.from_numpy(m).cuda() if masked else None).cpu().numpy()
    for i in range(B):
        # stc_istd_errors takes both images as img_as_float32 images (no resize)
        want = M.istd_sums_f(M.img_as_float32(a[i]), M.img_as_float32(b[i]), (m[i] >= 128) if masked else None)
        np.testing.assert_array_equal(got[i][[2, 5]], want[[2, 5]])
        np.testing.assert_allclose(got[i][[0, 1, 3, 4]], want[[0, 1, 3, 4]], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(got[i][6], want[6], rtol=1e-9)


@pytest.mark.parametrize("B,H,W", [(2, 256, 256), (1, 480, 640), (1, 7, 7), (2, 13, 29)])
def test_istd_ssim_vs_oracle(B, H, W):
    a, b, _ = _pair(B * 7 + W, B, H, W)
    got = metrics.istd_ssim(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()).cpu().numpy()
    for i in range(B):
        assert abs(got[i] - M.ssim(a[i], b[i])) < 1e-9 * max(1.0, abs(got[i]))


@pytest.mark.parametrize("hw,ohw,aa", [((20, 30), (20, 30), False), ((48, 64), (19, 26), False),
                                       ((48, 64), (19, 26), True), ((11, 9), (40, 33), True), ((5, 7), (1, 1), False)])
def test_image_resize_vs_oracle(hw, ohw, aa):
    """skimage transform.resize restatement on the GPU (bilinear float64, edge mode, optional
    gaussian anti-aliasing) vs the oracle (scipy gaussian_filter + numpy bilinear): 1e-12."""
    rng = np.random.default_rng(hw[0] * 31 + ohw[1])
    u = rng.integers(0, 256, (*hw, 3), dtype=np.uint8)
    got = metrics.resize_f64(torch.from_numpy(u).cuda(), metrics.IMG_U8F32, ohw, aa).cpu().numpy()
    want = M.resize(M.img_as_float32(u), ohw, anti_aliasing=aa)
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-12)
    m = rng.integers(0, 256, hw, dtype=np.uint8)
    got = metrics.resize_f64(torch.from_numpy(m).cuda(), metrics.IMG_U8F64, ohw, aa).cpu().numpy()
    np.testing.assert_allclose(got, M.resize(M.img_as_float64(m), ohw, anti_aliasing=aa), rtol=0, atol=1e-12)


@pytest.mark.parametrize("size", [None, 32])
def test_all_metrics_resize_branches_vs_oracle(tmp_path, size):
    """all_metrics with img2 / mask larger than img1 (infer's 256x192-style outputs scored against
    bigger ground truth) and the ``size`` branch, vs the oracle's eval.py restatement.
    LAB sums rtol 1e-6 (float32 gamma of img1: powf ulps); PSNR / SSIM 1e-9."""
    from PIL import Image
    rng = np.random.default_rng(11)
    for d in ("d1", "d2", "mk"):
        (tmp_path / d).mkdir()
    trip = []
    for i in range(2):
        a = rng.integers(0, 256, (24, 32, 3), dtype=np.uint8)
        b = rng.integers(0, 256, (60, 80, 3), dtype=np.uint8)
        m = ((rng.random((60, 80)) < 0.4) * 255).astype(np.uint8)
        Image.fromarray(a).save(tmp_path / "d1" / f"{i}.png")
        Image.fromarray(b).save(tmp_path / "d2" / f"{i}.png")
        Image.fromarray(m).save(tmp_path / "mk" / f"{i}.png")
        trip.append((a, b, m))
    r = metrics.all_metrics(str(tmp_path / "d1"), str(tmp_path / "d2"), size=size, maskdir=str(tmp_path / "mk"))
    w = M.all_metrics_arrays(trip, size=size)
    for k in w:
        assert abs(r[k] - w[k]) <= 1e-6 * abs(w[k]), (k, r[k], w[k])
    r2 = metrics.all_metrics(str(tmp_path / "d1"), str(tmp_path / "d2"), size=size)
    w2 = M.all_metrics_arrays([(a, b, None) for a, b, _ in trip], size=size)
    for k in w2:
        if not math.isnan(w2[k]):
            tol = 1e-9 if k in ("psnr", "ssim") else 1e-6
            assert abs(r2[k] - w2[k]) <= tol * max(1.0, abs(w2[k])), (k, r2[k], w2[k])


def test_all_metrics_end_to_end(tmp_path):
    from PIL import Image
    a, b, m = _pair(5, 3, 64, 48)
    for d in ("d1", "d2", "mk"):
        (tmp_path / d).mkdir()
    for i in range(3):
        Image.fromarray(a[i]).save(tmp_path / "d1" / f"{i}.png")
        Image.fromarray(b[i]).save(tmp_path / "d2" / f"{i}.png")
        Image.fromarray(m[i]).save(tmp_path / "mk" / f"{i}.png")
    r = metrics.all_metrics(str(tmp_path / "d1"), str(tmp_path / "d2"), maskdir=str(tmp_path / "mk"))
    w = M.all_metrics_arrays([(a[i], b[i], m[i]) for i in range(3)])
    for k in w:
        assert abs(r[k] - w[k]) < 1e-6 * abs(w[k]), k
    r2 = metrics.all_metrics(str(tmp_path / "d1"), str(tmp_path / "d2"))
    assert math.isnan(r2["rmse_non"])
    assert abs(r2["psnr"] - np.mean([M.psnr(a[i], b[i]) for i in range(3)])) < 1e-6
    assert abs(r2["ssim"] - np.mean([M.ssim(a[i], b[i]) for i in range(3)])) < 1e-9
