"""GPU parity of the ISTD metrics (stc_istd_errors / stc_istd_ssim) with the CPU oracle
(oracle/istd_metrics.py) on random and structured uint8 pairs, with and without masks, and
all_metrics() end to end over PNG directories.  Tolerances: LAB sums rtol 1e-5 (fp32 colour
conversion on both sides, powf/cbrtf vs numpy ulps); squared error and SSIM rtol 1e-9 (fp64)."""
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
        want = M.istd_sums(a[i], b[i], m[i] if masked else None)
        np.testing.assert_array_equal(got[i][[2, 5]], want[[2, 5]])
        np.testing.assert_allclose(got[i][[0, 1, 3, 4]], want[[0, 1, 3, 4]], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(got[i][6], want[6], rtol=1e-9)


@pytest.mark.parametrize("B,H,W", [(2, 256, 256), (1, 480, 640), (1, 7, 7), (2, 13, 29)])
def test_istd_ssim_vs_oracle(B, H, W):
    a, b, _ = _pair(B * 7 + W, B, H, W)
    got = metrics.istd_ssim(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()).cpu().numpy()
    for i in range(B):
        assert abs(got[i] - M.ssim(a[i], b[i])) < 1e-9 * max(1.0, abs(got[i]))


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
    s = sum(M.istd_sums(a[i], b[i], m[i]) for i in range(3))
    assert abs(r["rmse"] - s[0] / s[2]) < 1e-5 * r["rmse"]
    assert abs(r["mae_non"] - s[4] / s[5]) < 1e-5 * r["mae_non"]
    assert abs(r["rmse_all"] - (s[0] + s[3]) / (s[2] + s[5])) < 1e-5 * r["rmse_all"]
    r2 = metrics.all_metrics(str(tmp_path / "d1"), str(tmp_path / "d2"))
    assert math.isnan(r2["rmse_non"])
    assert abs(r2["psnr"] - np.mean([M.psnr(a[i], b[i]) for i in range(3)])) < 1e-6
    assert abs(r2["ssim"] - np.mean([M.ssim(a[i], b[i]) for i in range(3)])) < 1e-9
