"""GPU parity of stc_prepare_batch with the numpy oracle (bit-exact fp32): flips, crops, the
zero-padded crop of a small image, 1- and 3-channel tensors sharing one draw per sample."""
import numpy as np
import pytest
import torch

from oracle import prepare_ref as P
from stcgan_amd import data

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("H,W,crop,flip_prob", [(286, 286, 256, 0.5), (480, 640, 256, 0.5), (200, 300, 256, 0.5),
                                                (256, 256, None, 1.0), (256, 256, None, None)])
def test_prepare_bit_exact(H, W, crop, flip_prob):
    rng = np.random.default_rng(H + W)
    img = rng.integers(0, 256, (3, H, W, 3), dtype=np.uint8)
    mask = rng.integers(0, 256, (3, H, W), dtype=np.uint8)
    outs, params = data.prepare_samples([torch.from_numpy(img).cuda(), torch.from_numpy(mask).cuda()],
                                        flip_prob=flip_prob, crop_size=crop, rng=np.random.RandomState(7))
    _, geom = data.augment_params(3, H, W, flip_prob, crop, rng=np.random.RandomState(7))
    for b in range(3):
        f, oy, ox = params[b]
        for src, got in ((img, outs[0]), (mask, outs[1])):
            want = P.prepare_one(src[b], f, oy, ox, *geom)
            np.testing.assert_array_equal(got[b].cpu().numpy(), want)
