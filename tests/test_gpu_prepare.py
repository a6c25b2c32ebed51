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


@pytest.mark.parametrize("H,W,oh,ow,C", [(48, 64, 19, 25, 3), (30, 40, 16, 16, 1), (32, 48, 16, 24, 3),
                                         (37, 29, 11, 7, 3)])
def test_resize_area_bit_exact(H, W, oh, ow, C):
    rng = np.random.default_rng(H * W)
    img = rng.integers(0, 256, (2, H, W, C), dtype=np.uint8)
    got = data.resize_area(torch.from_numpy(img).cuda(), (oh, ow)).cpu().numpy()
    for b in range(2):
        np.testing.assert_array_equal(got[b], P.resize_area_one(img[b], oh, ow))


def test_resize_then_flip_crop_pipeline():
    rng = np.random.default_rng(11)
    img = rng.integers(0, 256, (2, 60, 80, 3), dtype=np.uint8)
    outs, params = data.prepare_samples([torch.from_numpy(img).cuda()], flip_prob=0.5, crop_size=24, resize=32,
                                        rng=np.random.RandomState(5))
    for b in range(2):
        f, oy, ox = params[b]
        r = P.resize_area_one(img[b], 32, 32)
        if f:
            r = np.fliplr(r)
        np.testing.assert_array_equal(outs[0][b].cpu().numpy(), r[oy:oy + 24, ox:ox + 24].transpose(2, 0, 1))
