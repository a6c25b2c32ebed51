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


@pytest.mark.parametrize("H,W,oh,ow,C", [(6, 8, 12, 16, 3), (30, 40, 45, 70, 1), (48, 64, 48, 80, 3), (17, 23, 9, 40, 3),
                                         (5, 5, 5, 5, 1)])
@pytest.mark.parametrize("u8", [True, False])
def test_resize_linear_bit_exact(H, W, oh, ow, C, u8):
    rng = np.random.default_rng(H * W + oh)
    img = rng.integers(0, 256, (2, H, W, C), dtype=np.uint8)
    v = np.stack([P.normalise(im) for im in img])
    src = torch.from_numpy(img if u8 else v).cuda()
    got = data.resize_linear(src, (oh, ow)).cpu().numpy()
    for b in range(2):
        np.testing.assert_array_equal(got[b], P.resize_linear_one(v[b], oh, ow))


@pytest.mark.parametrize("H,W,C", [(24, 32, 3), (31, 17, 1), (40, 40, 3)])
@pytest.mark.parametrize("u8", [True, False])
def test_warp_affine_bit_exact(H, W, C, u8):
    rng = np.random.default_rng(H + 7 * W + C)
    img = rng.integers(0, 256, (4, H, W, C), dtype=np.uint8)
    v = np.stack([P.normalise(im) for im in img])
    mats = np.stack([P.rotation_matrix(W, H, 0, 1.043), P.rotation_matrix(W, H, -13.7, 1),
                     P.rotation_matrix(W, H, 90, 1), P.rotation_matrix(W, H, 4.2, 0.95)])
    got = data.warp_affine(torch.from_numpy(img if u8 else v).cuda(), mats).cpu().numpy()
    for b in range(4):
        np.testing.assert_array_equal(got[b], P.warp_affine_one(v[b], mats[b]))


def _oracle_chain(u8, resize, scale, angle, params, geom):
    pad_h, pad_w, OH, OW = geom
    v = P.normalise(u8)
    h, w = v.shape[:2]
    rows, cols = resize
    v = P.resize_area_one(u8, rows, cols) if (rows < h and cols < w) else P.resize_linear_one(v, rows, cols)
    if scale is not None:
        v = P.warp_affine_one(v, P.rotation_matrix(cols, rows, 0, scale))
    if angle is not None:
        v = P.warp_affine_one(v, P.rotation_matrix(cols, rows, angle, 1))
    f, oy, ox = params
    if f:
        v = np.fliplr(v)
    v = np.pad(v, ((pad_h, pad_h), (pad_w, pad_w), (0, 0)))
    return v[oy:oy + OH, ox:ox + OW].transpose(2, 0, 1)


@pytest.mark.parametrize("H,W,resize,crop", [(20, 28, (15, 20), 12), (12, 16, (15, 20), 12), (12, 16, (15, 20), 18)])
def test_full_transform_chain_bit_exact(H, W, resize, crop):
    """transform.transforms(resize, scale=0.05, angle=15, flip_prob=0.5, crop_size) on (img, mask, target)."""
    rng = np.random.default_rng(H * 3 + crop)
    srcs = [rng.integers(0, 256, (3, H, W, 3), dtype=np.uint8), rng.integers(0, 256, (3, H, W), dtype=np.uint8),
            rng.integers(0, 256, (3, H, W, 3), dtype=np.uint8)]
    outs, params = data.prepare_samples([torch.from_numpy(s).cuda() for s in srcs], flip_prob=0.5, crop_size=crop,
                                        resize=resize, scale=0.05, angle=15, rng=np.random.RandomState(3))
    scales, angles, p2, geom = data.draw_params(3, *resize, 0.05, 15, 0.5, crop, rng=np.random.RandomState(3))
    np.testing.assert_array_equal(params, p2)
    for src, got in zip(srcs, outs):
        for b in range(3):
            want = _oracle_chain(src[b], resize, scales[b], angles[b], params[b], geom)
            np.testing.assert_array_equal(got[b].cpu().numpy(), want)


def test_istd_loader_end_to_end(tmp_path):
    """ISTDLoader (train transforms at toy size) against the oracle chain on the same PNG files; two
    ranks' shards concatenate to the single-rank batch."""
    from PIL import Image
    import os
    rng = np.random.default_rng(4)
    for sub in ("A", "B", "matte", "C_fixed"):
        os.makedirs(tmp_path / "train" / f"train_{sub}")
        for i in range(6):
            shape = (20, 26) if sub in ("B", "matte") else (20, 26, 3)
            Image.fromarray(rng.integers(0, 256, shape, dtype=np.uint8)).save(
                tmp_path / "train" / f"train_{sub}" / f"{i:02d}.png")
    kw = dict(resize=(15, 20), scale=0.05, angle=15, flip_prob=0.5, crop_size=12, shuffle=True, drop_last=True,
              workers=2)
    torch.manual_seed(0)
    ld = data.ISTDLoader(str(tmp_path), "train", 4, **kw)
    batches = list(ld)
    torch.manual_seed(0)
    plan = list(ld.schedule())
    assert len(batches) == 1 and len(plan) == 1
    sel, stream = plan[0]
    scales, angles, params, geom = data.draw_params(4, 15, 20, 0.05, 15, 0.5, 12, rng=stream)
    names, img, mask, target = batches[0]
    assert names == [f"{i:02d}" for i in sel]
    for k, (got, sub) in enumerate(((img, "A"), (mask, "B"), (target, "C_fixed"))):
        for b, i in enumerate(sel):
            u = np.asarray(Image.open(tmp_path / "train" / f"train_{sub}" / f"{i:02d}.png"))
            u = u if u.ndim == 2 else np.ascontiguousarray(u[:, :, ::-1])
            want = _oracle_chain(u, (15, 20), scales[b], angles[b], params[b], geom)
            np.testing.assert_array_equal(got[b].cpu().numpy(), want)
    shards = []
    for r in range(2):
        torch.manual_seed(0)
        shards.append(list(data.ISTDLoader(str(tmp_path), "train", 4, rank=r, world=2, **kw))[0])
    assert shards[0][0] + shards[1][0] == names
    for t in (1, 2, 3):
        torch.testing.assert_close(torch.cat([shards[0][t], shards[1][t]]), batches[0][t], rtol=0, atol=0)
