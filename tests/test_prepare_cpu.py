"""CPU checks of the batch-preparation host logic (stcgan_amd.data.augment_params: the reference's
random-draw order) and of its oracle (oracle/prepare_ref.py) on hand cases."""
import numpy as np

from oracle import prepare_ref as P
from stcgan_amd import data


def test_params_follow_reference_draw_order():
    rs = np.random.RandomState(3)
    params, geom = data.augment_params(4, 300, 400, flip_prob=0.5, crop_size=256, rng=rs)
    ref = np.random.RandomState(3)
    for i in range(4):
        flip = 0 if ref.rand() > 0.5 else 1
        oy, ox = ref.randint(low=0, high=300 - 256), ref.randint(low=0, high=400 - 256)
        assert tuple(params[i]) == (flip, oy, ox)
    assert geom == (0, 0, 256, 256)


def test_padding_geometry():
    _, geom = data.augment_params(1, 200, 300, None, 256, rng=np.random.RandomState(0))
    assert geom == (56, 0, 256, 256)


def test_oracle_hand_case():
    img = np.array([[[0], [255]], [[51], [102]]], np.uint8)  # 2x2, one channel
    out = P.prepare_one(img, 1, 0, 0, 0, 0, 2, 2)
    want = (np.array([[255, 0], [102, 51]], np.float32) / np.float32(255) - np.float32(0.5)) * np.float32(2)
    np.testing.assert_array_equal(out[0], want)
    padded = P.prepare_one(img, 0, 0, 0, 1, 1, 2, 2)  # top-left corner of the 1-pixel zero border
    assert padded[0, 0, 0] == 0.0 and padded[0, 0, 1] == 0.0 and padded[0, 1, 0] == 0.0 and padded[0, 1, 1] == -1.0


def test_area_oracle_cells_and_fast_path():
    # 4 -> 2 per axis is an integer scale: the block mean
    img = np.arange(16, dtype=np.uint8).reshape(4, 4) * 16
    r = P.resize_area_one(img, 2, 2)[:, :, 0]
    v = (img.astype(np.float32) / np.float32(255) - np.float32(0.5)) * np.float32(2)
    np.testing.assert_allclose(r, v.reshape(2, 2, 2, 2).mean(axis=(1, 3)), atol=2e-7)
    # 5 -> 2 (scale 2.5): cells [0,2.5) and [2.5,5): weights 0.4, 0.4, 0.2 | 0.2, 0.4, 0.4
    tab = P._area_tab(2, 5, 2.5)
    assert [s for s, _ in tab[0]] == [0, 1, 2] and [s for s, _ in tab[1]] == [2, 3, 4]
    np.testing.assert_allclose([a for _, a in tab[0]], [0.4, 0.4, 0.2], rtol=1e-6)
    np.testing.assert_allclose([a for _, a in tab[1]], [0.2, 0.4, 0.4], rtol=1e-6)


def test_draw_order_with_scale_and_angle():
    """transform.transforms(scale, angle, flip, crop): per sample uniform, uniform, rand, randint x2
    (transform.py:67, 91, 109, 141-142)."""
    scales, angles, params, geom = data.draw_params(3, 300, 400, 0.05, 15, 0.5, 256, rng=np.random.RandomState(9))
    ref = np.random.RandomState(9)
    for i in range(3):
        assert scales[i] == ref.uniform(low=0.95, high=1.05)
        assert angles[i] == ref.uniform(low=-15, high=15)
        flip = 0 if ref.rand() > 0.5 else 1
        assert tuple(params[i]) == (flip, ref.randint(low=0, high=44), ref.randint(low=0, high=144))
    assert geom == (0, 0, 256, 256)


def test_crop_of_exact_size_raises_like_reference():
    # np.random.randint(low=0, high=0) raises in RandomCrop when an image side equals the crop side
    import pytest
    with pytest.raises(ValueError):
        data.draw_params(1, 256, 300, crop_size=256, rng=np.random.RandomState(0))


def test_rotation_matrix_matches_oracle():
    for cols, rows, a, s in ((400, 300, 12.5, 1.0), (256, 256, 0, 1.04), (7, 5, -90, 0.5)):
        np.testing.assert_array_equal(data.rotation_matrix(cols, rows, a, s), P.rotation_matrix(cols, rows, a, s))


def test_linear_resize_oracle_known_answer():
    # 2 -> 4 per axis: weights (1), (.75,.25), (.25,.75), (1) with the borders clamped
    v = np.array([[[0.0], [1.0]], [[2.0], [3.0]]], np.float32)
    r = P.resize_linear_one(v, 4, 4)[:, :, 0]
    row = lambda a, b: [a, .75 * a + .25 * b, .25 * a + .75 * b, b]  # noqa: E731
    top, bot = row(0., 1.), row(2., 3.)
    want = np.array([top, [.75 * t + .25 * u for t, u in zip(top, bot)], [.25 * t + .75 * u for t, u in zip(top, bot)],
                     bot], np.float32)
    np.testing.assert_allclose(r, want, atol=1e-7)
    np.testing.assert_array_equal(P.resize_linear_one(v, 2, 2), v)


def test_warp_oracle_known_answers():
    rng = np.random.default_rng(1)
    v = P.normalise(rng.integers(0, 256, (6, 8, 3), dtype=np.uint8))
    np.testing.assert_array_equal(P.warp_affine_one(v, P.rotation_matrix(8, 6, 0, 1)), v)
    np.testing.assert_array_equal(P.warp_affine_one(v, P.rotation_matrix(8, 6, 180, 1)), v[::-1, ::-1])
    sq = P.normalise(rng.integers(0, 256, (5, 5, 1), dtype=np.uint8))
    np.testing.assert_array_equal(P.warp_affine_one(sq, P.rotation_matrix(5, 5, 90, 1)), np.rot90(sq))
    # a pure shift by half a pixel: every output is the mean of two neighbours (weights 16/32)
    M = np.array([[1, 0, 0.5], [0, 1, 0]], np.float64)
    w = P.warp_affine_one(v, M)
    np.testing.assert_allclose(w[:, 1:], (v[:, :-1] * np.float32(.5) + v[:, 1:] * np.float32(.5)), atol=1e-7)
    np.testing.assert_allclose(w[:, 0], v[:, 0] * np.float32(.5), atol=1e-7)  # the zero border


class _Probe:
    """A dataset whose items are the reference transforms' draws on the global np.random."""

    def __init__(self, n, H, W, aug):
        self.n, self.H, self.W, self.aug = n, H, W, aug

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        s, a, p, _ = data.draw_params(1, self.H, self.W, rng=np.random, **self.aug)
        return i, float(s[0]), float(a[0]), p[0].tolist()


def _worker_init(wid):
    np.random.seed(42 + wid)


def _loader_schedule(loader, H, W):
    out = []
    for sel, rng in loader.schedule():
        s, a, p, _ = data.draw_params(len(sel), H, W, rng=rng, **loader.aug)
        out.append([(i, float(s[k]), float(a[k]), p[k].tolist()) for k, i in enumerate(sel)])
    return out


def _make_istd(root, n):
    import os
    from PIL import Image
    rng = np.random.default_rng(0)
    for sub in ("A", "B", "matte", "C_fixed"):
        d = os.path.join(root, "train", f"train_{sub}")
        os.makedirs(d)
        for i in range(n):
            shape = (6, 8) if sub in ("B", "matte") else (6, 8, 3)
            Image.fromarray(rng.integers(0, 256, shape, dtype=np.uint8)).save(os.path.join(d, f"{i:03d}.png"))


def test_loader_streams_match_torch_dataloader(tmp_path):
    """ISTDLoader's sample order and transform draws equal a real torch DataLoader's (shuffle from
    torch's global generator, workers seeded 42 + id, batch s on worker s % workers)."""
    import torch
    from torch.utils.data import DataLoader
    _make_istd(str(tmp_path), 10)
    aug = dict(scale=0.05, angle=15, flip_prob=0.5, crop_size=4)
    for workers in (0, 2):
        probe = _Probe(10, 6, 8, aug)
        dl = DataLoader(probe, batch_size=3, shuffle=True, drop_last=True, num_workers=workers,
                        worker_init_fn=_worker_init, collate_fn=list)
        ours = data.ISTDLoader(str(tmp_path), "train", 3, shuffle=True, drop_last=True, workers=workers, **aug)
        for epoch in range(2):
            torch.manual_seed(100 + epoch)
            np.random.seed(5 + epoch)
            want = [list(b) for b in dl]
            torch.manual_seed(100 + epoch)
            np.random.seed(5 + epoch)
            got = _loader_schedule(ours, 6, 8)
            assert got == want, (workers, epoch)
    assert len(ours) == 3


def test_loader_files_and_shards(tmp_path):
    _make_istd(str(tmp_path), 5)
    ld = data.ISTDLoader(str(tmp_path), "train", 4, datas=("target", "img", "mask"))
    assert ld.datas == ["img", "mask", "target"] and ld.names == [f"{i:03d}" for i in range(5)]
    assert len(ld) == 2
    im = ld._read("img", 0)
    from PIL import Image
    rgb = np.asarray(Image.open(str(tmp_path / "train" / "train_A" / "000.png")))
    np.testing.assert_array_equal(im, rgb[:, :, ::-1])  # BGR, as cv.imread
    assert ld._read("mask", 0).shape == (6, 8)
    assert [data.shard_bounds(10, r, 4) for r in range(4)] == [(0, 3), (3, 6), (6, 8), (8, 10)]
    assert [data.shard_bounds(8, r, 2) for r in range(2)] == [(0, 4), (4, 8)]
