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
