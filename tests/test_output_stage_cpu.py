"""CPU checks of the infer() output-stage oracle (oracle/output_stage.py): hand-derived cases of
OpenCV's float32 INTER_LINEAR geometry and of float2uint's truncation (STCGAN/utils.py:63-65).
cv2 is absent here, so these cases -- not OpenCV itself -- pin the restatement (parity unpinned
against cv2; see the oracle's header)."""
import numpy as np

from oracle import output_stage as O

F32 = np.float32


def _scalar_resize(img, oh, ow):
    """Pixel-by-pixel float32 restatement (slow; small images only) -- cross-checks the vectorised
    oracle's indexing."""
    h, w = img.shape
    out = np.zeros((oh, ow), F32)
    for dy in range(oh):
        fy = F32((dy + 0.5) * (1.0 / (oh / h)) - 0.5)
        sy = int(np.floor(fy))
        fy = F32(fy - F32(sy))
        rows = (min(max(sy, 0), h - 1), min(max(sy + 1, 0), h - 1))
        for dx in range(ow):
            fx = F32((dx + 0.5) * (1.0 / (ow / w)) - 0.5)
            sx = int(np.floor(fx))
            fx = F32(fx - F32(sx))
            two = sx + 1 < w
            if sx < 0:
                sx, fx = 0, F32(0)
            if sx >= w - 1:
                sx, fx = w - 1, F32(0)
            hv = []
            for r in rows:
                a = F32(img[r, sx] * F32(F32(1) - fx))
                hv.append(F32(a + F32(img[r, sx + 1] * fx)) if two else a)
            out[dy, dx] = F32(F32(hv[0] * F32(F32(1) - fy)) + F32(hv[1] * fy))
    return out


def test_identity_size_is_plain_float2uint():
    rng = np.random.default_rng(0)
    x = np.tanh(rng.standard_normal((2, 3, 12, 16))).astype(F32)
    got = O.infer_output(x, 12, 16)
    want = ((x * F32(0.5) + F32(0.5)) * F32(255)).astype(np.uint8).transpose(0, 2, 3, 1)
    np.testing.assert_array_equal(got, want)


def test_float2uint_truncates():
    v = np.array([0.0, 0.999999, 1.0 / 255 - 1e-7, 1.0 / 255, 0.5, 1.0], F32)
    np.testing.assert_array_equal(O.float2uint(v), [0, 254, 0, 1, 127, 255])


def test_upscale_edges_and_weights():
    # W=2 -> OW=4 (scale 0.5): dx=0 clamps left (weight 0), dx=1: 0.75/0.25, dx=2: 0.25/0.75,
    # dx=3: single term past the right edge
    img = np.array([[0.25, 0.75]], F32)
    r = O.resize_linear(img, 1, 4)
    np.testing.assert_array_equal(r[0], np.array([0.25, 0.375, 0.625, 0.75], F32))


def test_downscale_rows_exact_midpoint():
    # H=4 -> OH=3 (scale 4/3): output row 1 samples source y=1.5 -> mean of rows 1 and 2
    img = np.array([[0.0], [0.25], [0.75], [1.0]], F32)
    r = O.resize_linear(img, 3, 1)
    assert r[1, 0] == F32(0.5)


def test_constant_image_stays_constant():
    for (h, w, oh, ow) in ((256, 256, 192, 256), (480, 640, 192, 256), (384, 512, 192, 256)):
        img = np.full((h, w, 3), 0.5, F32)
        r = O.resize_linear(img, oh, ow)
        assert r.shape == (oh, ow, 3)
        np.testing.assert_array_equal(r, 0.5)


def test_exact_2x_downscale_is_area_mean():
    img = np.arange(16, dtype=F32).reshape(4, 4) / F32(16)
    r = O.resize_linear(img, 2, 2)
    want = np.array([[img[0:2, 0:2].sum(), img[0:2, 2:4].sum()], [img[2:4, 0:2].sum(), img[2:4, 2:4].sum()]], F32) * F32(0.25)
    np.testing.assert_allclose(r, want, rtol=0, atol=1e-7)


def test_vectorised_oracle_matches_scalar_loop():
    rng = np.random.default_rng(1)
    for (h, w, oh, ow) in ((16, 12, 6, 10), (10, 10, 7, 13), (5, 40, 9, 16), (48, 64, 19, 25)):
        img = rng.random((h, w), dtype=np.float32)
        np.testing.assert_array_equal(O.resize_linear(img, oh, ow), _scalar_resize(img, oh, ow))
