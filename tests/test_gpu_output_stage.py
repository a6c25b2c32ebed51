"""GPU parity of the infer() output stage (stc_infer_output) against the CPU oracle
(oracle/output_stage.py): uint8 images bit-exact at the reference's sizes -- 256x256 and the
native 480x640 ISTD resolution resized to 256x192, an exact 2x downscale (INTER_AREA branch), the
identity size -- and STCGAN.infer() end to end (PNG files == oracle of the generator outputs)."""
import numpy as np
import pytest
import torch

from oracle import output_stage as O
from stcgan_amd import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,C,H,W", [(2, 1, 256, 256), (2, 3, 256, 256), (3, 3, 480, 640), (2, 1, 480, 640),
                                     (2, 3, 384, 512), (1, 3, 192, 256), (1, 1, 7, 9), (0, 3, 256, 256)])
def test_infer_output_bit_exact(B, C, H, W):
    g = torch.Generator().manual_seed(B * 1000 + C * 100 + H)
    x = torch.tanh(torch.randn((B, C, H, W), generator=g) * 2)
    if B:
        x[0, 0, :4, :4] = 1.0  # saturated corners: 255 exactly
        x[-1, -1, -4:, -4:] = -1.0
    got = ops.infer_output(x.cuda(), 192, 256).cpu().numpy()
    want = O.infer_output(x.numpy(), 192, 256)
    assert got.shape == want.shape == (B, 192, 256, C)
    np.testing.assert_array_equal(got, want)


def test_infer_end_to_end_writes_reference_pngs(tmp_path):
    import types
    from PIL import Image
    from stcgan_amd.stcgan import STCGAN

    torch.manual_seed(3)
    args = types.SimpleNamespace(devices=["cuda:0"], tasks=["infer", "train"], lr_G=5e-5, lr_D=2e-5, beta1=0.5,
                                 beta2=0.999, ngf=8, dtype="fp32", infered=str(tmp_path), load_weights_g1=None,
                                 load_weights_g2=None, load_weights_d1=None, load_weights_d2=None)
    tr = STCGAN(args)
    x = torch.rand((2, 3, 256, 256)) * 2 - 1
    tr.valid_loader = [(["a", "b"], x, None, None)]
    res = tr.infer()
    with torch.no_grad():
        m = tr.G1(x.cuda())
        y = tr.G2([x.cuda(), m])
    m_ref = O.infer_output(m.cpu().numpy())
    y_ref = O.infer_output(y.cpu().numpy())
    for i, name in enumerate(["a", "b"]):
        assert res[i][0] == name
        np.testing.assert_array_equal(res[i][1], m_ref[i, :, :, 0])
        np.testing.assert_array_equal(res[i][2], y_ref[i])
        mk = np.asarray(Image.open(tmp_path / "mask" / f"{name}.png"))
        sl = np.asarray(Image.open(tmp_path / "shadowless" / f"{name}.png"))[:, :, ::-1]  # file RGB -> BGR
        np.testing.assert_array_equal(mk, m_ref[i, :, :, 0])
        np.testing.assert_array_equal(sl, y_ref[i])
