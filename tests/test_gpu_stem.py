"""The first-layer conv kernel (csrc/stem_bf16.hip: Conv2d k4 s2 p1, 8 input channels, 64 outputs, activation
epilogue) -- G's outermost down conv (STCGAN/networks.py:99) and D's first conv (:165-166) -- against the im2col GEMM
tile + stc_bn_apply (no table), which it must equal bit for bit (same K order and MFMA), and against torch fp32."""
import pytest
import torch
import torch.nn.functional as F

from stcgan_amd import _lib as L
from stcgan_amd import ops

pytestmark = pytest.mark.gpu

DEV = "cuda"
BF = torch.bfloat16


@pytest.mark.parametrize("case", [(2, 256, 1, False), (2, 256, 2, False), (3, 256, 1, True), (1, 512, 2, True)],
                         ids=["w256_one_out", "w256_two_out", "w256_bias", "w512_two_out_bias"])
def test_stem_conv_act(case):
    B, W, nout, with_bias = case
    g = torch.Generator(device=DEV).manual_seed(W + nout)
    x = torch.randn((B, W, W, 8), generator=g, device=DEV).to(BF)
    w = (torch.randn((64, 8, 4, 4), generator=g, device=DEV) * 0.1)
    b = torch.randn(64, generator=g, device=DEV) * 0.1 if with_bias else None
    wp = ops.pack(L.PACK_CONV_FWD, w, 64, 8, BF)
    Ho = W // 2
    # y1 dense; y2 the second half of a 128-channel buffer (the generator's skip concat)
    y1 = torch.full((B, Ho, Ho, 64), float("nan"), device=DEV, dtype=BF)
    y2b = torch.full((B, Ho, Ho, 128), float("nan"), device=DEV, dtype=BF)
    y2v = L.nhwc_view(y2b, 64) if nout == 2 else None
    assert ops.conv_act(L.CONV_S2, B, L.nhwc_view(x), 8, wp, 64, L.nhwc_view(y1), 0.2, BF, y2v, 0.0, bias=b)
    # reference path: the im2col tile's raw output, then the activation pass
    raw = torch.empty((B, Ho, Ho, 64), device=DEV, dtype=BF)
    ops.conv(L.CONV_S2, B, L.nhwc_view(x), 8, wp, 64, L.nhwc_view(raw), BF, bias=b)
    r1 = torch.empty_like(y1)
    r2 = torch.full((B, Ho, Ho, 128), float("nan"), device=DEV, dtype=BF)
    ops.bn_apply(B, L.nhwc_view(raw), 64, BF, None, L.nhwc_view(r1), 0.2,
                 L.nhwc_view(r2, 64) if nout == 2 else None, 0.0)
    torch.cuda.synchronize()
    assert torch.equal(y1, r1)
    if nout == 2:
        assert torch.equal(y2b[..., 64:], r2[..., 64:])
        assert torch.isnan(y2b[..., :64].float()).all()  # (the other half of the buffer untouched)
    ref = F.conv2d(x.permute(0, 3, 1, 2).float(), w.to(BF).float(), b, 2, 1)
    got = F.leaky_relu(ref, 0.2)
    err = float((y1.permute(0, 3, 1, 2).float() - got).abs().max())
    assert err <= 1e-2 * float(got.abs().max())
