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


class _BNT:
    def __init__(self, C, seed):
        g = torch.Generator().manual_seed(seed)
        self.scale = (torch.rand(C, generator=g) + 0.5).to(DEV)
        self.shift = (torch.randn(C, generator=g) * 0.2).to(DEV)
        self.mean = (torch.randn(C, generator=g) * 0.1).to(DEV)
        self.rstd = (torch.rand(C, generator=g) + 0.5).to(DEV)
        self.gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)


@pytest.mark.parametrize("with_other", [False, True], ids=["no_other", "g_other"])
def test_stem_bn_backward(with_other):
    """G's output-layer input gradient (dq 256x256x8 -> the 128-channel concat gradient at 128x128) with the
    up-path BN's backward sums on channels 64..127: the streaming kernel against the im2col tile + the separate BN
    backward (same outputs bit for bit, sums within fp32 reordering)."""
    B, Cin, Cout, C, ch_off = 4, 8, 128, 64, 64
    g = torch.Generator(device=DEV).manual_seed(7 + with_other)
    wt = torch.randn((Cin, Cout, 4, 4), generator=g, device=DEV) * 0.05  # the ConvT weight [8][128]
    w = ops.pack(L.PACK_CONVT_DGRAD, wt, Cout, Cin, BF)
    dq = (torch.randn((B, 256, 256, Cin), generator=g, device=DEV) * 0.5).to(BF)
    x = torch.randn((B, 128, 128, C), generator=g, device=DEV).to(BF)
    go = torch.randn((B, 128, 128, C), generator=g, device=DEV).to(BF) if with_other else None
    bn = _BNT(C, 55)
    st = (bn.scale, bn.shift, bn.mean, bn.rstd)
    assert ops.conv_query(L.CONV_S2, B, 128, 128, Cin, Cout, BF)[2][4] != ops.HALO_CFG
    out1 = torch.zeros((B, 128, 128, Cout), device=DEV, dtype=BF)
    dx1 = torch.empty((B, 128, 128, C), device=DEV, dtype=BF)
    dg1, db1 = ops.conv_bn_backward(L.CONV_S2, B, L.nhwc_view(dq), Cin, w, Cout, L.nhwc_view(out1), BF,
                                    bn_x=L.nhwc_view(x), C=C, bn_state=st, gamma=bn.gamma, s_self=0.0, ch_off=ch_off,
                                    g_other=None if go is None else L.nhwc_view(go), s_other=0.2,
                                    dxv=L.nhwc_view(dx1))
    out2 = torch.zeros((B, 128, 128, Cout), device=DEV, dtype=BF)
    ops.conv(L.CONV_S2, B, L.nhwc_view(dq), Cin, w, Cout, L.nhwc_view(out2), BF)
    dx2 = torch.empty((B, 128, 128, C), device=DEV, dtype=BF)
    dg2, db2 = ops.bn_backward(B, L.nhwc_view(x), C, BF, L.nhwc_view(dx2), g1=L.nhwc_view(out2, ch_off), s1=0.0,
                               g2=None if go is None else L.nhwc_view(go), s2=0.2,
                               bn_state=(bn.scale, bn.shift, bn.mean, bn.rstd, bn.gamma))
    torch.cuda.synchronize()
    assert torch.equal(out1, out2)
    for a, b_, nm in ((dg1, dg2, "dgamma"), (db1, db2, "dbeta")):
        err = float((a - b_).abs().max())
        assert err <= 1e-4 * float(b_.abs().max()) + 1e-5, f"{nm}: {err:.3e}"
    err = float((dx1.float() - dx2.float()).abs().max())
    assert err <= 1e-2 * float(dx2.float().abs().max()), f"dx: {err:.3e}"


@pytest.mark.parametrize("B", [32, 3])
def test_stem_logits_dgrad_bn_backward(B):
    """The PatchGAN logits layer's input gradient (dy 30x30, 1 channel padded to 8 -> 31x31x512) with layer 4's
    BatchNorm-backward sums: the streaming kernel against the im2col conv + the separate BN backward."""
    Cin, Cout, C = 8, 512, 512
    g = torch.Generator(device=DEV).manual_seed(11 + B)
    wt = torch.zeros((Cin, Cout, 4, 4), device=DEV)
    wt[:1] = torch.randn((1, Cout, 4, 4), generator=g, device=DEV) * 0.05  # conv weight [1 (padded 8)][512]
    w = ops.pack(L.PACK_CONV_S1_DGRAD, wt, Cout, Cin, BF)
    dy = torch.zeros((B, 30, 30, Cin), device=DEV, dtype=BF)
    dy[..., :1] = (torch.randn((B, 30, 30, 1), generator=g, device=DEV) * 0.5).to(BF)
    x = torch.randn((B, 31, 31, C), generator=g, device=DEV).to(BF)
    bn = _BNT(C, 57)
    st = (bn.scale, bn.shift, bn.mean, bn.rstd)
    out1 = torch.zeros((B, 31, 31, Cout), device=DEV, dtype=BF)
    dx1 = torch.empty((B, 31, 31, C), device=DEV, dtype=BF)
    dg1, db1 = ops.conv_bn_backward(L.CONV_S1_DGRAD, B, L.nhwc_view(dy), Cin, w, Cout, L.nhwc_view(out1), BF,
                                    bn_x=L.nhwc_view(x), C=C, bn_state=st, gamma=bn.gamma, s_self=0.2,
                                    dxv=L.nhwc_view(dx1))
    out2 = torch.zeros((B, 31, 31, Cout), device=DEV, dtype=BF)
    ops.conv(L.CONV_S1_DGRAD, B, L.nhwc_view(dy), Cin, w, Cout, L.nhwc_view(out2), BF)
    dx2 = torch.empty((B, 31, 31, C), device=DEV, dtype=BF)
    dg2, db2 = ops.bn_backward(B, L.nhwc_view(x), C, BF, L.nhwc_view(dx2), g1=L.nhwc_view(out2), s1=0.2,
                               bn_state=(bn.scale, bn.shift, bn.mean, bn.rstd, bn.gamma))
    torch.cuda.synchronize()
    assert torch.equal(out1, out2)
    ref = torch.nn.functional.conv_transpose2d(dy.permute(0, 3, 1, 2).float(), wt.to(BF).float(), None, 1, 1)
    assert float((out1.permute(0, 3, 1, 2).float() - ref).abs().max()) <= 1e-2 * float(ref.abs().max())
    for a, b_, nm in ((dg1, dg2, "dgamma"), (db1, db2, "dbeta")):
        err = float((a - b_).abs().max())
        assert err <= 1e-4 * float(b_.abs().max()) + 1e-5, f"{nm}: {err:.3e}"
    err = float((dx1.float() - dx2.float()).abs().max())
    assert err <= 1e-2 * float(dx2.float().abs().max()), f"dx: {err:.3e}"
