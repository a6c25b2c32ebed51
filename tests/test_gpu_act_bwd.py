"""Input-gradient conv with the activation backward of a layer without BatchNorm in its epilogue
(stc_conv_bwd_act, csrc/igemm_bf16.hpp BNB epilogue with bnb_act): G's outermost level (LeakyReLU into conv_1,
ReLU into the skip, STCGAN/networks.py:99-106) and the PatchGAN's first layer (LeakyReLU, networks.py:165-166).
It must equal the two-call form -- the conv into a gradient tensor, then stc_bn_bwd_apply with no table -- bit for
bit, and torch fp32 within the bf16 tolerance; the train step with and without it must be bit-identical."""
import types

import pytest
import torch
import torch.nn.functional as F

from stcgan_amd import _lib as L
from stcgan_amd import ops
from stcgan_amd.stcgan import STCGAN

pytestmark = pytest.mark.gpu

DEV = "cuda"
BF = torch.bfloat16


@pytest.mark.parametrize("B,with_other", [(4, True), (4, False), (32, True), (7, False)],
                         ids=["b4_skip", "b4_single", "b32_skip", "b7_single"])
def test_conv_act_backward_matches_two_call_form(B, with_other):
    """conv_1's input gradient (dr_1 at 64x64x128 -> 128x128x64, the ConvT geometry of a conv-s2 input gradient)."""
    Cin, Cout, Hg = 128, 64, 64
    g = torch.Generator(device=DEV).manual_seed(31 + B + with_other)
    w = torch.randn((Cin, Cout, 4, 4), generator=g, device=DEV) * 0.05  # conv_1 weight [128][64]
    wd = ops.pack(L.PACK_CONV_DGRAD, w, Cout, Cin, BF)
    dy = (torch.randn((B, Hg, Hg, Cin), generator=g, device=DEV) * 0.5).to(BF)
    x = torch.randn((B, 2 * Hg, 2 * Hg, Cout), generator=g, device=DEV).to(BF)  # the activation's input
    x[:, :3, :3] = 0  # exact zeros: act'(0) takes the slope branch in both forms
    go = (torch.randn((B, 2 * Hg, 2 * Hg, Cout), generator=g, device=DEV) * 0.5).to(BF) if with_other else None
    s_self, s_other = 0.2, 0.0
    out1 = torch.full((B, 2 * Hg, 2 * Hg, Cout), float("nan"), device=DEV, dtype=BF)
    assert ops.conv_act_backward(L.CONVT_S2, B, L.nhwc_view(dy), Cin, wd, Cout, L.nhwc_view(out1), BF,
                                 act_x=L.nhwc_view(x), s_self=s_self,
                                 g_other=None if go is None else L.nhwc_view(go), s_other=s_other)
    # the two-call form: conv into a gradient tensor, then the activation backward with no table
    ga = torch.empty((B, 2 * Hg, 2 * Hg, Cout), device=DEV, dtype=BF)
    ops.conv(L.CONVT_S2, B, L.nhwc_view(dy), Cin, wd, Cout, L.nhwc_view(ga), BF)
    out2 = torch.empty_like(out1)
    if go is None:
        ops.bn_backward(B, L.nhwc_view(x), Cout, BF, L.nhwc_view(out2), g1=L.nhwc_view(ga), s1=s_self)
    else:
        ops.bn_backward(B, L.nhwc_view(x), Cout, BF, L.nhwc_view(out2), g1=L.nhwc_view(go), s1=s_other,
                        g2=L.nhwc_view(ga), s2=s_self)
    torch.cuda.synchronize()
    assert torch.equal(out1, out2)
    # torch fp32: the conv's input gradient through the activations
    gin = F.conv_transpose2d(dy.permute(0, 3, 1, 2).float(), w.to(BF).float(), None, 2, 1)
    xs = x.permute(0, 3, 1, 2).float()
    ref = gin * torch.where(xs > 0, 1.0, s_self)
    if go is not None:
        ref = ref + go.permute(0, 3, 1, 2).float() * torch.where(xs > 0, 1.0, s_other)
    err = float((out1.permute(0, 3, 1, 2).float() - ref).abs().max())
    assert err <= 1e-2 * float(ref.abs().max()), err


def test_conv_act_backward_declines_small_grid():
    """A grid the halo kernels do not take (too few blocks): nothing launched, the caller runs the two-call form."""
    B, Cin, Cout, Hg = 2, 128, 64, 64
    wd = ops.pack(L.PACK_CONV_DGRAD, torch.zeros((Cin, Cout, 4, 4), device=DEV), Cout, Cin, BF)
    dy = torch.zeros((B, Hg, Hg, Cin), device=DEV, dtype=BF)
    x = torch.zeros((B, 2 * Hg, 2 * Hg, Cout), device=DEV, dtype=BF)
    out = torch.full_like(x, 7.0)
    assert not ops.conv_act_backward(L.CONVT_S2, B, L.nhwc_view(dy), Cin, wd, Cout, L.nhwc_view(out), BF,
                                     act_x=L.nhwc_view(x), s_self=0.2)
    torch.cuda.synchronize()
    assert bool((out == 7.0).all())


def _train(fuse, loss_type):
    prev = ops.FUSE_ACT_BWD
    ops.FUSE_ACT_BWD = fuse
    try:
        torch.manual_seed(5)
        a = types.SimpleNamespace(devices=["cuda:0"], tasks=["train"], lr_G=5e-5, lr_D=2e-5, beta1=0.5, beta2=0.999,
                                  D_loss_fn="standard", D_loss_type=loss_type, ngf=64, dtype="bf16",
                                  load_weights_g1=None, load_weights_g2=None, load_weights_d1=None,
                                  load_weights_d2=None)
        tr = STCGAN(a)
        g = torch.Generator().manual_seed(13)
        x, m, y = (torch.rand((4, c, 256, 256), generator=g).cuda() * 2 - 1 for c in (3, 1, 3))
        losses = [{k: float(v) for k, v in tr.train_step(x, m, y).items()} for _ in range(2)]
        torch.cuda.synchronize()
        state = {n: {k: v.cpu() for k, v in getattr(tr, n).state_dict().items()} for n in ("G1", "G2", "D1", "D2")}
    finally:
        ops.FUSE_ACT_BWD = prev
    return state, losses


@pytest.mark.parametrize("loss_type", ["normal", "rel_avg"])
def test_train_step_bit_identical_with_fused_act_backward(loss_type):
    ref_state, ref_losses = _train(False, loss_type)
    state, losses = _train(True, loss_type)
    assert losses == ref_losses
    for n, sd in ref_state.items():
        for k, v in sd.items():
            assert torch.equal(state[n][k], v), (n, k)
