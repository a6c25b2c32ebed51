"""Deep split-K conv + train-mode BatchNorm + activation in one post-GEMM launch (stc_conv_fwd_bn_act,
splitk_bn_act_kernel) against the three launches it replaces (stc_conv_fwd_ex's split-K reduce with partial
statistics, stc_bn_finalize, stc_bn_apply) -- the Conv -> BatchNorm2d -> LeakyReLU / ReLU of the generator's
deep levels, STCGAN/networks.py:104-128.

The raw conv output is bit-identical where the fused launch keeps the reduce's slab order (> 1024 rows; below
that it sums slab groups: within one bf16 step); mean / rstd / scale / shift / running statistics
agree to 1e-5 relative (two-pass fp64 vs Chan-merged partials); the activations are bit-identical to
stc_bn_apply run with the fused launch's own tables, and a second call is bit-identical to the first.
"""
import pytest
import torch

from stcgan_amd import _lib as L
from stcgan_amd import ops


@pytest.fixture(autouse=True)
def _fused_on(monkeypatch):
    monkeypatch.setattr(ops, "FUSE_BN_ACT", True)  # opt-in in the product path

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16

# (kind, B, gh, gw, cin, cout, crop): conv_s2 output grid / ConvT input grid gh x gw; crop: activations cover
# (H - crop) x (W - crop) of the output (the decoder's odd levels)
CASES = [
    (L.CONV_S2, 32, 8, 8, 256, 512, 0),
    (L.CONV_S2, 32, 4, 4, 512, 512, 0),
    (L.CONV_S2, 32, 2, 2, 512, 512, 0),
    (L.CONV_S2, 5, 3, 3, 512, 512, 0),
    (L.CONVT_S2, 32, 1, 1, 512, 512, 0),
    (L.CONVT_S2, 32, 4, 4, 1024, 512, 0),
    (L.CONVT_S2, 32, 2, 2, 1024, 512, 1),
]


def R_WIDE(kind, B, gh, gw):
    """GEMM rows few enough (<= 1024) that the fused launch splits each row's slabs into >= 2 groups (and the
    separate path may take the wide reduce): the fp32 sums differ from the separate path's in order."""
    return (4 if kind == L.CONVT_S2 else 1) * B * gh * gw <= 1024


def _io(kind, B, gh, gw, cin, cout, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    xh, xw, yh, yw = (gh, gw, 2 * gh, 2 * gw) if kind == L.CONVT_S2 else (2 * gh, 2 * gw, gh, gw)
    x = (torch.randn((B, xh, xw, cin), device=DEV, generator=g) * 0.5).to(BF)
    taps, nph = (4, 4) if kind == L.CONVT_S2 else (16, 1)
    w = (torch.randn((nph, cout, taps, cin), device=DEV, generator=g) * 0.05).to(BF)
    return x, w, yh, yw


def _bn(cout, seed):
    torch.manual_seed(seed)
    bn = torch.nn.BatchNorm2d(cout).to(DEV)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-0.1, 0.1)
        bn.running_var.uniform_(0.9, 1.1)
    return bn


def _close(a, b, rel):
    scale = max(float(b.abs().max()), 1e-6)
    return float((a - b).abs().max()) <= rel * scale


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"k{c[0]}B{c[1]}g{c[2]}c{c[4]}-{c[5]}crop{c[6]}")
def test_fused_bn_act_matches_separate(case):
    kind, B, gh, gw, cin, cout, crop = case
    x, w, yh, yw = _io(kind, B, gh, gw, cin, cout)
    ah, aw = yh - crop, yw - crop
    xv = L.nhwc_view(x)
    # separate launches
    y0 = torch.zeros((B, yh, yw, cout), device=DEV, dtype=BF)
    bn0 = _bn(cout, 5)
    t0 = torch.empty((2, cout), device=DEV)
    part, nch = ops.conv_stats(kind, B, xv, cin, w, cout, L.nhwc_view(y0), BF)
    m0, r0 = ops.bn_finalize_part(part, nch, cout, bn0, t0[0], t0[1])
    # fused, twice, with two activations (LeakyReLU 0.2 + ReLU) into a wider concat buffer
    assert L.lib().stc_conv_fwd_bn_act_ok(L.dtype_code(BF), kind, B, xv, cin, cout, L.nhwc_view(y0)) == 1
    outs = []
    for _ in range(2):
        bn1 = _bn(cout, 5)
        t1 = torch.empty((2, cout), device=DEV)
        y1 = torch.zeros((B, yh, yw, cout), device=DEV, dtype=BF)
        a1 = torch.full((B, ah, aw, cout), 7.0, device=DEV, dtype=BF)
        a2 = torch.full((B, ah, aw, 2 * cout), 7.0, device=DEV, dtype=BF)
        st = ops.conv_bn_act(kind, B, xv, cin, w, cout, L.nhwc_view(y1), BF, bn1, t1[0], t1[1],
                             L.nhwc_view(a1, 0, ah, aw), 0.2, L.nhwc_view(a2, cout, ah, aw), 0.0)
        assert st is not None
        torch.cuda.synchronize()
        outs.append((y1, a1, a2, st[0], st[1], t1, bn1.running_mean.clone(), bn1.running_var.clone(),
                     int(bn1.num_batches_tracked)))
    y1, a1, a2, m1, r1, t1, rm1, rv1, nbt1 = outs[0]
    if R_WIDE(kind, B, gh, gw):
        # slab groups (fused) / lanes over the splits (wide reduce) sum in another fp32 order: the bf16 raw
        # outputs agree to one bf16 rounding step (plus fp32 cancellation near zero)
        d = (y1.float() - y0.float()).abs()
        tol = y0.float().abs() * 2.0 ** -7 + 1e-5 * float(y0.float().abs().max())  # + fp32 cancellation
        assert bool((d <= tol).all()), "raw conv output off by > 1 bf16 step"
    else:
        assert torch.equal(y1, y0), "raw conv output differs from the split-K reduce"
    assert _close(m1, m0, 1e-5) and _close(r1, r0, 1e-5)
    assert _close(t1[0], t0[0], 1e-5) and _close(t1[1], t0[1], 1e-5)
    assert _close(rm1, bn0.running_mean, 1e-5) and _close(rv1, bn0.running_var, 1e-5)
    assert nbt1 == int(bn0.num_batches_tracked) == 1
    # activations == stc_bn_apply over the raw output with the fused launch's tables
    e1 = torch.zeros_like(a1)
    e2 = torch.full_like(a2, 7.0)
    ops.bn_apply(B, L.nhwc_view(y1, 0, ah, aw), cout, BF, (t1[0], t1[1]), L.nhwc_view(e1), 0.2,
                 L.nhwc_view(e2, cout, ah, aw), 0.0)
    torch.cuda.synchronize()
    assert torch.equal(a1, e1) and torch.equal(a2, e2)
    assert bool((a2[..., :cout] == 7.0).all()), "write outside the activation view"
    for u, v in zip(outs[0][:8], outs[1][:8]):
        assert torch.equal(u, v), "fused BatchNorm launch is not deterministic"


def test_fused_bn_act_declines_shallow_layers():
    """Only split-K layers with <= 2048 GEMM rows take the fused launch; conv_bn_act returns None otherwise."""
    x, w, yh, yw = _io(L.CONV_S2, 32, 32, 32, 64, 128)
    y = torch.zeros((32, yh, yw, 128), device=DEV, dtype=BF)
    assert L.lib().stc_conv_fwd_bn_act_ok(L.dtype_code(BF), L.CONV_S2, 32, L.nhwc_view(x), 64, 128,
                                          L.nhwc_view(y)) == 0
    bn = _bn(128, 1)
    t = torch.empty((2, 128), device=DEV)
    assert ops.conv_bn_act(L.CONV_S2, 32, L.nhwc_view(x), 64, w, 128, L.nhwc_view(y), BF, bn, t[0], t[1],
                           L.nhwc_view(y), 0.2) is None
    assert int(bn.num_batches_tracked) == 0
