"""BatchNorm finalize fused into the producing conv (stc_conv_fwd_bnfin / stc_conv_bwd_bnfin, csrc/bnfin.hpp)
against the separate kernels it replaces (stc_conv_fwd_ex + stc_bn_finalize; stc_conv_bwd_bn + the dbeta/dgamma
reduction of stc_bn_bwd_apply) -- the BatchNorm2d train forward / backward of STCGAN/networks.py:107,109,170,179.

Both merge the same chunk partials in a fixed order (the fused form in two levels), so they agree to fp64
rounding of the merge: mean / rstd / scale / shift / running statistics to 1e-5 relative, dbeta / dgamma to
1e-5 of max|.|.  Covered: the in-epilogue path (one and several channel tiles, one and two merge levels), the
split-K reduction path, the wide split-K path (its separate-launch fallback) and the fp32 parity path; a second
call is bit-identical to the first (deterministic), and the ticket counters are left at zero.
"""
import pytest
import torch

from stcgan_amd import _lib as L
from stcgan_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16

# (kind, B, gh, gw, cin, cout): output grid gh x gw (ConvT: input grid)
CASES = [
    (L.CONV_S2, 2, 32, 32, 64, 128),     # 16 tiles: one merge level
    (L.CONV_S2, 8, 32, 32, 64, 128),     # 64 tiles: two levels
    (L.CONV_S2, 8, 16, 16, 128, 512),    # several channel tiles
    (L.CONVT_S2, 8, 16, 16, 256, 128),   # 4 phases x tiles
    (L.CONV_S2, 8, 4, 4, 512, 512),      # split-K reduction
    (L.CONV_S2, 8, 1, 1, 512, 512),      # wide split-K reduction (separate finalize launch)
]


def _io(kind, B, gh, gw, cin, cout, dt, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    if kind == L.CONVT_S2:
        xh, xw, yh, yw = gh, gw, 2 * gh, 2 * gw
    else:
        xh, xw, yh, yw = 2 * gh, 2 * gw, gh, gw
    x = (torch.randn((B, xh, xw, cin), device=DEV, generator=g) * 0.5).to(dt)
    taps, nph = (4, 4) if kind == L.CONVT_S2 else (16, 1)
    w = (torch.randn((nph, cout, taps, cin), device=DEV, generator=g) * 0.05).to(dt)
    y = torch.zeros((B, yh, yw, cout), device=DEV, dtype=dt)
    return x, w, y


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


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"k{c[0]}B{c[1]}g{c[2]}c{c[4]}-{c[5]}")
@pytest.mark.parametrize("dt", [BF, torch.float32], ids=["bf16", "fp32"])
def test_fwd_fused_finalize_matches_separate(case, dt):
    kind, B, gh, gw, cin, cout = case
    if dt == torch.float32 and cin * cout > 128 * 128:
        pytest.skip("fp32 parity path: one shape suffices")
    x, w, y = _io(kind, B, gh, gw, cin, cout, dt)
    xv, yv = L.nhwc_view(x), L.nhwc_view(y)
    # separate kernels
    bn0 = _bn(cout, 5)
    t0 = torch.empty((2, cout), device=DEV)
    part, nch = ops.conv_stats(kind, B, xv, cin, w, cout, yv, dt)
    m0, r0 = ops.bn_finalize_part(part, nch, cout, bn0, t0[0], t0[1])
    y0 = y.clone()
    # fused, twice (fresh module state each time): deterministic and counters back at zero
    outs = []
    for _ in range(2):
        bn1 = _bn(cout, 5)
        t1 = torch.empty((2, cout), device=DEV)
        y.zero_()
        m1, r1 = ops.conv_stats_fin(kind, B, xv, cin, w, cout, yv, dt, bn1, t1[0], t1[1])
        torch.cuda.synchronize()
        outs.append((m1, r1, t1, bn1.running_mean.clone(), bn1.running_var.clone(), int(bn1.num_batches_tracked)))
        cnt = bn1.__dict__["_stc_fin"][(str(w.device), "fwd")][0]
        assert int(cnt.abs().sum()) == 0, "ticket counters not left at zero"
    assert torch.equal(y, y0), "conv output differs"
    m1, r1, t1, rm1, rv1, nbt1 = outs[0]
    assert _close(m1, m0, 1e-5) and _close(r1, r0, 1e-5)
    assert _close(t1[0], t0[0], 1e-5) and _close(t1[1], t0[1], 1e-5)
    assert _close(rm1, bn0.running_mean, 1e-5) and _close(rv1, bn0.running_var, 1e-5)
    assert nbt1 == int(bn0.num_batches_tracked) == 1
    m2, r2, t2, rm2, rv2, _ = outs[1]
    for a, b in ((m1, m2), (r1, r2), (t1, t2), (rm1, rm2), (rv1, rv2)):
        assert torch.equal(a, b), "fused finalize is not deterministic"


@pytest.mark.parametrize("case", [c for c in CASES if c[0] == L.CONV_S2],
                         ids=lambda c: f"B{c[1]}g{c[2]}c{c[4]}-{c[5]}")
def test_bwd_fused_sums_match_separate(case):
    """Input-gradient conv (ConvT geometry over conv_s2's output grid) with the BN-backward reduction of the
    BatchNorm on its output fused in: dbeta/dgamma from the in-launch finalize vs stc_bn_bwd_apply's own."""
    kind, B, gh, gw, cin, cout = case
    # the dgrad of conv_s2 (cin -> cout, output grid gh x gw) is a ConvT from dy [B, gh, gw, cout] to
    # [B, 2gh, 2gw, cin]; its output feeds a BatchNorm over cin channels
    g = torch.Generator(device=DEV).manual_seed(11)
    dy = (torch.randn((B, gh, gw, cout), device=DEV, generator=g) * 0.5).to(BF)
    wd = (torch.randn((4, cin, 4, cout), device=DEV, generator=g) * 0.05).to(BF)
    bx = (torch.randn((B, 2 * gh, 2 * gw, cin), device=DEV, generator=g)).to(BF)
    scale = torch.rand(cin, device=DEV, generator=g) + 0.5
    shift = torch.rand(cin, device=DEV, generator=g) - 0.5
    mean = torch.randn(cin, device=DEV, generator=g) * 0.1
    rstd = torch.rand(cin, device=DEV, generator=g) + 0.5
    gamma = torch.rand(cin, device=DEV, generator=g) + 0.5
    res = []
    for fused in (False, True, True):
        bn = _bn(cin, 3)
        out = torch.zeros((B, 2 * gh, 2 * gw, cin), device=DEV, dtype=BF)
        dx = torch.zeros((B, 2 * gh, 2 * gw, cin), device=DEV, dtype=BF)
        dg, db = ops.conv_bn_backward(L.CONVT_S2, B, L.nhwc_view(dy), cout, wd, cin, L.nhwc_view(out), BF,
                                      bn_x=L.nhwc_view(bx), C=cin, bn_state=(scale, shift, mean, rstd), gamma=gamma,
                                      s_self=0.2, dxv=L.nhwc_view(dx), bn=bn if fused else None)
        torch.cuda.synchronize()
        res.append((out, dx, dg.clone(), db.clone()))
        if fused:
            cnt = bn.__dict__["_stc_fin"][(str(dy.device), "bwd")][0]
            assert int(cnt.abs().sum()) == 0
    (o0, x0, g0, b0), (o1, x1, g1, b1), (o2, x2, g2, b2) = res
    assert torch.equal(o0, o1)
    assert _close(g1, g0, 1e-5) and _close(b1, b0, 1e-5)
    assert float((x1.float() - x0.float()).abs().max()) <= 1e-2 * float(x0.float().abs().max())
    assert torch.equal(g1, g2) and torch.equal(b1, b2) and torch.equal(x1, x2)
