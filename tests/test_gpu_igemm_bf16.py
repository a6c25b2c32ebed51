"""bf16 LDS-DMA implicit-GEMM kernel (csrc/igemm_bf16.hip) against torch fp32 references.

Every conv kind on the ST-CGAN path (Conv2d k4 s2/s1, ConvTranspose2d k4 s2 as 4 phases, the
conv-s1 input gradient), every tile configuration, split-K on/off, ragged M and N, channel-offset
output views (the zero-copy skip concat), and the BatchNorm statistics fused into the epilogue /
split-K reduction.  Operands are rounded to bf16 before the fp32 reference, so the only
differences are fp32 summation order and the final bf16 rounding of the output:
tolerance 1e-2 * max|ref| on outputs, 2e-3 relative on the per-channel mean/variance.
"""
import pytest
import torch
import torch.nn.functional as F

from stcgan_amd import _lib as L
from stcgan_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def rnd(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(shape, generator=g) * scale


def q(t):
    return t.to(BF).float()


def run(kind, B, x_nchw, w, Cin, Cout, out_shape, force=None, co=0, extra_c=0, bias=None):
    """Runs stc_conv_fwd_ex with stats; returns (y NCHW fp32, mean, var) on the CPU."""
    pack_mode = {L.CONV_S2: L.PACK_CONV_FWD, L.CONV_S1: L.PACK_CONV_FWD, L.CONVT_S2: L.PACK_CONVT_FWD,
                 L.CONV_S1_DGRAD: L.PACK_CONV_S1_DGRAD}[kind]
    xg = nhwc(x_nchw).to(DEV, BF)
    wp = ops.pack(pack_mode, w.to(DEV), Cout, Cin, BF)
    Ho, Wo = out_shape
    Ctot = Cout + extra_c
    y = torch.full((B, Ho, Wo, Ctot), float("nan"), device=DEV, dtype=BF)
    part, nch = ops.conv_stats(kind, B, L.nhwc_view(xg), Cin, wp, Cout, L.nhwc_view(y, co), BF,
                               bias=None if bias is None else bias.to(DEV), force=force)
    bn = torch.nn.BatchNorm2d(Cout).to(DEV)
    t = torch.empty((2, Cout), device=DEV)
    mean, rstd = ops.bn_finalize_part(part, nch, Cout, bn, t[0], t[1])
    var = 1.0 / rstd.double() ** 2 - bn.eps
    torch.cuda.synchronize()
    yo = nchw(y[..., co:co + Cout].float()).cpu()
    return yo, mean.cpu().double(), var.cpu()


def check(got, ref, mean, var, what, tol=1e-2):
    scale = float(ref.abs().max()) + 1e-12
    err = float((got - ref).abs().max())
    assert err <= tol * scale, f"{what}: max err {err:.3e} vs scale {scale:.3e}"
    rm = ref.double().mean(dim=(0, 2, 3))
    rv = ref.double().var(dim=(0, 2, 3), unbiased=False)
    sd = float(rv.max().sqrt()) + 1e-12
    assert float((mean - rm).abs().max()) <= 2e-3 * sd, f"{what}: mean err {float((mean - rm).abs().max()):.3e}"
    assert float(((var - rv).abs() / (rv + 1e-12)).max()) <= 2e-3 * 4, f"{what}: var err"


CASES = [  # B, Cin, Cout, H(grid), W(grid)
    (2, 64, 128, 32, 32),
    (2, 128, 256, 16, 16),
    (4, 512, 512, 4, 4),
    (3, 64, 96, 10, 14),     # ragged M and N (N not a tile multiple)
    (2, 8, 64, 64, 64),      # Cin = 8: a K-step spans 8 taps
    (1, 256, 64, 7, 9),
]
CFGS = ([None] + [(c, 1) for c in range(20)] + [(0, 2), (5, 4), (8, 2), (12, 4), (14, 2), (17, 4)] +
        [(c, 1) for c in (29, 30, 31, 32, 33, 34, 35)] + [(29, 4), (31, 2), (33, 2)])  # loader-wave tiles


@pytest.mark.parametrize("force", CFGS, ids=lambda f: "auto" if f is None else f"cfg{f[0]}_ks{f[1]}")
@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
def test_conv_s2(case, force):
    B, Cin, Cout, Hg, Wg = case
    x = q(rnd(B, Cin, 2 * Hg, 2 * Wg, seed=1))
    w = q(rnd(Cout, Cin, 4, 4, seed=2, scale=0.05))
    ref = F.conv2d(x, w, None, 2, 1)
    y, mean, var = run(L.CONV_S2, B, x, w, Cin, Cout, (Hg, Wg), force=force)
    check(y, ref, mean, var, f"conv s2 {case} {force}")


@pytest.mark.parametrize("force", [None, (0, 1), (1, 1), (3, 1), (5, 2), (8, 1), (9, 1), (13, 1), (11, 2), (14, 1),
                                   (15, 1), (16, 1), (17, 2), (18, 1), (19, 1), (29, 1), (30, 2), (31, 1), (32, 1), (33, 1),
                                   (34, 1), (35, 1)],
                         ids=lambda f: "auto" if f is None else f"cfg{f[0]}_ks{f[1]}")
@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
def test_convT_s2(case, force):
    B, Cin, Cout, Hg, Wg = case
    x = q(rnd(B, Cin, Hg, Wg, seed=3))
    w = q(rnd(Cin, Cout, 4, 4, seed=4, scale=0.05))
    ref = F.conv_transpose2d(x, w, None, 2, 1)
    y, mean, var = run(L.CONVT_S2, B, x, w, Cin, Cout, (2 * Hg, 2 * Wg), force=force)
    check(y, ref, mean, var, f"convT {case} {force}")


@pytest.mark.parametrize("force", [None, (0, 1), (6, 1), (0, 4), (14, 1), (17, 1)], ids=lambda f: "auto" if f is None else f"cfg{f[0]}_ks{f[1]}")
def test_conv_s1_and_dgrad(force):
    B, Cin, Cout, H = 2, 256, 512, 17   # PatchGAN layer 4 geometry (32x32 -> 31x31), smaller
    x = q(rnd(B, Cin, H, H, seed=5))
    w = q(rnd(Cout, Cin, 4, 4, seed=6, scale=0.05))
    ref = F.conv2d(x, w, None, 1, 1)
    y, mean, var = run(L.CONV_S1, B, x, w, Cin, Cout, (H - 1, H - 1), force=force)
    check(y, ref, mean, var, f"conv s1 {force}")
    # input gradient: dx = conv_transpose2d(dy, w, stride 1, pad 1), N = Cin, reduction over Cout
    dy = q(rnd(B, Cout, H - 1, H - 1, seed=7))
    ref = F.conv_transpose2d(dy, w, None, 1, 1)
    y, mean, var = run(L.CONV_S1_DGRAD, B, dy, w, Cout, Cin, (H, H), force=force)
    check(y, ref, mean, var, f"conv s1 dgrad {force}")


@pytest.mark.parametrize("force", [None, (1, 1), (0, 2)], ids=lambda f: "auto" if f is None else f"cfg{f[0]}_ks{f[1]}")
def test_channel_offset_view_and_bias(force):
    """Output into the second half of a concat buffer (zero-copy skip) with a bias epilogue."""
    B, Cin, Cout, Hg, Wg = 2, 128, 128, 16, 16
    x = q(rnd(B, Cin, 2 * Hg, 2 * Wg, seed=8))
    w = q(rnd(Cout, Cin, 4, 4, seed=9, scale=0.05))
    b = rnd(Cout, seed=10)
    ref = F.conv2d(x, w, b, 2, 1)
    y, mean, var = run(L.CONV_S2, B, x, w, Cin, Cout, (Hg, Wg), force=force, co=64, extra_c=64, bias=b)
    check(y, ref, mean, var, f"offset view {force}")


@pytest.mark.parametrize("case", [(L.CONV_S2, 4, 512, 512, 4, 4, (12, 4)), (L.CONV_S2, 2, 128, 256, 16, 16, (0, 2)),
                                  (L.CONVT_S2, 2, 512, 256, 4, 4, (5, 4)), (L.CONV_S2, 3, 64, 96, 10, 14, (11, 2)),
                                  (L.CONV_S2, 32, 512, 512, 8, 8, None), (L.CONVT_S2, 32, 1024, 512, 4, 4, None)],
                         ids=lambda c: "x".join(map(str, c[:6])) + ("" if c[6] is None else f"_cfg{c[6][0]}ks{c[6][1]}"))
def test_splitk_inlaunch_matches_reduction_launch(case):
    """Split-K combined in the launch (each tile's last arriver sums the slabs in split order and runs the epilogue)
    against the separate reduction launch: the same outputs bit for bit (same sums in the same order, no bias), the
    BatchNorm statistics from other chunks (tile partials vs reduction-block partials) within fp32 rounding."""
    kind, B, Cin, Cout, Hg, Wg, force = case
    if kind == L.CONVT_S2:
        x = q(rnd(B, Cin, Hg, Wg, seed=11))
        w = q(rnd(Cin, Cout, 4, 4, seed=12, scale=0.05))
        out = (2 * Hg, 2 * Wg)
    else:
        x = q(rnd(B, Cin, 2 * Hg, 2 * Wg, seed=11))
        w = q(rnd(Cout, Cin, 4, 4, seed=12, scale=0.05))
        out = (Hg, Wg)
    _, _, plan = ops.conv_query(kind, B, Hg, Wg, Cin, Cout, BF, force=force)
    assert plan[2] > 1, f"not a split-K plan: {plan}"
    old = ops.set_splitk_inlaunch(True)
    try:
        y1, m1, v1 = run(kind, B, x, w, Cin, Cout, out, force=force)
        ops.set_splitk_inlaunch(False)
        y0, m0, v0 = run(kind, B, x, w, Cin, Cout, out, force=force)
    finally:
        ops.set_splitk_inlaunch(old)
    assert torch.equal(y1, y0)
    assert float((m1 - m0).abs().max()) <= 1e-5 * (float(v0.max()) ** 0.5 + 1e-12)
    assert float(((v1 - v0).abs() / (v0 + 1e-12)).max()) <= 1e-4


@pytest.mark.parametrize("case", [(L.CONV_S2, 32, 512, 1024, 8, 8), (L.CONVT_S2, 32, 512, 512, 2, 2),
                                  (L.CONV_S2, 32, 1024, 512, 4, 4), (L.CONVT_S2, 32, 1024, 512, 4, 4)],
                         ids=lambda c: "x".join(map(str, c)))
def test_splitk_inlaunch_bn_backward_matches_reduction_launch(case):
    """The fused BatchNorm-backward form of an input-gradient conv on an in-launch split-K plan (the last arriver's
    epilogue writes the {dn, dn*xhat} partials, nphase * mtiles chunks) against the reduction launch (which computes
    them itself): the conv output bit for bit, the BN input gradient bit for bit apart from fp32 rounding of the
    per-channel sums, dgamma / dbeta within fp32 rounding."""
    kind, B, Cin, Cout, Hg, Wg = case
    _, _, plan = ops.conv_query(kind, B, Hg, Wg, Cin, Cout, BF)
    if not 2 <= plan[2] <= 4:
        pytest.skip(f"the automatic plan is not a 2-4 split plan here: {plan}")
    gen = torch.Generator(device=DEV)
    if kind == L.CONVT_S2:
        wt = q(rnd(Cin, Cout, 4, 4, seed=61, scale=0.05))
        w = ops.pack(L.PACK_CONVT_FWD, wt.to(DEV), Cout, Cin, BF)
        dy = torch.randn((B, Hg, Wg, Cin), generator=gen.manual_seed(62), device=DEV).to(BF)
        Ho, Wo = 2 * Hg, 2 * Wg
    else:
        wt = q(rnd(Cout, Cin, 4, 4, seed=61, scale=0.05))
        w = ops.pack(L.PACK_CONV_FWD, wt.to(DEV), Cout, Cin, BF)
        dy = torch.randn((B, 2 * Hg, 2 * Wg, Cin), generator=gen.manual_seed(62), device=DEV).to(BF)
        Ho, Wo = Hg, Wg
    C = Cout
    x = torch.randn((B, Ho, Wo, C), generator=gen.manual_seed(63), device=DEV).to(BF)
    go = torch.randn((B, Ho, Wo, C), generator=gen.manual_seed(64), device=DEV).to(BF)
    g = torch.Generator().manual_seed(65)
    st = tuple((torch.rand(C, generator=g) + 0.5).to(DEV) if i in (0, 3) else (torch.randn(C, generator=g) * 0.2).to(DEV)
               for i in range(4))
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    res = []
    old = ops.set_splitk_inlaunch(True)
    try:
        for mode in (True, False):
            ops.set_splitk_inlaunch(mode)
            out = torch.zeros((B, Ho, Wo, Cout), device=DEV, dtype=BF)
            dx = torch.empty((B, Ho, Wo, C), device=DEV, dtype=BF)
            dg, db = ops.conv_bn_backward(kind, B, L.nhwc_view(dy), Cin, w, Cout, L.nhwc_view(out), BF,
                                          bn_x=L.nhwc_view(x), C=C, bn_state=st, gamma=gamma, s_self=0.2,
                                          g_other=L.nhwc_view(go), s_other=0.0, dxv=L.nhwc_view(dx))
            torch.cuda.synchronize()
            res.append((out, dx.float(), dg, db))
    finally:
        ops.set_splitk_inlaunch(old)
    (o1, dx1, g1, b1), (o0, dx0, g0, b0) = res
    assert torch.equal(o1, o0)
    for a, b in ((g1, g0), (b1, b0)):
        assert float((a - b).abs().max()) <= 1e-5 * (float(b.abs().max()) + 1e-6)
    assert float((dx1 - dx0).abs().max()) <= 1e-2 * (float(dx0.abs().max()) + 1e-6)


def test_plan_query_consistent():
    for kind, gh in ((L.CONV_S2, 64), (L.CONVT_S2, 8), (L.CONV_S1, 31)):
        ws, nch, plan = ops.conv_query(kind, 32, gh, gh, 256, 512, BF)
        assert plan[4] >= 0 and plan[2] >= 1 and nch >= 1
        assert (ws > 0) == (plan[2] > 1)


NARROW = [  # kind, B, Cin, N, grid H, grid W
    ("convT", 2, 128, 3, 20, 24),    # generator output layer (bias + tanh, NCHW fp32)
    ("convT", 2, 128, 1, 16, 16),
    ("convT", 1, 64, 8, 9, 13),      # first-layer input gradient (N = 8 padded channels), ragged tiles
    ("convT", 3, 64, 4, 33, 17),
    ("conv_s1", 2, 512, 1, 30, 30),  # PatchGAN logits 31x31 -> 30x30 (the two-pass taps GEMM + gather)
    ("conv_s1", 32, 512, 1, 30, 30),  # ... at the train step's batch
    ("conv_s1", 3, 256, 1, 7, 9),    # ... with 256 channels, ragged
    ("conv_s1", 1, 128, 2, 11, 9),
]


@pytest.mark.parametrize("out", ["nchw_f32", "nhwc_bf16"])
@pytest.mark.parametrize("case", NARROW, ids=lambda c: "_".join(map(str, c)))
def test_narrow_halo(case, out):
    """bf16 narrow-N layers (N <= 8/16) on the LDS-halo MFMA kernel (csrc/narrow_bf16.hip)."""
    kind, B, Cin, N, GH, GW = case
    x_shape = (B, Cin, GH, GW) if kind == "convT" else (B, Cin, GH + 1, GW + 1)
    x = q(rnd(*x_shape, seed=31))
    b = rnd(N, seed=32)
    if kind == "convT":
        w = q(rnd(Cin, N, 4, 4, seed=33, scale=0.05))
        ref = F.conv_transpose2d(x, w, b, 2, 1)
        wp = ops.pack(L.PACK_CONVT_FWD, w.to(DEV), N, Cin, BF)
        kd, Ho, Wo = L.CONVT_S2, 2 * GH, 2 * GW
    else:
        w = q(rnd(N, Cin, 4, 4, seed=34, scale=0.05))
        ref = F.conv2d(x, w, b, 1, 1)
        wp = ops.pack(L.PACK_CONV_FWD, w.to(DEV), N, Cin, BF)
        kd, Ho, Wo = L.CONV_S1, GH, GW
    assert ops.plan_of(kd, B, GH, GW, Cin, N, BF)[3] == 1
    xg = nhwc(x).to(DEV, BF)
    tanh = out == "nchw_f32"
    if tanh:
        ref = torch.tanh(ref)
        y = torch.full((B, N, Ho, Wo), float("nan"), device=DEV)
        ops.conv(kd, B, L.nhwc_view(xg), Cin, wp, N, L.nchw_view(y), BF, bias=b.to(DEV), tanh=True, out_f32=True)
        got = y.cpu()
    else:
        y = torch.full((B, Ho, Wo, N), float("nan"), device=DEV, dtype=BF)
        ops.conv(kd, B, L.nhwc_view(xg), Cin, wp, N, L.nhwc_view(y), BF, bias=b.to(DEV))
        got = nchw(y.float()).cpu()
    scale = float(ref.abs().max())
    err = float((got - ref).abs().max())
    tol = 2e-5 if tanh else 8e-3  # fp32 output: summation order only; bf16 output: final rounding
    assert err <= tol * max(scale, 1.0) * (1 if tanh else 1) + (1e-5 if tanh else 0), f"narrow {case} {out}: {err:.3e}"


NARROW_STREAM = [  # B, Cin, N, grid H, grid W: the streaming ConvT kernel's shapes (16-row strips, 64-column blocks)
    (2, 128, 3, 32, 64),     # generator output layer (G2: 3 channels)
    (3, 128, 1, 16, 128),    # G1: 1 channel, two column blocks
    (2, 64, 8, 32, 64),      # first-layer input gradient (N = 8 padded channels)
    (1, 64, 8, 48, 192),
    (32, 128, 3, 128, 128),  # full size (bench workload)
    (32, 64, 8, 128, 128),
]


@pytest.mark.parametrize("out", ["nchw_f32", "nhwc_bf16"])
@pytest.mark.parametrize("case", NARROW_STREAM, ids=lambda c: "_".join(map(str, c)))
def test_narrow_stream(case, out):
    """The streaming ConvT kernel (csrc/narrow_bf16.hip narrow_stream_kernel, the default for these shapes) vs torch
    fp32 and vs the tiled K-split kernel forced on the same inputs (same MFMA products, another summation order)."""
    B, Cin, N, GH, GW = case
    assert ops.kernel_name(L.CONVT_S2, B, GH, GW, Cin, N, BF)[0].startswith("narrow_stream_kernel")
    x = q(rnd(B, Cin, GH, GW, seed=41))
    b = rnd(N, seed=42)
    w = q(rnd(Cin, N, 4, 4, seed=43, scale=0.05))
    ref = F.conv_transpose2d(x, w, b, 2, 1)
    wp = ops.pack(L.PACK_CONVT_FWD, w.to(DEV), N, Cin, BF)
    xg = nhwc(x).to(DEV, BF)
    tanh = out == "nchw_f32"
    outs = []
    for force in (None, (4, 1)):
        if tanh:
            y = torch.full((B, N, 2 * GH, 2 * GW), float("nan"), device=DEV)
            ops.conv(L.CONVT_S2, B, L.nhwc_view(xg), Cin, wp, N, L.nchw_view(y), BF, bias=b.to(DEV), tanh=True,
                     out_f32=True, force=force)
            outs.append(y.cpu())
        else:
            y = torch.full((B, 2 * GH, 2 * GW, N), float("nan"), device=DEV, dtype=BF)
            ops.conv(L.CONVT_S2, B, L.nhwc_view(xg), Cin, wp, N, L.nhwc_view(y), BF, bias=b.to(DEV), force=force)
            outs.append(nchw(y.float()).cpu())
    if tanh:
        ref = torch.tanh(ref)
    scale = max(float(ref.abs().max()), 1.0)
    tol = 2e-5 if tanh else 8e-3
    for got, what in zip(outs, ("stream", "tiled")):
        assert not torch.isnan(got).any(), f"{what}: unwritten outputs"
        err = float((got - ref).abs().max())
        assert err <= tol * scale + (1e-5 if tanh else 0), f"narrow {what} {case} {out}: {err:.3e}"
    # the two kernels differ only in fp32 summation order (bf16 outputs: at most one rounding step apart)
    d = float((outs[0] - outs[1]).abs().max())
    assert d <= (1e-5 if tanh else 8e-3 * scale), f"stream vs tiled {case} {out}: {d:.3e}"


def test_narrow_stream_offset_view():
    """G2's output layer writing into a channel-offset NHWC view (the cat / objective buffers), NaN guard around it."""
    B, Cin, N, GH, GW = 2, 128, 3, 16, 64
    x = q(rnd(B, Cin, GH, GW, seed=44))
    w = q(rnd(Cin, N, 4, 4, seed=45, scale=0.05))
    ref = F.conv_transpose2d(x, w, None, 2, 1)
    wp = ops.pack(L.PACK_CONVT_FWD, w.to(DEV), N, Cin, BF)
    buf = torch.full((B, 2 * GH, 2 * GW, 8), float("nan"), device=DEV, dtype=BF)
    yv = L.nhwc_view(buf, c0=4)
    ops.conv(L.CONVT_S2, B, L.nhwc_view(nhwc(x).to(DEV, BF)), Cin, wp, N, yv, BF)
    got = nchw(buf[..., 4:4 + N].float()).cpu()
    assert torch.isnan(buf[..., :4].float()).all() and torch.isnan(buf[..., 4 + N:].float()).all()
    assert float((got - ref).abs().max()) <= 8e-3 * max(float(ref.abs().max()), 1.0)


WGRAD = [  # kind, stride, B, Cin, Cout, H, W (input grid of the forward layer)
    ("conv", 2, 2, 64, 128, 32, 32),
    ("conv", 2, 2, 8, 64, 64, 64),     # first layer: Cg = 8, 16 taps per 128-column tile
    ("conv", 2, 4, 512, 512, 4, 4),    # small pixel count, many column tiles
    ("conv", 1, 2, 256, 512, 17, 17),  # PatchGAN layer 4 geometry
    ("conv", 2, 3, 32, 96, 10, 14),    # ragged R / columns
    ("convT", 2, 2, 128, 64, 16, 16),
    ("convT", 2, 2, 1024, 512, 2, 2),
    ("convT", 2, 1, 64, 8, 9, 13),     # R = 64 (64-row tile), odd grid
    ("conv", 1, 2, 512, 8, 17, 17),    # PatchGAN logits (N = 8 padded): R <= 16 -> swapped 128x16 tile
    ("conv", 1, 1, 64, 8, 9, 11),      # R = 8, ragged
    ("conv", 2, 2, 16, 64, 40, 24),    # R = 64 with Cg = 16
    # pixel-mapping modes of the K-step addressing (wgrad_bf16.hip WbParams::pmode)
    ("conv", 2, 1, 16, 128, 128, 128),  # mode 1: 64 x 64 grid (a step inside one row), many splits
    ("conv", 2, 5, 16, 64, 8, 8),       # mode 3: 4 x 4 grids, 80 pixels (partial last step)
    ("convT", 2, 3, 64, 32, 1, 1),      # mode 3: 1 x 1 grids, 3 pixels
    ("conv", 2, 2, 32, 64, 256, 16),    # mode 2 with GW = 8 (8 rows per step)
]


@pytest.mark.parametrize("case", WGRAD, ids=lambda c: "_".join(map(str, c)))
def test_wgrad_bf16_dma(case, force=None):
    """bf16 weight gradient on the LDS-DMA / transposed-read kernel (csrc/wgrad_bf16.hip)."""
    kind, s, B, Cin, Cout, H, W = case
    x = q(rnd(B, Cin, H, W, seed=41))
    if kind == "conv":
        w = torch.zeros(Cout, Cin, 4, 4, requires_grad=True)
        y = F.conv2d(x, w, None, s, 1)
        dy = q(rnd(*y.shape, seed=42))
        (gw,) = torch.autograd.grad(y, w, dy)
        # D = dy (R = Cout), G = x (Cg = Cin)
        dW = ops.wgrad(B, s, L.nhwc_view(nhwc(dy).to(DEV, BF)), Cout, L.nhwc_view(nhwc(x).to(DEV, BF)), Cin, Cin, BF,
                       device=DEV, force=force)
    else:
        w = torch.zeros(Cin, Cout, 4, 4, requires_grad=True)
        y = F.conv_transpose2d(x, w, None, 2, 1)
        dy = q(rnd(*y.shape, seed=43))
        (gw,) = torch.autograd.grad(y, w, dy)
        # D = x (R = Cin), G = dy (Cg = Cout)
        dW = ops.wgrad(B, 2, L.nhwc_view(nhwc(x).to(DEV, BF)), Cin, L.nhwc_view(nhwc(dy).to(DEV, BF)), Cout, Cout, BF,
                       device=DEV, force=force)
    torch.cuda.synchronize()
    got = dW.cpu()
    err = float((got - gw).abs().max())
    scale = float(gw.abs().max())
    assert err <= 2e-5 * scale + 1e-6, f"wgrad {case}: {err:.3e} vs {scale:.3e}"  # exact products, fp32 sums


class _BNT:
    def __init__(self, C, seed):
        g = torch.Generator().manual_seed(seed)
        self.scale = (torch.rand(C, generator=g) + 0.5).to(DEV)
        self.shift = (torch.randn(C, generator=g) * 0.2).to(DEV)
        self.mean = (torch.randn(C, generator=g) * 0.1).to(DEV)
        self.rstd = (torch.rand(C, generator=g) + 0.5).to(DEV)
        self.gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)


FUSED = [  # kind, B, Cin(dy), Cout(conv out), grid H, W (GEMM grid), C (BN), ch_off, with g_other
    ("convT", 2, 128, 64, 16, 16, 64, 0, True),     # G down path: conv-s2 dgrad, skip gradient as g_other
    ("convT", 4, 512, 512, 2, 2, 512, 0, True),     # deep level: split-K reduction path
    ("conv_s2", 2, 64, 256, 16, 16, 128, 128, False),  # G up path: second half of the concat gradient
    ("s1_dgrad", 2, 256, 128, 15, 15, 128, 0, False),  # PatchGAN layer-4 input gradient
]


@pytest.mark.parametrize("case", FUSED, ids=lambda c: "_".join(map(str, c)))
def test_conv_bn_backward_fused(case):
    """stc_conv_bwd_bn (BN-backward reduction in the conv epilogue) == conv + separate BN backward."""
    kind, B, Cin, Cout, GH, GW, C, ch_off, other = case
    kd = {"convT": L.CONVT_S2, "conv_s2": L.CONV_S2, "s1_dgrad": L.CONV_S1_DGRAD}[kind]
    if kd == L.CONVT_S2:
        dy_hw, out_hw = (GH, GW), (2 * GH, 2 * GW)
        w = ops.pack(L.PACK_CONVT_FWD, rnd(Cin, Cout, 4, 4, seed=51, scale=0.05).to(DEV), Cout, Cin, BF)
    elif kd == L.CONV_S2:
        dy_hw, out_hw = (2 * GH, 2 * GW), (GH, GW)
        w = ops.pack(L.PACK_CONV_FWD, rnd(Cout, Cin, 4, 4, seed=51, scale=0.05).to(DEV), Cout, Cin, BF)
    else:
        dy_hw, out_hw = (GH - 1, GW - 1), (GH, GW)
        w = ops.pack(L.PACK_CONV_S1_DGRAD, rnd(Cin, Cout, 4, 4, seed=51, scale=0.05).to(DEV), Cout, Cin, BF)
    dy = (torch.randn((B, *dy_hw, Cin), generator=torch.Generator().manual_seed(52)) * 0.5).to(DEV, BF)
    x = torch.randn((B, *out_hw, C), generator=torch.Generator().manual_seed(53)).to(DEV, BF)
    go = torch.randn((B, *out_hw, C), generator=torch.Generator().manual_seed(54)).to(DEV, BF) if other else None
    bn = _BNT(C, 55)
    st = (bn.scale, bn.shift, bn.mean, bn.rstd)
    # fused
    out1 = torch.zeros((B, *out_hw, Cout), device=DEV, dtype=BF)
    dx1 = torch.empty((B, *out_hw, C), device=DEV, dtype=BF)
    dg1, db1 = ops.conv_bn_backward(kd, B, L.nhwc_view(dy), Cin, w, Cout, L.nhwc_view(out1), BF, bn_x=L.nhwc_view(x),
                                    C=C, bn_state=st, gamma=bn.gamma, s_self=0.2, ch_off=ch_off,
                                    g_other=None if go is None else L.nhwc_view(go), s_other=0.0,
                                    dxv=L.nhwc_view(dx1))
    # reference: conv, then the two-pass BN backward
    out2 = torch.zeros((B, *out_hw, Cout), device=DEV, dtype=BF)
    ops.conv(kd, B, L.nhwc_view(dy), Cin, w, Cout, L.nhwc_view(out2), BF)
    dx2 = torch.empty((B, *out_hw, C), device=DEV, dtype=BF)
    dg2, db2 = ops.bn_backward(B, L.nhwc_view(x), C, BF, L.nhwc_view(dx2), g1=L.nhwc_view(out2, ch_off), s1=0.2,
                               g2=None if go is None else L.nhwc_view(go), s2=0.0,
                               bn_state=(bn.scale, bn.shift, bn.mean, bn.rstd, bn.gamma))
    torch.cuda.synchronize()
    assert torch.equal(out1, out2)
    for a, b_, nm in ((dg1, dg2, "dgamma"), (db1, db2, "dbeta")):
        err = float((a - b_).abs().max())
        assert err <= 1e-4 * float(b_.abs().max()) + 1e-5, f"{nm} {case}: {err:.3e}"
    err = float((dx1.float() - dx2.float()).abs().max())
    assert err <= 1e-2 * float(dx2.float().abs().max()), f"dx {case}: {err:.3e}"


WGRAD_FORCED = [  # (case, tile config, pixel splits): the 8-wave tiles on ragged / offset shapes
    (("conv", 2, 2, 64, 256, 32, 32), 3, 0),
    (("conv", 2, 2, 64, 256, 32, 32), 4, 2),
    (("conv", 2, 2, 64, 256, 32, 32), 5, 1),
    (("conv", 1, 2, 256, 512, 17, 17), 3, 0),
    (("conv", 2, 3, 32, 96, 10, 14), 3, 3),    # R, columns and pixels all ragged for a 256 tile
    (("conv", 2, 3, 32, 96, 10, 14), 5, 0),
    (("convT", 2, 2, 128, 64, 16, 16), 4, 0),
    (("convT", 2, 2, 1024, 512, 2, 2), 3, 1),
    (("conv", 2, 2, 8, 64, 64, 64), 5, 0),      # Cg = 8: 16 taps per 128 columns
    (("conv", 1, 2, 512, 8, 17, 17), 0, 4),     # R = 8 on a 128-row tile
    (("conv", 2, 1, 16, 128, 128, 128), 0, 3),  # mode 1 with an odd split count
    (("conv", 2, 5, 16, 64, 8, 8), 0, 2),       # mode 3, split boundary inside the pixel range
    # loader-wave tiles (4 DMA-only waves, 4- / 3-stage ring): every pixel mode, ragged, split / unsplit
    (("conv", 2, 2, 64, 256, 32, 32), 6, 0),
    (("conv", 2, 2, 64, 256, 32, 32), 7, 1),
    (("conv", 2, 3, 32, 96, 10, 14), 6, 3),
    (("conv", 2, 3, 32, 96, 10, 14), 7, 0),
    (("convT", 2, 2, 128, 64, 16, 16), 7, 2),
    (("conv", 2, 1, 16, 128, 128, 128), 6, 3),
    (("conv", 2, 5, 16, 64, 8, 8), 7, 2),
    (("conv", 1, 2, 512, 8, 17, 17), 6, 4),
    # halo tile (stride 2, 16 channels x 16 taps per tile): K-step widths 16 / 32 / 64 (+ a 128-wide grid: two steps
    # per row), both roles (conv: D = dy; convT: D = x), ragged R, several channel groups, splits across images
    (("conv", 2, 2, 64, 128, 32, 32), 8, 0),
    (("conv", 2, 2, 64, 128, 32, 32), 8, 3),
    (("conv", 2, 1, 32, 256, 64, 64), 8, 2),
    (("conv", 2, 1, 16, 128, 128, 128), 8, 1),
    (("conv", 2, 1, 48, 96, 256, 64), 8, 5),
    (("conv", 2, 1, 16, 128, 64, 256), 8, 2),
    (("convT", 2, 2, 128, 64, 16, 16), 8, 0),
    (("convT", 2, 3, 256, 32, 32, 32), 8, 4),
    (("convT", 2, 1, 128, 16, 64, 64), 8, 1),
    # 8-wide grids (a K-step = one whole 8 x 8 image; 17-position plane lines): both roles, ragged R, splits
    (("conv", 2, 4, 64, 128, 16, 16), 8, 0),
    (("conv", 2, 5, 32, 96, 16, 16), 8, 2),
    (("convT", 2, 3, 128, 64, 8, 8), 8, 0),
    (("convT", 2, 2, 48, 128, 8, 8), 8, 3),
    # the stride-1 halo tile (PatchGAN layer 4: D = dy 31 x 31 run as 32 x 32, G = x 32 x 32)
    (("conv", 1, 2, 64, 128, 32, 32), 8, 0),
    (("conv", 1, 1, 256, 512, 32, 32), 8, 3),
    (("conv", 1, 3, 32, 96, 32, 32), 8, 2),
]


@pytest.mark.parametrize("case,cfg,ns", WGRAD_FORCED, ids=lambda c: "_".join(map(str, c)) if isinstance(c, tuple) else str(c))
def test_wgrad_bf16_forced_tiles(case, cfg, ns):
    """Every weight-gradient tile configuration (a per-call plan of stc_conv_wgrad_ex) against autograd."""
    test_wgrad_bf16_dma(case, force=(cfg, ns))


@pytest.mark.parametrize("case", [("convT", 2, 2, 1024, 512, 2, 2), ("conv", 2, 4, 512, 512, 4, 4),
                                  ("convT", 2, 32, 1024, 512, 4, 4), ("conv", 2, 32, 512, 512, 8, 8),
                                  ("conv", 2, 3, 32, 96, 10, 14)],
                         ids=lambda c: "_".join(map(str, c)))
def test_wgrad_channel_major_direct_store(case):
    """Single-split weight gradients whose tiles are wider than one tap's channels store torch layout from the tile
    with channel-group-major columns (8 channels x 16 taps per 128 columns, no transposing reduce): bit-identical
    to the tap-major slab + reduce (force {-1, -1}), and the plan reports no slab."""
    kind, s, B, Cin, Cout, H, W = case
    x = nhwc(q(rnd(B, Cin, H, W, seed=71))).to(DEV, BF)
    if kind == "conv":
        Ho, Wo = (H + 1) // 2, (W + 1) // 2
        dy = nhwc(q(rnd(B, Cout, Ho, Wo, seed=72))).to(DEV, BF)
        D, R, G, Cg = dy, Cout, x, Cin
    else:
        dy = nhwc(q(rnd(B, Cout, 2 * H, 2 * W, seed=73))).to(DEV, BF)
        D, R, G, Cg = x, Cin, dy, Cout
    a = ops.wgrad(B, s, L.nhwc_view(D), R, L.nhwc_view(G), Cg, Cg, BF, device=DEV)
    b = ops.wgrad(B, s, L.nhwc_view(D), R, L.nhwc_view(G), Cg, Cg, BF, device=DEV, force=(-1, -1))
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("B,Cin,H,W,rows,dt", [(4, 512, 31, 31, 1, BF), (2, 64, 9, 13, 2, BF), (3, 128, 17, 5, 1, torch.float32),
                                              (1, 64, 6, 7, 2, torch.float32), (32, 512, 31, 31, 1, BF)])
def test_wgrad_rows_narrow_s1(B, Cin, H, W, rows, dt):
    """stc_conv_wgrad_rows (the PatchGAN logits layer: conv s1, 1-2 real output channels padded to 8):
    vs torch autograd; padded rows zero."""
    x = q(rnd(B, Cin, H, W, seed=71)) if dt == BF else rnd(B, Cin, H, W, seed=71)
    w = torch.zeros(8, Cin, 4, 4, requires_grad=True)
    y = F.conv2d(x, w, None, 1, 1)
    dy = rnd(*y.shape, seed=72)
    dy[:, rows:] = 0
    dy = q(dy) if dt == BF else dy
    (gw,) = torch.autograd.grad(y, w, dy)
    dW = ops.wgrad(B, 1, L.nhwc_view(nhwc(dy).to(DEV, dt)), 8, L.nhwc_view(nhwc(x).to(DEV, dt)), Cin, Cin, dt,
                   device=DEV, rows=rows, rows_kernel=True)
    torch.cuda.synchronize()
    got = dW.cpu()
    err = float((got - gw).abs().max())
    scale = float(gw.abs().max())
    assert err <= 2e-5 * scale + 1e-6, f"wgrad rows: {err:.3e} vs {scale:.3e}"
    assert float(got[rows:].abs().max()) == 0.0


def test_wgrad_halo_plan_automatic():
    """The train step's stride-2 weight gradients with an 8..128-wide grid and 16-channel groups take the halo tile
    (plan config 8); the narrow first layers (Cg = 8) and the deep 4x4 .. 1x1 grids keep the im2col tiles."""
    for (B, gh, R, Cg) in ((32, 64, 128, 64), (32, 32, 256, 128), (32, 16, 512, 256), (32, 64, 256, 64),
                           (32, 32, 512, 128), (32, 16, 1024, 256), (32, 31, 512, 256), (32, 8, 512, 512),
                           (32, 8, 1024, 512)):
        assert ops.wgrad_query(B, gh, gh, R, Cg, BF)[1][0] == 8, (B, gh, R, Cg)
    for (B, gh, R, Cg) in ((32, 128, 64, 8), (32, 4, 512, 512), (32, 2, 512, 512)):
        assert ops.wgrad_query(B, gh, gh, R, Cg, BF)[1][0] != 8, (B, gh, R, Cg)
