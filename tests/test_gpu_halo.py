"""The halo kernels (csrc/halo_bf16.hip) against torch fp32 references and the im2col tile.

Conv2d k4 s2 p1 (STCGAN/networks.py:104-105, 167-169, 176-178) and the ConvTranspose2d input gradient (its
geometry, networks.py:112-128 backward), ConvTranspose2d k4 s2 p1 (networks.py:112-128, one sub-pixel phase per
block) and the Conv2d input gradient (its geometry), with the A operand staged as input rows in LDS.  Checked: every output
width the kernel takes (16, 32, 64 columns: 16, 8 and 4 output rows per 256-row tile), several 64-channel
chunks, ragged N, channel-offset input and output views (the concat buffers), bias, the BatchNorm statistics
and the fused BatchNorm-backward sums of the epilogue, the automatic plan at the train step's sizes.
Operands are bf16-exact, so the references differ by fp32 summation order and the final bf16 rounding only:
1e-2 * max|ref| on outputs (as tests/test_gpu_igemm_bf16.py), 2e-3 on the statistics.  Against the im2col tile
(a different but fixed K order) the outputs agree to the same bound.
"""
import pytest
import torch
import torch.nn.functional as F

from stcgan_amd import _lib as L
from stcgan_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16
HALO = (ops.HALO_CFG, 1)   # the 8-wave block (one per CU)
HALO2 = (ops.HALO_CFG, 2)  # the 4-wave block (two per CU)
HALO64 = (ops.HALO_CFG, 3)  # the 4-wave 256 x 64 block (conv-s2)
HALO64W8 = (ops.HALO_CFG, 4)  # the 8-wave 256 x 64 block (conv-s2, grids <= 32 wide; else the 4-wave one)
HALO_G1 = (ops.HALO_CFG, 5)  # ConvT: one phase per block
HALO_T2 = (ops.HALO_CFG, 6)  # ConvT: the two phases of a row parity per block, at any size


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def rnd(*shape, seed=0, scale=1.0, dev="cpu"):
    g = torch.Generator(device=dev).manual_seed(seed)
    return torch.randn(shape, generator=g, device=dev) * scale


def q(t):
    return t.to(BF).float()


def run(B, x, w, Cin, Cout, GH, GW, force, co_in=0, extra_in=0, co=0, extra_c=0, bias=None):
    """stc_conv_fwd_ex (with statistics) of NCHW fp32 x; returns (y NCHW fp32, mean, var, plan)."""
    xb = torch.zeros((B, 2 * GH, 2 * GW, Cin + extra_in), device=DEV, dtype=BF)
    xb[..., co_in:co_in + Cin] = nhwc(x).to(DEV, BF)
    wp = ops.pack(L.PACK_CONV_FWD, w.to(DEV), Cout, Cin, BF)
    y = torch.full((B, GH, GW, Cout + extra_c), float("nan"), device=DEV, dtype=BF)
    part, nch = ops.conv_stats(L.CONV_S2, B, L.nhwc_view(xb, co_in), Cin, wp, Cout, L.nhwc_view(y, co), BF,
                               bias=None if bias is None else bias.to(DEV), force=force)
    _, nq, plan = ops.conv_query(L.CONV_S2, B, GH, GW, Cin, Cout, BF, force=force)
    assert nq == nch
    bn = torch.nn.BatchNorm2d(Cout).to(DEV)
    t = torch.empty((2, Cout), device=DEV)
    mean, rstd = ops.bn_finalize_part(part, nch, Cout, bn, t[0], t[1])
    var = 1.0 / rstd.double() ** 2 - bn.eps
    torch.cuda.synchronize()
    return nchw(y[..., co:co + Cout].float()), mean.double(), var, plan


def check(got, ref, mean, var, what, tol=1e-2):
    scale = float(ref.abs().max()) + 1e-12
    err = float((got - ref).abs().max())
    assert err <= tol * scale, f"{what}: max err {err:.3e} vs scale {scale:.3e}"
    rm = ref.double().mean(dim=(0, 2, 3))
    rv = ref.double().var(dim=(0, 2, 3), unbiased=False)
    sd = float(rv.max().sqrt()) + 1e-12
    assert float((mean - rm).abs().max()) <= 2e-3 * sd, f"{what}: mean err {float((mean - rm).abs().max()):.3e}"
    assert float(((var - rv).abs() / (rv + 1e-12)).max()) <= 8e-3, f"{what}: var err"


CASES = [  # B, Cin, Cout, GH, GW
    (2, 64, 128, 8, 64),     # 4 output rows per tile (e2 / D layer 2 width), two tiles per image
    (1, 128, 256, 16, 32),   # 8 rows per tile, two 64-channel chunks, two N tiles (e3 / D layer 3)
    (1, 256, 512, 16, 16),   # 16 rows per tile (a whole 16x16 image), 4 chunks (e4)
    (3, 64, 96, 4, 64),      # ragged N (96 of a 128 tile), 3 images
    (1, 192, 40, 8, 32),     # 3 chunks, N = 40
    (4, 128, 128, 8, 8),     # 8-wide grid: a 256-row tile = 4 whole 8 x 8 images
    (8, 64, 64, 4, 8),       # 8-wide grid, 4-row images: a tile spans 8 images
]


@pytest.mark.parametrize("shape", [HALO, HALO2, HALO64, HALO64W8], ids=["8wave", "4wave", "n64", "n64w8"])
@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
def test_halo_conv_s2(case, shape):
    B, Cin, Cout, GH, GW = case
    x = q(rnd(B, Cin, 2 * GH, 2 * GW, seed=1, dev=DEV))
    w = q(rnd(Cout, Cin, 4, 4, seed=2, scale=0.05, dev=DEV))
    ref = F.conv2d(x, w, None, 2, 1)
    y, mean, var, plan = run(B, x, w, Cin, Cout, GH, GW, shape)
    assert plan[4] == ops.HALO_CFG and plan[0] == 256 and plan[1] == (64 if shape in (HALO64, HALO64W8) else 128)
    check(y, ref, mean, var, f"halo {case}")
    # the im2col tile on the same operands: equal up to the summation order
    y2, _, _, plan2 = run(B, x, w, Cin, Cout, GH, GW, (0, 1))
    assert plan2[4] == 0
    scale = float(ref.abs().max())
    assert float((y - y2).abs().max()) <= 1e-2 * scale


@pytest.mark.parametrize("shape", [HALO, HALO2, HALO64, HALO64W8], ids=["8wave", "4wave", "n64", "n64w8"])
def test_halo_views_and_bias(shape):
    """Input from a channel slice of a wider buffer (the concat buffers), output into the second half of one,
    with a bias epilogue."""
    B, Cin, Cout, GH, GW = 2, 64, 128, 8, 32
    x = q(rnd(B, Cin, 2 * GH, 2 * GW, seed=3, dev=DEV))
    w = q(rnd(Cout, Cin, 4, 4, seed=4, scale=0.05, dev=DEV))
    b = rnd(Cout, seed=5, dev=DEV)
    ref = F.conv2d(x, w, b, 2, 1)
    y, mean, var, _ = run(B, x, w, Cin, Cout, GH, GW, shape, co_in=64, extra_in=64, co=64, extra_c=64, bias=b)
    check(y, ref, mean, var, "halo views+bias")


def test_halo_plan_automatic_at_train_sizes():
    """The train step's conv-s2 layers with 64-channel chunks and enough blocks take the halo kernel; the
    others keep their im2col plans."""
    for (gh, cin, cout) in ((64, 64, 128), (32, 128, 256), (64, 64, 256), (32, 128, 512), (16, 256, 1024)):
        plan = ops.conv_query(L.CONV_S2, 32, gh, gh, cin, cout, BF)[2]
        assert plan[4] == ops.HALO_CFG and plan[1] == 128, (gh, cin, cout)
    # e4 (16 x 16, N = 512): 128 blocks of 128 channels, 256 of 64 -> the 256 x 64 halo block
    plan = ops.conv_query(L.CONV_S2, 32, 16, 16, 256, 512, BF)[2]
    assert plan[4] == ops.HALO_CFG and plan[1] == 64
    for (gh, cin, cout) in ((128, 8, 64), (8, 512, 512)):
        assert ops.conv_query(L.CONV_S2, 32, gh, gh, cin, cout, BF)[2][4] != ops.HALO_CFG, (gh, cin, cout)


def test_halo_full_size_e4_n64():
    """G's fourth down conv at the bench size (bs 32, 32x32x256 -> 16x16x512, the 8-wave 256 x 64 halo block) with
    statistics, vs the fp32 convolution of the same bf16 operands and the 8-wave 256 x 128 block (the same
    64-channel stages, so the same K order per output); the 4-wave 256 x 64 block against the 4-wave 256 x 128
    one likewise (32-channel stages)."""
    B, Cin, Cout, GH = 32, 256, 512, 16
    x = q(rnd(B, Cin, 2 * GH, 2 * GH, seed=8, dev=DEV))
    w = q(rnd(Cout, Cin, 4, 4, seed=9, scale=0.05, dev=DEV))
    ref = F.conv2d(x, w, None, 2, 1)
    y, mean, var, plan = run(B, x, w, Cin, Cout, GH, GH, None)
    assert plan[4] == ops.HALO_CFG and plan[1] == 64
    check(y, ref, mean, var, "halo e4 full size")
    for shape_a, shape_b in ((None, HALO), (HALO64, HALO2)):
        ya, ma, _, pa = run(B, x, w, Cin, Cout, GH, GH, shape_a)
        yb, mb, _, pb = run(B, x, w, Cin, Cout, GH, GH, shape_b)
        assert pa[1] == 64 and pb[1] == 128
        assert torch.equal(ya, yb)  # same K order per output: the N tile does not change the sums
        assert float((ma - mb).abs().max()) <= 1e-6 * (float(mb.abs().max()) + 1e-6)


def test_halo_full_size_e2():
    """G's second down conv at the bench size (bs 32, 128x128x64 -> 64x64x128) on the automatic plan, vs the
    fp32 convolution of the same bf16 operands."""
    B, Cin, Cout, GH = 32, 64, 128, 64
    x = q(rnd(B, Cin, 2 * GH, 2 * GH, seed=6, dev=DEV))
    w = q(rnd(Cout, Cin, 4, 4, seed=7, scale=0.05, dev=DEV))
    ref = F.conv2d(x, w, None, 2, 1)
    y, mean, var, plan = run(B, x, w, Cin, Cout, GH, GH, None)
    assert plan[4] == ops.HALO_CFG
    check(y, ref, mean, var, "halo e2 full size")


class _BNT:
    def __init__(self, C, seed):
        g = torch.Generator().manual_seed(seed)
        self.scale = (torch.rand(C, generator=g) + 0.5).to(DEV)
        self.shift = (torch.randn(C, generator=g) * 0.2).to(DEV)
        self.mean = (torch.randn(C, generator=g) * 0.1).to(DEV)
        self.rstd = (torch.rand(C, generator=g) + 0.5).to(DEV)
        self.gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)


@pytest.mark.parametrize("case", [(8, 64, 256, 64, 64, 128, 128), (32, 256, 1024, 16, 16, 512, 512),
                                  (32, 128, 512, 32, 32, 256, 256), (64, 256, 1024, 16, 16, 512, 512)],
                         ids=["d2_dgrad_8wave", "d4_dgrad_8wave", "d3_dgrad_4wave", "gw16_4wave"])
def test_halo_conv_bn_backward(case):
    """The ConvT input gradient at its train-step size (conv-s2 geometry, automatic plan = halo) with the
    BatchNorm-backward reduction fused into the epilogue: output vs torch, sums vs the separate reduction."""
    B, Cin, Cout, GH, GW, C, ch_off = case
    assert ops.conv_query(L.CONV_S2, B, GH, GW, Cin, Cout, BF)[2][4] == ops.HALO_CFG
    wt = q(rnd(Cout, Cin, 4, 4, seed=51, scale=0.05, dev=DEV))
    w = ops.pack(L.PACK_CONV_FWD, wt, Cout, Cin, BF)
    dy = q(rnd(B, Cin, 2 * GH, 2 * GW, seed=52, scale=0.5, dev=DEV))
    dyb = nhwc(dy).to(BF)
    x = torch.randn((B, GH, GW, C), generator=torch.Generator(device=DEV).manual_seed(53), device=DEV).to(BF)
    go = torch.randn((B, GH, GW, C), generator=torch.Generator(device=DEV).manual_seed(54), device=DEV).to(BF)
    bn = _BNT(C, 55)
    st = (bn.scale, bn.shift, bn.mean, bn.rstd)
    out1 = torch.zeros((B, GH, GW, Cout), device=DEV, dtype=BF)
    dx1 = torch.empty((B, GH, GW, C), device=DEV, dtype=BF)
    dg1, db1 = ops.conv_bn_backward(L.CONV_S2, B, L.nhwc_view(dyb), Cin, w, Cout, L.nhwc_view(out1), BF,
                                    bn_x=L.nhwc_view(x), C=C, bn_state=st, gamma=bn.gamma, s_self=0.2, ch_off=ch_off,
                                    g_other=L.nhwc_view(go), s_other=0.0, dxv=L.nhwc_view(dx1))
    out2 = torch.zeros((B, GH, GW, Cout), device=DEV, dtype=BF)
    ops.conv(L.CONV_S2, B, L.nhwc_view(dyb), Cin, w, Cout, L.nhwc_view(out2), BF)
    dx2 = torch.empty((B, GH, GW, C), device=DEV, dtype=BF)
    dg2, db2 = ops.bn_backward(B, L.nhwc_view(x), C, BF, L.nhwc_view(dx2), g1=L.nhwc_view(out2, ch_off), s1=0.2,
                               g2=L.nhwc_view(go), s2=0.0, bn_state=(bn.scale, bn.shift, bn.mean, bn.rstd, bn.gamma))
    torch.cuda.synchronize()
    assert torch.equal(out1, out2)
    ref = F.conv2d(dy, wt, None, 2, 1)
    assert float((nchw(out1.float()) - ref).abs().max()) <= 1e-2 * float(ref.abs().max())
    for a, b_, nm in ((dg1, dg2, "dgamma"), (db1, db2, "dbeta")):
        err = float((a - b_).abs().max())
        assert err <= 1e-4 * float(b_.abs().max()) + 1e-5, f"{nm} {case}: {err:.3e}"
    err = float((dx1.float() - dx2.float()).abs().max())
    assert err <= 1e-2 * float(dx2.float().abs().max()), f"dx {case}: {err:.3e}"


def run_t(B, x, w, Cin, Cout, GH, GW, force):
    """ConvTranspose2d (stc_conv_fwd_ex with statistics) of NCHW fp32 x [B, Cin, GH, GW]."""
    xb = nhwc(x).to(DEV, BF)
    wp = ops.pack(L.PACK_CONVT_FWD, w.to(DEV), Cout, Cin, BF)
    y = torch.full((B, 2 * GH, 2 * GW, Cout), float("nan"), device=DEV, dtype=BF)
    part, nch = ops.conv_stats(L.CONVT_S2, B, L.nhwc_view(xb), Cin, wp, Cout, L.nhwc_view(y), BF, force=force)
    _, nq, plan = ops.conv_query(L.CONVT_S2, B, GH, GW, Cin, Cout, BF, force=force)
    assert nq == nch
    bn = torch.nn.BatchNorm2d(Cout).to(DEV)
    t = torch.empty((2, Cout), device=DEV)
    mean, rstd = ops.bn_finalize_part(part, nch, Cout, bn, t[0], t[1])
    var = 1.0 / rstd.double() ** 2 - bn.eps
    torch.cuda.synchronize()
    return nchw(y.float()), mean.double(), var, plan


TCASES = [  # B, Cin, Cout, GH, GW (input grid)
    (2, 64, 128, 8, 64),
    (1, 128, 256, 16, 32),   # two chunks, two N tiles
    (1, 256, 512, 16, 16),
    (3, 64, 96, 4, 64),      # ragged N
    (2, 128, 64, 8, 64),     # N = 64: the 256 x 64 tile
    (1, 192, 40, 8, 32),     # N = 40 on the 256 x 64 tile, 3 chunks
    (4, 128, 128, 8, 8),     # 8-wide grid (tiles span images): the d4 geometry
    (8, 64, 64, 4, 8),
]


@pytest.mark.parametrize("shape", [HALO, HALO2, HALO_T2], ids=["8wave", "4wave", "phase_pair"])
@pytest.mark.parametrize("case", TCASES, ids=lambda c: "x".join(map(str, c)))
def test_halo_convT(case, shape):
    B, Cin, Cout, GH, GW = case
    x = q(rnd(B, Cin, GH, GW, seed=11, dev=DEV))
    w = q(rnd(Cin, Cout, 4, 4, seed=12, scale=0.05, dev=DEV))
    ref = F.conv_transpose2d(x, w, None, 2, 1)
    y, mean, var, plan = run_t(B, x, w, Cin, Cout, GH, GW, shape)
    assert plan[4] == ops.HALO_CFG and plan[1] == (64 if Cout <= 64 else 128)
    check(y, ref, mean, var, f"halo convT {case}")
    y2, _, _, plan2 = run_t(B, x, w, Cin, Cout, GH, GW, (0, 1))
    assert plan2[4] == 0
    assert float((y - y2).abs().max()) <= 1e-2 * float(ref.abs().max())


@pytest.mark.parametrize("case", [(32, 256, 64, 64, 64), (32, 128, 64, 64, 64)], ids=["d1", "e2_dgrad_geometry"])
def test_halo_convT_phase_pair_equals_single_phase(case):
    """The phase-pair block (GEOM 4, automatic at these train-step sizes) sums every phase's taps in the single-phase
    block's order (the same 4 x 1 waves of 64 x 64): outputs and BatchNorm partials bit-identical to GEOM 1, and
    within bf16 rounding of torch."""
    B, Cin, Cout, GH, GW = case
    x = q(rnd(B, Cin, GH, GW, seed=21, dev=DEV))
    w = q(rnd(Cin, Cout, 4, 4, seed=22, scale=0.05, dev=DEV))
    y1, m1, v1, _ = run_t(B, x, w, Cin, Cout, GH, GW, None)
    y2, m2, v2, _ = run_t(B, x, w, Cin, Cout, GH, GW, HALO_G1)
    assert torch.equal(y1, y2) and torch.equal(m1, m2) and torch.equal(v1, v2)
    ref = F.conv_transpose2d(x, w, None, 2, 1)
    check(y1, ref, m1, v1, f"halo convT phase pair {case}")


def test_halo_convT_plan_automatic_at_train_sizes():
    """The generators' ConvT layers (forward and the conv-s2 input gradients) with 64-channel chunks and whole-row
    tiles take the halo kernel at the train-step size."""
    for (gh, cin, cout) in ((32, 512, 128), (16, 1024, 256), (64, 256, 64), (32, 256, 128), (16, 512, 256),
                            (64, 128, 64)):
        assert ops.conv_query(L.CONVT_S2, 32, gh, gh, cin, cout, BF)[2][4] == ops.HALO_CFG, (gh, cin, cout)
    # d4 (8 x 8 grid, 1024 -> 512): the 256 x 64 block (256 blocks; 128-channel tiles would leave half the chip idle)
    plan = ops.conv_query(L.CONVT_S2, 32, 8, 8, 1024, 512, BF)[2]
    assert plan[4] == ops.HALO_CFG and plan[1] == 64
    for (gh, cin, cout) in ((128, 128, 1), (4, 1024, 512)):
        assert ops.conv_query(L.CONVT_S2, 32, gh, gh, cin, cout, BF)[2][4] != ops.HALO_CFG, (gh, cin, cout)


@pytest.mark.parametrize("case", [(32, 256, 128, 32, 32, 128, 0), (32, 128, 64, 64, 64, 64, 0)],
                         ids=["e3_dgrad", "e2_dgrad_n64"])
def test_halo_convT_bn_backward(case):
    """The conv-s2 input gradient (ConvT geometry) at its train-step size with the fused BatchNorm-backward sums."""
    B, Cin, Cout, GH, GW, C, ch_off = case
    assert ops.conv_query(L.CONVT_S2, B, GH, GW, Cin, Cout, BF)[2][4] == ops.HALO_CFG
    wt = q(rnd(Cin, Cout, 4, 4, seed=61, scale=0.05, dev=DEV))
    w = ops.pack(L.PACK_CONVT_FWD, wt, Cout, Cin, BF)
    dy = q(rnd(B, Cin, GH, GW, seed=62, scale=0.5, dev=DEV))
    dyb = nhwc(dy).to(BF)
    oh, ow = 2 * GH, 2 * GW
    x = torch.randn((B, oh, ow, C), generator=torch.Generator(device=DEV).manual_seed(63), device=DEV).to(BF)
    go = torch.randn((B, oh, ow, C), generator=torch.Generator(device=DEV).manual_seed(64), device=DEV).to(BF)
    bn = _BNT(C, 65)
    st = (bn.scale, bn.shift, bn.mean, bn.rstd)
    out1 = torch.zeros((B, oh, ow, Cout), device=DEV, dtype=BF)
    dx1 = torch.empty((B, oh, ow, C), device=DEV, dtype=BF)
    dg1, db1 = ops.conv_bn_backward(L.CONVT_S2, B, L.nhwc_view(dyb), Cin, w, Cout, L.nhwc_view(out1), BF,
                                    bn_x=L.nhwc_view(x), C=C, bn_state=st, gamma=bn.gamma, s_self=0.2, ch_off=ch_off,
                                    g_other=L.nhwc_view(go), s_other=0.0, dxv=L.nhwc_view(dx1))
    out2 = torch.zeros((B, oh, ow, Cout), device=DEV, dtype=BF)
    ops.conv(L.CONVT_S2, B, L.nhwc_view(dyb), Cin, w, Cout, L.nhwc_view(out2), BF)
    dx2 = torch.empty((B, oh, ow, C), device=DEV, dtype=BF)
    dg2, db2 = ops.bn_backward(B, L.nhwc_view(x), C, BF, L.nhwc_view(dx2), g1=L.nhwc_view(out2, ch_off), s1=0.2,
                               g2=L.nhwc_view(go), s2=0.0, bn_state=(bn.scale, bn.shift, bn.mean, bn.rstd, bn.gamma))
    torch.cuda.synchronize()
    assert torch.equal(out1, out2)
    ref = F.conv_transpose2d(dy, wt, None, 2, 1)
    assert float((nchw(out1.float()) - ref).abs().max()) <= 1e-2 * float(ref.abs().max())
    for a, b_, nm in ((dg1, dg2, "dgamma"), (db1, db2, "dbeta")):
        err = float((a - b_).abs().max())
        assert err <= 1e-4 * float(b_.abs().max()) + 1e-5, f"{nm} {case}: {err:.3e}"
    err = float((dx1.float() - dx2.float()).abs().max())
    assert err <= 1e-2 * float(dx2.float().abs().max()), f"dx {case}: {err:.3e}"


# ---- Conv2d k4 s1 p1 (the PatchGAN's stride-1 layer, STCGAN/networks.py:172-178) and its input gradient

def run_s1(kind, B, x, w, Cin, Cout, out_hw, force):
    """stc_conv_fwd_ex (with statistics) of kind CONV_S1 / CONV_S1_DGRAD on NCHW fp32 x (w: the conv weight)."""
    pack = L.PACK_CONV_FWD if kind == L.CONV_S1 else L.PACK_CONV_S1_DGRAD
    xb = nhwc(x).to(DEV, BF)
    wp = ops.pack(pack, w.to(DEV), Cout, Cin, BF)
    Ho, Wo = out_hw
    y = torch.full((B, Ho, Wo, Cout), float("nan"), device=DEV, dtype=BF)
    part, nch = ops.conv_stats(kind, B, L.nhwc_view(xb), Cin, wp, Cout, L.nhwc_view(y), BF, force=force)
    _, nq, plan = ops.conv_query(kind, B, Ho, Wo, Cin, Cout, BF, force=force)
    assert nq == nch
    bn = torch.nn.BatchNorm2d(Cout).to(DEV)
    t = torch.empty((2, Cout), device=DEV)
    mean, rstd = ops.bn_finalize_part(part, nch, Cout, bn, t[0], t[1])
    var = 1.0 / rstd.double() ** 2 - bn.eps
    torch.cuda.synchronize()
    return nchw(y.float()), mean.double(), var, plan


S1CASES = [  # B, conv Cin, conv Cout (32 x 32 -> 31 x 31)
    (1, 64, 128),
    (2, 128, 200),   # ragged N
    (1, 256, 512),   # the PatchGAN layer's channels
]


@pytest.mark.parametrize("shape", [HALO, HALO2], ids=["8wave", "4wave"])
@pytest.mark.parametrize("case", S1CASES, ids=lambda c: "x".join(map(str, c)))
def test_halo_conv_s1(case, shape):
    """Forward on the 32 x 32 grid with the last row / column masked: output, and statistics over the 31 x 31
    pixels only."""
    B, Cin, Cout = case
    x = q(rnd(B, Cin, 32, 32, seed=71, dev=DEV))
    w = q(rnd(Cout, Cin, 4, 4, seed=72, scale=0.05, dev=DEV))
    ref = F.conv2d(x, w, None, 1, 1)
    y, mean, var, plan = run_s1(L.CONV_S1, B, x, w, Cin, Cout, (31, 31), shape)
    assert plan[4] == ops.HALO_CFG
    check(y, ref, mean, var, f"halo s1 {case}")
    y2, _, _, plan2 = run_s1(L.CONV_S1, B, x, w, Cin, Cout, (31, 31), (0, 1))
    assert plan2[4] == 0
    assert float((y - y2).abs().max()) <= 1e-2 * float(ref.abs().max())


@pytest.mark.parametrize("shape", [HALO, HALO2], ids=["8wave", "4wave"])
@pytest.mark.parametrize("case", S1CASES, ids=lambda c: "x".join(map(str, c)))
def test_halo_conv_s1_dgrad(case, shape):
    """Input gradient dx = conv_transpose2d(dy, w, stride 1, pad 1): 31 x 31 x Cout -> 32 x 32 x Cin."""
    B, Cin, Cout = case
    if Cout % 64:
        pytest.skip("the reduction (conv Cout) needs 64-channel chunks")
    dy = q(rnd(B, Cout, 31, 31, seed=73, dev=DEV))
    w = q(rnd(Cout, Cin, 4, 4, seed=74, scale=0.05, dev=DEV))
    ref = F.conv_transpose2d(dy, w, None, 1, 1)
    y, mean, var, plan = run_s1(L.CONV_S1_DGRAD, B, dy, w, Cout, Cin, (32, 32), shape)
    assert plan[4] == ops.HALO_CFG
    check(y, ref, mean, var, f"halo s1 dgrad {case}")
    y2, _, _, plan2 = run_s1(L.CONV_S1_DGRAD, B, dy, w, Cout, Cin, (32, 32), (0, 1))
    assert plan2[4] == 0
    assert float((y - y2).abs().max()) <= 1e-2 * float(ref.abs().max())


def test_halo_s1_plan_automatic_at_train_size():
    assert ops.conv_query(L.CONV_S1, 32, 31, 31, 256, 512, BF)[2][4] == ops.HALO_CFG
    assert ops.conv_query(L.CONV_S1_DGRAD, 32, 32, 32, 512, 256, BF)[2][4] == ops.HALO_CFG
    # other grids keep the im2col tiles
    assert ops.conv_query(L.CONV_S1, 32, 15, 15, 256, 512, BF)[2][4] != ops.HALO_CFG
    assert ops.conv_query(L.CONV_S1, 32, 30, 30, 512, 1, BF)[2][4] != ops.HALO_CFG


def test_halo_conv_s1_full_size():
    """The PatchGAN's layer 4 forward at the bench size (bs 32, 32x32x256 -> 31x31x512), automatic plan."""
    B, Cin, Cout = 32, 256, 512
    x = q(rnd(B, Cin, 32, 32, seed=75, dev=DEV))
    w = q(rnd(Cout, Cin, 4, 4, seed=76, scale=0.05, dev=DEV))
    ref = F.conv2d(x, w, None, 1, 1)
    y, mean, var, plan = run_s1(L.CONV_S1, B, x, w, Cin, Cout, (31, 31), None)
    assert plan[4] == ops.HALO_CFG
    check(y, ref, mean, var, "halo s1 full size")


def test_halo_conv_s1_dgrad_bn_backward():
    """The stride-1 layer's input gradient at the bench size with the fused BatchNorm-backward sums of the layer
    below (PatchGAN layer 3's BN, 256 channels)."""
    B, Cin, Cout, C = 32, 512, 256, 256   # GEMM: 31x31x512 -> 32x32x256
    assert ops.conv_query(L.CONV_S1_DGRAD, B, 32, 32, Cin, Cout, BF)[2][4] == ops.HALO_CFG
    wt = q(rnd(Cin, Cout, 4, 4, seed=81, scale=0.05, dev=DEV))  # conv weight [512][256]
    w = ops.pack(L.PACK_CONV_S1_DGRAD, wt, Cout, Cin, BF)
    dy = q(rnd(B, Cin, 31, 31, seed=82, scale=0.5, dev=DEV))
    dyb = nhwc(dy).to(BF)
    x = torch.randn((B, 32, 32, C), generator=torch.Generator(device=DEV).manual_seed(83), device=DEV).to(BF)
    bn = _BNT(C, 85)
    st = (bn.scale, bn.shift, bn.mean, bn.rstd)
    out1 = torch.zeros((B, 32, 32, Cout), device=DEV, dtype=BF)
    dx1 = torch.empty((B, 32, 32, C), device=DEV, dtype=BF)
    dg1, db1 = ops.conv_bn_backward(L.CONV_S1_DGRAD, B, L.nhwc_view(dyb), Cin, w, Cout, L.nhwc_view(out1), BF,
                                    bn_x=L.nhwc_view(x), C=C, bn_state=st, gamma=bn.gamma, s_self=0.2,
                                    dxv=L.nhwc_view(dx1))
    out2 = torch.zeros((B, 32, 32, Cout), device=DEV, dtype=BF)
    ops.conv(L.CONV_S1_DGRAD, B, L.nhwc_view(dyb), Cin, w, Cout, L.nhwc_view(out2), BF)
    dx2 = torch.empty((B, 32, 32, C), device=DEV, dtype=BF)
    dg2, db2 = ops.bn_backward(B, L.nhwc_view(x), C, BF, L.nhwc_view(dx2), g1=L.nhwc_view(out2), s1=0.2,
                               bn_state=(bn.scale, bn.shift, bn.mean, bn.rstd, bn.gamma))
    torch.cuda.synchronize()
    assert torch.equal(out1, out2)
    ref = F.conv_transpose2d(dy, wt, None, 1, 1)
    assert float((nchw(out1.float()) - ref).abs().max()) <= 1e-2 * float(ref.abs().max())
    for a, b_, nm in ((dg1, dg2, "dgamma"), (db1, db2, "dbeta")):
        err = float((a - b_).abs().max())
        assert err <= 1e-4 * float(b_.abs().max()) + 1e-5, f"{nm}: {err:.3e}"
    err = float((dx1.float() - dx2.float()).abs().max())
    assert err <= 1e-2 * float(dx2.float().abs().max()), f"dx: {err:.3e}"
