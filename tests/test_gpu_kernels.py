"""Per-kernel parity of the HIP path against torch-CPU fp32 references of the same op.

Tolerances (fp32): the f32 MFMA is an exact fmaf chain in a different summation
order than mkldnn, so errors scale like eps32 * sqrt(K) * |values|; every
check below uses max-abs error <= 2e-5 * max|ref| + 1e-6 unless stated.
bf16 checks use 2e-2 relative to max|ref| (8-bit mantissa operands, fp32 accumulation).
"""
import pytest
import torch
import torch.nn.functional as F

from stcgan_amd import _lib as L
from stcgan_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def close(got, ref, tol=2e-5, what=""):
    got = got.detach().float().cpu()
    ref = ref.detach().float().cpu()
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    scale = float(ref.abs().max()) + 1e-12
    err = float((got - ref).abs().max())
    assert err <= tol * scale + 1e-6, f"{what}: max err {err:.3e} vs scale {scale:.3e}"
    return err


def rnd(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(shape, generator=g) * scale


CONV_CASES = [  # B, Cin, Cout, H, W
    (2, 4, 64, 64, 64),      # first layer (padded channels), N=64 tile
    (2, 64, 128, 32, 32),    # 128x128 tile
    (2, 128, 256, 16, 16),
    (1, 512, 512, 4, 4),     # small M -> split-K
    (2, 512, 512, 2, 2),     # bottleneck M = 2
    (3, 32, 96, 10, 14),     # ragged tiles
    (2, 16, 1, 16, 16),      # N = 1 (last layer)
    (2, 8, 3, 12, 12),       # N = 3
]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("stride", [2, 1])
def test_conv_fwd(case, stride, dt):
    B, Cin, Cout, H, W = case
    if Cin < ops.vec(dt):
        pytest.skip("Cin below the vector width (padded at the model edge)")
    x = rnd(B, Cin, H, W, seed=1)
    w = rnd(Cout, Cin, 4, 4, seed=2, scale=0.05)
    sc = torch.rand(Cin, generator=torch.Generator().manual_seed(3)) + 0.5
    sh = rnd(Cin, seed=4, scale=0.2)
    bias = rnd(Cout, seed=5)
    ref = F.conv2d(F.leaky_relu(x * sc[None, :, None, None] + sh[None, :, None, None], 0.2), w, bias, stride, 1)
    xg = nhwc(x).to(DEV, dt)
    wp = ops.pack(L.PACK_CONV_FWD, w.to(DEV), Cout, Cin, dt)
    Ho, Wo = ref.shape[2], ref.shape[3]
    y = torch.full((B, Ho, Wo, Cout), float("nan"), device=DEV, dtype=torch.float32)
    ops.conv(L.CONV_S2 if stride == 2 else L.CONV_S1, B, L.nhwc_view(xg), Cin, wp, Cout, L.nhwc_view(y), dt,
             pro=(sc.to(DEV), sh.to(DEV)), slope=0.2, bias=bias.to(DEV), out_f32=True)
    if dt == torch.bfloat16:
        xr = (x * sc[None, :, None, None] + sh[None, :, None, None])
        ref = F.conv2d(F.leaky_relu(xr, 0.2), w, bias, stride, 1)
        close(nchw(y), ref, tol=3e-2, what="conv bf16")
    else:
        close(nchw(y), ref, what="conv fwd")


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CONV_CASES)
def test_convT_fwd(case, dt):
    B, Cin, Cout, H, W = case
    if Cin < ops.vec(dt) or (4 * Cin) % (32 if dt == torch.float32 else 64):
        pytest.skip("K = 4*Cin not a whole number of K-steps")
    x = rnd(B, Cin, H, W, seed=11)
    w = rnd(Cin, Cout, 4, 4, seed=12, scale=0.05)
    ref = F.conv_transpose2d(F.relu(x), w, None, 2, 1)
    xg = nhwc(x).to(DEV, dt)
    wp = ops.pack(L.PACK_CONVT_FWD, w.to(DEV), Cout, Cin, dt)
    y = torch.full((B, 2 * H, 2 * W, Cout), float("nan"), device=DEV, dtype=torch.float32)
    ops.conv(L.CONVT_S2, B, L.nhwc_view(xg), Cin, wp, Cout, L.nhwc_view(y), dt, slope=0.0, out_f32=True)
    close(nchw(y), ref, tol=3e-2 if dt == torch.bfloat16 else 2e-5, what="convT fwd")


NARROW_CASES = [  # kind, B, Cin, N, H, W  (GEMM grid = input grid for convT, output grid for conv s1)
    ("convT", 2, 128, 3, 20, 24),   # G output layer geometry (partial 16x16 tiles)
    ("convT", 2, 128, 1, 16, 16),
    ("convT", 1, 64, 8, 9, 13),     # first-layer input-gradient geometry, N = 8
    ("convT", 2, 64, 4, 32, 32),
    ("conv_s1", 2, 512, 1, 31, 31),  # PatchGAN logits: 31x31 -> 30x30
    ("conv_s1", 1, 256, 2, 12, 10),
]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", NARROW_CASES)
def test_narrow_n_paths(case, dt):
    kind, B, Cin, N, H, W = case
    x = rnd(B, Cin, H, W, seed=17)
    sc = torch.rand(Cin, generator=torch.Generator().manual_seed(18)) + 0.5
    sh = rnd(Cin, seed=19, scale=0.2)
    b = rnd(N, seed=20)
    xa = F.relu(x * sc[None, :, None, None] + sh[None, :, None, None])
    xg = nhwc(x).to(DEV, dt)
    if dt == torch.bfloat16:
        xa = F.relu(nchw(xg.float().cpu()) * sc[None, :, None, None] + sh[None, :, None, None])
        xa = xa.to(torch.bfloat16).float()
    if kind == "convT":
        w = rnd(Cin, N, 4, 4, seed=21, scale=0.05)
        wq = w.to(torch.bfloat16).float() if dt == torch.bfloat16 else w
        ref = torch.tanh(F.conv_transpose2d(xa, wq, b, 2, 1))
        wp = ops.pack(L.PACK_CONVT_FWD, w.to(DEV), N, Cin, dt)
        y = torch.empty((B, N, 2 * H, 2 * W), device=DEV)
        ops.conv(L.CONVT_S2, B, L.nhwc_view(xg), Cin, wp, N, L.nchw_view(y), dt, pro=(sc.to(DEV), sh.to(DEV)),
                 slope=0.0, bias=b.to(DEV), tanh=True, out_f32=True)
    else:
        w = rnd(N, Cin, 4, 4, seed=22, scale=0.05)
        wq = w.to(torch.bfloat16).float() if dt == torch.bfloat16 else w
        ref = torch.tanh(F.conv2d(xa, wq, b, 1, 1))
        wp = ops.pack(L.PACK_CONV_FWD, w.to(DEV), N, Cin, dt)
        y = torch.empty((B, N, H - 1, W - 1), device=DEV)
        ops.conv(L.CONV_S1, B, L.nhwc_view(xg), Cin, wp, N, L.nchw_view(y), dt, pro=(sc.to(DEV), sh.to(DEV)),
                 slope=0.0, bias=b.to(DEV), tanh=True, out_f32=True)
    assert ops.plan_of(L.CONVT_S2 if kind == "convT" else L.CONV_S1, B, H if kind == "convT" else H - 1,
                       W if kind == "convT" else W - 1, Cin, N, dt)[3] == 1
    # fp32: one serial fmaf chain per output over K = 16*Cin (8192 terms for the logits layer)
    close(y, ref, tol=3e-5 if dt == torch.float32 else 1e-3, what=f"narrow {kind}")


def test_convT_tanh_bias_nchw_out():
    B, Cin, Cout, H, W = 2, 32, 3, 8, 8
    x = rnd(B, Cin, H, W, seed=21)
    w = rnd(Cin, Cout, 4, 4, seed=22, scale=0.1)
    b = rnd(Cout, seed=23)
    ref = torch.tanh(F.conv_transpose2d(x, w, b, 2, 1))
    xg = nhwc(x).to(DEV)
    wp = ops.pack(L.PACK_CONVT_FWD, w.to(DEV), Cout, Cin, torch.float32)
    y = torch.empty((B, Cout, 2 * H, 2 * W), device=DEV)
    ops.conv(L.CONVT_S2, B, L.nhwc_view(xg), Cin, wp, Cout, L.nchw_view(y), torch.float32, bias=b.to(DEV),
             tanh=True, out_f32=True)
    close(y, ref, what="convT tanh nchw")


@pytest.mark.parametrize("case", CONV_CASES[1:6])
@pytest.mark.parametrize("stride", [2, 1])
def test_conv_dgrad(case, stride):
    B, Cin, Cout, H, W = case
    x = rnd(B, Cin, H, W, seed=31).requires_grad_(True)
    w = rnd(Cout, Cin, 4, 4, seed=32, scale=0.05)
    y = F.conv2d(x, w, None, stride, 1)
    dy = rnd(*y.shape, seed=33)
    (gx,) = torch.autograd.grad(y, x, dy)
    dyg = nhwc(dy).to(DEV)
    dt = torch.float32
    if stride == 2:
        if H % 2 or W % 2:
            pytest.skip("odd input of a stride-2 conv: last row/col grad is outside the 2x grid")
        wp = ops.pack(L.PACK_CONV_DGRAD, w.to(DEV), Cin, Cout, dt)
        out = torch.empty((B, H, W, Cin), device=DEV)
        ops.conv(L.CONVT_S2, B, L.nhwc_view(dyg), Cout, wp, Cin, L.nhwc_view(out), dt)
    else:
        wp = ops.pack(L.PACK_CONV_S1_DGRAD, w.to(DEV), Cin, Cout, dt)
        out = torch.empty((B, H, W, Cin), device=DEV)
        ops.conv(L.CONV_S1_DGRAD, B, L.nhwc_view(dyg), Cout, wp, Cin, L.nhwc_view(out), dt)
    close(nchw(out), gx, what="conv dgrad")


@pytest.mark.parametrize("case", CONV_CASES[1:6])
def test_convT_dgrad(case):
    B, Cin, Cout, H, W = case
    x = rnd(B, Cin, H, W, seed=41).requires_grad_(True)
    w = rnd(Cin, Cout, 4, 4, seed=42, scale=0.05)
    y = F.conv_transpose2d(x, w, None, 2, 1)
    dy = rnd(*y.shape, seed=43)
    (gx,) = torch.autograd.grad(y, x, dy)
    dt = torch.float32
    wp = ops.pack(L.PACK_CONVT_DGRAD, w.to(DEV), Cin, Cout, dt)
    out = torch.empty((B, H, W, Cin), device=DEV)
    ops.conv(L.CONV_S2, B, L.nhwc_view(nhwc(dy).to(DEV)), Cout, wp, Cin, L.nhwc_view(out), dt)
    close(nchw(out), gx, what="convT dgrad")


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CONV_CASES[:6])
@pytest.mark.parametrize("stride", [2, 1])
def test_conv_wgrad(case, stride, dt):
    B, Cin, Cout, H, W = case
    if Cin < ops.vec(dt) or Cout % ops.vec(dt):
        pytest.skip("channels below the vector width (padded at the model edge)")
    x = rnd(B, Cin, H, W, seed=51)
    w = rnd(Cout, Cin, 4, 4, seed=52, scale=0.05).requires_grad_(True)
    sc = torch.rand(Cin, generator=torch.Generator().manual_seed(53)) + 0.5
    sh = rnd(Cin, seed=54, scale=0.2)
    xa = F.leaky_relu(x * sc[None, :, None, None] + sh[None, :, None, None], 0.2)
    y = F.conv2d(xa, w, None, stride, 1)
    dy = rnd(*y.shape, seed=55)
    (gw,) = torch.autograd.grad(y, w, dy)
    xg = nhwc(x).to(DEV, dt)
    dyg = nhwc(dy).to(DEV, dt)
    if dt == torch.bfloat16:  # reference on the bf16-rounded operands
        xb = nchw(xg.float().cpu())
        xa = F.leaky_relu(xb * sc[None, :, None, None] + sh[None, :, None, None], 0.2)
        w2 = w.detach().clone().requires_grad_(True)
        y = F.conv2d(xa, w2, None, stride, 1)
        (gw,) = torch.autograd.grad(y, w2, nchw(dyg.float().cpu()))
    dW = ops.wgrad(B, stride, L.nhwc_view(dyg), Cout, L.nhwc_view(xg), Cin, Cin, dt,
                   gpro=(sc.to(DEV), sh.to(DEV)), gslope=0.2, device=DEV)
    # bf16: operands (incl. the prologue output) are bf16-rounded before the MFMA
    close(dW, gw, tol=1e-2 if dt == torch.bfloat16 else 2e-5, what="conv wgrad")


@pytest.mark.parametrize("case", CONV_CASES[1:6])
def test_convT_wgrad_bf16(case):
    B, Cin, Cout, H, W = case
    if Cout % 8:
        pytest.skip()
    dt = torch.bfloat16
    x = rnd(B, Cin, H, W, seed=64)
    dy = rnd(B, Cout, 2 * H, 2 * W, seed=65)
    xg, dyg = nhwc(x).to(DEV, dt), nhwc(dy).to(DEV, dt)
    xb = F.relu(nchw(xg.float().cpu())).to(torch.bfloat16).float()
    w = torch.zeros(Cin, Cout, 4, 4, requires_grad=True)
    y = F.conv_transpose2d(xb, w, None, 2, 1)
    (gw,) = torch.autograd.grad(y, w, nchw(dyg.float().cpu()))
    dW = ops.wgrad(B, 2, L.nhwc_view(xg), Cin, L.nhwc_view(dyg), Cout, Cout, dt, dslope=0.0, device=DEV)
    close(dW, gw, tol=2e-5, what="convT wgrad bf16")  # exact bf16 products, fp32 sums


@pytest.mark.parametrize("case", CONV_CASES[1:6])
def test_convT_wgrad(case):
    B, Cin, Cout, H, W = case
    x = rnd(B, Cin, H, W, seed=61)
    w = rnd(Cin, Cout, 4, 4, seed=62, scale=0.05).requires_grad_(True)
    y = F.conv_transpose2d(F.relu(x), w, None, 2, 1)
    dy = rnd(*y.shape, seed=63)
    (gw,) = torch.autograd.grad(y, w, dy)
    dW = ops.wgrad(B, 2, L.nhwc_view(nhwc(x).to(DEV)), Cin, L.nhwc_view(nhwc(dy).to(DEV)), Cout, Cout,
                   torch.float32, dslope=0.0, device=DEV)
    close(dW, gw, what="convT wgrad")


class _BN:
    def __init__(self, C, seed):
        g = torch.Generator().manual_seed(seed)
        self.weight = (torch.rand(C, generator=g) + 0.5).to(DEV)
        self.bias = (torch.randn(C, generator=g) * 0.1).to(DEV)
        self.running_mean = (torch.randn(C, generator=g) * 0.1).to(DEV)
        self.running_var = (torch.rand(C, generator=g) + 0.5).to(DEV)
        self.num_batches_tracked = torch.zeros((), dtype=torch.long, device=DEV)
        self.momentum, self.eps = 0.1, 1e-5


@pytest.mark.parametrize("shape", [(4, 64, 16, 16), (2, 512, 1, 1), (3, 128, 15, 20), (32, 8, 2, 2)])
def test_bn_stats_and_backward(shape):
    B, C, H, W = shape
    x = rnd(B, C, H, W, seed=71) * 3 + 1.5  # non-zero mean: exercises the shifted sums
    bn = _BN(C, 72)
    rm0, rv0 = bn.running_mean.cpu().clone(), bn.running_var.cpu().clone()
    xg = nhwc(x).to(DEV)
    tab = torch.empty((2, C), device=DEV)
    mean, rstd = ops.bn_train_table(B, L.nhwc_view(xg), C, torch.float32, bn, tab[0], tab[1])
    ref_m = x.mean(dim=(0, 2, 3))
    ref_v = x.var(dim=(0, 2, 3), unbiased=False)
    close(mean, ref_m, tol=1e-6, what="mean")
    close(rstd, torch.rsqrt(ref_v + 1e-5), tol=1e-5, what="rstd")
    n = B * H * W
    close(bn.running_mean, 0.9 * rm0 + 0.1 * ref_m, tol=1e-6, what="running_mean")
    close(bn.running_var, 0.9 * rv0 + 0.1 * ref_v * n / max(n - 1, 1), tol=1e-5, what="running_var")
    assert int(bn.num_batches_tracked) == 1
    # backward: n = BN(x); dn = g1*relu'(n) + g2*lrelu'(n)
    xr = x.clone().requires_grad_(True)
    gam = bn.weight.cpu().clone().requires_grad_(True)
    bet = bn.bias.cpu().clone().requires_grad_(True)
    nrm = F.batch_norm(xr, None, None, gam, bet, True, 0.0, 1e-5)
    g1 = rnd(*x.shape, seed=73)
    g2 = rnd(*x.shape, seed=74)
    out = (F.relu(nrm) * g1).sum() + (F.leaky_relu(nrm, 0.2) * g2).sum()
    gx, gg, gb = torch.autograd.grad(out, (xr, gam, bet))
    dx = torch.empty_like(xg)
    dg, db = ops.bn_backward(B, L.nhwc_view(xg), C, torch.float32, L.nhwc_view(dx),
                             g1=L.nhwc_view(nhwc(g1).to(DEV)), s1=0.0, g2=L.nhwc_view(nhwc(g2).to(DEV)), s2=0.2,
                             bn_state=(tab[0], tab[1], mean, rstd, bn.weight))
    close(nchw(dx), gx, tol=1e-4, what="bn dx")
    close(dg, gg, tol=1e-5, what="dgamma")
    close(db, gb, tol=1e-5, what="dbeta")


def test_act_backward_no_bn():
    x = rnd(2, 16, 8, 8, seed=81)
    g1, g2 = rnd(2, 16, 8, 8, seed=82), rnd(2, 16, 8, 8, seed=83)
    ref = g1 * (x > 0).float() + g2 * torch.where(x > 0, 1.0, 0.2)
    xg = nhwc(x).to(DEV)
    dx = torch.empty_like(xg)
    ops.bn_backward(2, L.nhwc_view(xg), 16, torch.float32, L.nhwc_view(dx), g1=L.nhwc_view(nhwc(g1).to(DEV)),
                    s1=0.0, g2=L.nhwc_view(nhwc(g2).to(DEV)), s2=0.2)
    close(nchw(dx), ref, tol=1e-6, what="act bwd")


def test_gather_scatter_roundtrip():
    x, m, y = rnd(2, 3, 10, 12, seed=91), rnd(2, 1, 10, 12, seed=92), rnd(2, 3, 10, 12, seed=93)
    dst = torch.empty((2, 10, 12, 8), device=DEV)
    ops.gather([x.to(DEV), m.to(DEV), y.to(DEV)], dst, torch.float32)
    ref = torch.cat([x, m, y, torch.zeros(2, 1, 10, 12)], 1)
    close(nchw(dst), ref, tol=0.0, what="gather")
    outs = [torch.zeros(2, 3, 10, 12, device=DEV), None, torch.zeros(2, 3, 10, 12, device=DEV)]
    ops.scatter(dst, outs, [3, 1, 3], torch.float32)
    close(outs[0], x, tol=0.0, what="scatter x")
    close(outs[2], y, tol=0.0, what="scatter y")


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
@pytest.mark.parametrize("chans,H,W", [((3,), 16, 32), ((3, 1), 32, 64), ((3, 1, 3), 16, 16), ((4,), 64, 12)])
def test_gather_runs(dt, chans, H, W):
    """The vectorised gather (gather4: W % 4 == 0, aligned planes): NCHW fp32 sources -> NHWC [B, H, W, Cpad], exact
    (bf16: the round-to-nearest-even cast), padding channels zero."""
    B = 3
    srcs = [rnd(B, c, H, W, seed=200 + i) for i, c in enumerate(chans)]
    cpad = 8 if dt == torch.bfloat16 or sum(chans) > 4 else 4
    dst = torch.full((B, H, W, cpad), float("nan"), device=DEV, dtype=dt)
    ops.gather([t.to(DEV) for t in srcs], dst, dt)
    ref = torch.cat(srcs + [torch.zeros(B, cpad - sum(chans), H, W)], 1).to(dt)
    assert torch.equal(nchw(dst).cpu(), ref)


def test_tanh_bias_bwd_and_chan_sum():
    y = torch.tanh(rnd(2, 3, 8, 8, seed=101))
    gy = rnd(2, 3, 8, 8, seed=102)
    dq = torch.empty((2, 8, 8, 4), device=DEV)
    db = ops.tanh_bias_bwd(y.to(DEV), gy.to(DEV), L.nhwc_view(dq), torch.float32)
    ref = gy * (1 - y * y)
    close(nchw(dq)[:, :3], ref, tol=1e-6, what="tanh bwd")
    assert float(dq[..., 3].abs().max()) == 0.0
    close(db, ref.sum(dim=(0, 2, 3)), tol=1e-6, what="dbias")
    s = ops.chan_sum(2, L.nhwc_view(dq), 4, 3, torch.float32, DEV)
    close(s, ref.sum(dim=(0, 2, 3)), tol=1e-6, what="chan_sum")


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
@pytest.mark.parametrize("B,C,H,W", [(32, 3, 256, 256), (32, 1, 256, 256), (3, 3, 10, 12), (2, 1, 6, 10)],
                         ids=["c3_256", "c1_256", "quad_small", "scalar_w10"])
def test_tanh_bias_bwd_paths(dt, B, C, H, W):
    """The output layer's tanh + bias backward (4 pixels per thread where W % 4 == 0, else per pixel): dq to the
    per-element formula within fp32 rounding (bf16: the output cast), padding channels zero, dbias within fp32
    reordering of the per-channel sum."""
    g = torch.Generator().manual_seed(B * 7 + C)
    y = torch.tanh(torch.randn(B, C, H, W, generator=g)).to(DEV)
    gy = torch.randn(B, C, H, W, generator=g).to(DEV)
    cpad = 4 if dt == torch.float32 else 8
    dq = torch.full((B, H, W, cpad), float("nan"), device=DEV, dtype=dt)
    db = ops.tanh_bias_bwd(y, gy, L.nhwc_view(dq), dt)
    ref = gy * (1 - y * y)
    err = float((nchw(dq)[:, :C].float() - ref).abs().max())
    assert err <= (2e-6 if dt == torch.float32 else 8e-3) * float(ref.abs().max()), err  # (bf16: the output cast)
    assert float(dq[..., C:].float().abs().max()) == 0.0
    rs = ref.double().sum(dim=(0, 2, 3))
    assert float((db.double() - rs).abs().max()) <= 1e-5 * float(ref.abs().sum(dim=(0, 2, 3)).max())


@pytest.mark.parametrize("n", [1, 1000, 393216])
def test_losses(n):
    from stcgan_amd import loss as sl
    p = rnd(n, seed=111).to(DEV).requires_grad_(True)
    t = rnd(n, seed=112).to(DEV)
    for fn, ref in [(lambda a: sl.l1_loss(a, t), lambda a: F.l1_loss(a, t.cpu())),
                    (lambda a: sl.mse_const(a, 1.0), lambda a: F.mse_loss(a, torch.ones_like(a))),
                    (lambda a: sl.mse_const(a, 0.0), lambda a: F.mse_loss(a, torch.zeros_like(a))),
                    (lambda a: sl.bce_logits_const(a, -1.0),
                     lambda a: F.binary_cross_entropy_with_logits(a, -torch.ones_like(a)))]:
        v = fn(p)
        (g,) = torch.autograd.grad(v * 3.0, p)
        pc = p.detach().cpu().requires_grad_(True)
        rv = ref(pc)
        (rg,) = torch.autograd.grad(rv * 3.0, pc)
        close(v, rv, tol=1e-5, what="loss value")
        close(g, rg, tol=1e-6, what="loss grad")


def test_adam_matches_torch():
    from stcgan_amd.optim import Adam
    ps = [rnd(1000, seed=121).to(DEV), rnd(37, 5, seed=122).to(DEV), rnd(70000, seed=123).to(DEV)]
    ps = [torch.nn.Parameter(p) for p in ps]
    refs = [torch.nn.Parameter(p.detach().cpu().clone()) for p in ps]
    opt = Adam(ps, lr=5e-5, betas=(0.5, 0.999))
    ropt = torch.optim.Adam(refs, lr=5e-5, betas=(0.5, 0.999))
    for step in range(3):
        for i, (p, r) in enumerate(zip(ps, refs)):
            g = rnd(*p.shape, seed=200 + 10 * step + i)
            p.grad = g.to(DEV)
            r.grad = g.clone()
        opt.step()
        ropt.step()
    for p, r in zip(ps, refs):
        close(p, r, tol=1e-6, what="adam param")
