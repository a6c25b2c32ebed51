"""C3 (the bf16 train step of BASELINE config 3: ngf=64, bs=32, 256x256) checked layer by layer.

A whole-step comparison in bf16 cannot be tight: the generator's backward passes eight BatchNorm
backwards, each of which removes the mean and the x_hat-component of its incoming gradient, and the
relative bf16 storage noise (2^-9 per element) grows through them to 13-20 % at the innermost levels.
That is a property of the algorithm in bf16, not of an implementation: the oracle's own bf16 mode
(oracle/stcgan_ref.py Precision) moves its generator gradients by 13 % median / 20 % worst per tensor
under a 1e-6 relative perturbation of the weights (scripts/bf16_sensitivity.py; fp32: 0.3 %).

So every layer is checked on its OWN inputs instead: one G1 / G2 / D forward + backward at the C3 size
runs with engine.TRACE on, which keeps the HIP path's bf16 buffers of every level (the saved raw conv
outputs, activations and BatchNorm tables of the forward; the gradient entering and leaving every layer
of the backward).  Each layer's forward conv + BatchNorm statistics + activation, its weight gradient,
its input gradient and its fused activation + BatchNorm backward are recomputed from those bf16 inputs
with torch fp32 on the GPU (native convolutions, MIOpen off) and compared -- one layer deep, so the
tolerance is the layer's own bf16 rounding, not an amplified one:
  * weight and BatchNorm-parameter gradients (fp32 results): relative L2 <= 2e-3;
  * bf16 tensors (activations, raw outputs, gradients between layers): relative L2 <= 1e-2 and max
    |error| <= 2 % of the tensor's max (a bf16 rounding flip is 2^-8 of one element);
  * BatchNorm batch statistics (fp32): mean and rstd relative L2 <= 1e-4.
A wrong tile, a mis-indexed tap or a wrong BN term shows up at full size as an O(1) error in one check."""
import pytest
import torch
import torch.nn.functional as F

from fixture_init import fixture_state, pm_one, uniform

pytestmark = pytest.mark.gpu

DEV = "cuda"
BS = 32


def f(t, c=None):
    """NHWC (bf16/fp32) -> NCHW fp32 (first c channels)."""
    x = t.float().permute(0, 3, 1, 2)
    return (x if c is None else x[:, :c]).contiguous()


def q(t):
    return t.to(torch.bfloat16).float()


def rel(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return float((a - b).norm() / (b.norm() + 1e-30))


class Checker:
    def __init__(self):
        self.fails, self.worst = [], {}

    def fp32(self, what, got, want, tol=2e-3):
        e = rel(got, want)
        self.worst[what] = e
        if not e <= tol:
            self.fails.append((what, e))

    def bf16(self, what, got, want, tol=1e-2):
        e = rel(got, want)
        m = float((got.float() - want.float()).abs().max() / (want.float().abs().max() + 1e-30))
        self.worst[what] = e
        if not (e <= tol and m <= 0.02):
            self.fails.append((what, e, m))


def _wgrad_ref(fn, x, w, g):
    w = w.detach().clone().requires_grad_(True)
    x = x.detach().clone().requires_grad_(True)
    y = fn(x, w)
    gx, gw = torch.autograd.grad(y, (x, w), g)
    return gx, gw


def _bn_bwd_ref(raw, mean, rstd, gamma, dn):
    """Training-mode BatchNorm backward given dn = dL/d(BN output) (NCHW fp32)."""
    xh = (raw - mean[None, :, None, None]) * rstd[None, :, None, None]
    n = dn.shape[0] * dn.shape[2] * dn.shape[3]
    dgam = (dn * xh).sum(dim=(0, 2, 3))
    dbet = dn.sum(dim=(0, 2, 3))
    dx = gamma[None, :, None, None] * rstd[None, :, None, None] * (
        dn - dbet[None, :, None, None] / n - xh * dgam[None, :, None, None] / n)
    return dx, dgam, dbet


@pytest.fixture(autouse=True)
def _native_conv():
    prev = torch.backends.cudnn.enabled
    torch.backends.cudnn.enabled = False  # torch's own fp32 convolutions (no algorithm search)
    yield
    torch.backends.cudnn.enabled = prev


@pytest.mark.parametrize("name", ["G1", "G2"])
def test_c3_generator_layers(name):
    from stcgan_amd import engine, networks
    cin, cout = (3, 1) if name == "G1" else (4, 3)
    net = networks.get_generator(cin, cout, ngf=64)
    net.load_state_dict(fixture_state(net.state_dict(), 11 if name == "G1" else 12, "ref"))
    net.to(DEV).set_compute_dtype("bf16").train()
    x = uniform((BS, cin, 256, 256), 5100).to(DEV)
    gy = (uniform((BS, cout, 256, 256), 5101) * 1e-3).to(DEV)
    engine.TRACE = {}
    try:
        y = net(x)
        y.backward(gy)
        torch.cuda.synchronize()
        tr = engine.TRACE["G"][0]
    finally:
        engine.TRACE = None
    sv, plan = tr["saved"], net._plan
    S, rd, ad, cr, rq = sv["S"], sv["rd"], sv["ad"], sv["cr"], sv["rq"]
    Lv, co = plan.L, plan.co
    C = Checker()
    # ---------------- forward, down path: conv_k -> (BN) -> activations
    xin = f(sv["xin"], cin)
    prev = xin
    for k in range(Lv):
        w = plan.conv[k].weight.detach()
        r = F.conv2d(prev, q(w), None, 2, 1)
        if rd[k].data_ptr() == (ad[k].data_ptr() if ad[k] is not None else -1):
            # activation epilogue (no BatchNorm, ops.conv_act): no raw tensor -- the activation of the
            # bf16-rounded conv output is checked below against the torch conv
            rdk = q(r)
        else:
            C.bf16(f"fwd conv{k} raw", f(rd[k]), q(r))
            rdk = f(rd[k])
        if k in plan.bnd:
            mean, rstd = sv["st_d"][k]
            C.fp32(f"fwd bn_d{k} mean", mean, r.mean(dim=(0, 2, 3)), 1e-4)
            C.fp32(f"fwd bn_d{k} rstd", rstd, torch.rsqrt(r.var(dim=(0, 2, 3), unbiased=False) + 1e-5), 1e-4)
            sc, sh = sv["tab_d"][k][0], sv["tab_d"][k][1]
            n = rdk * sc[None, :, None, None] + sh[None, :, None, None]
        else:
            n = rdk
        if k < Lv - 1:
            C.bf16(f"fwd act{k} (conv{k + 1} input)", f(ad[k]), q(F.leaky_relu(n, 0.2)))
            prev = f(ad[k])
        C.bf16(f"fwd skip{k}", f(cr[k], co[k]), q(F.relu(n)))
    # ---------------- forward, up path: convT_k -> BN_up -> ReLU into the parent's concat
    for k in range(Lv - 1, 0, -1):
        w = plan.convT[k].weight.detach()
        r = F.conv_transpose2d(f(cr[k]), q(w), None, 2, 1)
        C.bf16(f"fwd convT{k} raw", f(rq[k]), q(r))
        mean, rstd = sv["st_u"][k]
        C.fp32(f"fwd bn_u{k} mean", mean, r.mean(dim=(0, 2, 3)), 1e-4)
        C.fp32(f"fwd bn_u{k} rstd", rstd, torch.rsqrt(r.var(dim=(0, 2, 3), unbiased=False) + 1e-5), 1e-4)
        sc, sh = sv["tab_u"][k][0], sv["tab_u"][k][1]
        n = f(rq[k]) * sc[None, :, None, None] + sh[None, :, None, None]
        C.bf16(f"fwd up{k} (ReLU half)", f(cr[k - 1])[:, co[k - 1]:], q(F.relu(n)))
    w0 = plan.convT[0].weight.detach()
    y_ref = torch.tanh(F.conv_transpose2d(f(cr[0]), q(w0), plan.convT[0].bias.detach(), 2, 1))
    C.fp32("fwd output (tanh)", y.detach(), y_ref, 1e-3)
    # ---------------- backward, up path
    ydet = y.detach()
    C.bf16("bwd dq0 (tanh')", f(tr[("dq", 0)], cout), q(gy * (1 - ydet * ydet)))
    C.fp32("bwd convT0 bias grad", plan.convT[0].bias.grad, (gy * (1 - ydet * ydet)).sum(dim=(0, 2, 3)), 2e-3)
    for k in range(Lv):
        cout_t = cout if k == 0 else co[k - 1]
        g = f(tr[("dq", k)], cout_t)
        xk = f(cr[k])
        wT = plan.convT[k].weight
        gx, gw = _wgrad_ref(lambda a, b: F.conv_transpose2d(a, b, None, 2, 1), xk, q(wT.detach()), g)
        C.fp32(f"bwd convT{k} weight grad", wT.grad, gw)
        gc = f(tr[("gcat", k)])[:, :, :S[k + 1][0], :S[k + 1][1]]
        C.bf16(f"bwd convT{k} input grad", gc, q(gx))
        if k == Lv - 1:
            break
        # BN_up[k+1] (+ the ReLU of the concat): its output's gradient is the second half of gcat[k]
        bn = plan.bnu[k + 1]
        mean, rstd = sv["st_u"][k + 1]
        sc, sh = sv["tab_u"][k + 1][0], sv["tab_u"][k + 1][1]
        raw = f(rq[k + 1])
        n = raw * sc[None, :, None, None] + sh[None, :, None, None]
        dn = gc[:, co[k]:] * (n > 0)
        dx, dgam, dbet = _bn_bwd_ref(raw, mean, rstd, bn.weight.detach(), dn)
        C.bf16(f"bwd bn_u{k + 1} input grad", f(tr[("dq", k + 1)]), q(dx))
        C.fp32(f"bwd bn_u{k + 1} gamma grad", bn.weight.grad, dgam, 1e-2)
        C.fp32(f"bwd bn_u{k + 1} beta grad", bn.bias.grad, dbet, 1e-2)
    # innermost: ReLU backward of the raw conv output (no BN)
    C.bf16("bwd innermost relu", f(tr[("dr", Lv - 1)]), q(f(tr[("gcat", Lv - 1)]) * (f(rd[Lv - 1]) > 0)))
    # ---------------- backward, down path
    for k in range(Lv - 1, -1, -1):
        d = f(tr[("dr", k)])
        inp = xin if k == 0 else f(ad[k - 1])
        wk = plan.conv[k].weight
        gx, gw = _wgrad_ref(lambda a, b: F.conv2d(a, b, None, 2, 1), inp, q(wk.detach()), d)
        C.fp32(f"bwd conv{k} weight grad", wk.grad, gw)
        if k == 0:
            break
        ga = f(tr[("ga", k)])
        C.bf16(f"bwd conv{k} input grad", ga, q(gx))
        # r_{k-1}: skip half (ReLU) + conv_k input (LeakyReLU), then BN_down[k-1] (absent at level 0)
        raw = f(rd[k - 1])
        g1 = f(tr[("gcat", k - 1)])[:, :co[k - 1], :S[k][0], :S[k][1]]
        if k - 1 in plan.bnd:
            bn = plan.bnd[k - 1]
            mean, rstd = sv["st_d"][k - 1]
            sc, sh = sv["tab_d"][k - 1][0], sv["tab_d"][k - 1][1]
            n = raw * sc[None, :, None, None] + sh[None, :, None, None]
            dn = g1 * (n > 0) + ga * torch.where(n > 0, 1.0, 0.2)
            dx, dgam, dbet = _bn_bwd_ref(raw, mean, rstd, bn.weight.detach(), dn)
            C.fp32(f"bwd bn_d{k - 1} gamma grad", bn.weight.grad, dgam, 1e-2)
            C.fp32(f"bwd bn_d{k - 1} beta grad", bn.bias.grad, dbet, 1e-2)
        else:
            dx = g1 * (raw > 0) + ga * torch.where(raw > 0, 1.0, 0.2)
        C.bf16(f"bwd dr{k - 1}", f(tr[("dr", k - 1)]), q(dx))
    print(f"C3 {name} layer checks: {len(C.worst)}; worst:",
          sorted(C.worst.items(), key=lambda kv: -kv[1])[:6])
    assert not C.fails, C.fails[:10]


@pytest.mark.parametrize("name", ["D1", "D2"])
def test_c3_discriminator_layers(name):
    from stcgan_amd import engine, networks
    cin = 4 if name == "D1" else 7
    net = networks.get_discriminator(cin, ndf=64)
    net.load_state_dict(fixture_state(net.state_dict(), 13 if name == "D1" else 14, "ref"))
    net.to(DEV).set_compute_dtype("bf16").train()
    x = uniform((BS, cin, 256, 256), 5200).to(DEV)
    x[:, 3:4] = pm_one((BS, 1, 256, 256), 5201).to(DEV)
    engine.TRACE = {}
    try:
        c = net(x)
        gout = (uniform(tuple(c.shape), 5202) * 1e-3).to(DEV)
        c.backward(gout)
        torch.cuda.synchronize()
        tr = engine.TRACE["D"][0]
    finally:
        engine.TRACE = None
    sv, plan = tr["saved"], net._plan
    raw, act, stats, tabs = sv["raw"], sv["act"], sv["stats"], sv["tabs"]
    C = Checker()
    n_l = plan.n
    for i, cv in enumerate(plan.convs):
        s = plan.strides[i]
        inp = f(act[i], cin if i == 0 else None)
        w = cv.weight.detach()
        if i == n_l - 1:
            r = F.conv2d(inp, q(w), cv.bias.detach(), 1, 1)
            C.fp32("fwd logits", c.detach(), r, 1e-3)
            break
        r = F.conv2d(inp, q(w), cv.bias.detach() if cv.bias is not None else None, s, 1)
        if raw[i + 1].data_ptr() == act[i + 1].data_ptr():  # activation epilogue: no raw tensor (ops.conv_act)
            rawi = q(r)
        else:
            C.bf16(f"fwd conv{i} raw", f(raw[i + 1]), q(r))
            rawi = f(raw[i + 1])
        if tabs[i + 1] is not None:
            mean, rstd = stats[i + 1]
            C.fp32(f"fwd bn{i} mean", mean, r.mean(dim=(0, 2, 3)), 1e-4)
            C.fp32(f"fwd bn{i} rstd", rstd, torch.rsqrt(r.var(dim=(0, 2, 3), unbiased=False) + 1e-5), 1e-4)
            sc, sh = tabs[i + 1]
            n = rawi * sc[None, :, None, None] + sh[None, :, None, None]
        else:
            n = rawi
        C.bf16(f"fwd act{i + 1}", f(act[i + 1]), q(F.leaky_relu(n, 0.2)))
    # backward
    for i in range(n_l - 1, -1, -1):
        cv = plan.convs[i]
        s = plan.strides[i]
        g = f(tr[("g", i)], cv.out_channels)
        if i == n_l - 1:
            C.bf16("bwd logits grad", g, q(gout))
        inp = f(act[i], cin if i == 0 else None)
        gx, gw = _wgrad_ref(lambda a, b: F.conv2d(a, b, None, s, 1), inp, q(cv.weight.detach()), g)
        C.fp32(f"bwd conv{i} weight grad", cv.weight.grad, gw)
        if cv.bias is not None:
            C.fp32(f"bwd conv{i} bias grad", cv.bias.grad, g.sum(dim=(0, 2, 3)))
        if i == 0:
            break
        ga = f(tr[("ga", i)])
        C.bf16(f"bwd conv{i} input grad", ga, q(gx))
        rw = f(raw[i])
        if tabs[i] is not None:
            bn = plan.bns[i - 2]
            mean, rstd = stats[i]
            sc, sh = tabs[i]
            n = rw * sc[None, :, None, None] + sh[None, :, None, None]
            dn = ga * torch.where(n > 0, 1.0, 0.2)
            dx, dgam, dbet = _bn_bwd_ref(rw, mean, rstd, bn.weight.detach(), dn)
            C.fp32(f"bwd bn{i - 1} gamma grad", bn.weight.grad, dgam, 1e-2)
            C.fp32(f"bwd bn{i - 1} beta grad", bn.bias.grad, dbet, 1e-2)
        else:
            dx = ga * torch.where(rw > 0, 1.0, 0.2)
        C.bf16(f"bwd g{i - 1}", f(tr[("g", i - 1)], plan.convs[i - 1].out_channels), q(dx))
    print(f"C3 {name} layer checks: {len(C.worst)}; worst:",
          sorted(C.worst.items(), key=lambda kv: -kv[1])[:6])
    assert not C.fails, C.fails[:10]
