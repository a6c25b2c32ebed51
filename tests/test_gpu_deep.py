"""stc_deep_conv (csrc/deep_bf16.hip): the generator's innermost levels in one launch per layer.

Kernel level: each launch against torch fp32 on the same bf16 operands -- Conv2d k4 s2 p1 and ConvTranspose2d
k4 s2 p1 (STCGAN/networks.py:104-105, :119-121, :126-128) at the deep levels' shapes (1x1 - 8x8 grids, bs 32 and
odd 480x640 sizes), sources read raw with the BatchNorm affine (from statistics partials or a table) + activation
applied in the kernel, two sources (the U-Net concat), split K with the in-launch reduction, the tile statistics
partials and the designated table / running-statistics outputs.  Network level: the generator forward with the
deep path equals the per-layer path within bf16 rounding, and two runs are bit-identical (the split-K sum order
is fixed whatever the arrival order)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def _nchw(t):
    return t.permute(0, 3, 1, 2).float()


def _rel(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return float((a - b).norm() / (b.norm() + 1e-30))


def _bn(C, g):
    bn = torch.nn.BatchNorm2d(C).to(DEV)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, generator=g, device=DEV) + 0.5)
        bn.bias.copy_(torch.rand(C, generator=g, device=DEV) - 0.5)
        bn.running_mean.copy_(torch.rand(C, generator=g, device=DEV) * 0.1)
        bn.running_var.copy_(torch.rand(C, generator=g, device=DEV) + 0.5)
    return bn


CASES = [  # kind, B, input H, W, Cin per source, Cout, sources with a BatchNorm table
    ("conv", 32, 8, 8, [512], 512, False),      # e5-shaped (16 -> 8x8 -> 4x4 at 256x256): the activation as input
    ("conv", 32, 4, 4, [512], 512, True),       # e6
    ("conv", 32, 2, 2, [512], 512, True),       # e7 (1x1 output: 4 of 16 taps kept)
    ("convT", 32, 1, 1, [512], 512, False),     # d7 (1x1 input: one tap per phase)
    ("convT", 32, 2, 2, [512, 512], 512, True),  # d6 (concat of two sources)
    ("convT", 32, 4, 4, [512, 512], 512, True),  # d5
    ("conv", 32, 16, 16, [512], 512, False),    # e4 / d4 shapes
    ("convT", 32, 8, 8, [512, 512], 512, True),
    ("conv", 8, 15, 20, [256], 512, True),      # 480x640 shapes (odd input)
    ("convT", 8, 4, 5, [512, 512], 512, True),
    ("conv", 2, 4, 4, [64], 64, True),          # ngf=8 widths
    ("convT", 2, 2, 2, [64, 64], 64, True),
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}-B{c[1]}-{c[2]}x{c[3]}-{'+'.join(map(str, c[4]))}" for c in CASES])
def test_deep_conv_vs_torch(case):
    from stcgan_amd import _lib as L, ops
    kind, B, H, W, cins, cout, use_tab = case
    g = torch.Generator(device=DEV)
    g.manual_seed(H * 100 + W + sum(cins))
    cin = sum(cins)
    convt = kind == "convT"
    # raw sources (bf16 NHWC) with a (scale, shift) table and an activation each
    raws = [(torch.randn((B, H, W, c), generator=g, device=DEV) * 2 + 0.3).to(torch.bfloat16) for c in cins]
    slopes = ([0.2] if not convt else [0.0, 0.0])[:len(cins)]
    srcs, acts = [], []
    for r, sl in zip(raws, slopes):
        C = r.shape[3]
        x = _nchw(r)
        if use_tab:
            sc = torch.rand(C, generator=g, device=DEV) + 0.5
            sh = torch.rand(C, generator=g, device=DEV) - 0.5
            srcs.append(ops.deep_src(L.nhwc_view(r), C, table=(sc, sh), slope=sl))
            n = torch.addcmul(sh[None, :, None, None], x, sc[None, :, None, None])  # (one rounding, as fmaf)
        else:
            srcs.append(ops.deep_src(L.nhwc_view(r), C, slope=sl if convt else 1.0))
            n = x
        acts.append(F.leaky_relu(n, sl if (use_tab or convt) else 1.0).to(torch.bfloat16).float())
    a = torch.cat(acts, 1)
    w = (torch.randn((cin, cout, 4, 4) if convt else (cout, cin, 4, 4), generator=g, device=DEV) * 0.02)
    wq = w.to(torch.bfloat16).float()
    if convt:
        ref = F.conv_transpose2d(a, wq, None, 2, 1)
        wp = ops.pack(L.PACK_CONVT_FWD, w, cout, cin, torch.bfloat16)
        kd = L.CONVT_S2
    else:  # (an odd input is zero-padded to even first: the pad / crop generator, src/models/stcgan_g.py:120-132)
        ref = F.conv2d(F.pad(a, (0, W % 2, 0, H % 2)), wq, None, 2, 1)
        wp = ops.pack(L.PACK_CONV_FWD, w, cout, cin, torch.bfloat16)
        kd = L.CONV_S2
    Ho, Wo = ref.shape[2], ref.shape[3]
    y = torch.empty((B, Ho, Wo, cout), dtype=torch.bfloat16, device=DEV)
    bn = _bn(cout, g)
    rm0, rv0 = bn.running_mean.clone(), bn.running_var.clone()
    tab = torch.empty((2, cout), device=DEV)
    st = (torch.empty(cout, device=DEV), torch.empty(cout, device=DEV))
    tickets = {}
    ops.deep_conv(kd, B, srcs, wp, cout, L.nhwc_view(y), tickets, "k", bn=ops.deep_bn(bn, tab, st))
    torch.cuda.synchronize()
    assert int(tickets["k"].abs().sum()) == 0  # (left zero for the next launch)
    got = _nchw(y)
    assert _rel(got, ref) < 1e-2
    assert float((got - ref).abs().max()) <= 0.02 * float(ref.abs().max()) + 1e-6
    # the output's BatchNorm: batch statistics of the fp32 conv output, table, running statistics, batch count
    mean, var = ref.mean(dim=(0, 2, 3)), ref.var(dim=(0, 2, 3), unbiased=False)
    assert _rel(st[0], mean) < 2e-3
    assert _rel(st[1], torch.rsqrt(var + bn.eps)) < 2e-3
    assert _rel(tab[0], bn.weight.detach() * torch.rsqrt(var + bn.eps)) < 2e-3
    assert _rel(tab[1], bn.bias.detach() - mean * tab[0]) < 2e-3
    n = B * Ho * Wo
    assert torch.allclose(bn.running_mean, 0.9 * rm0 + 0.1 * mean, rtol=2e-3, atol=1e-5)
    assert torch.allclose(bn.running_var, 0.9 * rv0 + 0.1 * var * n / (n - 1), rtol=2e-3, atol=1e-5)
    assert int(bn.num_batches_tracked) == 1
    # bit-identical on a second launch (fixed split and merge orders, whatever the arrival order)
    y2 = torch.empty_like(y)
    tab2 = torch.empty_like(tab)
    st2 = (torch.empty_like(st[0]), torch.empty_like(st[1]))
    ops.deep_conv(kd, B, srcs, wp, cout, L.nhwc_view(y2), tickets, "k", bn=ops.deep_bn(bn, tab2, st2, running=False))
    torch.cuda.synchronize()
    assert torch.equal(y, y2) and torch.equal(tab, tab2) and torch.equal(st[0], st2[0])
    assert int(tickets["k"].abs().sum()) == 0


@pytest.mark.parametrize("ngf,B", [(64, 8), (8, 4)])
def test_generator_deep_path_matches_per_layer_path(ngf, B):
    """G forward (train) with the deep levels on stc_deep_conv vs the per-layer path: outputs, saved raw outputs,
    BatchNorm statistics and running statistics within bf16 rounding; the deep path bit-reproducible."""
    from stcgan_amd import engine, networks
    g = torch.Generator(device=DEV)
    g.manual_seed(17)
    x = torch.rand((B, 3, 256, 256), generator=g, device=DEV) * 2 - 1
    torch.manual_seed(3)
    net = networks.get_generator(3, 1, ngf=ngf)
    for m in net.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            torch.nn.init.uniform_(m.weight, 0.5, 1.5)
    net = net.to(DEV).set_compute_dtype("bf16").train()
    state0 = {k: v.clone() for k, v in net.state_dict().items()}
    runs = {}
    prev = engine.DEEP
    try:
        for tag, deep in (("deep", True), ("deep2", True), ("layer", False)):
            engine.DEEP = deep
            net.load_state_dict(state0)
            engine.TRACE = {}
            y = net(x.clone().requires_grad_(True))
            torch.cuda.synchronize()
            runs[tag] = (y.detach().clone(), engine.TRACE["G"][0]["saved"],
                         {k: v.clone() for k, v in net.state_dict().items()})
            engine.TRACE = None
    finally:
        engine.DEEP = prev
        engine.TRACE = None
    yd, sd, std = runs["deep"]
    assert torch.equal(yd, runs["deep2"][0])
    for k in std:
        assert torch.equal(std[k], runs["deep2"][2][k]), k
    yl, sl, stl = runs["layer"]
    assert _rel(yd, yl) < 2e-2
    Lv = len(sd["rd"])
    for k in range(1, Lv):
        assert _rel(sd["rd"][k].float(), sl["rd"][k].float()) < 3e-2, ("rd", k)
        assert _rel(sd["rq"][k].float(), sl["rq"][k].float()) < 3e-2, ("rq", k)
        assert _rel(sd["cr"][k].float(), sl["cr"][k].float()) < 3e-2, ("cr", k)
    for k in sd["st_d"]:
        assert _rel(sd["st_d"][k][0], sl["st_d"][k][0]) < 3e-2 and _rel(sd["st_d"][k][1], sl["st_d"][k][1]) < 3e-2
    for k in std:
        if "num_batches_tracked" in k:
            assert torch.equal(std[k], stl[k]), k
        elif "running" in k:
            assert _rel(std[k], stl[k]) < 3e-2, k
