"""A/B of the one-wave-per-SIMD halo kernels (csrc/halo_wide.hpp, configurations 1-3) against this round's
starting kernels (halo_bf16.hip's automatic choice, force shape 7) on every halo GEMM shape of one train step
(bs 32, 256x256, bf16): per candidate the output vs a torch fp32 convolution of the same bf16 operands (max error
/ max |ref|), the BatchNorm statistics vs the fp64 moments of that reference, and the time (HIP events over 20
launches, interleaved rounds, median and min).  Usage: python scripts/ab_wide.py [--quick]
(env AB_SHAPES=i,j,..: a subset of SHAPES; AB_CANDS=name,..: a subset of the candidates; STC_LIB_PATH: a
diagnostic library -- its error columns then mean nothing)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from stcgan_amd import _lib as L  # noqa: E402
from stcgan_amd import ops  # noqa: E402

BF = torch.bfloat16
SHAPES = [  # (kind, GEMM grid, cin, cout, what)
    (L.CONV_S1, 31, 256, 512, "D c4 fwd (k4 s1)"),
    (L.CONV_S1_DGRAD, 32, 512, 256, "D c4 dgrad"),
    (L.CONV_S2, 64, 64, 128, "e2 / D c2 fwd"),
    (L.CONV_S2, 32, 128, 256, "e3 / D c3 fwd"),
    (L.CONV_S2, 64, 64, 256, "d2 dgrad (ConvT 256->64)"),
    (L.CONV_S2, 32, 128, 512, "d3 dgrad (ConvT 512->128)"),
    (L.CONV_S2, 16, 256, 1024, "d4 dgrad (ConvT 1024->256)"),
    (L.CONVT_S2, 32, 512, 128, "d3 fwd"),
    (L.CONVT_S2, 16, 1024, 256, "d4 fwd"),
    (L.CONVT_S2, 32, 256, 128, "e3 / D c3 dgrad"),
    (L.CONVT_S2, 16, 512, 256, "e4 dgrad"),
    (L.CONV_S2, 16, 256, 512, "e4 fwd"),
]
CANDS = (("legacy", (ops.HALO_CFG, 7)), ("w1_256x256", (ops.HALO_CFG, 8)), ("w2_4x128x64", (ops.HALO_CFG, 9)),
         ("w3_2x128x128", (ops.HALO_CFG, 10)), ("w4_ld4", (ops.HALO_CFG, 11)))


def make(kind, B, gh, cin, cout, dev, g):
    convt = kind == L.CONVT_S2
    ih, oh = {L.CONV_S2: (2 * gh, gh), L.CONVT_S2: (gh, 2 * gh), L.CONV_S1: (gh + 1, gh),
              L.CONV_S1_DGRAD: (gh - 1, gh)}[kind]
    x = torch.randn((B, cin, ih, ih), generator=g, device=dev).to(BF).float()
    if convt or kind == L.CONV_S1_DGRAD:
        w = (torch.randn((cin, cout, 4, 4), generator=g, device=dev) * 0.05).to(BF).float()
        wp = ops.pack(L.PACK_CONVT_FWD if convt else L.PACK_CONV_S1_DGRAD, w, cout, cin, BF)
        ref = F.conv_transpose2d(x, w, None, 2 if convt else 1, 1)
    else:
        w = (torch.randn((cout, cin, 4, 4), generator=g, device=dev) * 0.05).to(BF).float()
        wp = ops.pack(L.PACK_CONV_FWD, w, cout, cin, BF)
        ref = F.conv2d(x, w, None, 2 if kind == L.CONV_S2 else 1, 1)
    assert ref.shape[-1] == oh, (ref.shape, oh)
    xb = x.permute(0, 2, 3, 1).contiguous().to(BF)
    return xb, wp, ref, oh


def main():
    quick = "--quick" in sys.argv
    dev = torch.device("cuda", 0)
    B = 32
    g = torch.Generator(device=dev).manual_seed(0)
    sel = os.environ.get("AB_SHAPES")
    shapes = [SHAPES[int(i)] for i in sel.split(",")] if sel else SHAPES
    keep = os.environ.get("AB_CANDS")
    keep = set(keep.split(",")) if keep else None
    for kind, gh, cin, cout, what in shapes:
        xb, wp, ref, oh = make(kind, B, gh, cin, cout, dev, g)
        rm = ref.double().mean(dim=(0, 2, 3))
        rv = ref.double().var(dim=(0, 2, 3), unbiased=False)
        scale = float(ref.abs().max())
        fl = 2.0 * ref.numel() * cin * (4 if kind == L.CONVT_S2 else 16)
        times, res = {}, {}
        cands = []
        for name, force in CANDS:
            plan = ops.conv_query(kind, B, gh, gh, cin, cout, BF, force=force)[2]
            if (name != "legacy" and plan[3] <= 0) or (keep and name not in keep):
                continue
            cands.append((name, force, plan))
        for rnd in range(2 if quick else 5):
            for name, force, plan in cands:
                y = torch.full((B, oh, oh, cout), float("nan"), device=dev, dtype=BF)
                part, nch = ops.conv_stats(kind, B, L.nhwc_view(xb), cin, wp, cout, L.nhwc_view(y), BF, force=force)
                torch.cuda.synchronize()
                if rnd == 0:
                    bn = torch.nn.BatchNorm2d(cout).to(dev)
                    t = torch.empty((2, cout), device=dev)
                    mean, rstd = ops.bn_finalize_part(part, nch, cout, bn, t[0], t[1])
                    var = 1.0 / rstd.double() ** 2 - bn.eps
                    got = y.float().permute(0, 3, 1, 2)
                    err = float((got - ref).abs().max()) / scale
                    sd = float(rv.max().sqrt())
                    merr = float((mean.double() - rm).abs().max()) / sd
                    verr = float(((var - rv).abs() / (rv + 1e-12)).max())
                    res[name] = (err, merr, verr)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    ops.conv_stats(kind, B, L.nhwc_view(xb), cin, wp, cout, L.nhwc_view(y), BF, force=force)
                e1.record()
                e1.synchronize()
                times.setdefault(name, []).append(e0.elapsed_time(e1) / 20 * 1e3)
        line = f"{what:28s} k{kind} grid{gh} cin{cin} cout{cout}:"
        for name, force, plan in cands:
            t = sorted(times[name])
            e = res[name]
            ok = e[0] <= 1e-2 and e[1] <= 2e-3 and e[2] <= 8e-3
            line += (f"\n    {name:14s} plan{list(plan)} med {t[len(t) // 2]:7.1f} us min {t[0]:7.1f} "
                     f"({fl / t[0] / 1e6:5.0f} TF, {fl / t[0] / 1e6 / 2516:.3f})  err {e[0]:.2e} mean {e[1]:.1e} "
                     f"var {e[2]:.1e} {'ok' if ok else 'FAIL'}")
        print(line, flush=True)


if __name__ == "__main__":
    main()
