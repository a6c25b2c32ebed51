"""stc_deep_conv plan sweep: every (tile, K splits) for the deep levels' shapes at bs 32 (256x256) and 8 (480x640),
timed alone with HIP events (median of 15 launches; sources with a BatchNorm table and the output's BatchNorm, as in
the generator).
Prints one line per plan and the best per shape.  usage: deep_tune.py [--quick]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))

import torch  # noqa: E402

from stcgan_amd import _lib as L, ops  # noqa: E402

DEV = "cuda"
# (name, kind, B, input H, W, source channels, Cout)
SHAPES = [("e4", "conv", 32, 16, 16, [512], 512), ("e5", "conv", 32, 8, 8, [512], 512),
          ("e6", "conv", 32, 4, 4, [512], 512), ("e7", "conv", 32, 2, 2, [512], 512),
          ("d7", "convT", 32, 1, 1, [512], 512), ("d6", "convT", 32, 2, 2, [512, 512], 512),
          ("d5", "convT", 32, 4, 4, [512, 512], 512), ("d4", "convT", 32, 8, 8, [512, 512], 512)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    ap.add_argument("--phases", action="store_true", help="wall-clock phase stamps of the automatic plan, no sweep")
    ap.add_argument("--force", default=None, help="phases of this plan: tile,splits")
    a = ap.parse_args()
    g = torch.Generator(device=DEV)
    g.manual_seed(1)
    best = {}
    for name, kind, B, H, W, cins, cout in SHAPES:
        if a.only and name not in a.only.split(","):
            continue
        convt = kind == "convT"
        cin = sum(cins)
        raws = [(torch.randn((B, H, W, c), generator=g, device=DEV)).to(torch.bfloat16) for c in cins]
        bns = []
        for c in cins:
            bn = torch.nn.BatchNorm2d(c).to(DEV)
            bns.append(bn)
        tabs = [(torch.rand(c, generator=g, device=DEV) + 0.5, torch.rand(c, generator=g, device=DEV) - 0.5)
                for c in cins]
        srcs = [ops.deep_src(L.nhwc_view(r), r.shape[3], table=t, slope=0.0) for r, t in zip(raws, tabs)]
        bn_o = torch.nn.BatchNorm2d(cout).to(DEV)
        tab_o = torch.empty((2, cout), device=DEV)
        st_o = (torch.empty(cout, device=DEV), torch.empty(cout, device=DEV))
        dbn = ops.deep_bn(bn_o, tab_o, st_o, running=False)
        w = torch.randn((cin, cout, 4, 4) if convt else (cout, cin, 4, 4), generator=g, device=DEV) * 0.02
        wp = ops.pack(L.PACK_CONVT_FWD if convt else L.PACK_CONV_FWD, w, cout, cin, torch.bfloat16)
        kd = L.CONVT_S2 if convt else L.CONV_S2
        Ho, Wo = (2 * H, 2 * W) if convt else ((H + 1) // 2, (W + 1) // 2)
        y = torch.empty((B, Ho, Wo, cout), dtype=torch.bfloat16, device=DEV)
        tickets = {}
        gh, gw = (H, W) if convt else (Ho, Wo)
        auto = ops.deep_query(kd, B, gh, gw, H, W, cin, cout)[2]
        if a.phases:
            fo = tuple(int(v) for v in a.force.split(",")) if a.force else None
            for plan_force in (fo,):
                auto = ops.deep_query(kd, B, gh, gw, H, W, cin, cout, force=fo)[2]
                nb = auto[4]
                stamps = torch.zeros((nb, 8), dtype=torch.int64, device=DEV)
                for _ in range(3):
                    ops.deep_conv(kd, B, srcs, wp, cout, L.nhwc_view(y), tickets, "p", bn=dbn, force=fo)
                torch.cuda.synchronize()
                L.lib().stc_deep_debug_next(L.ptr(stamps))
                ops.deep_conv(kd, B, srcs, wp, cout, L.nhwc_view(y), tickets, "p", bn=dbn, force=fo)
                torch.cuda.synchronize()
                st = stamps.cpu().double() * 10e-3  # (100 MHz wall clock -> us)
                t0 = float(st[:, 0].min())
                def q(col, rows=None):
                    v = st[:, col] if rows is None else st[rows, col]
                    v = v[v > 0] - t0
                    return (round(float(v.min()), 2), round(float(v.median()), 2), round(float(v.max()), 2)) if v.numel() else None
                red = st[:, 3] > 0
                fin = st[:, 5] > 0
                print(f"== {name} plan {auto} blocks {nb}: start {q(0)} tables {q(1)} kloop_done {q(2)} "
                      f"reduce_go {q(3, red)} stats_done {q(4)} finalize_go {q(5, fin)} end {q(6)} "
                      f"(min / median / max us from the first block's start)", flush=True)
                # the per-layer path's GEMM on the same operands (activations as its input), HIP events
                if not convt or len(cins) == 1:
                    xa = raws[0]
                    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                    for _ in range(3):
                        ops.conv_stats(kd, B, L.nhwc_view(xa), cin, wp, cout, L.nhwc_view(y), torch.bfloat16)
                    ev[0].record()
                    for _ in range(10):
                        ops.conv_stats(kd, B, L.nhwc_view(xa), cin, wp, cout, L.nhwc_view(y), torch.bfloat16)
                    ev[1].record()
                    torch.cuda.synchronize()
                    print(f"   {name} per-layer GEMM (+ split-K reduce) {ev[0].elapsed_time(ev[1]) * 100:.1f} us, "
                          f"plan {ops.conv_query(kd, B, gh, gw, cin, cout, torch.bfloat16)[2]}", flush=True)
            continue
        res = []
        for t in range(6):
            for s in (1, 2, 4, 8, 16, 32, 64):
                try:
                    plan = ops.deep_query(kd, B, gh, gw, H, W, cin, cout, force=(t, s))[2]
                except RuntimeError:
                    continue
                if plan[2] != s or plan[4] > 2048:
                    continue
                for _ in range(3):
                    ops.deep_conv(kd, B, srcs, wp, cout, L.nhwc_view(y), tickets, (t, s), bn=dbn, force=(t, s))
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(15)]
                for e0, e1 in evs:
                    e0.record()
                    ops.deep_conv(kd, B, srcs, wp, cout, L.nhwc_view(y), tickets, (t, s), bn=dbn, force=(t, s))
                    e1.record()
                torch.cuda.synchronize()
                ts = sorted(e0.elapsed_time(e1) * 1e3 for e0, e1 in evs)
                us = ts[len(ts) // 2]
                res.append((us, plan))
                print(f"{name} tile {plan[0]}x{plan[1]} splits {plan[2]} taps {plan[3]} blocks {plan[4]}: {us:.1f} us",
                      flush=True)
        res.sort()
        best[name] = {"best": res[0], "auto": auto, "auto_us": next((u for u, p in res if p == auto), None)}
        print(f"== {name}: best {res[0][0]:.1f} us {res[0][1]}, automatic plan {auto}: {best[name]['auto_us']}",
              flush=True)
    print(json.dumps(best))


if __name__ == "__main__":
    main()
