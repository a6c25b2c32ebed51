"""stc_deep_conv plan sweep: every (tile, K splits) for the deep levels' shapes at bs 32 (256x256) and 8 (480x640),
timed alone with HIP events (median of 15 launches, sources with BatchNorm partials as in the generator).
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
        parts = []
        for r in raws:
            nch = ops.stats_chunks(B, H, W)
            part = torch.empty((nch, r.shape[3], 4), dtype=torch.float32, device=DEV)
            L.check(L.lib().stc_chan_stats(L.BF16, B, L.nhwc_view(r), r.shape[3], L.ptr(part), nch, L.stream()), "s")
            parts.append((part, nch))
        srcs = [ops.deep_src(L.nhwc_view(r), r.shape[3], part=p, nch=n, bn=bn, slope=0.0)
                for r, (p, n), bn in zip(raws, parts, bns)]
        w = torch.randn((cin, cout, 4, 4) if convt else (cout, cin, 4, 4), generator=g, device=DEV) * 0.02
        wp = ops.pack(L.PACK_CONVT_FWD if convt else L.PACK_CONV_FWD, w, cout, cin, torch.bfloat16)
        kd = L.CONVT_S2 if convt else L.CONV_S2
        Ho, Wo = (2 * H, 2 * W) if convt else ((H + 1) // 2, (W + 1) // 2)
        y = torch.empty((B, Ho, Wo, cout), dtype=torch.bfloat16, device=DEV)
        tickets = {}
        gh, gw = (H, W) if convt else (Ho, Wo)
        auto = ops.deep_query(kd, B, gh, gw, H, W, cin, cout)[3]
        res = []
        for t in range(6):
            for s in (1, 2, 4, 8, 16, 32, 64):
                try:
                    plan = ops.deep_query(kd, B, gh, gw, H, W, cin, cout, force=(t, s))[3]
                except RuntimeError:
                    continue
                if plan[2] != s or plan[4] > 2048:
                    continue
                for _ in range(3):
                    ops.deep_conv(kd, B, srcs, wp, cout, L.nhwc_view(y), tickets, (t, s), force=(t, s))
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(15)]
                for e0, e1 in evs:
                    e0.record()
                    ops.deep_conv(kd, B, srcs, wp, cout, L.nhwc_view(y), tickets, (t, s), force=(t, s))
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
