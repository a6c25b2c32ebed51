"""Split-K sweep for the deep (latency-bound) layers of one ST-CGAN bf16 train step: every conv
problem with M*nphase <= 8192 (the 16x16 ... 1x1 U-Net levels), tile configs of <= 128 rows,
ksplit 1..64.  Uses the recorder and HIP-graph timer of tune_bf16.py.  Output: JSON to argv[1]."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import tune_bf16 as T  # noqa: E402
from tune_bf16 import BF, L, ops  # noqa: E402

CFGS = (5, 12, 19, 4, 10, 0, 2)
KS = (1, 2, 4, 8, 16, 32, 64)


def main():
    probs = T.record()
    out = []
    names = {0: "conv_s2", 1: "conv_s1", 2: "convT", 3: "s1_dgrad"}
    tot_auto = tot_best = 0.0
    for prob, (count, _) in sorted(probs.items(), key=lambda kv: -kv[0][1] * kv[0][2] * kv[0][3] * kv[0][8] * kv[0][9]):
        kind, B, gh, gw, xh, xw, yh, yw, cin, cout = prob
        nph = 4 if kind == L.CONVT_S2 else 1
        if B * gh * gw * nph > 8192:
            continue
        ws, nch, plan = ops.conv_query(kind, B, gh, gw, cin, cout, BF)
        if plan[4] < 0:
            continue
        taps = 4 if kind == L.CONVT_S2 else 16
        K = taps * cin
        flops = 2.0 * B * gh * gw * nph * cout * K
        t_auto = T.bench(prob, None)
        res = {}
        for cfg in CFGS:
            for ks in KS:
                if (K // 64) < ks:
                    continue
                t = T.bench(prob, (cfg, ks), reps=10)
                if t is not None:
                    res[(cfg, ks)] = t
        best = min(res, key=res.get)
        tot_auto += t_auto * count
        tot_best += res[best] * count
        print(f"{names[kind]:8s} M={B * gh * gw:6d}x{nph} N={cout:4d} K={K:5d} n={count} auto{plan[4]},{plan[2]}"
              f" {t_auto:7.1f}us | best cfg{best[0]},ks{best[1]} {res[best]:7.1f}us {flops / res[best] / 1e6:6.1f}TF | "
              + " ".join(f"{c},{k}:{v:.1f}" for (c, k), v in sorted(res.items(), key=lambda kv: kv[1])[:6]), flush=True)
        out.append({"prob": prob, "count": count, "auto": [plan[4], plan[2], t_auto], "best": [best[0], best[1], res[best]],
                    "all": {f"{k[0]},{k[1]}": v for k, v in res.items()}})
    print(f"deep layers, one step: auto {tot_auto / 1e3:.3f} ms, best {tot_best / 1e3:.3f} ms")
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
