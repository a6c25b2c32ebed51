"""Per-kernel timeline of the last forward(s) of a rocprofv3 kernel trace of scripts/fwd_timeline.py:
each kernel's duration and the idle gap before it, grouped totals (GEMM / BN / other) and the span.
usage: fwd_timeline_read.py <kernel_trace.csv> [generators]  (a generator forward starts at its input gather;
the last ``generators`` of them, default 2 = one G1+G2 forward)"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
ngen = int(sys.argv[2]) if len(sys.argv) > 2 else 2
starts = [i for i, v in enumerate(iv) if "gather" in v[2]]
sel = iv[starts[-ngen]:]
span = sel[-1][1] - sel[0][0]
groups = {}
prev_end = None
lines = []
for s, e, n in sel:
    short = n.replace("void ", "").replace("stc::", "")
    short = short.split("(")[0][:70]
    gap = 0 if prev_end is None else s - prev_end
    prev_end = max(e, prev_end or e)
    lines.append(f"{(e - s) / 1e3:8.1f} us  gap {gap / 1e3:6.1f}  {short}")
    key = ("gemm" if any(t in n for t in ("halo_conv", "igemm", "stem_conv", "narrow", "logits")) else
           "bn" if "bn_" in n else "reduce" if "reduce" in n else "other")
    g = groups.setdefault(key, [0, 0])
    g[0] += 1
    g[1] += e - s
busy = sum(e - s for s, e, _ in sel)
print(f"kernels {len(sel)}  span {span / 1e3:.1f} us  kernel sum {busy / 1e3:.1f} us  idle {(span - busy) / 1e3:.1f} us")
for k, (c, t) in sorted(groups.items(), key=lambda kv: -kv[1][1]):
    print(f"  {k:7s} {c:4d} launches {t / 1e3:8.1f} us")
print("\n".join(lines))
