"""Concurrency profile of a rocprofv3 kernel trace over the last train steps: the time during which 0, 1, 2
and 3+ kernels run at once (queue-level overlap), the kernels that run ALONE the longest (the exposed
critical path), and per-stream busy time.
usage: trace_concurrency.py <kernel_trace.csv> [last_fraction | adamA:adamB] [n_show]
  adamA:adamB -- the window from the end of the adam_pack launch #adamA to the end of #adamB (0-based; two per
  train step, D then G), e.g. 5:25 = the 10 timed steps of `bench.py --warmup 3 --steps 10`"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
frac = float(sys.argv[2]) if len(sys.argv) > 2 and ":" not in sys.argv[2] else 0.5
nshow = int(sys.argv[3]) if len(sys.argv) > 3 else 20
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Stream_Id") or r.get("Queue_Id"))
            for r in rows)
t_beg, t_end = iv[0][0], max(e for _, e, _, _ in iv)
if ":" in (sys.argv[2] if len(sys.argv) > 2 else ""):
    a, b = (int(v) for v in sys.argv[2].split(":"))
    ad = [v for v in iv if "adam_pack" in v[2]]
    w0, w1 = ad[a][1], ad[b][1]
    iv = [v for v in iv if v[0] >= w0 and v[1] <= w1]
    print(f"window: adam #{a} .. #{b} ({(w1 - w0) / 1e6:.3f} ms)")
else:
    cut = t_end - (t_end - t_beg) * frac
    iv = [v for v in iv if v[0] >= cut]
ev = []
for i, (s, e, n, q) in enumerate(iv):
    ev.append((s, 1, i))
    ev.append((e, -1, i))
ev.sort()
conc = defaultdict(int)
alone = defaultdict(int)
running = set()
last = ev[0][0]
for t, d, i in ev:
    if t > last:
        conc[min(len(running), 3)] += t - last
        if len(running) == 1:
            (j,) = running
            alone[iv[j][2]] += t - last
    last = t
    if d > 0:
        running.add(i)
    else:
        running.discard(i)
span = iv[-1][1] - iv[0][0]
print(f"span {span / 1e6:.3f} ms over {len(iv)} launches")
for k in sorted(conc):
    print(f"  {k if k < 3 else '3+'} kernels running: {conc[k] / 1e6:8.3f} ms  ({conc[k] / span * 100:5.1f} %)")
per_q = defaultdict(int)
for s, e, n, q in iv:
    per_q[q] += e - s
print("per stream busy:", {q: round(v / 1e6, 3) for q, v in per_q.items()})
print("running alone (exposed), by kernel:")
for n, v in sorted(alone.items(), key=lambda kv: -kv[1])[:nshow]:
    print(f"  {v / 1e6:8.3f} ms  {n[:110]}")
