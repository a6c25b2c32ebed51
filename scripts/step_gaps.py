"""Idle gaps inside the last full train step of a rocprofv3 kernel trace (between the last two G-side
Adam launches): total idle, the largest gaps with their neighbours, and a size histogram.
usage: step_gaps.py <kernel_trace.csv> [n_show]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
ad = [i for i, v in enumerate(iv) if "adam_pack" in v[2]]
seg = iv[ad[-3]:ad[-1] + 1]
t0 = seg[0][1]
cur_e, gaps = seg[0][1], []
for i, (s, e, n) in enumerate(seg[1:], 1):
    if s > cur_e:
        gaps.append((s - cur_e, (cur_e - t0) / 1e3, n[:60], seg[i - 1][2][:50]))
    cur_e = max(cur_e, e)
span = seg[-1][0] - t0
print(f"step span {span / 1e3:.1f} us, idle {sum(g[0] for g in gaps) / 1e3:.1f} us in {len(gaps)} gaps, "
      f"{len(seg)} launches")
for g in sorted(gaps, reverse=True)[:int(sys.argv[2]) if len(sys.argv) > 2 else 15]:
    print(f"{g[0] / 1e3:7.1f} us at t={g[1]:8.1f}  before {g[2]}  after {g[3]}")
