"""GPU occupancy of a rocprofv3 kernel trace: wall time of the last N steps' span, summed kernel time,
the union of busy intervals (overlap across streams counted once) and the idle time between them.
usage: trace_gaps.py <kernel_trace.csv> [last_fraction]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
t_end = iv[-1][1]
t_beg = iv[0][0]
cut = t_end - (t_end - t_beg) * frac
iv = [v for v in iv if v[0] >= cut]
span = iv[-1][1] - iv[0][0]
busy, cur_s, cur_e = 0, iv[0][0], iv[0][1]
gaps = []
for s, e, n in iv[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, n))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
tot = sum(e - s for s, e, _ in iv)
print(f"kernels {len(iv)}  span {span / 1e6:.3f} ms  busy(union) {busy / 1e6:.3f} ms  "
      f"sum {tot / 1e6:.3f} ms  idle {(span - busy) / 1e6:.3f} ms in {len(gaps)} gaps")
gaps.sort(reverse=True)
for g, n in gaps[:15]:
    print(f"  gap {g / 1e3:8.1f} us before {n[:90]}")
