"""Per-launch durations of one kernel family inside one train step of a rocprofv3 kernel trace.
usage: trace_family.py <kernel_trace.csv> <regex> [adamA:adamB]
  window: from the end of adam_pack launch #adamA to the end of #adamB (two per step: D then G; default the
  trace's last whole step).  Prints each matching launch (start offset, duration, workgroups) and the sum."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = re.compile(sys.argv[2])
iv = sorted(rows, key=lambda r: int(r["Start_Timestamp"]))
ad = [r for r in iv if "adam_pack" in r["Kernel_Name"]]
if len(sys.argv) > 3:
    a, b = (int(v) for v in sys.argv[3].split(":"))
else:
    a, b = len(ad) - 3, len(ad) - 1
w0, w1 = int(ad[a]["End_Timestamp"]), int(ad[b]["End_Timestamp"])
tot = 0.0
n = 0
for r in iv:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < w0 or e > w1 or not pat.search(r["Kernel_Name"]):
        continue
    d = (e - s) / 1e3
    tot += d
    n += 1
    g = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
    wg = int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or 1)
    print(f"{(s - w0) / 1e3:9.1f} us  {d:7.1f} us  blocks {g // max(wg, 1):6d}  {r['Kernel_Name'][:90]}")
print(f"{n} launches, {tot:.1f} us in window {(w1 - w0) / 1e3:.1f} us")
