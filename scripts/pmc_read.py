"""Average PMC counters per dispatch for kernels matching a substring: pmc_read.py <dir> <substr>"""
import csv
import glob
import sys
from collections import defaultdict

d, sub = sys.argv[1], sys.argv[2]
vals = defaultdict(list)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    per = defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            per[r["Dispatch_Id"]][r["Counter_Name"]] = per[r["Dispatch_Id"]].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
    for disp, c in per.items():
        for k, v in c.items():
            vals[k].append(v)
for k in sorted(vals):
    v = vals[k]
    print(f"{k:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
