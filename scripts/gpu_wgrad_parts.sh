#!/bin/bash
# Weight-gradient calls of the train step under a rocprofv3 kernel trace: the tile vs the ordered reduce per problem.
set -o pipefail
O=gpurun_out/${1:-r04_wparts}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o w -- python3 scripts/ab_wgrad_parts.py > $O/run.log 2>&1 || exit 1
python3 - $O/tr/w_kernel_trace.csv <<'PY' | tee $O/parts.txt
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
    k = r["Kernel_Name"]
    if "wgrad" in k or "reduce" in k:
        print(f"{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:8.1f} us  grid {r['Grid_Size_X']:>8} x {r['Grid_Size_Z']:>3}  {k[:90]}")
PY
grep "plan" $O/run.log
