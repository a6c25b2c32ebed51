#!/bin/bash
# Kernel-level durations of the logits-layer weight gradient (rocprofv3 kernel trace of scripts/ab_rows.py).
set -o pipefail
O=gpurun_out/${1:-r04_rows2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o rows -- python3 scripts/ab_rows.py > $O/rows.log 2>&1 || exit 1
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} python3 scripts/prof_summary.py {} 12 > $O/summary.txt
cat $O/summary.txt
