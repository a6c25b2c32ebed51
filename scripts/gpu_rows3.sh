#!/bin/bash
# Logits-layer weight gradient: kernel durations of the shipped build and of the loads-only diagnostic build.
set -o pipefail
O=gpurun_out/${1:-r04_rows5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o rows -- python3 scripts/ab_rows.py > $O/rows.log 2>&1 || exit 1
STC_LIB_PATH=ab/lib_noepi.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_noepi -o rows -- python3 scripts/ab_rows.py > $O/rows_noepi.log 2>&1 || exit 1
for d in prof prof_noepi; do echo "== $d"; python3 scripts/prof_summary.py $O/$d/rows_kernel_stats.csv 3; done | tee $O/summary.txt
