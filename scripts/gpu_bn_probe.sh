#!/bin/bash
# BN element-wise passes: HBM rate per shape (scripts/bn_bw.py) and the per-launch kernel trace of one
# single-stream train step (scripts/step_breakdown.py under rocprofv3).  Output: gpurun_out/$1/
set -o pipefail
O=gpurun_out/${1:-bn_probe}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python scripts/bn_bw.py > $O/bn_bw.txt 2>&1 || { cat $O/bn_bw.txt; exit 1; }
cat $O/bn_bw.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o steps -- python scripts/step_breakdown.py > $O/step_breakdown.txt 2>&1 || exit 1
T=$(ls $O/tr/*/steps_kernel_trace.csv $O/tr/steps_kernel_trace.csv 2>/dev/null | head -1)
python scripts/trace_family.py $T 'bn_' > $O/bn_launches.txt
python scripts/trace_family.py $T '.' > $O/all_launches.txt
tail -1 $O/bn_launches.txt; tail -1 $O/all_launches.txt
