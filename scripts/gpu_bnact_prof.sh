#!/bin/bash
# GPU box: kernel trace of the G1+G2 train-mode forward with and without the fused deep BatchNorm launch.
set -o pipefail
O=gpurun_out/bnact_prof
mkdir -p $O
export TMPDIR=/tmp
for v in 0 1; do
  STC_BN_ACT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$v -o fwd \
    -- python scripts/g1g2_fwd.py --reps 5 > $O/run$v.log 2>&1 || exit 1
  python scripts/prof_summary.py $O/t$v/fwd_kernel_stats.csv 30 > $O/summary$v.txt || exit 1
  python scripts/trace_gaps.py $O/t$v/fwd_kernel_trace.csv 0.6 > $O/gaps$v.txt 2>&1 || true
done
head -32 $O/summary0.txt $O/summary1.txt
