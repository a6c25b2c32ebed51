#!/bin/bash
# GPU box: kernel stats of the bench workload with the separate finalize kernels and with the fused finalize.
set -o pipefail
O=gpurun_out/bnfin_prof
mkdir -p $O
export TMPDIR=/tmp
for v in 0 1; do
  STC_BNFIN=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$v -o steps \
    -- python scripts/train_steps.py --steps 6 --warmup 2 > $O/run$v.log 2>&1 || exit 1
  grep "ms/step" $O/run$v.log
  python scripts/prof_summary.py $O/t$v/steps_kernel_stats.csv 40 > $O/summary$v.txt
done
head -30 $O/summary0.txt
head -30 $O/summary1.txt
