#!/bin/bash
# Kernel trace of the bench workload's overlapped train step (scripts/train_steps.py: 4 timed steps after 2
# warm-up), then its concurrency profile (scripts/trace_concurrency.py: exposed kernels = running alone).
set -o pipefail
O=gpurun_out/${1:-r04_trace}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o steps -- python scripts/train_steps.py --steps 4 --warmup 2 > $O/train_steps.log 2>&1 || exit 1
python scripts/trace_concurrency.py $O/tr/steps_kernel_trace.csv 3:7 40 > $O/concurrency.txt
python scripts/prof_summary.py $O/tr/steps_kernel_stats.csv 40 > $O/summary.txt 2>/dev/null || true
cat $O/concurrency.txt
