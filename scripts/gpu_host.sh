#!/bin/bash
# Is the eager step host-bound?  Host enqueue vs GPU time (scripts/host_vs_gpu.py) and the step time with extra
# host time per step (train_steps.py --host-sleep-us).  Output: gpurun_out/$1/
set -o pipefail
O=gpurun_out/${1:-host}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python scripts/host_vs_gpu.py > $O/host_vs_gpu.txt 2>&1 || { tail $O/host_vs_gpu.txt; exit 1; }
head -4 $O/host_vs_gpu.txt
for s in 0 500 1000 2000 0; do
  timeout -k 10 200 python scripts/train_steps.py --steps 20 --warmup 3 --host-sleep-us $s > $O/sleep_$s.txt 2>&1 || exit 1
  echo "sleep $s: $(tail -1 $O/sleep_$s.txt)"
done
