#!/bin/bash
# Stream-priority A/B of the eager step (scripts/train_steps.py --main/--lane/--side-priority), configs interleaved.
set -o pipefail
O=gpurun_out/${1:-prio}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for cfg in "0 0 0" "-1 0 0" "-1 -1 0" "0 -1 0"; do
    set -- $cfg
    timeout -k 10 200 python scripts/train_steps.py --steps 20 --warmup 3 --main-priority $1 --lane-priority $2 --side-priority $3 > $O/run.txt 2>&1 || { tail $O/run.txt; exit 1; }
    echo "main=$1 lane=$2 side=$3: $(tail -1 $O/run.txt | cut -d' ' -f1)" | tee -a $O/ab.txt
  done
done
