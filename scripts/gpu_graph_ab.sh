#!/bin/bash
# Eager vs HIP-graph bench lines, interleaved on one box.
set -o pipefail
O=gpurun_out/${1:-graph_ab}
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for mode in eager graph; do
    flag=""; [ $mode = graph ] && flag="--graph"
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras $flag > $O/$mode$i.json 2> $O/$mode$i.err || { tail -5 $O/$mode$i.err; exit 1; }
    python -c "import json;d=json.load(open('$O/$mode$i.json'));print('$mode', d['value'], d['ms_per_step'], d['config']['step_launch'])"
  done
done
