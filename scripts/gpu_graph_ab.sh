#!/bin/bash
# GPU box: bench.py eager vs --graph (the step replayed as one HIP graph), alternating processes.
set -o pipefail
O=gpurun_out/graph_ab
mkdir -p $O
: > $O/ab.log
for i in 1 2 3; do
  for g in "" "--graph"; do
    r=$(timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-extras --no-cpu-baseline $g 2>$O/err.log | tail -1) || exit 1
    echo "${g:-eager} $i: $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("step_launch"))')" >> $O/ab.log
  done
done
cat $O/ab.log
