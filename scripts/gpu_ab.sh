#!/bin/bash
# Tests, then interleaved bench A/B of two library/flag settings on one box.  usage: gpu_ab.sh <tag> "<tests>" [reps]
set -o pipefail
O=gpurun_out/${1:-ab}
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$2" ]; then
  timeout -k 10 900 python -u -m pytest $2 -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for i in $(seq 1 ${3:-2}); do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench$i.json 2> $O/bench$i.err || exit 1
  python -c "import json;d=json.load(open('$O/bench$i.json'));print('bench', d['value'], d['ms_per_step'], d['roofline'].get('g1g2_forward_frac'))"
done
timeout -k 10 200 python scripts/host_vs_gpu.py > $O/host_vs_gpu.txt 2>&1 && head -3 $O/host_vs_gpu.txt | tail -2
