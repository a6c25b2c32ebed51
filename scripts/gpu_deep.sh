#!/bin/bash
# stc_deep_conv: GPU tests, then the north-star forward with the deep path on / off (eager, graph) and a kernel
# trace of the deep forward.  usage: gpu_deep.sh <tag>
set -o pipefail
O=gpurun_out/${1:-deep}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_deep.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for d in 0 1; do
  timeout -k 10 240 python scripts/fwd_timeline.py --reps 5 --deep $d --levels ${LEVELS:-3} > $O/fwd_deep$d.json 2> $O/fwd_deep$d.err || exit 1
  echo "deep=$d $(cat $O/fwd_deep$d.json)"
done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o fwd -- python scripts/fwd_timeline.py --reps 2 --no-graph --deep 1 --levels ${LEVELS:-3} > $O/trace_run.log 2>&1 || exit 1
python scripts/fwd_timeline_read.py $(ls $O/tr/*/fwd_kernel_trace.csv $O/tr/fwd_kernel_trace.csv 2>/dev/null | head -1) 2 > $O/timeline.txt
head -8 $O/timeline.txt
if [ -n "$EXTRA" ]; then
  timeout -k 10 300 python scripts/exchange_timeline.py > $O/exchange_timeline.json 2> $O/exchange_timeline.err || exit 1
  timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 240 --timeout-method thread -k "shards" > $O/dist.log 2>&1 || { tail -20 $O/dist.log; exit 1; }
  tail -2 $O/dist.log
fi
