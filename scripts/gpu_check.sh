#!/bin/bash
# quick GPU check: the listed test files (-k filter optional), the north-star forward + its kernel trace, two
# bench lines.  usage: gpu_check.sh <tag> "<test files>" ["<-k expr>"]
set -o pipefail
O=gpurun_out/${1:-check}
mkdir -p $O
export TMPDIR=/tmp
K=${3:+-k "$3"}
eval timeout -k 10 600 python -u -m pytest $2 -x -q --timeout 200 --timeout-method thread $K > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 240 python scripts/fwd_timeline.py --reps 5 > $O/fwd.json 2> $O/fwd.err || exit 1
echo "fwd $(cat $O/fwd.json)"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o fwd -- python scripts/fwd_timeline.py --reps 2 --no-graph > $O/trace_run.log 2>&1 || exit 1
python scripts/fwd_timeline_read.py $(ls $O/tr/*/fwd_kernel_trace.csv $O/tr/fwd_kernel_trace.csv 2>/dev/null | head -1) 2 > $O/timeline.txt
head -1 $O/timeline.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench$i.json 2> $O/bench$i.err || exit 1
  python -c "import json;d=json.load(open('$O/bench$i.json'));print('bench', d['value'], d['ms_per_step'])"
done
