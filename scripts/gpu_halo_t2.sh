#!/bin/bash
# halo ConvT phase pair (GEOM 4): halo tests, the north-star forward and its kernel trace, one bench line
set -o pipefail
O=gpurun_out/${1:-halo_t2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_halo.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 240 python scripts/fwd_timeline.py --reps 5 --deep 0 > $O/fwd.json 2> $O/fwd.err || exit 1
echo "fwd $(cat $O/fwd.json)"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o fwd -- python scripts/fwd_timeline.py --reps 2 --no-graph --deep 0 > $O/trace_run.log 2>&1 || exit 1
python scripts/fwd_timeline_read.py $(ls $O/tr/*/fwd_kernel_trace.csv $O/tr/fwd_kernel_trace.csv 2>/dev/null | head -1) 2 > $O/timeline.txt
head -6 $O/timeline.txt
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['value'], d['ms_per_step'], d.get('g1g2_forward'))"
fi
