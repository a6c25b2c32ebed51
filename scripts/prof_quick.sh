#!/bin/bash
# rocprof kernel stats of a short bf16 bench (no extras, no CPU leg): prof_quick.sh <tag>
set -o pipefail
OUT=gpurun_out/pq_${1:-x}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > $OUT/bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o k -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > $OUT/rocprof.log 2>&1 || exit $?
python scripts/prof_summary.py $OUT/trace/k_kernel_stats.csv 45 > $OUT/summary.txt
tail -1 $OUT/bench.log | cut -c1-200
head -46 $OUT/summary.txt
