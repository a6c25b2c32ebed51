#!/bin/bash
# Round-3 final: the whole GPU suite, the default bench line (CPU baseline + extras), rocprof stats and PMC
# traffic of the bench command, and the single-stream per-launch breakdown.  Each step time-limited.
set -o pipefail
O=gpurun_out/r03_final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1
rc=$?
echo "suite rc=$rc" >> $O/suite.log
tail -3 $O/suite.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1 || exit 1
tail -1 $O/bench_default.log > $O/bench_default.json
BENCH_ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-extras" timeout -k 10 1000 bash scripts/profile_round.sh r03_final/prof || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/single -o steps \
  -- python scripts/step_breakdown.py > $O/step_breakdown.txt 2>&1 || exit 1
python scripts/prof_summary.py $O/single/steps_kernel_stats.csv 45 > $O/single_summary.txt
cut -c1-400 $O/bench_default.json
