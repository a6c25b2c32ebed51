#!/bin/bash
# Round final profile: rocprof stats + PMC traffic / MFMA busy of the bench command (scripts/profile_round.sh) and
# the single-stream per-launch step breakdown.  Output: gpurun_out/$1/
set -o pipefail
O=gpurun_out/${1:-r05_final}
mkdir -p $O
export TMPDIR=/tmp
BENCH_ARGS="--steps 5 --warmup 2 --no-cpu-baseline" timeout -k 10 1000 bash scripts/profile_round.sh ${1:-r05_final} || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/single -o steps \
  -- python scripts/step_breakdown.py > $O/step_breakdown.txt 2>&1 || exit 1
python scripts/prof_summary.py $O/single/steps_kernel_stats.csv 45 > $O/single_summary.txt
tail -2 $O/step_breakdown.txt
