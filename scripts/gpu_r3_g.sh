#!/bin/bash
# Round 3 profile: overlap bit-identity + C3 tests, then bench line / rocprof stats / PMC passes of the
# bench command, and the single-stream per-launch breakdown.  Each step time-limited.
set -o pipefail
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_overlap.py "tests/test_gpu_configs.py::test_c3_bf16_train_step_ngf64_vs_bf16_oracle" \
  -v --timeout 240 --timeout-method thread > $O/g_tests.log 2>&1
echo "tests rc=$?" >> $O/g_tests.log
BENCH_ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-extras" timeout -k 10 1000 bash scripts/profile_round.sh r03_prof &&
export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_prof/single -o steps \
  -- python scripts/step_breakdown.py > gpurun_out/r03_prof/single_breakdown.txt 2>&1 &&
python scripts/prof_summary.py gpurun_out/r03_prof/single/steps_kernel_stats.csv 45 > gpurun_out/r03_prof/single_summary.txt
