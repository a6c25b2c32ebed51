#!/bin/bash
# Per-step kernel profile of the bench workload: rocprofv3 kernel trace + stats of scripts/train_steps.py,
# the kernel summary and the trace's busy/idle analysis.  Output: gpurun_out/$1/
OUT=gpurun_out/${1:-steps}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o steps \
  -- python scripts/train_steps.py --steps ${STEPS:-4} --warmup 2 ${STEP_ARGS} > $OUT/rocprof.log 2>&1 || exit $?
grep "ms/step" $OUT/rocprof.log
python scripts/prof_summary.py $OUT/trace/steps_kernel_stats.csv 45 > $OUT/summary.txt
python scripts/trace_gaps.py $OUT/trace/steps_kernel_trace.csv 0.5 > $OUT/gaps.txt
head -20 $OUT/gaps.txt
