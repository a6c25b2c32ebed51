#!/bin/bash
# GPU box: in-step A/B of the round-3 loader-tile plans (conv: STC_PLAN_R2 restores the round-2 plan;
# weight gradient: STC_WPLAN_R2), alternating processes; then a kernel trace of the step.
set -o pipefail
O=gpurun_out/plans
mkdir -p $O
: > $O/ab.log
for i in 1 2 3; do
  for arm in "new" "conv_r2" "wgrad_r2" "both_r2"; do
    case $arm in
      new) E="";; conv_r2) E="STC_PLAN_R2=1";; wgrad_r2) E="STC_WPLAN_R2=1";; both_r2) E="STC_PLAN_R2=1 STC_WPLAN_R2=1";;
    esac
    r=$(env $E timeout -k 10 200 python -u scripts/train_steps.py --steps 20 --warmup 5 2>&1 | grep "ms/step") || exit 1
    echo "$arm $i: $r" >> $O/ab.log
  done
done
cat $O/ab.log
STEPS=6 timeout -k 10 400 bash scripts/gpu_steps.sh plans/steps || exit 1
python scripts/trace_concurrency.py gpurun_out/plans/steps/trace/steps_kernel_trace.csv 0.6 30 > $O/concurrency.txt
head -45 $O/concurrency.txt
