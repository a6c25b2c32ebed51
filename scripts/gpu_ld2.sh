#!/bin/bash
# GPU box: the 2-loader-wave conv tiles (64 KiB, two blocks per CU like the plain tiles): correctness of the
# forced configs, isolated times, then the in-step A/B (STC_PLAN_LD2=1 vs the default plan).
set -o pipefail
O=gpurun_out/ld2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_igemm_bf16.py -q -x --timeout 200 --timeout-method thread -k "cfg33 or cfg34 or cfg35 or auto" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_loaders.py > $O/loaders.log 2>&1 || exit 1
cat $O/loaders.log
: > $O/ab.log
for i in 1 2 3; do
  for v in 0 1; do
    if [ $v = 1 ]; then E="STC_PLAN_LD2=1"; else E=""; fi
    r=$(env $E timeout -k 10 200 python -u scripts/train_steps.py --steps 20 --warmup 5 2>&1 | grep "ms/step") || exit 1
    echo "ld2=$v $i: $r" >> $O/ab.log
  done
done
cat $O/ab.log
