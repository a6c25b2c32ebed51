#!/bin/bash
# GPU box: first-layer row-halo conv -- bit-identity vs the GEMM tile, model suites, in-step A/B, per-launch times.
set -o pipefail
O=gpurun_out/halo8
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_halo8.py -q -x --timeout 100 --timeout-method thread > $O/unit.log 2>&1
rc=$?; tail -3 $O/unit.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread \
  -k "c3 or model or configs or streams or dist or extras or graph or overlap or objective" > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
: > $O/ab.log
for i in 1 2 3 4; do
  for v in 0 1; do
    r=$(STC_HALO8=$v timeout -k 10 200 python -u scripts/train_steps.py --steps 20 --warmup 5 2>&1 | grep "ms/step") || exit 1
    echo "halo8=$v $i: $r" >> $O/ab.log
  done
done
cat $O/ab.log
for v in 0 1; do
  STC_HALO8=$v timeout -k 10 200 python -u scripts/step_breakdown.py > $O/breakdown$v.txt 2>&1 || exit 1
  grep -E "cin8 cout64|conv-family" $O/breakdown$v.txt | head -12
done
