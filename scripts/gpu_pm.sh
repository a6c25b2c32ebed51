#!/bin/bash
# GPU box: phase-major block order for the 4-phase ConvT GEMMs (STC_PHASE_MAJOR=0 restores the z-major grid):
# tests, isolated conv timings both ways, in-step A/B.
set -o pipefail
O=gpurun_out/pm
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread \
  -k "igemm or c3 or model or configs or streams" > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  STC_PHASE_MAJOR=$v timeout -k 10 240 python -u scripts/diag_gemm.py > $O/diag$v.log 2>&1 || exit 1
done
paste -d'\n' $O/diag0.log $O/diag1.log | grep -v amdgpu
: > $O/ab.log
for i in 1 2 3; do
  for v in 0 1; do
    r=$(STC_PHASE_MAJOR=$v timeout -k 10 200 python -u scripts/train_steps.py --steps 20 --warmup 5 2>&1 | grep "ms/step") || exit 1
    echo "phase_major=$v $i: $r" >> $O/ab.log
  done
done
cat $O/ab.log
