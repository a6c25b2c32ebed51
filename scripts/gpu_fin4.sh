#!/bin/bash
# GPU box: kernel + model tests with the loader-wave plans and the fused finalize on, train-step A/B
# (HEAD / this tree with separate finalize / fused), weight-gradient plan sweep.
set -o pipefail
O=gpurun_out/fin4
mkdir -p $O
STC_BNFIN=1 timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread \
  -k "igemm or kernels or streams or c3 or model or dist or extras or bn or graph or overlap" > $O/suite.log 2>&1
rc=$?
echo "suite rc=$rc" >> $O/suite.log
tail -4 $O/suite.log
[ $rc -eq 0 ] || exit $rc
: > $O/ab.log
for i in 1 2 3; do
  r=$(timeout -k 10 200 python -u ab/head/scripts/train_steps.py --steps 20 --warmup 5 2>&1 | grep "ms/step") || exit 1
  echo "head $i: $r" >> $O/ab.log
  for v in 0 1; do
    r=$(STC_BNFIN=$v timeout -k 10 200 python -u scripts/train_steps.py --steps 20 --warmup 5 2>&1 | grep "ms/step") || exit 1
    echo "bnfin=$v $i: $r" >> $O/ab.log
  done
done
cat $O/ab.log
WG_CFGS=0,3,5,6,7 WG_SPLITS=0,4,8,16,32 timeout -k 10 500 python -u scripts/tune_wgrad.py $O/tune_wgrad.json > $O/tune_wgrad.log 2>&1 || exit 1
tail -3 $O/tune_wgrad.log
