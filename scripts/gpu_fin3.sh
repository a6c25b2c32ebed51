#!/bin/bash
# GPU box: BN-finalize tests + train-step A/B (HEAD / separate finalize / fused finalize), then plan sweeps
# of the loader-wave tiles (conv: configs 0, 29-31; weight gradient: 0, 6, 7).
set -o pipefail
O=gpurun_out/fin3
mkdir -p $O
STC_BNFIN=1 timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread \
  -k "streams or c3 or model or dist or extras or bn" > $O/suite.log 2>&1
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
TUNE_CFGS=0,29,30,31 TUNE_KS=1,2,4 timeout -k 10 500 python -u scripts/tune_bf16.py $O/tune_bf16.json > $O/tune_bf16.log 2>&1 || exit 1
tail -3 $O/tune_bf16.log
WG_CFGS=0,6,7 WG_SPLITS=0,4,8,16,32,64 timeout -k 10 400 python -u scripts/tune_wgrad.py $O/tune_wgrad.json > $O/tune_wgrad.log 2>&1 || exit 1
tail -3 $O/tune_wgrad.log
