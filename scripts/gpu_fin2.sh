#!/bin/bash
# GPU box: BN-finalize tests + A/B of train-step time: HEAD library (ab/head), this tree with the separate
# finalize kernels (STC_BNFIN=0) and with the finalize fused into the producers (STC_BNFIN=1).
set -o pipefail
O=gpurun_out/fin2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread \
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
timeout -k 10 300 python -u scripts/ab_loaders.py > $O/loaders.log 2>&1
cat $O/loaders.log
timeout -k 10 300 python -u scripts/ab_wgrad_loaders.py > $O/wloaders.log 2>&1; cat $O/wloaders.log
