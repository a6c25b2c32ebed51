#!/bin/bash
# GPU box: activation epilogue (first conv of G / D without the raw tensor + bn_apply pass): tests, then the
# in-step A/B (STC_ACT_EPI=0 restores conv + bn_apply).
set -o pipefail
O=gpurun_out/act
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread \
  -k "c3 or model or configs or streams or dist or extras or graph or overlap or objective" > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
: > $O/ab.log
for i in 1 2 3; do
  for v in 0 1; do
    r=$(STC_ACT_EPI=$v timeout -k 10 200 python -u scripts/train_steps.py --steps 20 --warmup 5 2>&1 | grep "ms/step") || exit 1
    echo "act_epi=$v $i: $r" >> $O/ab.log
  done
done
cat $O/ab.log
