#!/bin/bash
# GPU box: deep split-K conv + BatchNorm + activation in one post-GEMM launch (STC_BN_ACT): its tests and the
# model-level suites, then the in-step A/B and the G1+G2 forward (STC_BN_ACT=0 restores reduce/finalize/apply).
set -o pipefail
O=gpurun_out/bnact
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bn_act.py -q -x --timeout 100 --timeout-method thread > $O/unit.log 2>&1
rc=$?; tail -3 $O/unit.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread \
  -k "c3 or model or configs or streams or dist or extras or graph or overlap or objective" > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
: > $O/ab.log
for i in 1 2 3; do
  for v in 0 1; do
    r=$(STC_BN_ACT=$v timeout -k 10 200 python -u scripts/train_steps.py --steps 20 --warmup 5 2>&1 | grep "ms/step") || exit 1
    echo "bn_act=$v $i: $r" >> $O/ab.log
  done
done
for v in 0 1 0 1; do
  STC_BN_ACT=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > $O/bench$v.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('$O/bench$v.log').read().strip().splitlines()[-1]); r=d['roofline']; print('bn_act=$v', d['ms_per_step'], 'ms/step  g1g2_forward', r['g1g2_forward'])" >> $O/ab.log
done
cat $O/ab.log
