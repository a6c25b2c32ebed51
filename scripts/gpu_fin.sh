#!/bin/bash
# GPU box: the full GPU suite, then an A/B of the BatchNorm finalize fused into the producing conv
# (STC_BNFIN=1, default) against the separate finalize kernels (STC_BNFIN=0), alternating processes.
set -o pipefail
O=gpurun_out/fin
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/suite.log 2>&1
rc=$?
echo "suite rc=$rc" >> $O/suite.log
tail -15 $O/suite.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
: > $O/ab.log
for i in 1 2 3; do
  for v in 0 1; do
    r=$(STC_BNFIN=$v timeout -k 10 200 python -u scripts/train_steps.py --steps 20 --warmup 5 2>&1 | grep "ms/step") || exit 1
    echo "bnfin=$v $i: $r" >> $O/ab.log
  done
done
cat $O/ab.log
