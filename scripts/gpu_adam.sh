#!/bin/bash
# GPU box: Adam launch variants -- state hashes (bit-identity across processes), optimiser-step timings, and
# the in-step A/B of the default variant against streaming stores.
set -o pipefail
O=gpurun_out/adam
mkdir -p $O
: > $O/hash.log
for v in 0 0 1 2 3; do
  STC_ADAM_VARIANT=$v timeout -k 10 200 python -u scripts/ab_adam_variant.py hash 2>&1 | grep "state hash" >> $O/hash.log || exit 1
done
cat $O/hash.log
timeout -k 10 200 python -u scripts/ab_adam_variant.py > $O/times.log 2>&1 || exit 1
cat $O/times.log
: > $O/ab.log
for i in 1 2 3 4 5; do
  for v in 0 2; do
    r=$(STC_ADAM_VARIANT=$v timeout -k 10 200 python -u scripts/train_steps.py --steps 20 --warmup 5 2>&1 | grep "ms/step") || exit 1
    echo "adam_variant=$v $i: $r" >> $O/ab.log
  done
done
cat $O/ab.log
