#!/bin/bash
# GPU box: Adam streaming-load / streaming-pack-store variants: state hashes, optimiser-step times, in-step A/B.
set -o pipefail
O=gpurun_out/adam2
mkdir -p $O
for v in 10; do
  STC_ADAM_VARIANT=$v timeout -k 10 200 python -u scripts/ab_adam_variant.py hash 2>&1 | grep -E "state hash" || exit 1
done
AB_VARIANTS=2,10 timeout -k 10 200 python -u scripts/ab_adam_variant.py 2>&1 | grep " us" || exit 1
for i in 1 2 3 4; do
  for v in 2 10; do
    r=$(STC_ADAM_VARIANT=$v timeout -k 10 200 python -u scripts/train_steps.py --steps 20 --warmup 5 2>&1 | grep "ms/step") || exit 1
    echo "adam_variant=$v $i: $r"
  done
done
