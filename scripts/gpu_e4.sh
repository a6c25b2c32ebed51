#!/bin/bash
# e4 forward on the 256 x 64 halo block: halo tests, per-shape A/B, same-box step A/B against ab/lib_base.so.
set -o pipefail
O=gpurun_out/r04_e4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_halo.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python -u scripts/ab_conv.py > $O/ab_conv.log 2>&1 || exit 1
cat $O/ab_conv.log
for r in 1 2; do
  STC_LIB_PATH=ab/lib_base.so timeout -k 10 200 python -u scripts/train_steps.py --steps 20 --warmup 3 > $O/base_$r.log 2>&1 || exit 1
  timeout -k 10 200 python -u scripts/train_steps.py --steps 20 --warmup 3 > $O/now_$r.log 2>&1 || exit 1
done
grep -H "ms/step" $O/*.log
