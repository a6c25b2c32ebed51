#!/bin/bash
# e4 forward on the 256 x 64 halo block: halo tests, single-stream step breakdown (per-launch HIP events) with the
# current library, the 8-wave 256 x 64 variant (ab/lib_n64w8.so) and ab/lib_base.so, per-shape A/B.
set -o pipefail
O=gpurun_out/r04_e4b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_halo.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in now n64w8 base; do
  if [ $v = now ]; then L=; else L=ab/lib_$v.so; fi
  STC_LIB_PATH=$L timeout -k 10 300 python -u scripts/step_breakdown.py > $O/$v.txt 2>&1 || exit 1
done
grep -H "grid16x16 cin256 cout512" $O/now.txt $O/n64w8.txt $O/base.txt
timeout -k 10 200 python -u scripts/ab_conv.py > $O/ab_conv.log 2>&1 || exit 1
grep "e4 fwd" $O/ab_conv.log
