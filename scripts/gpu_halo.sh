#!/bin/bash
# Halo conv-s2 kernel: its GPU tests, then per-layer timings of the halo vs the im2col tile at the train-step
# shapes (scripts/ab_conv.py).  Output: gpurun_out/$1/
set -o pipefail
O=gpurun_out/${1:-r04_halo}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_halo.py -v --timeout 120 --timeout-method thread -x > $O/halo_tests.log 2>&1
rc=$?
tail -3 $O/halo_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_conv.py > $O/ab_conv.log 2>&1 || exit 1
cat $O/ab_conv.log
# variant libraries (diagnostic builds under ab/): the same timings with each
for lib in $AB_LIBS; do
  echo "== $lib" | tee -a $O/ab_conv.log
  STC_LIB_PATH=$lib timeout -k 10 300 python -u scripts/ab_conv.py 2>&1 | tee -a $O/ab_conv.log || exit 1
done
