#!/bin/bash
# Weight-gradient kernels: their GPU tests, then the plan sweep over the train step's problems (scripts/tune_wgrad.py,
# configs $WG_CFGS, splits $WG_SPLITS).  Output: gpurun_out/$1/
set -o pipefail
O=gpurun_out/${1:-r04_wgrad}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_igemm_bf16.py -k wgrad -v --timeout 120 --timeout-method thread -x > $O/wgrad_tests.log 2>&1
rc=$?
tail -3 $O/wgrad_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/tune_wgrad.py $O/tune.json > $O/tune.log 2>&1 || exit 1
cat $O/tune.log
