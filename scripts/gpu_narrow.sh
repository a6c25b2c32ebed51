#!/bin/bash
# Streaming narrow ConvT kernel: GPU tests (vs torch fp32 and the tiled kernel) and the per-launch A/B.
set -o pipefail
O=gpurun_out/${1:-r04_narrow}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_igemm_bf16.py -k "narrow" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 120 python -u scripts/ab_narrow.py 2>&1 | tee $O/ab.log
