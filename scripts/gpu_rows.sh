#!/bin/bash
# MFMA logits-layer weight gradient and the streaming narrow ConvT: GPU tests + per-call timings.
set -o pipefail
O=gpurun_out/${1:-r04_rows}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_igemm_bf16.py -k "rows or narrow" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 120 python -u scripts/ab_rows.py 2>&1 | tee $O/ab_rows.log
timeout -k 10 120 python -u scripts/ab_narrow.py 2>&1 | tee $O/ab_narrow.log
