#!/bin/bash
# Statistics pass after the 16-byte stores: conv / model GPU tests, then the per-shape A/B and the epilogue timing.
set -o pipefail
O=gpurun_out/${1:-r04_epi}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_halo.py tests/test_gpu_igemm_bf16.py tests/test_gpu_model.py tests/test_gpu_c3_layers.py tests/test_gpu_stem.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u scripts/ab_epi.py 2>&1 | tee $O/ab_epi.log
timeout -k 10 200 python -u scripts/ab_conv.py > $O/ab_conv.log 2>&1 && cut -c1-120 $O/ab_conv.log
