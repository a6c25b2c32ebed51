#!/bin/bash
# Round 3: K-split narrow kernel -- parity tests of the kernels, then the tile sweep (old vs new).
set -o pipefail
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_igemm_bf16.py tests/test_gpu_kernels.py -x -q --timeout 240 \
  --timeout-method thread > $O/e_kernels.log 2>&1 &&
timeout -k 10 200 python -u scripts/narrow_sweep.py > $O/e_narrow_sweep.log 2>&1
echo "rc=$?" >> $O/e_narrow_sweep.log
