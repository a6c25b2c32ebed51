#!/bin/bash
# Weight-gradient GPU tests (every tile, the rows path, the split reduces) and the per-problem tile / reduce profile.
set -o pipefail
O=gpurun_out/${1:-r04_wtests}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_igemm_bf16.py tests/test_gpu_kernels.py -k "wgrad or rows" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash scripts/gpu_wgrad_parts.sh ${1:-r04_wtests}_parts > /dev/null && cat gpurun_out/${1:-r04_wtests}_parts/parts.txt | grep reduce | sort | uniq -c | sort -rn | head -20
