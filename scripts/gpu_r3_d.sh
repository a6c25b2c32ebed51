#!/bin/bash
# Round 3: optimiser overlapped with the backward + graph capture with the discriminator lanes.
# Each GPU step time-limited; nothing after a failed step.
set -o pipefail
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_dist.py -x -v --timeout 240 \
  --timeout-method thread > $O/d_graph_dist.log 2>&1 &&
timeout -k 10 400 python -u scripts/ab_overlap.py --steps 10 --rounds 3 > $O/d_ab_overlap.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread > $O/d_suite.log 2>&1
echo "rc=$?" >> $O/d_suite.log
