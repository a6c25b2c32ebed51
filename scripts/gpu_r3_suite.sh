#!/bin/bash
# Full GPU suite (no -x: every failure reported) + a short bench; each step time-limited.
set -o pipefail
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/suite.log 2>&1
rc=$?
echo "suite rc=$rc" >> $O/suite.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $O/bench.log 2>&1
fi
