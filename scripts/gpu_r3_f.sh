#!/bin/bash
# Round 3: full GPU suite (every failure reported), the default bench line (extras + CPU baseline) and the
# ATen call sites left in a step; each step time-limited, nothing after a crash or a timeout.
set -o pipefail
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/f_suite.log 2>&1
rc=$?
echo "rc=$rc" >> $O/f_suite.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/f_bench.json 2> $O/f_bench.err &&
timeout -k 10 200 python -u scripts/torch_ops.py > $O/f_torch_ops.log 2>&1
