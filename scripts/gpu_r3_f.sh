#!/bin/bash
# Round 3: full GPU suite, then the default bench line (extras + CPU baseline), each time-limited.
set -o pipefail
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread > $O/f_suite.log 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/f_bench.json 2> $O/f_bench.err
echo "rc=$?" >> $O/f_suite.log
