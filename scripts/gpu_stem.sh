#!/bin/bash
# First-layer stem conv: its GPU tests, the C3 per-layer checks that run through it, a per-layer timing against the
# im2col tile, then the default bench line.  Output: gpurun_out/$1/
set -o pipefail
O=gpurun_out/${1:-r04_stem}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stem.py tests/test_gpu_c3_layers.py -v --timeout 300 --timeout-method thread -x > $O/stem_tests.log 2>&1
rc=$?
tail -3 $O/stem_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_stem.py > $O/ab_stem.log 2>&1 || exit 1
cat $O/ab_stem.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | cut -c1-300
