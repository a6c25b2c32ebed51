#!/bin/bash
# The GPU test suite (every -m gpu test, one process), then the default bench line.  Output: gpurun_out/$1/
set -o pipefail
O=gpurun_out/${1:-r04_suite}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -x ${PYTEST_ARGS} > $O/suite.log 2>&1
rc=$?
echo "suite rc=$rc" >> $O/suite.log
tail -3 $O/suite.log
[ $rc -eq 0 ] || exit $rc
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit 1
  tail -1 $O/bench.log | cut -c1-600
fi
