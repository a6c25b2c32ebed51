#!/bin/bash
# GPU box: row-halo first layers on by default -- the model-level suites through it, and the bench line.
set -o pipefail
O=gpurun_out/halo8b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread \
  -k "halo8 or c3 or model or configs or streams or dist or extras or graph or overlap or objective or kernels" > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  STC_HALO8=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/bench$v.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('$O/bench$v.log').read().strip().splitlines()[-1]); r=d['roofline']; print('halo8=$v', d['value'], d['ms_per_step'], 'g1g2', r['g1g2_forward'])"
done
