#!/bin/bash
# GPU box: BN-backward dgrad epilogue with the first row group's loads issued before the tile staging --
# correctness suites, in-step timing, and the bench line (dominant-kernel roofline).
set -o pipefail
O=gpurun_out/bnb
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread \
  -k "igemm_bf16 or bnfin or c3 or model or configs or kernels" > $O/suite.log 2>&1
rc=$?; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python -u scripts/train_steps.py --steps 20 --warmup 5 2>&1 | grep "ms/step" || exit 1
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $O/bench.log 2>&1 || exit 1
python -c "
import json; d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]); r=d['roofline']
print(d['value'], d['ms_per_step'], r['frac'], r['frac_in_situ'], r['kernel'][:150]); print(r['g1g2_forward'])
print({k: (v['avg_us'], v['tflops']) for k, v in r['per_kernel'].items()})"
