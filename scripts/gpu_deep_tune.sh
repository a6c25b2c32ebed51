#!/bin/bash
# stc_deep_conv: GPU tests, the phase stamps of the automatic plans, the plan sweep (scripts/deep_tune.py) and the
# forward with the deep path on / off.
set -o pipefail
O=gpurun_out/${1:-deep_tune}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_deep.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u scripts/deep_tune.py --phases > $O/phases.log 2>&1 || { tail -5 $O/phases.log; exit 1; }
grep "==" $O/phases.log | cut -c1-260
if [ -z "$NO_SWEEP" ]; then
  timeout -k 10 500 python -u scripts/deep_tune.py ${TUNE_ARGS} > $O/tune.log 2>&1 || { tail -5 $O/tune.log; exit 1; }
  grep "==" $O/tune.log
fi
timeout -k 10 240 python scripts/fwd_timeline.py --reps 5 --deep 0 > $O/fwd_deep0.json 2> $O/fwd_deep0.err || exit 1
echo "deep=0 $(cat $O/fwd_deep0.json)"
for lv in ${LEVELS:-2 3}; do
  timeout -k 10 240 python scripts/fwd_timeline.py --reps 5 --deep 1 --levels $lv > $O/fwd_deep1_l$lv.json 2> $O/fwd_deep1_l$lv.err || exit 1
  echo "deep=1 levels=$lv $(cat $O/fwd_deep1_l$lv.json)"
done
