#!/bin/bash
# Same-box step A/B: the library at this round's session start (ab/lib_start.so) against the current one, alternating.
set -o pipefail
O=gpurun_out/${1:-r04_absession}
mkdir -p $O
for r in 1 2; do
  STC_LIB_PATH=ab/lib_start.so timeout -k 10 200 python -u scripts/train_steps.py --steps 20 --warmup 3 > $O/start_$r.log 2>&1 || exit 1
  timeout -k 10 200 python -u scripts/train_steps.py --steps 20 --warmup 3 > $O/now_$r.log 2>&1 || exit 1
done
grep -H "ms/step" $O/*.log
