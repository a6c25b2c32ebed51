#!/bin/bash
# A/B of the default library vs the one built without packed-FP32 VALU ops (Makefile EXTRA=...):
# the side-stream bit-identity tests (3 runs each) and the step time.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NOPK=$PWD/shadow-removal-istd_amd/stcgan_amd/libstcgan_hip_nopk.so
for lib in default nopk; do
  if [ $lib = nopk ]; then export STC_LIB_PATH=$NOPK; else unset STC_LIB_PATH; fi
  for i in 1 2 3; do
    timeout -k 10 200 python -u -m pytest -q tests/test_gpu_extras.py tests/test_gpu_streams.py -k "side_stream or schedules" \
      --timeout 150 --timeout-method thread 2>&1 | tail -1 | sed "s/^/$lib run $i: /" || exit 1
  done
  timeout -k 10 120 python scripts/train_steps.py --steps 15 --warmup 3 --repeat 4 | tail -2 | sed "s/^/$lib: /" || exit 1
done
