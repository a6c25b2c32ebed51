#!/bin/bash
# Round-3 stream-hazard / packed-FP32 diagnosis on one GPU (each step time-limited, chained with &&).
set -o pipefail
O=gpurun_out/r3
mkdir -p $O
PK=$PWD/scripts/micro/libstcgan_hip_rows_packed.so
timeout -k 10 180 python -u tests/test_gpu_stream_hazards.py > $O/probe.log 2>&1 &&
timeout -k 10 120 python -u scripts/rows_stress.py --iters 2000 --load --tag shipped > $O/rows.log 2>&1 &&
STC_LIB_PATH=$PK timeout -k 10 120 python -u scripts/rows_stress.py --iters 2000 --load --tag packed >> $O/rows.log 2>&1 &&
( STC_LIB_PATH=$PK timeout -k 10 150 python -u scripts/rows_stress.py --iters 3000 --load --tag packed-2proc-a >> $O/rows.log 2>&1 & pa=$!
  STC_LIB_PATH=$PK timeout -k 10 150 python -u scripts/rows_stress.py --iters 3000 --load --tag packed-2proc-b >> $O/rows.log 2>&1 & pb=$!
  wait $pa && wait $pb ) &&
( timeout -k 10 150 python -u scripts/rows_stress.py --iters 3000 --load --tag shipped-2proc-a >> $O/rows.log 2>&1 & pa=$!
  timeout -k 10 150 python -u scripts/rows_stress.py --iters 3000 --load --tag shipped-2proc-b >> $O/rows.log 2>&1 & pb=$!
  wait $pa && wait $pb ) &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_stream_hazards.py \
  tests/test_gpu_streams.py tests/test_gpu_extras.py tests/test_gpu_configs.py::test_c3_bf16_train_step_ngf64_vs_bf16_oracle > $O/t1.log 2>&1
