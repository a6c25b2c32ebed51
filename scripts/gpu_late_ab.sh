#!/bin/bash
# Early real-input D backward: its tests, an interleaved A/B (train_steps.py --ab-attr early=0,1) and the bench line.
set -o pipefail
O=gpurun_out/${1:-late}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_model.py tests/test_gpu_extras.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python scripts/train_steps.py --steps 20 --warmup 3 --ab-attr late=0,1 --repeat 8 > $O/ab.txt 2>&1 || { tail $O/ab.txt; exit 1; }
grep -v amdgpu $O/ab.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['value'], d['ms_per_step'])"
