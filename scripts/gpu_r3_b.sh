#!/bin/bash
set -o pipefail
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 600 python -u scripts/graph_capture_probe.py > $O/graph_probe.log 2>&1
echo "probe rc=$?" >> $O/graph_probe.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -q -x --timeout 280 --timeout-method thread > $O/graph_test.log 2>&1
echo "graph test rc=$?" >> $O/graph_test.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $O/bench_graph.log 2>&1
echo "bench rc=$?" >> $O/bench_graph.log
TUNE_CFGS=0,1,2,4,5,11,23,24,25,26,27,28 TUNE_KS=1,2,4 timeout -k 10 600 python -u scripts/tune_bf16.py $O/tune_new.json > $O/tune_new.log 2>&1
echo "tune rc=$?" >> $O/tune_new.log
