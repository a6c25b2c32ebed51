#!/bin/bash
# graph-capture probe (subprocesses), the GPU suite minus the graph test, c3 layer prints, eager bench
set -o pipefail
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 600 python -u scripts/graph_capture_probe.py > $O/graph_probe.log 2>&1
echo "probe rc=$?" >> $O/graph_probe.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "not test_captured_step" > $O/suite.log 2>&1
echo "suite rc=$?" >> $O/suite.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_c3_layers.py tests/test_gpu_configs.py -m gpu -q -s --timeout 300 --timeout-method thread -k "layers or bf16_oracle" > $O/c3.log 2>&1
echo "c3 rc=$?" >> $O/c3.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-graph > $O/bench.log 2>&1
echo "bench rc=$?" >> $O/bench.log
