#!/bin/bash
set -o pipefail
O=gpurun_out/r3
mkdir -p $O
PROBE_LOG=1 timeout -k 10 600 python -u scripts/graph_capture_probe.py > $O/graph_probe2.log 2>&1
echo "probe rc=$?" >> $O/graph_probe2.log
