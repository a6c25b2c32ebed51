#!/bin/bash
# Host cost per call site of the train step (scripts/host_ops.py) and per launch ingredient (scripts/host_micro.py).
set -o pipefail
O=gpurun_out/${1:-hostprof}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python scripts/host_micro.py > $O/host_micro.txt 2>&1 || { tail $O/host_micro.txt; exit 1; }
cat $O/host_micro.txt
timeout -k 10 200 python scripts/host_ops.py > $O/host_ops.txt 2>&1 || { tail $O/host_ops.txt; exit 1; }
head -40 $O/host_ops.txt
