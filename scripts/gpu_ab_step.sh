#!/bin/bash
# Step-time A/B of diagnostic library builds (scripts/ab_step.py under each of $AB_LIBS, then the in-tree
# library).  Output: gpurun_out/$1/ab_step.log
set -o pipefail
O=gpurun_out/${1:-r04_abstep}
mkdir -p $O
export TMPDIR=/tmp
for lib in $AB_LIBS; do
  STC_LIB_PATH=$lib timeout -k 10 300 python -u scripts/ab_step.py >> $O/ab_step.log 2>&1 || exit 1
done
timeout -k 10 300 python -u scripts/ab_step.py >> $O/ab_step.log 2>&1 || exit 1
cat $O/ab_step.log
