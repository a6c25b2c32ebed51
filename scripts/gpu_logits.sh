#!/bin/bash
# Kernel durations of the PatchGAN logits conv: the two-pass taps form and the tiled kernel (rocprofv3 of ab_logits.py).
set -o pipefail
O=gpurun_out/${1:-r04_logits}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o lg -- python3 scripts/ab_logits.py > $O/run.log 2>&1 || exit 1
python3 scripts/prof_summary.py $O/prof/lg_kernel_stats.csv 8 | tee $O/summary.txt
