#!/bin/bash
# North-star forward: eager / host-enqueue / HIP-graph timing, then a kernel trace of eager forwards
# and its per-kernel timeline (scripts/fwd_timeline.py, fwd_timeline_read.py).  usage: gpu_fwd_timeline.sh <tag>
set -o pipefail
O=gpurun_out/${1:-fwd}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python scripts/fwd_timeline.py --reps 5 > $O/fwd_time.json 2> $O/fwd_time.err || exit 1
cat $O/fwd_time.json
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o fwd -- python scripts/fwd_timeline.py --reps 2 --no-graph > $O/trace_run.log 2>&1 || exit 1
python scripts/fwd_timeline_read.py $(ls $O/tr/*/fwd_kernel_trace.csv $O/tr/fwd_kernel_trace.csv 2>/dev/null | head -1) 2 > $O/timeline.txt
head -8 $O/timeline.txt
