#!/bin/bash
# stc_deep_conv PMC passes (one launch set of scripts/deep_tune.py --phases --only $1): L2 hits / misses, HBM fetch
set -o pipefail
O=gpurun_out/deep_pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o run -- python3 $R/scripts/deep_tune.py --phases --only ${1:-e5} > $R/$O/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/$O/p1 -o run -- python3 $R/scripts/deep_tune.py --phases --only ${1:-e5} > $R/$O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $R/$O/p2 -o run -- python3 $R/scripts/deep_tune.py --phases --only ${1:-e5} > $R/$O/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE -d $R/$O/p3 -o run -- python3 $R/scripts/deep_tune.py --phases --only ${1:-e5} > $R/$O/p3.log 2>&1 || exit 1
echo done
