#!/bin/bash
# Streaming Cin = 8 kernels: strip height 8 (shipped) against 4 and 16 (tuning builds), scripts/ab_stem.py each.
set -o pipefail
O=gpurun_out/${1:-r04_stemrb}
mkdir -p $O
timeout -k 10 200 python -u scripts/ab_stem.py > $O/rb8.log 2>&1 || exit 1
for v in rb4 rb16; do STC_LIB_PATH=ab/lib_$v.so timeout -k 10 200 python -u scripts/ab_stem.py > $O/$v.log 2>&1 || exit 1; done
for v in rb8 rb4 rb16; do echo "== $v"; grep us $O/$v.log; done
