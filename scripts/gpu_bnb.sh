#!/bin/bash
# Fused BN-backward epilogue: the shipped library against builds with 8 / 16 rows of BN-input loads in flight.
set -o pipefail
O=gpurun_out/${1:-r04_bnb}
mkdir -p $O
timeout -k 10 200 python -u scripts/ab_bnb.py > $O/shipped.log 2>&1 || exit 1
for v in bnbg8 bnbg16; do STC_LIB_PATH=ab/lib_$v.so timeout -k 10 200 python -u scripts/ab_bnb.py > $O/$v.log 2>&1 || exit 1; done
for v in shipped bnbg8 bnbg16; do echo "== $v"; grep us $O/$v.log; done
