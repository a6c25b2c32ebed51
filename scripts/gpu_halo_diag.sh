#!/bin/bash
# What bounds the halo conv kernels: the per-shape A/B (scripts/ab_conv.py) under the shipped library and the
# diagnostic builds without the LDS-DMA (STC_EXP_NODMA), without the MFMAs (NOMFMA) and without the epilogue (NOEPI).
set -o pipefail
O=gpurun_out/${1:-r04_halodiag}
mkdir -p $O
timeout -k 10 200 python -u scripts/ab_conv.py > $O/shipped.log 2>&1 || exit 1
for v in nodma nomfma noepi; do
  STC_LIB_PATH=ab/lib_$v.so timeout -k 10 200 python -u scripts/ab_conv.py > $O/$v.log 2>&1 || exit 1
done
for v in shipped nodma nomfma noepi; do echo "== $v"; grep -i "halo\|us" $O/$v.log | head -16; done
