#!/bin/bash
# GPU box: scripts/diag_gemm.py with the shipped library and each diagnostic variant (ab/lib_*.so).
set -o pipefail
O=gpurun_out/diag
mkdir -p $O
: > $O/diag.log
for v in shipped ${VARIANTS:-nodma nomfma noepi}; do
  if [ $v = shipped ]; then L=""; else L=$PWD/ab/lib_$v.so; fi
  STC_LIB_PATH=$L timeout -k 10 240 python -u scripts/diag_gemm.py >> $O/diag.log 2>&1 || exit 1
done
cat $O/diag.log
