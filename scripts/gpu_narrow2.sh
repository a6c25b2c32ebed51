#!/bin/bash
# Streaming narrow ConvT: ring-depth variants and the diagnostic builds (no DMA / no MFMA / no epilogue).
set -o pipefail
O=gpurun_out/${1:-r04_narrow2}
mkdir -p $O
timeout -k 10 120 python -u scripts/ab_narrow.py > $O/ab.log 2>&1 || exit 1
for v in nodma nomfma noepi; do
  echo "== $v" >> $O/ab.log
  STC_LIB_PATH=ab/lib_$v.so timeout -k 10 120 python -u scripts/ab_narrow.py >> $O/ab.log 2>&1 || exit 1
done
cat $O/ab.log
