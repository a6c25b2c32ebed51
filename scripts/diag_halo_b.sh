#!/bin/bash
# Diagnostic variants of the library (under ab/, git-ignored): the halo kernels' B operand without LDS reads
# (fragments from registers), and without its LDS-DMA stream too -- for scripts/diag_gemm.py
set -e
mkdir -p "$(dirname "$0")/../ab"
cd "$(dirname "$0")/../shadow-removal-istd_amd/csrc"
for v in nobread:-DSTC_EXP_NOBREAD=1 nob:"-DSTC_EXP_NOBREAD=1 -DSTC_EXP_NOBDMA=1"; do
  n=${v%%:*}; f=${v#*:}
  make -j8 OUT=../../ab/lib_$n.so BUILD=../../build/csrc_$n EXTRA="$f" > /dev/null
done
