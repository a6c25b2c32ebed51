#!/bin/bash
# Diagnostic variants of the library for scripts/diag_gemm.py (what the DMA, the MFMAs and the
# epilogue each cost in the bf16 conv / weight-gradient tiles); outputs under ab/ (git-ignored).
set -e
mkdir -p "$(dirname "$0")/../ab"
cd "$(dirname "$0")/../shadow-removal-istd_amd/csrc"
for v in nodma:-DSTC_EXP_NODMA=1 nomfma:-DSTC_EXP_NOMFMA=1 noepi:-DSTC_EXP_NOEPI=1; do
  n=${v%%:*}; f=${v#*:}
  make -j8 OUT=../../ab/lib_$n.so BUILD=../../build/csrc_$n EXTRA="$f" > /dev/null
done
