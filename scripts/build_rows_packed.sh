#!/bin/bash
# Diagnostic variant of the library whose logits-layer weight gradient keeps the compiler's packed
# v_pk_fma_f32 accumulations (STC_ROWS_PACKED); used only by scripts/rows_stress.py via STC_LIB_PATH.
set -e
cd "$(dirname "$0")/../shadow-removal-istd_amd/csrc"
make -j8 OUT=../../scripts/micro/libstcgan_hip_rows_packed.so BUILD=../../build/csrc_rows_packed EXTRA=-DSTC_ROWS_PACKED
