# Diagnostic timing of the halo_wide kernels (scripts/ab_wide.py) under diagnostic libraries in diaglib/
# (built with STC_EXP_* switches; outputs meaningless, times only).  Usage: bash scripts/diag_wide.sh LOG
set -e
LOG=${1:-gpurun_out/diag.log}
export AB_SHAPES=${AB_SHAPES:-0,1,3} AB_CANDS=${AB_CANDS:-legacy,w2_4x128x64,w4_ld4}
for v in main ${VARIANTS:-noadma nobdma nodma}; do
  if [ $v = main ]; then unset STC_LIB_PATH; else export STC_LIB_PATH=$PWD/diaglib/lib_$v.so; fi
  echo "=== $v" >> $LOG
  timeout -k 10 200 python -u scripts/ab_wide.py --quick >> $LOG 2>&1
done
