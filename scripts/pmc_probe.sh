#!/bin/bash
# PMC passes on one conv problem: pmc_probe.sh <tag> <pmc_kernel.py args...>
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python scripts/pmc_kernel.py "$@" > $OUT/run.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o k -- python scripts/pmc_kernel.py "$@" > $OUT/trace.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/p1 -o k -- python scripts/pmc_kernel.py "$@" > $OUT/p1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d $OUT/p2 -o k -- python scripts/pmc_kernel.py "$@" > $OUT/p2.log 2>&1 || exit $?
cat $OUT/run.log
