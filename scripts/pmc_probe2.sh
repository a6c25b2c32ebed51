#!/bin/bash
# Memory-side PMC passes on one conv problem: pmc_probe2.sh <tag> <pmc_kernel.py args...>
# L2 hit/miss and EA reads, TCP->TCC read latency, and the SQ wait/issue split.
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/pmc2_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python scripts/pmc_kernel.py "$@" > $OUT/run.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv -d $OUT/p1 -o k -- python scripts/pmc_kernel.py "$@" > $OUT/p1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum --output-format csv -d $OUT/p2 -o k -- python scripts/pmc_kernel.py "$@" > $OUT/p2.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d $OUT/p3 -o k -- python scripts/pmc_kernel.py "$@" > $OUT/p3.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d $OUT/p4 -o k -- python scripts/pmc_kernel.py "$@" > $OUT/p4.log 2>&1 || exit $?
cat $OUT/run.log
for p in p1 p2 p3 p4; do python scripts/pmc_read.py $OUT/$p igemm_bf16; done
