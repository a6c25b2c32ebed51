#!/bin/bash
# GPU box: (1) the split reduction of the new library bit-identical to ab/lib_base.so, (2) wgrad/conv
# timings (scripts/diag_gemm.py), (3) PMC passes on the dominant weight-gradient kernel.
set -o pipefail
O=gpurun_out/wg
mkdir -p $O
export TMPDIR=/tmp
STC_LIB_PATH=$PWD/ab/lib_base.so timeout -k 10 120 python -u scripts/wgrad_dump.py $O/base.npz > $O/dump.log 2>&1 || exit 1
timeout -k 10 120 python -u scripts/wgrad_dump.py $O/new.npz >> $O/dump.log 2>&1 || exit 1
python scripts/wgrad_dump.py --compare $O/base.npz $O/new.npz >> $O/dump.log 2>&1; echo "compare rc=$?" >> $O/dump.log
timeout -k 10 240 python -u scripts/diag_gemm.py > $O/diag.log 2>&1 || exit 1
A="32 2 64 64 128 128 128 64 50"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d $O/p1 -o k -- python scripts/pmc_wgrad.py $A > $O/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/p2 -o k -- python scripts/pmc_wgrad.py $A > $O/p2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv -d $O/p3 -o k -- python scripts/pmc_wgrad.py $A > $O/p3.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum --output-format csv -d $O/p4 -o k -- python scripts/pmc_wgrad.py $A > $O/p4.log 2>&1 || exit 1
cat $O/dump.log $O/diag.log
for p in p1 p2 p3 p4; do python scripts/pmc_read.py $O/$p wgrad_bf16_kernel; done
