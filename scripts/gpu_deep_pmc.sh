#!/bin/bash
# stc_deep_conv PMC passes over scripts/deep_tune.py --phases --only $1 (one pass per counter group)
set -o pipefail
O=gpurun_out/deep_pmc_${1:-e5}
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVES" \
           "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_FLAT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_SENDMSG"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $R/$O/p$i -o run -- python3 $R/scripts/deep_tune.py --phases --only ${1:-e5} > $R/$O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/$O/p$i.log; }
done
echo done
