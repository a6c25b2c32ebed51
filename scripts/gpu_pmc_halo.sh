#!/bin/bash
# PMC passes over single halo-conv problems (scripts/pmc_kernel.py, automatic plan): where the halo tile's waves wait.
# Output: gpurun_out/$1/
set -o pipefail
O=gpurun_out/${1:-r04_pmc_halo}
mkdir -p $O
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
for prob in "e2fwd 0 32 64 64 64 128" "d3fwd 2 32 32 32 512 128" "c4fwd 1 32 31 31 256 512"; do
  set -- $prob
  n=$1; shift
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/${n}_p$i -o run -- python scripts/pmc_kernel.py $@ -1 0 20 > $O/${n}_p$i.log 2>&1 || exit 1
  done
  echo "== $n" >> $O/pmc.txt
  python scripts/pmc_read.py $O/${n}_p1 halo_conv >> $O/pmc.txt
  python scripts/pmc_read.py $O/${n}_p2 halo_conv >> $O/pmc.txt
done
cat $O/pmc.txt
