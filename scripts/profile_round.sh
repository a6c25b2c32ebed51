#!/bin/bash
# Round profile on the GPU box: bench JSON, rocprofv3 kernel-trace stats of the same bench command,
# and two PMC passes (FETCH_SIZE, WRITE_SIZE) for per-launch HBM traffic.  Output: gpurun_out/$1/
set -o pipefail
OUT=gpurun_out/${1:-r01_bf16}
ARGS=${BENCH_ARGS:---steps 5 --warmup 2 --no-cpu-baseline}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py $ARGS > $OUT/bench.log 2>&1 || exit $?
tail -1 $OUT/bench.log > $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python bench.py $ARGS > $OUT/rocprof.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o bench -- python bench.py $ARGS > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o bench -- python bench.py $ARGS > $OUT/pmc_write.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_mfma -o bench -- python bench.py $ARGS > $OUT/pmc_mfma.log 2>&1 || exit $?
python scripts/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_traffic.json $OUT/pmc_mfma > $OUT/pmc_traffic.txt
python scripts/prof_summary.py $OUT/trace/bench_kernel_stats.csv 40 > $OUT/summary.txt
echo "$ARGS" > $OUT/command.txt
cat $OUT/bench.json | cut -c1-300
