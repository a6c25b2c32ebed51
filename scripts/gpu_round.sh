#!/bin/bash
# One GPU-box session: GPU tests, smoke, a short bench.  Every GPU step has its own time
# limit; the script stops at the first abort/fault/timeout (exit code >= 2 from a step),
# and continues past ordinary test failures (exit code 1) so the bench still reports.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 30 "gpurun_out/$name.log"
  if [ $rc -ge 2 ] && [ $rc -ne 5 ]; then echo "== stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = quick ]; then  # selected test files (TESTS=...), then the default bench line
  step pytest_sel 600 python -u -m pytest ${TESTS:-tests/test_gpu_configs.py} -m gpu -v -rf -s --timeout 300 --timeout-method thread
  step bench 600 python bench.py
fi
if [ "$MODE" = prof ] || [ "$MODE" = all_prof ]; then
  export TMPDIR=/tmp
  step rocprof 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
       -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS}
fi
if [ "$MODE" = pmc ] || [ "$MODE" = all_prof ]; then
  export TMPDIR=/tmp
  PDT=${PMC_DTYPE:-bf16}
  step pmc_fetch 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o g \
       -- python scripts/g1g2_fwd.py --dtype $PDT
  step pmc_write 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o g \
       -- python scripts/g1g2_fwd.py --dtype $PDT
  python scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_traffic.json
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ] || [ "$MODE" = all_prof ]; then
  step bench 600 python bench.py --steps 5 --warmup 2
  step bench_bf16 600 python bench.py --steps 5 --warmup 2 --dtype bf16 --no-cpu-baseline
fi
