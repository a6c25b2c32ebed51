# GPU tests + two bench runs
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?; tail -3 gpurun_out/t_all.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$i.log 2>&1 || exit $?
  echo "bench $i: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_$i.log)"
done
