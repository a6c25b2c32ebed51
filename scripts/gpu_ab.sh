# A/B bench of the in-tree library against ab/lib_prev.so on the same box (alternating runs)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?; tail -3 gpurun_out/t_all.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  STC_LIB_PATH=$PWD/ab/lib_prev.so timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_prev_$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_new_$i.log 2>&1 || exit $?
  for f in prev new; do echo "$f $i: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_${f}_$i.log)"; done
done
