cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?; tail -3 gpurun_out/t_all.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u scripts/tune_wgrad.py gpurun_out/tune_wgrad.json > gpurun_out/tune_wgrad.log 2>&1 || exit $?
cat gpurun_out/tune_wgrad.log | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_bf16.log 2>&1 || exit $?
tail -c 1500 gpurun_out/bench_bf16.log
