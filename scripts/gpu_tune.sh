cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_igemm_bf16.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_bf16.log 2>&1; rc=$?; tail -2 gpurun_out/t_bf16.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u scripts/tune_bf16.py gpurun_out/tune4.json > gpurun_out/tune4.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/tune4.log
