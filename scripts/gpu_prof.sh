cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/profile_round.sh r01_bf16c || exit $?
timeout -k 10 300 python scripts/step_breakdown.py > gpurun_out/r01_bf16c/step_breakdown.txt 2>&1 || exit $?
tail -2 gpurun_out/r01_bf16c/step_breakdown.txt
head -30 gpurun_out/r01_bf16c/summary.txt
