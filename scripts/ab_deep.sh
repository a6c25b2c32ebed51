# stc_deep_conv phase stamps for a few forced plans (A/B of the tile / split choices)
set -o pipefail
mkdir -p gpurun_out/ab_deep
timeout -k 10 120 python -u scripts/deep_tune.py --phases --only e5,e6,d5 > gpurun_out/ab_deep/auto.log 2>&1 || exit 1
grep "==\|per-layer" gpurun_out/ab_deep/auto.log | cut -c1-220
for f in 2,8 3,8 2,16 0,8; do
  timeout -k 10 120 python -u scripts/deep_tune.py --phases --only e5 --force $f > gpurun_out/ab_deep/f$f.log 2>&1 || exit 1
  grep "==" gpurun_out/ab_deep/f$f.log | cut -c1-220
done
