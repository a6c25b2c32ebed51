set -o pipefail
mkdir -p gpurun_out/adam
for v in 0 0 2 2; do
  STC_ADAM_VARIANT=$v timeout -k 10 200 python -u scripts/ab_adam_variant.py hash 2>&1 | grep -E "state hash|Error" || exit 1
done
