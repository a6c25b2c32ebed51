#!/bin/bash
# Three default bench lines and the train_steps.py timing in one call (box-to-box / run-to-run spread).
set -o pipefail
O=gpurun_out/${1:-bench3}
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench$i.json 2> $O/bench$i.err || exit 1
  python -c "import json;d=json.load(open('$O/bench$i.json'));print('bench', d['value'], d['ms_per_step'], d['roofline']['g1g2_forward_frac'])"
  timeout -k 10 200 python scripts/train_steps.py --steps 20 --warmup 3 > $O/ts$i.txt 2>&1 || exit 1
  echo "train_steps $(tail -1 $O/ts$i.txt | cut -d' ' -f1)"
done
