#!/bin/bash
# bench.py launch modes: the default (auto probe) three times, then eager and graph once each.
set -o pipefail
O=gpurun_out/${1:-launch}
mkdir -p $O
export TMPDIR=/tmp
for run in auto1 eager auto2 graph auto3; do
  case $run in auto*) a="";; eager) a="--launch eager";; graph) a="--launch graph";; esac
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras $a > $O/$run.json 2> $O/$run.err || { tail -5 $O/$run.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$run.json'));print('$run', d['value'], d['ms_per_step'], d['config']['step_launch'], d.get('launch_probe'))"
done
