#!/bin/bash
# A/B on one box: the in-tree library against ab/lib_*.so variants, alternating processes (train step
# timing, scripts/train_steps.py) -- each run time-limited.
set -o pipefail
O=gpurun_out/r3
mkdir -p $O
: > $O/h_ab.log
for i in 1 2 3; do
  for v in base ${VARIANTS:-setprio}; do
    if [ $v = base ]; then L=""; else L=$PWD/ab/lib_$v.so; fi
    r=$(STC_LIB_PATH=$L timeout -k 10 200 python -u scripts/train_steps.py --steps 20 --warmup 5 2>&1 | grep "ms/step") || exit 1
    echo "$v $i: $r" >> $O/h_ab.log
  done
done
cat $O/h_ab.log
timeout -k 10 400 python -u scripts/train_steps.py --steps 20 --warmup 5 --repeat 8 --ab-attr overlap_optim=0,1 > $O/h_overlap.log 2>&1
tail -3 $O/h_overlap.log
