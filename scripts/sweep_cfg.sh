#!/bin/bash
# Time one bf16 conv problem under several forced tile configs: sweep_cfg.sh "<kind B gh gw cin cout>" "cfgs..."
PROB=$1; shift
for c in $@; do
  printf "cfg %-3s " $c
  timeout -k 5 60 python scripts/pmc_kernel.py $PROB $c 1 50 2>/dev/null | tail -1 || exit $?
done
