#!/bin/bash
# A/B: priority by remaining fraction (in-tree, MG_FWD_PRIO=1) vs longest-remaining-first
# (variants/prio2, MG_FWD_PRIO=2), static lists, forward kernel at 1/8 and 1/4 shard sizes.
set -u
mkdir -p gpurun_out
out=gpurun_out/ab_prio2.log
: > $out
kb() { MULTIGRAD_LPT=static timeout -k 10 300 python tools/kernel_bench.py "$@" --iters 50 >> $out 2>&1; }
for rep in 1 2; do
  kb --tag p8_frac_$rep --params 1250000 --halos 16777216 || exit $?
  kb --tag p8_lrf_$rep --so variants/prio2/_C.so --params 1250000 --halos 16777216 || exit $?
  kb --tag p4_frac_$rep --params 2500000 --halos 33554432 || exit $?
  kb --tag p4_lrf_$rep --so variants/prio2/_C.so --params 2500000 --halos 33554432 || exit $?
done
grep -o '"tag": "[^"]*"\|"fwd_internal_us": [0-9.]*' $out | paste - -
