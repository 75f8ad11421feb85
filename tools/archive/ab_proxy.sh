#!/bin/bash
# A/B the variants under variants/* at the per-rank proxy size (1/8 of the headline).
set -u
mkdir -p gpurun_out
out=gpurun_out/ab_proxy.log
: > $out
timeout -k 10 300 python tools/kernel_bench.py --tag base --params 1250000 --halos 16777216 --iters 50 >> $out 2>&1 || exit $?
MULTIGRAD_LPT=0 timeout -k 10 300 python tools/kernel_bench.py --tag base_nolpt --params 1250000 --halos 16777216 --iters 50 >> $out 2>&1 || exit $?
for d in variants/*/; do
  n=$(basename $d)
  timeout -k 10 300 python tools/kernel_bench.py --tag $n --so $d/_C.so --params 1250000 --halos 16777216 --iters 50 >> $out 2>&1 || exit $?
done
grep tag $out
