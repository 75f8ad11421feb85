#!/bin/bash
# A/B the kernel variants under variants/* against the in-tree _C.so (one process each).
set -u
mkdir -p gpurun_out
out=gpurun_out/ab.log
: > $out
timeout -k 10 300 python tools/kernel_bench.py --tag base "$@" >> $out 2>&1 || exit $?
for d in variants/*/; do
  n=$(basename $d)
  timeout -k 10 300 python tools/kernel_bench.py --tag $n --so $d/_C.so "$@" >> $out 2>&1 || exit $?
done
grep tag $out
