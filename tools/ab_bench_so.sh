#!/bin/bash
# A/B the headline bench between the in-tree _C.so and variants/<name>/_C.so on the same
# box, alternating runs: bash tools/ab_bench_so.sh <name> [bench args...]
set -u
name=$1; shift
mkdir -p gpurun_out
cp multigrad_amd/_C.so /tmp/_C_base.so
for rep in 1 2 3; do
  for v in base $name; do
    if [ $v = base ]; then cp /tmp/_C_base.so multigrad_amd/_C.so; else cp variants/$v/_C.so multigrad_amd/_C.so; fi
    ms=$(timeout -k 10 200 python3 bench.py "$@" 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || exit 1
    echo "$v $ms"
  done
done
cp /tmp/_C_base.so multigrad_amd/_C.so
