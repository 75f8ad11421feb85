#!/bin/bash
# Per-rank proxy steps for the 2- and 4-GPU owner shards (1/2, 1/4 of the headline):
# static LPT lists with priority feedback vs dynamic work queues.
set -eu
mkdir -p gpurun_out
for frac in 2 4; do
  P=$((10000000 / frac)); H=$((134217728 / frac))
  for mode in static dynamic; do
    MULTIGRAD_LPT=$mode timeout -k 10 300 python bench.py --params $P --halos $H --steps 100 \
      --warmup 10 > gpurun_out/lpt_${frac}_$mode.log 2>&1
    grep -o '"ms_per_step": [0-9.]*' gpurun_out/lpt_${frac}_$mode.log | sed "s/^/1\/$frac $mode /"
  done
done
