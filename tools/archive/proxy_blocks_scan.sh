#!/bin/bash
# Per-rank proxy step (1/8 of the headline) against the forward grid cap.
set -eu
mkdir -p gpurun_out
for nb in 1024 960 896 814 768 704 651; do
  MULTIGRAD_FWD_MAX_BLOCKS=$nb timeout -k 10 300 python bench.py --params 1250000 --halos 16777216 \
    --steps 200 --warmup 20 > gpurun_out/proxy_nb$nb.log 2>&1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/proxy_nb$nb.log | sed "s/^/blocks $nb /"
done
