#!/bin/bash
# After making the priority-feedback static schedule the default: GPU tests, the 1-GPU
# bench and the per-rank proxy of the 8-GPU owner step, static (default) vs dynamic.
set -eu
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
tail -1 gpurun_out/pytest_gpu.log
for mode in auto dynamic; do
  MULTIGRAD_LPT=$mode timeout -k 10 300 python bench.py > gpurun_out/bench_$mode.log 2>&1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_$mode.log | sed "s/^/full $mode /"
  MULTIGRAD_LPT=$mode timeout -k 10 300 python bench.py --params 1250000 --halos 16777216 \
    --steps 200 --warmup 20 > gpurun_out/proxy_$mode.log 2>&1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/proxy_$mode.log | sed "s/^/proxy $mode /"
done
