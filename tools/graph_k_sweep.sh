#!/bin/bash
# Block-graph length sweep (owner-shard proxy and the fused 1-GPU step): ms/step of eager
# launches and of K-step graph replays for K = 1..32, and K = 16 with kernel arguments forced
# into device memory.   bash tools/graph_k_sweep.sh [ROWS]   -> gpurun_out/gk/
set -u
rows=${1:-owner_proxy,fused}
out=gpurun_out/gk
mkdir -p $out
for K in 2 4 8 16 32; do
  timeout -k 10 400 python3 benchmarks/graph_modes.py --rows $rows --modes eager,graph-K --K $K \
    --repeats 2 --steps 256 > $out/K$K.log 2>&1 || { echo "K=$K failed"; exit 1; }
  echo "K=$K $(grep '^{' $out/K$K.log | tr '\n' ' ')"
done
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 400 python3 benchmarks/graph_modes.py --rows $rows \
  --modes eager,graph-K --K 16 --repeats 2 --steps 256 > $out/K16_devkernarg.log 2>&1 \
  || { echo "devkernarg failed"; exit 1; }
echo "K=16 HIP_FORCE_DEV_KERNARG=1 $(grep '^{' $out/K16_devkernarg.log | tr '\n' ' ')"
