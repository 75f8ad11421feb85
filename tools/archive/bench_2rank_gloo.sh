#!/bin/bash
# Rehearsal of the multi-rank bench flow on ONE GPU: 2 ranks share cuda:0 and stage their
# collectives through gloo (RCCL refuses two ranks on one device).  Validates rendezvous,
# data placement, the owner / ZeRO schedules, timing and the JSON line -- not RCCL speed.
set -eu
mkdir -p gpurun_out
for pl in owner hashed; do
  MULTIGRAD_DEVICE_COMM=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) \
    bench.py --gpus 2 --steps 10 --warmup 2 --placement $pl --halos 16777216 \
    > gpurun_out/bench2_$pl.log 2>&1
  grep '^{' gpurun_out/bench2_$pl.log
done
