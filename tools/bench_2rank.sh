#!/bin/bash
# Two ranks sharing one GPU (gloo for the device collectives: RCCL refuses two ranks on one
# GPU) run bench.py's hashed placement; the JSON's config.autotune block records every
# exchange schedule the setup timed (serial two-shot, side stream, fused exchange, RCCL)
#   bash tools/bench_2rank.sh [bench args...]   -> stdout: the bench JSON line
set -u
port=$(python3 -c "import socket;s=socket.socket();s.bind(('127.0.0.1',0));print(s.getsockname()[1])")
HSA_ENABLE_IPC_MODE_LEGACY=0 MULTIGRAD_DEVICE_COMM=0 OMP_NUM_THREADS=1 \
  timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
  --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --placement hashed "$@"
