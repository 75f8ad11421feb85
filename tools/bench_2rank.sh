#!/bin/bash
# NPROC (default 2) ranks sharing one GPU (gloo for the host-side collectives: RCCL refuses
# two ranks on one GPU) run bench.py, by default its hashed placement; the JSON's
# config.autotune block records every exchange schedule the setup timed (serial two-shot,
# side stream, fused exchange, RCCL/gloo)
#   [NPROC=n] bash tools/bench_2rank.sh [bench args...]   -> stdout: the bench JSON line
set -u
port=$(python3 -c "import socket;s=socket.socket();s.bind(('127.0.0.1',0));print(s.getsockname()[1])")
HSA_ENABLE_IPC_MODE_LEGACY=0 MULTIGRAD_DEVICE_COMM=0 OMP_NUM_THREADS=1 \
  timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=${NPROC:-2} \
  --master-addr 127.0.0.1 --master-port $port bench.py --gpus ${NPROC:-2} --placement ${PLACEMENT:-hashed} "$@"
