#!/bin/bash
# Two ranks sharing one MI355X (gloo control plane; the one-shot and two-shot peer-memory
# kernels need no RCCL): the launch-bound floor of the multi-rank steps (tiny problem) and a
# mid-size run.  Both ranks' kernels share the GPU, so GPU-bound times are ~2x a real rank's.
set -u
mkdir -p gpurun_out
export MULTIGRAD_DEVICE_COMM=0 HSA_ENABLE_IPC_MODE_LEGACY=0 OMP_NUM_THREADS=1
for cfg in "8000 80000 400" "1000000 4000000 100"; do
  set -- $cfg
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 200)) bench.py --gpus 2 \
    --params $1 --halos $2 --steps $3 --warmup 10 ${EXTRA:-} > gpurun_out/b2r_$1.log 2>&1 || exit $?
  grep '^{' gpurun_out/b2r_$1.log | python -c "
import json,sys
d=json.loads(sys.stdin.read())
print('params=$1 halos=$2 hashed ms/step', d['ms_per_step'], 'owner ms/step', d['owner_ms_per_step'], d['config']['grad_collective'][:40], d['config']['chunks'])"
done
