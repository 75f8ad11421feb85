#!/bin/bash
# Hashed two-shot step with two ranks on one GPU: launch floor (tiny) and mid size, for
# graph / eager / chunks + side stream.
set -u
mkdir -p gpurun_out
export MULTIGRAD_DEVICE_COMM=0 HSA_ENABLE_IPC_MODE_LEGACY=0 OMP_NUM_THREADS=1
run() {  # label env...
  local label=$1; shift
  local envs=("$@")
  for cfg in "8000 80000 400" "1000000 4000000 100"; do
    read -r P H K <<< "$cfg"
    env "${envs[@]}" timeout -k 10 240 python -m torch.distributed.run \
      --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 200)) \
      bench.py --gpus 2 --params $P --halos $H --steps $K --warmup 10 \
      > gpurun_out/b2v.log 2>&1 || return $?
    grep '^{' gpurun_out/b2v.log | python -c "
import json,sys
d=json.loads(sys.stdin.read())
print('$label params=$P hashed ms/step', d['ms_per_step'], 'graph', d['config']['graph'], 'owner ms/step', d['owner_ms_per_step'])"
  done
}
run default MULTIGRAD_X=0
run eager MULTIGRAD_GRAPH=0
run chunks4_side MULTIGRAD_GRAPH=0 MULTIGRAD_CHUNKS=4 MULTIGRAD_TWOSHOT_SIDE_STREAM=1
