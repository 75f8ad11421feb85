#!/bin/bash
# Hashed two-shot step with two ranks on ONE GPU at the 2-GPU proxy size (1e7 params,
# 1.34e8 halos over 2 ranks): 1 chunk on the compute stream vs C chunks whose exchanges run
# on a side stream (capped grid).  Both ranks share the GPU, so this measures the overhead
# of the overlapped schedule, not its gain (the exchange is local memory here).
set -u
mkdir -p gpurun_out
export MULTIGRAD_DEVICE_COMM=0 HSA_ENABLE_IPC_MODE_LEGACY=0 OMP_NUM_THREADS=1
run() {  # label env...
  local label=$1; shift
  env "$@" timeout -k 10 300 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 200)) \
    bench.py --gpus 2 --params ${P:-10000000} --halos ${H:-134217728} --steps ${K:-30} --warmup 5 \
    --placement hashed --no-count-launches > gpurun_out/b2o_$label.log 2>&1 || return $?
  grep '^{' gpurun_out/b2o_$label.log | python -c "
import json,sys
d=json.loads(sys.stdin.read())
print('$label hashed ms/step', d['ms_per_step'], 'chunks', d['config']['chunks'])"
}
run same1 MULTIGRAD_X=0 || exit $?
run side4 MULTIGRAD_CHUNKS=4 MULTIGRAD_TWOSHOT_SIDE_STREAM=1 || exit $?
run side2 MULTIGRAD_CHUNKS=2 MULTIGRAD_TWOSHOT_SIDE_STREAM=1 || exit $?
run side4_b1024 MULTIGRAD_CHUNKS=4 MULTIGRAD_TWOSHOT_SIDE_STREAM=1 MULTIGRAD_TWOSHOT_BLOCKS=1024 || exit $?
run same4 MULTIGRAD_CHUNKS=4 || exit $?
