#!/bin/bash
# bench.py's multi-rank path with two ranks sharing one MI355X (hashed + owner placements,
# both schedules' autotune incl. the chunk-count candidates): full JSON lines kept.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2
mkdir -p "$O"
cd "$R"
export MULTIGRAD_DEVICE_COMM=0 HSA_ENABLE_IPC_MODE_LEGACY=0 OMP_NUM_THREADS=1
for cfg in "1000000 4000000 60" "10000000 33554432 20"; do
  set -- $cfg
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 200)) bench.py --gpus 2 \
    --params $1 --halos $2 --steps $3 --warmup 5 > "$O/b2r_$1.log" 2>&1 || { tail -20 "$O/b2r_$1.log"; exit 1; }
  grep '^{' "$O/b2r_$1.log" | cut -c1-300
done
