#!/bin/bash
# Round 5: full-size (1e7 floats) peer-memory exchanges with 4 and 8 ranks sharing one GPU
# (exchange grids capped to 1/ranks-per-GPU of the GPU), hashed placement; then the device
# L-BFGS (BASELINE config 4) at 1e7 on 4 ranks.  Rehearsals: N processes time-slice one GPU,
# the step rates are not measurements.
set -o pipefail
O=gpurun_out/r5_multirank
mkdir -p $O
for n in 4 8; do
  NPROC=$n PLACEMENT=hashed timeout -k 10 900 bash tools/bench_2rank.sh --steps 20 --warmup 5 --no-count-launches \
    > $O/bench_n$n.json 2> $O/bench_n$n.err || { tail -30 $O/bench_n$n.err; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('$O/bench_n$n.json') if l.startswith('{')][-1])  # gloo prints to stdout too
print($n, d['value'], d['loss_last'], d['config']['grad_collective'])
print(json.dumps(d['peer_memory_selftest'])[:600])
print(json.dumps(d['config']['autotune'])[:800])"
done
port=$(python3 -c "import socket;s=socket.socket();s.bind(('127.0.0.1',0));print(s.getsockname()[1])")
HSA_ENABLE_IPC_MODE_LEGACY=0 MULTIGRAD_DEVICE_COMM=0 OMP_NUM_THREADS=1 timeout -k 10 900 \
  python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
  --master-port $port benchmarks/configs.py --which lbfgs > $O/lbfgs_n4.log 2>&1 || { tail -30 $O/lbfgs_n4.log; exit 1; }
grep config $O/lbfgs_n4.log
