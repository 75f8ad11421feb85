for fe in 1 0; do
  MULTIGRAD_FUSED_EPILOGUE=$fe MULTIGRAD_DEVICE_COMM=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus 2 --steps 100 --warmup 10 --halos 16777216 --params 2500000 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('epilogue=$fe', d['ms_per_step'], d['config']['sumstat_allreduce'])"
done
