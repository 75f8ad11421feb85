set -eu
mkdir -p gpurun_out
for g in "" "--no-graph"; do
  timeout -k 10 200 python bench.py --params 1250000 --halos 16777216 --steps 300 --warmup 20 $g > gpurun_out/gp.log 2>&1
  echo "proxy $g: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/gp.log)"
done
for g in 0 1; do
  MULTIGRAD_GRAPH=$g MULTIGRAD_DEVICE_COMM=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) \
    bench.py --gpus 2 --steps 200 --warmup 10 --halos 16777216 > gpurun_out/g2_$g.log 2>&1
  echo "2rank graph=$g: $(grep -o '"ms_per_step": [0-9.]*\|"graph": [a-z]*\|"loss_last": [0-9.e-]*' gpurun_out/g2_$g.log | tr '\n' ' ')"
done
