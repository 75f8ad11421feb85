set -eu
mkdir -p gpurun_out
for rep in 1 2; do
for g in "" "--no-graph"; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 $g > gpurun_out/gf.log 2>&1
  echo "full $g: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/gf.log)"
  timeout -k 10 200 python bench.py --params 1250000 --halos 16777216 --steps 1000 --warmup 50 $g > gpurun_out/gp.log 2>&1
  echo "proxy $g: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/gp.log)"
done
done
