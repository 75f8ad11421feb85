#!/bin/bash
# Per-rank proxy of the 8-GPU HASHED step on one GPU: all 1e7 parameters, 1/8 of the halos
# (every population present at ~3.4 halos/rank), kernel stats with the update pipelined
# (default) and unpipelined (separate forward / VJP+Adam kernels).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p "$R/gpurun_out/hprox"
cd /tmp
for pl in 1 0; do
  MULTIGRAD_PIPELINE=$pl timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/hprox/p$pl" -o k -- python3 "$R/bench.py" --params 10000000 --halos 16777216 \
    --steps 40 --warmup 5 > "$R/gpurun_out/hprox/bench_p$pl.log" 2>&1 || exit $?
  grep '^{' "$R/gpurun_out/hprox/bench_p$pl.log" | cut -c1-200
done
find "$R/gpurun_out/hprox" -name '*kernel_stats.csv'
