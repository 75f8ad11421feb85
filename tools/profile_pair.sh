#!/bin/bash
# Kernel-trace profiles of the headline bench and of the per-rank 8-GPU proxy.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
for cfg in "full|--steps 30 --warmup 5 --no-graph" "proxy|--params 1250000 --halos 16777216 --steps 100 --warmup 10 --no-graph"; do
  name=${cfg%%|*}; args=${cfg#*|}
  mkdir -p "$R/gpurun_out/prof_$name"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$name" -o bench -- python3 "$R/bench.py" $args > "$R/gpurun_out/prof_$name.log" 2>&1 || exit $?
done
echo done
