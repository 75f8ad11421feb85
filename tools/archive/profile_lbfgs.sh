#!/bin/bash
# Kernel-trace profile of the device L-BFGS config (1e7 params, 20 iterations).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p "$R/gpurun_out/prof_lbfgs"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_lbfgs" -o lbfgs -- python3 "$R/benchmarks/configs.py" --which lbfgs > "$R/gpurun_out/prof_lbfgs.log" 2>&1
echo rc=$?
