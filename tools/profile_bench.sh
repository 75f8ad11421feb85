#!/bin/bash
# Kernel-trace profile of the 1-GPU bench (no PMC counters in this run).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p "$R/gpurun_out/prof"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- python3 "$R/bench.py" "$@" > "$R/gpurun_out/prof_bench.log" 2>&1
rc=$?
echo "rocprof rc=$rc"
find "$R/gpurun_out/prof" -name '*stats*' | head
exit $rc
