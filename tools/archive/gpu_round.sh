#!/bin/bash
# One GPU session: tests, smoke, short bench. Stops at the first crash/timeout.
# Usage: bash tools/archive/gpu_round.sh [bench args...]
set -u
mkdir -p gpurun_out
ok_or_fail() {  # continue on pass (0) or ordinary test failure (1); stop on anything else
  local rc=$1 name=$2
  echo "[$name] rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "[$name] crashed/timed out -- stopping"; exit "$rc"; fi
}
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
ok_or_fail $? pytest_gpu
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
ok_or_fail $? smoke
tail -3 gpurun_out/smoke.log
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench.log 2>&1
ok_or_fail $? bench
tail -3 gpurun_out/bench.log
