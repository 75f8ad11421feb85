#!/bin/bash
# Round-end rehearsal on one GPU: GPU tests, smoke, default bench, 2-rank bench flow.
set -eu
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
grep '^{' gpurun_out/bench.log
bash tools/archive/bench_2rank_gloo.sh
