#!/bin/bash
# Round-2 GPU check: all GPU tests, smoke, 1-GPU bench (headline), bench refusing --gpus 2 on 1 GPU.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
grep '^{' gpurun_out/bench.log
timeout -k 10 120 python bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/bench_gpus2.log 2>&1
echo "bench --gpus 2 on one GPU exits with $? (expected 2)"
