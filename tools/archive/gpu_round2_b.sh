#!/bin/bash
# New GPU tests (RCCL group, 1/8-shard schedules, L-BFGS-B), smoke with build stamp,
# L-BFGS / L-BFGS-B throughput at 1e7 parameters.
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_rccl_gpu.py tests/test_kernels_gpu.py tests/test_lbfgsb_gpu.py \
  -x -v -k "rccl or eighth or group or lbfgsb" --timeout 200 --timeout-method thread > gpurun_out/pytest_new.log 2>&1
rc=$?; tail -12 gpurun_out/pytest_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
timeout -k 10 400 python benchmarks/configs.py --which lbfgs lbfgsb > gpurun_out/lbfgs_bench.log 2>&1
rc=$?; cat gpurun_out/lbfgs_bench.log | grep '^{'; exit $rc
