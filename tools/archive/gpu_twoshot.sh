#!/bin/bash
# Two-shot kernel tests (2 processes on one GPU) then the xgmi/engine GPU tests.
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_twoshot_gpu.py tests/test_xgmi_gpu.py -x -v \
  --timeout 200 --timeout-method thread > gpurun_out/pytest_twoshot.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_twoshot.log
exit $rc
