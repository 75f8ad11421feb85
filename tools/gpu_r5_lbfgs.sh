#!/bin/bash
# Round 5: device-collective L-BFGS -- GPU tests (2/4/8 processes on one GPU), then the
# BASELINE config-4 benchmark at 1e7 parameters with a rocprofv3 kernel summary.
set -o pipefail
O=gpurun_out/r5_lbfgs
mkdir -p $O
export MULTIGRAD_PROGRESS=0
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_lbfgs_comm_gpu.py tests/test_multirank_gpu.py tests/test_lbfgsb_gpu.py \
  "tests/test_kernels_gpu.py::test_device_lbfgs_population_engine" > $O/pytest.log 2>&1 || { tail -50 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u benchmarks/configs.py --which lbfgs lbfgsb > $O/configs.log 2>&1 || { tail -30 $O/configs.log; exit 1; }
cat $O/configs.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- \
  python -u $GRAFT_REPO_ROOT/benchmarks/configs.py --which lbfgs > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" | head -3
