#!/bin/bash
# Round 5: multi-dot rewrite -- kernel test, L-BFGS tests, config-4 benchmark + rocprof.
set -o pipefail
O=gpurun_out/r5_lbfgs2
mkdir -p $O
export MULTIGRAD_PROGRESS=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_kernels_gpu.py::test_multi_dot_and_lincomb_kernels" \
  "tests/test_kernels_gpu.py::test_device_lbfgs_population_engine" \
  tests/test_lbfgs_comm_gpu.py tests/test_lbfgsb_gpu.py > $O/pytest.log 2>&1 || { tail -50 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u benchmarks/configs.py --which lbfgs lbfgsb > $O/configs.log 2>&1 || { tail -30 $O/configs.log; exit 1; }
cat $O/configs.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- \
  python -u $GRAFT_REPO_ROOT/benchmarks/configs.py --which lbfgs > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
ls $GRAFT_REPO_ROOT/$O/prof
