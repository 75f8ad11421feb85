#!/bin/bash
# Euler-Maclaurin forward check on one MI355X: kernel numerics tests, then the headline bench
# alternating the in-tree build with variants/em0 (MG_FWD_EM=0, the per-edge tail path), then
# a kernel-trace profile of the in-tree bench.  Stops at the first failing step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/em
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 \
  --timeout-method thread > "$O/pytest_kernels.log" 2>&1
rc=$?; tail -5 "$O/pytest_kernels.log"; [ $rc -eq 0 ] || exit $rc
bash tools/archive/ab_script_so.sh em0 bench.py --steps 50 --warmup 5 --no-count-launches > "$O/ab.log" 2>&1
rc=$?; cut -c1-260 "$O/ab.log"; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o bench \
  -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-count-launches > "$O/prof_bench.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
