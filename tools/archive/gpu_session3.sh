#!/bin/bash
# Round-3 session check on one MI355X: the full GPU test suite, then the hashed per-rank
# proxy kernel stats at 1/8, 1/4, 1/2 of the halos (tiles layout).  Stops at the first
# failing step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
LAYOUT=tiles DIVS="8 4 2" bash tools/profile_hashed_proxy.sh
