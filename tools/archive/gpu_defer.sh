#!/bin/bash
# Deferred per-edge fallback of the residual lanes forwards (LMODE): kernel + engine GPU
# tests, then the headline bench alternating the in-tree build with variants/defer0.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/defer
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_generic_engine_gpu.py -x -v --timeout 120 \
  --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
bash tools/archive/ab_script_so.sh defer0 bench.py --steps 50 --warmup 5 --no-count-launches > "$O/ab.log" 2>&1
rc=$?; cut -c1-160 "$O/ab.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/dbg/eager_then_replay.py > "$O/eager_then_replay.log" 2>&1
rc=$?; grep -v amdgpu.ids "$O/eager_then_replay.log"; exit $rc
