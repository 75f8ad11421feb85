#!/bin/bash
# Headline bench: the in-tree build against lanes-kernel variants (variants/<name>/_C.so),
# alternating on one box.  Usage: bash tools/archive/gpu_lanes_ab.sh name...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/lanes_ab
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fallback or headline or pipelined" > "$O/pytest.log" 2>&1
rc=$?; tail -1 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
for v in "$@"; do
  bash tools/archive/ab_script_so.sh $v bench.py --steps 50 --warmup 5 --no-count-launches > "$O/ab_$v.log" 2>&1
  rc=$?; cut -c1-110 "$O/ab_$v.log"; [ $rc -eq 0 ] || exit $rc
done
