#!/bin/bash
# Hashed-shard kernels (recurrence tiles VJP) on one MI355X: kernel numerics tests (fp64
# oracle), the 1/8 hashed-shard per-rank kernels alternating the in-tree build with each
# variant named on the command line, then PMC counters of the tiles kernels at 1/8.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/vjprec
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 \
  --timeout-method thread > "$O/pytest_kernels.log" 2>&1
rc=$?; tail -3 "$O/pytest_kernels.log"; [ $rc -eq 0 ] || exit $rc
for v in "$@"; do
  bash tools/archive/ab_script_so.sh $v tools/uncached_theta_bench.py > "$O/ab_$v.log" 2>&1
  rc=$?; cut -c1-330 "$O/ab_$v.log"; [ $rc -eq 0 ] || exit $rc
done
bash tools/pmc_kernels.sh --layout tiles --halos 16777216
