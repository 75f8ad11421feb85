#!/bin/bash
# Fix-up launch size of the deferred lanes fallback (MULTIGRAD_FIX_BLOCKS): the headline
# bench alternating 64 / 8 / 1 workgroups, then a kernel-trace profile at each size.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/fixb
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fallback or headline" > "$O/pytest.log" 2>&1
rc=$?; tail -1 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for fb in 64 8 1; do
    line=$(MULTIGRAD_FIX_BLOCKS=$fb timeout -k 10 200 python3 bench.py --steps 50 --warmup 5 --no-count-launches 2>/dev/null | tail -1) || exit 1
    echo "fb=$fb $(echo $line | cut -c1-120)"
  done
done
export TMPDIR=/tmp
for fb in 64 1; do
  (cd /tmp && MULTIGRAD_FIX_BLOCKS=$fb timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof$fb" -o b \
    -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-count-launches > "$O/prof$fb.log" 2>&1) || exit 1
done
