#!/bin/bash
# Round-end rehearsal on one MI355X: every GPU test in ONE pytest process, the smoke entry
# point, the 1-GPU headline bench, and a kernel-trace profile of it (summaries are copied
# into profiles/ by hand afterwards).  Stops at the first failing step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/rehearsal"
O=$R/gpurun_out/rehearsal
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -5 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
rc=$?; tail -3 "$O/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > "$O/bench.log" 2>&1
rc=$?; grep '^{' "$O/bench.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o bench \
  -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-count-launches > "$O/prof_bench.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
