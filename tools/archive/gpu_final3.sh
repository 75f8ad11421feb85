#!/bin/bash
# Round-3 closing rehearsal on one MI355X: full GPU suite, smoke, the driver's bench command
# three times, a kernel-trace profile of the bench, and the hashed 1/8 per-rank proxy.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/final3
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit 1
tail -1 "$O/smoke.log"
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench$i.log" 2>&1 || exit 1
  grep '^{' "$O/bench$i.log" | cut -c1-160
done
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o b \
  -- python3 "$R/bench.py" --steps 20 --warmup 5 > "$O/prof.log" 2>&1) || exit 1
LAYOUT=tiles DIVS="8" bash tools/profile_hashed_proxy.sh
