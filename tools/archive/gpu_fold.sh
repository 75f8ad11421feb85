#!/bin/bash
# Sumstat epilogue folded into the fix-up launch (MULTIGRAD_FOLD_EPILOGUE): GPU tests, smoke,
# the headline bench alternating fold on/off, and a kernel-trace profile with the fold.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/fold
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit 1
tail -1 "$O/smoke.log"
for rep in 1 2 3; do
  for f in 1 0; do
    line=$(MULTIGRAD_FOLD_EPILOGUE=$f timeout -k 10 200 python3 bench.py --steps 50 --warmup 5 --no-count-launches 2>/dev/null | tail -1) || exit 1
    echo "fold=$f $(echo $line | cut -c1-120)"
  done
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench$i.log" 2>&1 || exit 1
  grep '^{' "$O/bench$i.log" | cut -c1-200
done
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o b \
  -- python3 "$R/bench.py" --steps 20 --warmup 5 > "$O/prof.log" 2>&1) || exit 1
