#!/bin/bash
# Round-3 check on one MI355X: full GPU suite, smoke, the headline bench (x2), a kernel-trace
# profile of the bench, and the generic-engine benchmarks with the reworked auto policy.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${S3B_OUT:-s3b}
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit 1
tail -1 "$O/smoke.log"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench$i.log" 2>&1 || exit 1
  grep '^{' "$O/bench$i.log" | cut -c1-200
done
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o bench \
  -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-count-launches > "$O/prof_bench.log" 2>&1) || exit 1
for m in plain randkey group; do
  timeout -k 10 240 python -u benchmarks/generic_engine.py --params 20000 --halos 400000 --steps 60 \
    --model $m --repeats 5 >> "$O/generic.log" 2>&1 || { echo "generic $m failed"; exit 1; }
done
grep speedup "$O/generic.log" | cut -c1-200
