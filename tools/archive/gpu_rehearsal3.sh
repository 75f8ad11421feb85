#!/bin/bash
# Round-3 rehearsal on one MI355X: smoke(), the driver's bench command (20 timed steps after
# 5 warmup) three times and a 50-step run, a kernel-trace profile of the bench, the
# generic-engine benchmarks (plain / per-step keys / 2-member group).  Stops at the first
# failing step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/rehearsal3
mkdir -p "$O"
cd "$R"
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
rc=$?; tail -2 "$O/smoke.log"; [ $rc -eq 0 ] || exit $rc
: > "$O/bench.log"
for args in "--steps 20 --warmup 5" "--steps 20 --warmup 5" "--steps 20 --warmup 5" "--steps 50 --warmup 5"; do
  timeout -k 10 300 python bench.py --gpus 1 $args >> "$O/bench.log" 2>&1 || { tail -5 "$O/bench.log"; exit 1; }
done
grep '^{' "$O/bench.log" | cut -c1-230
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o bench \
  -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-count-launches > "$O/prof_bench.log" 2>&1) || exit 1
: > "$O/generic.log"
for mdl in plain randkey group; do
  timeout -k 10 300 python benchmarks/generic_engine.py --model $mdl --params 20000 --halos 400000 --steps 60 >> "$O/generic.log" 2>&1 || exit 1
done
grep speedup "$O/generic.log"
