#!/bin/bash
# Round 5 final tree: the driver's bench command three times, the headline under rocprofv3
# (kernel stats), smoke().
set -o pipefail
O=gpurun_out/r5_final
mkdir -p $O
export MULTIGRAD_PROGRESS=0
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd_$r.json 2> $O/bench_$r.err || { tail -20 $O/bench_$r.err; exit 1; }
  tail -1 $O/bench_driver_cmd_$r.json | cut -c1-200
done
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 5 > $O/bench_2000.json 2> $O/bench_2000.err || { tail -20 $O/bench_2000.err; exit 1; }
tail -1 $O/bench_2000.json | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o k -- \
  python -u $GRAFT_REPO_ROOT/bench.py > $GRAFT_REPO_ROOT/$O/bench_under_rocprof.json 2> $GRAFT_REPO_ROOT/$O/prof.err || { tail -30 $GRAFT_REPO_ROOT/$O/prof.err; exit 1; }
head -6 $GRAFT_REPO_ROOT/$O/prof/k_kernel_stats.csv | cut -c1-140
