#!/bin/bash
# Round 5: bounded update with the wave-uniform both-bounded fast path -- tests, then bounded vs
# unbounded headline alternating on one box, then a rocprof pass of the bounded step.
set -o pipefail
O=gpurun_out/r5_bounded3
mkdir -p $O
export MULTIGRAD_PROGRESS=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_kernels_gpu.py::test_bounded_pipelined_update_matches_unpipelined" > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2 3; do
  for b in none both mixed; do
    timeout -k 10 300 python -u bench.py --steps 300 --warmup 5 --bounds $b --no-count-launches > $O/bench_${b}_$r.json 2> $O/bench_${b}_$r.err || { tail -20 $O/bench_${b}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_${b}_$r.json')); print('$b', $r, d['value'], d['ms_per_step'], d['config']['pipelined'])"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_bounded -o b -- \
  python -u $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 5 --bounds both --no-count-launches > $GRAFT_REPO_ROOT/$O/prof_bounded.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/$O/prof_bounded.log; exit 1; }
head -4 $GRAFT_REPO_ROOT/$O/prof_bounded/b_kernel_stats.csv | cut -c1-120
