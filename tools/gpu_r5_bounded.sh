#!/bin/bash
# Round 5: bounded pipelined Adam, direct-step eager policy, mid-run checkpoint load, LDS of
# the fused exchange -- targeted tests, then the headline bench unbounded / bounded
# (pipelined and unpipelined) and a rocprof kernel summary of the bounded pipelined step.
set -o pipefail
O=gpurun_out/r5_bounded
mkdir -p $O
export MULTIGRAD_PROGRESS=0
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_kernels_gpu.py::test_bounded_pipelined_update_matches_unpipelined" \
  "tests/test_kernels_gpu.py::test_pipelined_update_matches_unpipelined" \
  "tests/test_kernels_gpu.py::test_multi_dot_and_lincomb_kernels" \
  "tests/test_generic_engine_gpu.py::test_direct_steps_with_default_stream_work_match_eager" \
  "tests/test_generic_engine_gpu.py::test_graph_engine_replays_after_eager_steps_with_syncs" \
  "tests/test_twoshot_gpu.py::test_load_state_dict_mid_run_discards_nothing_pending" \
  "tests/test_twoshot_gpu.py::test_engine_hashed_fused_exchange_matches_serial" \
  > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 200 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 200 --warmup 5 --bounds both > $O/bench_bounds_both.json 2> $O/bench_bb.err || { tail -20 $O/bench_bb.err; exit 1; }
MULTIGRAD_PIPELINE=0 timeout -k 10 300 python -u bench.py --steps 200 --warmup 5 --bounds both > $O/bench_bounds_both_unpipelined.json 2> $O/bench_bbu.err || { tail -20 $O/bench_bbu.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 200 --warmup 5 --bounds mixed > $O/bench_bounds_mixed.json 2> $O/bench_bm.err || { tail -20 $O/bench_bm.err; exit 1; }
for f in $O/bench_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['config']['pipelined'], d['config']['device_ops_per_step'])"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o bb -- \
  python -u $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 5 --bounds both > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
head -6 $GRAFT_REPO_ROOT/$O/prof/bb_kernel_stats.csv | cut -c1-200
