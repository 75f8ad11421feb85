#!/bin/bash
# Round 6: static LPT lists at every size -- the schedule tests, the determinism test, the
# headline bench and the run_adam end-to-end record on the new default.
set -o pipefail
O=gpurun_out/r6_static
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_determinism_gpu.py tests/test_engine_cache_gpu.py \
  "tests/test_kernels_gpu.py::test_forward_schedules_agree" \
  "tests/test_kernels_gpu.py::test_forward_schedules_at_eighth_shard_vs_fp64" \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python bench.py --steps 300 --warmup 10 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench.json
python -c 'import json;d=json.load(open("'$O'/bench.json"));print(d["value"], d["ms_per_step"], d["loss_last"])'
timeout -k 10 400 python -u benchmarks/run_adam_e2e.py > $O/e2e.log 2>&1 || { tail -30 $O/e2e.log; exit 1; }
grep '^{' $O/e2e.log > $O/run_adam_e2e.json
python -c 'import json;d=json.load(open("'$O'/run_adam_e2e.json"));print([c["wall_s"] for c in d["calls"]], d["ratio_repeat"], d["step_ms"])'
