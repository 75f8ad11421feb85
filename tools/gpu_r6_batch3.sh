#!/bin/bash
# Round 6: SMF fused step (4-term EM), L-BFGS ZeRO timeout, engine cache; GD benchmark,
# run_adam end-to-end timing, 1-GPU headline.
set -o pipefail
O=gpurun_out/r6_b3
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_smf2_gpu.py \
  tests/test_engine_cache_gpu.py tests/test_lbfgs_comm_gpu.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for n in 10000 1000000 100000000; do
  timeout -k 10 300 python benchmarks/smf_gd_benchmark.py --num-halos $n --num-steps 1000 > $O/gd_${n}.log 2>&1 || { tail -20 $O/gd_${n}.log; exit 1; }
  echo "$n $(grep '^{' $O/gd_${n}.log | cut -c1-150)"
done
timeout -k 10 300 python benchmarks/run_adam_e2e.py > $O/e2e.log 2>&1 || { tail -20 $O/e2e.log; exit 1; }
grep '^{' $O/e2e.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-200 $O/bench.json
