#!/bin/bash
# Round 6: fused step of the 2-parameter SMF models (GPU tests + GD benchmark at 1e4/1e6/1e8
# halos), then the 8-process one-GPU re-partition rehearsal with set-up tracing.
set -o pipefail
O=gpurun_out/r6_smf2
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_smf2_gpu.py \
  > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for n in 10000 1000000 100000000; do
  timeout -k 10 300 python benchmarks/smf_gd_benchmark.py --num-halos $n --num-steps 1000 > $O/gd_$n.log 2>&1 || { tail -20 $O/gd_$n.log; exit 1; }
  grep '^{' $O/gd_$n.log | cut -c1-400
done
