#!/bin/bash
# Round 6: SMF fused step with 16-row LDS tiles: its GPU tests and the GD benchmark.
set -o pipefail
O=gpurun_out/r6_s2check
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_smf2_gpu.py tests/test_engine_cache_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for nh in 100000000 1000000 10000; do
  timeout -k 10 300 python benchmarks/smf_gd_benchmark.py --num-halos $nh --num-steps 1000 > $O/gd_$nh.log 2>&1 || { tail -20 $O/gd_$nh.log; exit 1; }
  grep '^{' $O/gd_$nh.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print("gd", d["num_halos"], round(d["value"],1), d["final_params"])'
done
