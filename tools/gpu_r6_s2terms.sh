#!/bin/bash
# Round 6: the SMF fused step with adaptive Euler-Maclaurin term counts (in-tree) vs always
# 4 terms (abvar/s2fixed): GPU tests, then the reference's GD benchmark at 1e8 and 1e4
# halos, alternating on one box.
set -o pipefail
O=gpurun_out/r6_s2terms
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_smf2_gpu.py tests/test_engine_cache_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2 3; do
  for v in base s2fixed; do
    so=""; [ $v != base ] && so=abvar/$v/_C.so
    for nh in 100000000 10000; do
      MULTIGRAD_EXT_SO=$so timeout -k 10 300 python benchmarks/smf_gd_benchmark.py --num-halos $nh --num-steps 1000 \
        > $O/${v}_${nh}_$rep.log 2>&1 || { tail -20 $O/${v}_${nh}_$rep.log; exit 1; }
      echo "$v $nh $rep $(grep '^{' $O/${v}_${nh}_$rep.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(round(d["value"],1), d["final_params"])')"
    done
  done
done
