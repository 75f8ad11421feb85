#!/bin/bash
# Round 6: the SMF fused step's wide forward launch (1024-thread workgroups over 4-row tiles
# when the grid does not fill the chip) vs the 256-thread launch (MULTIGRAD_SMF2_WIDE=0):
# GPU tests, then GD at 1e5 / 1e6 / 1e8 halos, alternating on one box.
set -o pipefail
O=gpurun_out/r6_s2wide
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_smf2_gpu.py tests/test_engine_cache_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
MULTIGRAD_SMF2_SCHEDULE=grid timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_smf2_gpu.py > $O/pytest_grid.log 2>&1 || { tail -40 $O/pytest_grid.log; exit 1; }
tail -2 $O/pytest_grid.log
for rep in 1 2 3; do
  for w in 1 0; do
    for nh in 100000 1000000 100000000; do
      MULTIGRAD_SMF2_WIDE=$w timeout -k 10 300 python benchmarks/smf_gd_benchmark.py --num-halos $nh --num-steps 1000 \
        > $O/w${w}_${nh}_$rep.log 2>&1 || { tail -20 $O/w${w}_${nh}_$rep.log; exit 1; }
      echo "wide=$w $nh $rep $(grep '^{' $O/w${w}_${nh}_$rep.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(round(d["value"],1), d["final_params"])')"
    done
  done
done
