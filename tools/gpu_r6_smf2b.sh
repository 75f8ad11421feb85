#!/bin/bash
# Round 6: SMF fused step after LDS staging: GPU tests, GD benchmark 1e4/1e6/1e8, kernel stats.
set -o pipefail
O=gpurun_out/r6_smf2b
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_smf2_gpu.py tests/test_lbfgs_comm_gpu.py \
  > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
for n in 10000 1000000 100000000; do
  timeout -k 10 300 python benchmarks/smf_gd_benchmark.py --num-halos $n --num-steps 1000 > $O/gd_${n}_$rep.log 2>&1 || { tail -20 $O/gd_${n}_$rep.log; exit 1; }
  echo "$n $rep $(grep '^{' $O/gd_${n}_$rep.log | cut -c1-200)"
done
done
export TMPDIR=/tmp
for n in 1000000 100000000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$n -o run -- python benchmarks/smf_gd_benchmark.py --num-halos $n --num-steps 1000 > $O/prof_$n.log 2>&1 || { tail -20 $O/prof_$n.log; exit 1; }
  find $O/prof_$n -name "*kernel_stats.csv" -exec head -5 {} \;
done
