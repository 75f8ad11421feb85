#!/bin/bash
# Round 6: SMF step kernel with the optimizer state prefetched before the slab sum
# (in-tree) vs loaded after the loss (abvar/nopre): tests, then GD at 1e6 and 1e8 halos,
# alternating on one box, and the step kernel's rocprof time.
set -o pipefail
O=gpurun_out/r6_s2pre
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_smf2_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2 3; do
  for v in base nopre; do
    so=""; [ $v != base ] && so=abvar/$v/_C.so
    for nh in 1000000 100000000; do
      MULTIGRAD_EXT_SO=$so timeout -k 10 300 python benchmarks/smf_gd_benchmark.py --num-halos $nh --num-steps 1000 \
        > $O/${v}_${nh}_$rep.log 2>&1 || { tail -20 $O/${v}_${nh}_$rep.log; exit 1; }
      echo "$v $nh $rep $(grep '^{' $O/${v}_${nh}_$rep.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(round(d["value"],1), d["final_params"])')"
    done
  done
done
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o gd1e6 -- python $R/benchmarks/smf_gd_benchmark.py --num-halos 1000000 --num-steps 1000 > $R/$O/prof.log 2>&1 || { tail -20 $R/$O/prof.log; exit 1; }
cd $R
find $O/prof -name "*kernel_stats.csv" -exec head -4 {} \;
