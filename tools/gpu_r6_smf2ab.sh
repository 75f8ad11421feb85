#!/bin/bash
# Round 6: SMF fused-step prefetch depth A/B (in-tree AHEAD=2 vs abvar/ahead1, ahead4) on the
# GD benchmark at 1e4 / 1e6 / 1e8 halos, alternating, then a rocprofv3 kernel trace.
set -o pipefail
O=gpurun_out/r6_smf2ab
mkdir -p $O
for rep in 1 2; do
  for v in base ahead1 ahead4; do
    so=""; [ $v != base ] && so=abvar/$v/_C.so
    for n in 10000 1000000 100000000; do
      MULTIGRAD_EXT_SO=$so timeout -k 10 300 python benchmarks/smf_gd_benchmark.py --num-halos $n --num-steps 1000 \
        > $O/${v}_${n}_$rep.log 2>&1 || { tail -20 $O/${v}_${n}_$rep.log; exit 1; }
      echo "$v $n $rep $(grep '^{' $O/${v}_${n}_$rep.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(round(d["value"],1), d["engine"]["schedule"])')"
    done
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for n in 10000 1000000 100000000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run -- python benchmarks/smf_gd_benchmark.py --num-halos $n --num-steps 1000 > $O/prof_$n.log 2>&1 || { tail -20 $O/prof_$n.log; exit 1; }
done
find $O -name "*kernel_stats.csv" | head
