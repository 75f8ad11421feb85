#!/bin/bash
# Round 6: SMF fused-step forward occupancy A/B (in-tree 5 waves/SIMD vs 4 and 6), GD 1e8.
set -o pipefail
O=gpurun_out/r6_mwab
mkdir -p $O
for rep in 1 2 3; do
  for v in base mw4 mw6; do
    so=""; [ $v != base ] && so=abvar/$v/_C.so
    MULTIGRAD_EXT_SO=$so timeout -k 10 300 python benchmarks/smf_gd_benchmark.py --num-halos 100000000 --num-steps 1000 \
      > $O/${v}_$rep.log 2>&1 || { tail -20 $O/${v}_$rep.log; exit 1; }
    echo "$v $rep $(grep '^{' $O/${v}_$rep.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(round(d["value"],1))')"
  done
done
