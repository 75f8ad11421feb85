#!/bin/bash
# Round 6: LDS staging depth of the SMF fused step's forward: 8 rows (in-tree) vs 4 and 16,
# the reference's GD benchmark at 1e8 halos, alternating on one box.
set -o pipefail
O=gpurun_out/r6_s2rows
mkdir -p $O
for rep in 1 2 3; do
  for v in base rows4 rows16; do
    so=""; [ $v != base ] && so=abvar/$v/_C.so
    MULTIGRAD_EXT_SO=$so timeout -k 10 300 python benchmarks/smf_gd_benchmark.py --num-halos 100000000 --num-steps 1000 \
      > $O/${v}_$rep.log 2>&1 || { tail -20 $O/${v}_$rep.log; exit 1; }
    echo "$v $rep $(grep '^{' $O/${v}_$rep.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(round(d["value"],1))')"
  done
done
