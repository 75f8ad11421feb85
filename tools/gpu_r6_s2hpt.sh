#!/bin/bash
# Round 6: parallelism of the SMF fused step's forward at 1e6 halos: LDS tile rows (16
# in-tree, abvar/rows4) x minimum halos per thread (MULTIGRAD_SMF2_HALOS_PER_THREAD).
set -o pipefail
O=gpurun_out/r6_s2hpt
mkdir -p $O
for rep in 1 2; do
  for v in base rows4; do
    so=""; [ $v != base ] && so=abvar/$v/_C.so
    for hpt in 16 4 1; do
      MULTIGRAD_SMF2_HALOS_PER_THREAD=$hpt MULTIGRAD_EXT_SO=$so timeout -k 10 300 python benchmarks/smf_gd_benchmark.py --num-halos 1000000 --num-steps 1000 \
        > $O/${v}_hpt${hpt}_$rep.log 2>&1 || { tail -20 $O/${v}_hpt${hpt}_$rep.log; exit 1; }
      echo "$v hpt$hpt $rep $(grep '^{' $O/${v}_hpt${hpt}_$rep.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(round(d["value"],1))')"
    done
  done
done
