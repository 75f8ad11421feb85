#!/bin/bash
# Round 6: static LPT lists (auto) vs dynamic queues for the pipelined owner proxies.
set -o pipefail
O=gpurun_out/r6_lptab
mkdir -p $O
for rep in 1 2 3; do
  for cfg in "1250000 16777216 p8" "2500000 33554432 p4"; do
    set -- $cfg
    for mode in auto dynamic; do
      MULTIGRAD_LPT=$mode timeout -k 10 300 python bench.py --params $1 --halos $2 --steps 400 --warmup 20 \
        > $O/${3}_${mode}_$rep.log 2>&1 || { tail -20 $O/${3}_${mode}_$rep.log; exit 1; }
      echo "$3 $mode $rep $(grep '^{' $O/${3}_${mode}_$rep.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["ms_per_step"])')"
    done
  done
done
