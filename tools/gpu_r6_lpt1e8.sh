#!/bin/bash
# Round 6: static LPT lists (the default) vs dynamic queues on the 1e8-parameter config
# (190 lane groups per wave), alternating on one box.
set -o pipefail
O=gpurun_out/r6_lpt1e8
mkdir -p $O
for rep in 1 2; do
  for mode in auto dynamic; do
    MULTIGRAD_LPT=$mode timeout -k 10 400 python benchmarks/configs.py --which adam1e8 > $O/${mode}_$rep.log 2>&1 || { tail -20 $O/${mode}_$rep.log; exit 1; }
    grep '^{' $O/${mode}_$rep.log | python -c 'import json,sys
for l in sys.stdin: d=json.loads(l); print("'$mode'", '$rep', d["config"], round(d["value"],1), d.get("ms_per_step"))'
  done
done
