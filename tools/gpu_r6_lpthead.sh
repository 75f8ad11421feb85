#!/bin/bash
# Round 6: the headline with static LPT lists vs the default (dynamic queues at >= 8 groups
# per wave): time and run-to-run reproducibility of the trajectory.
set -o pipefail
O=gpurun_out/r6_lpthead
mkdir -p $O
for rep in 1 2 3; do
  for mode in static auto; do
    MULTIGRAD_LPT=$mode timeout -k 10 300 python bench.py --steps 300 --warmup 10 \
      > $O/${mode}_$rep.log 2>&1 || { tail -20 $O/${mode}_$rep.log; exit 1; }
    echo "$mode $rep $(grep '^{' $O/${mode}_$rep.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["ms_per_step"], repr(d["loss_last"]))')"
  done
done
