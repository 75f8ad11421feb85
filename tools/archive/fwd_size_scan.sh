#!/bin/bash
# Forward time vs problem size (1/8, 1/4, 1/2, 1 x the headline) for each schedule.
for mode in 1 dynamic; do
for k in 1 2 8; do
  p=$((1250000*k)); h=$((16777216*k))
  MULTIGRAD_LPT=$mode timeout -k 10 300 python tools/kernel_bench.py --tag ${mode}_x$k --params $p --halos $h --iters 30 2>/dev/null | grep tag | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['tag'], d['halos'], 'fwd_int', d['fwd_internal_us'], 'nores', d['fwd_noresid_us'], d['S'][:2])"
done; done
