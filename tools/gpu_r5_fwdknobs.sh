#!/bin/bash
# Round 5: same-box A/B of the tiles-forward build switches on the hashed per-rank proxy
# (all 1e7 parameters, 1/8 of the halos): MG_FWD_UNROLL 1/4 and MG_FWD_MINWAVES 6 against
# the defaults (2, 8).
set -o pipefail
O=gpurun_out/r5_fwdknobs
mkdir -p $O
for v in fwdu1 fwdu4 fwdw6; do
  echo "== $v" | tee -a $O/ab.log
  bash tools/ab_bench_so.sh $v --placement hashed --layout tiles --halos 16777216 --steps 400 --warmup 20 \
    >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
done
cat $O/ab.log
