#!/bin/bash
# Round 6: what one more lane group costs a wave of the pipelined owner forward (fit of the
# per-wave busy time to rows and groups), at 1/8 and 1/4 of the headline.
set -o pipefail
O=gpurun_out/r6_tailfit
mkdir -p $O
for cfg in "1250000 16777216 p8" "2500000 33554432 p4"; do
  set -- $cfg
  PYTHONPATH=$PWD timeout -k 10 300 python -u tools/fwd_trace_step.py --so abvar/trace/_C.so \
    --params $1 --halos $2 --json $O/fit_$3.json > $O/fit_$3.log 2>&1 || { tail -30 $O/fit_$3.log; exit 1; }
  tail -1 $O/fit_$3.log
done
