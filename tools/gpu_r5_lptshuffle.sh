#!/bin/bash
# Round 5: static LPT lists handed to the waves in a random order (spreads the 3-group waves
# over the SIMDs) vs the heap order, at the 8-GPU owner-shard size.  Per-wave trace, twice each.
set -o pipefail
O=gpurun_out/lptshuffle; mkdir -p $O
for rep in 1 2; do for sh in "" "--shuffle"; do
  echo "== shuffle '$sh' rep $rep" >> $O/trace.txt
  PYTHONPATH=$PWD timeout -k 10 200 python -u tools/fwd_trace.py $sh \
    --so variants/trace/_C.so --params 1250000 --halos 16777216 >> $O/trace.txt 2>> $O/err.txt \
    || { tail $O/err.txt; exit 1; }
done; done
cat $O/trace.txt
