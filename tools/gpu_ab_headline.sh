#!/bin/bash
# Same-box A/B of the headline bench: in-tree _C.so vs variants/<name>/_C.so (alternating).
set -o pipefail
O=gpurun_out/ab_headline
mkdir -p $O
for v in "$@"; do
  echo "== $v" | tee -a $O/ab.log
  bash tools/ab_bench_so.sh $v --steps 400 --warmup 20 >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
done
cat $O/ab.log
