#!/bin/bash
# Same-box A/B: update arguments read from the kernarg segment (variants/ka) vs the in-tree
# build, on the headline and on the bounded headline.
set -o pipefail
O=gpurun_out/ab_ka
mkdir -p $O
echo "== headline" | tee $O/ab.log
bash tools/ab_bench_so.sh ka --steps 400 --warmup 20 | tee -a $O/ab.log || exit 1
echo "== bounds both" | tee -a $O/ab.log
bash tools/ab_bench_so.sh ka --steps 400 --warmup 20 --bounds both | tee -a $O/ab.log || exit 1
