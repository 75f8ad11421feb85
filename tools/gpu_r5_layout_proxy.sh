#!/bin/bash
# Round 5: which layout for hashed shards at N = 2 and 4?  Per-rank proxies on one GPU (all
# 1e7 parameters, 1/N of the 1.34e8 halos), unpipelined (a hashed rank must sum its gradient
# across ranks before Adam): tiles vs lanes (global slot order, residual VJP), alternating.
set -o pipefail
O=gpurun_out/r5_layout_proxy
mkdir -p $O
export MULTIGRAD_PIPELINE=0 MULTIGRAD_FUSED_VJP_ADAM=0 MULTIGRAD_PROGRESS=0
for rep in 1 2; do
  for n in 2 4; do
    h=$((134217728 / n))
    for lay in tiles lanes; do
      extra=""; [ $lay = lanes ] && extra="--lane-order global"
      timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --halos $h --layout $lay $extra --no-count-launches \
        > $O/n${n}_${lay}_$rep.json 2> $O/n${n}_${lay}_$rep.err || { tail -20 $O/n${n}_${lay}_$rep.err; exit 1; }
      python -c "import json; d=json.load(open('$O/n${n}_${lay}_$rep.json')); print('N=$n', '$lay', $rep, d['ms_per_step'], d['config']['layout'], d['config']['pipelined'])"
    done
  done
done
