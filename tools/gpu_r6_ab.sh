#!/bin/bash
# Round 6: in-tree build vs an A/B variant (abvar/$1/_C.so), headline bench and the 1/8 owner
# proxy, alternating on one box.   bash tools/gpu_r6_ab.sh VARIANT
set -o pipefail
V=$1
O=gpurun_out/r6_ab_$V
mkdir -p $O
for rep in 1 2 3; do
  for v in base $V; do
    so=""; [ $v != base ] && so=abvar/$v/_C.so
    MULTIGRAD_EXT_SO=$so timeout -k 10 300 python bench.py --steps 300 --warmup 10 --no-count-launches > $O/head_${v}_$rep.json 2> $O/head_${v}_$rep.err || { tail -20 $O/head_${v}_$rep.err; exit 1; }
    MULTIGRAD_EXT_SO=$so timeout -k 10 300 python bench.py --params 1250000 --halos 16777216 --steps 400 --warmup 20 --no-count-launches > $O/own8_${v}_$rep.json 2> $O/own8_${v}_$rep.err || { tail -20 $O/own8_${v}_$rep.err; exit 1; }
    echo "$v $rep head $(python -c "import json;d=json.load(open('$O/head_${v}_$rep.json'));print(d['ms_per_step'], d['loss_last'])") own8 $(python -c "import json;d=json.load(open('$O/own8_${v}_$rep.json'));print(d['ms_per_step'])")"
  done
done
