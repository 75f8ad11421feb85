#!/bin/bash
# Round 6: two-term Euler-Maclaurin groups (MG_EM2, in-tree on) vs off (abvar/em2off):
# headline bench and the 1/8 owner proxy, alternating, same box; then rocprof stats.
set -o pipefail
O=gpurun_out/r6_em2ab
mkdir -p $O
for rep in 1 2 3; do
  for v in base em2off; do
    so=""; [ $v != base ] && so=abvar/$v/_C.so
    MULTIGRAD_EXT_SO=$so timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-count-launches > $O/head_${v}_$rep.json 2> $O/head_${v}_$rep.err || { tail -20 $O/head_${v}_$rep.err; exit 1; }
    MULTIGRAD_EXT_SO=$so timeout -k 10 300 python bench.py --params 1250000 --halos 16777216 --steps 400 --warmup 20 --no-count-launches > $O/own8_${v}_$rep.json 2> $O/own8_${v}_$rep.err || { tail -20 $O/own8_${v}_$rep.err; exit 1; }
    echo "$v $rep head $(python -c "import json;d=json.load(open('$O/head_${v}_$rep.json'));print(d['ms_per_step'], d['value'], d['loss_last'])") own8 $(python -c "import json;d=json.load(open('$O/own8_${v}_$rep.json'));print(d['ms_per_step'])")"
  done
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o head -- python bench.py --steps 200 --warmup 10 --no-count-launches > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec head -4 {} \;
