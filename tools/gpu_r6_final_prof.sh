#!/bin/bash
# Round 6, final tree: headline bench and the 1/8 owner proxy, plain and under
# rocprofv3 --kernel-trace --stats.
set -o pipefail
O=gpurun_out/r6_final
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_default.json'));print('default', d['value'], d['ms_per_step'], d['steps'], d['warmup'])"
timeout -k 10 300 python bench.py --params 1250000 --halos 16777216 --steps 400 --warmup 20 > $O/own8.json 2> $O/own8.err || { tail -20 $O/own8.err; exit 1; }
python -c "import json;d=json.load(open('$O/own8.json'));print('own8', d['value'], d['ms_per_step'])"
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_head -o head -- python $R/bench.py --steps 200 --warmup 10 > $R/$O/prof_head.log 2>&1 || { tail -20 $R/$O/prof_head.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_own8 -o own8 -- python $R/bench.py --params 1250000 --halos 16777216 --steps 400 --warmup 20 > $R/$O/prof_own8.log 2>&1 || { tail -20 $R/$O/prof_own8.log; exit 1; }
cd $R
find $O -name "*kernel_stats.csv" -exec head -4 {} \;
