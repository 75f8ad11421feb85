#!/bin/bash
# Per-rank proxy of the 8-GPU owner step (1/8 of the parameters and halos, one GPU):
# in-tree build vs variants/<v> (round 3: defer1), alternating, then a rocprofv3 kernel
# trace of the in-tree build.   bash tools/owner_proxy_ab.sh [variant] [reps]
set -u
export TMPDIR=/tmp
v=${1:-defer1}; reps=${2:-3}
out=gpurun_out/owner_proxy
mkdir -p $out
cp multigrad_amd/_C.so /tmp/_C_base.so
trap 'cp /tmp/_C_base.so multigrad_amd/_C.so' EXIT
args="--params 1250000 --halos 16777216 --steps 400 --warmup 20 --no-count-launches"
for r in $(seq $reps); do
  for b in base $v; do
    if [ $b = base ]; then cp /tmp/_C_base.so multigrad_amd/_C.so; else cp variants/$b/_C.so multigrad_amd/_C.so; fi
    timeout -k 10 300 python3 bench.py $args > $out/${b}_$r.json 2> $out/${b}_$r.err || { echo "bench $b failed"; exit 1; }
    echo "$b rep=$r $(python3 -c "import json;d=json.load(open('$out/${b}_$r.json'));print(d['ms_per_step'], d['config']['graph'], d['config']['graph_steps'])")"
  done
done
cp /tmp/_C_base.so multigrad_amd/_C.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o k -- \
  python3 bench.py $args > $out/prof.json 2> $out/prof.err || { echo "rocprof failed"; exit 1; }
find $out/prof -name '*kernel_trace.csv' -delete
find $out/prof -type f ! -name '*.csv' -delete
echo "prof $(python3 -c "import json;d=json.load(open('$out/prof.json'));print(d['ms_per_step'])")"
