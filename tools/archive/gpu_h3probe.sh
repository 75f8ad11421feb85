#!/bin/bash
# Timing probe only: the degree-3 correction on every group (MG_EM_H3MAX=0.5, outside its
# accuracy range) against the in-tree build, headline bench, same box.
set -u
O=gpurun_out/h3probe
mkdir -p $O
bash tools/archive/ab_script_so.sh h3_05 bench.py --steps 300 --warmup 30 > $O/ab.log 2>&1 || exit 1
cut -c1-140 $O/ab.log
