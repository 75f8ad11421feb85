#!/bin/bash
# 1/R by its own v_exp (MG_EM_RI_EXP=1) against the in-tree build (dependent v_rcp),
# headline bench, same box.
set -u
O=gpurun_out/riexp
mkdir -p $O
bash tools/archive/ab_script_so.sh riexp bench.py --steps 300 --warmup 30 > $O/ab.log 2>&1 || exit 1
cut -c1-140 $O/ab.log
