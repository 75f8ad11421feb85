#!/bin/bash
# 5 waves per SIMD (MG_LANES_MINWAVES=5, 96 VGPRs with spills) against the in-tree build,
# headline bench, same box.
set -u
O=gpurun_out/mw5
mkdir -p $O
bash tools/archive/ab_script_so.sh mw5 bench.py --steps 300 --warmup 30 > $O/ab.log 2>&1 || exit 1
cut -c1-140 $O/ab.log
