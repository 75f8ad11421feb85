#!/bin/bash
# VERDICT r3 #1 evidence, one box: the headline step over 0-100% narrow populations (in-tree
# build vs round 2's per-edge kernel, variants/em0, with rocprof statistics of the in-tree
# runs), round 3's deferral list (variants/defer1) at the shares where it fell off the cliff,
# and a 2000-step headline run.   bash tools/cliff_evidence.sh   -> gpurun_out/narrow/
set -u
STEPS=200 bash tools/narrow_sweep.sh em0 0 0.01 0.1 0.5 1.0 || exit 1
out=gpurun_out/narrow
cp multigrad_amd/_C.so /tmp/_C_base.so
trap 'cp /tmp/_C_base.so multigrad_amd/_C.so' EXIT
cp variants/defer1/_C.so multigrad_amd/_C.so
for f in 0 0.01 0.1; do
  # round 3 as it was: no lane grouping by path, no per-edge kernel switch
  MULTIGRAD_LANE_CLASSES=0 MULTIGRAD_PER_EDGE_SHARE=2 \
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --narrow-frac $f \
    > $out/defer1_20_$f.json 2> $out/defer1_20_$f.err || { echo "defer1 $f failed"; exit 1; }
  echo "defer1(round3) narrow=$f $(grep -o '"value": [0-9.]*' $out/defer1_20_$f.json)"
done
cp /tmp/_C_base.so multigrad_amd/_C.so
timeout -k 10 600 python3 bench.py --steps 2000 --warmup 5 > $out/steps2000.json \
  2> $out/steps2000.err || { echo "2000-step run failed"; exit 1; }
echo "2000 steps: $(grep -o '"value": [0-9.]*' $out/steps2000.json) $(grep -o '"ms_per_step": [0-9.]*' $out/steps2000.json)"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $out/steps20.json 2> $out/steps20.err \
  || { echo "20-step run failed"; exit 1; }
echo "20 steps (driver command): $(grep -o '"value": [0-9.]*' $out/steps20.json)"
