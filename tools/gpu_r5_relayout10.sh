#!/bin/bash
# Round 5: the crossing bench in 10-step windows (re-layout on / off) -- what the window that
# holds the re-layout pays, step by step.
set -o pipefail
O=gpurun_out/r5_relayout10
mkdir -p $O
export MULTIGRAD_PROGRESS=0
A="--steps 400 --warmup 5 --narrow-frac 0.01 --narrow-guess -0.64 --phase-steps 10 --no-count-launches"
timeout -k 10 300 python -u bench.py $A > $O/on.json 2> $O/on.err || { tail -20 $O/on.err; exit 1; }
MULTIGRAD_RELAYOUT=0 timeout -k 10 300 python -u bench.py $A > $O/off.json 2> $O/off.err || { tail -20 $O/off.err; exit 1; }
for f in on off; do python -c "
import json; d=json.load(open('$O/$f.json'))
print('$f', d['value'], [round(p['ms_per_step'],3) for p in d['phases']][:20], d['config']['relayouts'])"; done
