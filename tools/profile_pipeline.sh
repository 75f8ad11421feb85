#!/bin/bash
# Kernel stats of the full 1-GPU bench and of the 8-GPU per-rank proxy, with and without
# the pipelined update (MULTIGRAD_PIPELINE).
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for pipe in 1 0; do
  for cfg in full proxy; do
    args="--steps 50 --warmup 5"
    [ $cfg = proxy ] && args="--params 1250000 --halos 16777216 --steps 200 --warmup 20"
    d=gpurun_out/prof_pipe${pipe}_$cfg
    MULTIGRAD_PIPELINE=$pipe timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
      python3 bench.py $args > $d.log 2>&1
    grep -o "\"ms_per_step\": [0-9.]*" $d.log
    f=$(find $d -name '*kernel_stats.csv' | head -1)
    python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]:
    print(f"  {float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):6d} calls {float(r['AverageNs'])/1e3:8.2f} us  {r['Name'][:90]}")
PY
  done
done
