#!/bin/bash
# Per-rank proxy of the N-GPU HASHED step on one GPU: all 1e7 parameters, 1/N of the halos
# (every population present), in the layout the hashed ranks use (lanes, local slot order,
# recomputing VJP; or tiles with LAYOUT=tiles), kernel stats.  The gradient collective is
# absent on one rank (the engine runs the replicated update); the two-shot kernel replaces
# it on N ranks.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
LAYOUT=${LAYOUT:-lanes}
mkdir -p "$R/gpurun_out/hprox"
cd /tmp
for div in ${DIVS:-8 4 2}; do
  h=$((134217728 / div))
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/hprox/${LAYOUT}_d$div" -o k -- python3 "$R/bench.py" --params 10000000 --halos $h \
    --layout $LAYOUT --lane-order local --steps 40 --warmup 5 > "$R/gpurun_out/hprox/bench_${LAYOUT}_d$div.log" 2>&1 || exit $?
  grep '^{' "$R/gpurun_out/hprox/bench_${LAYOUT}_d$div.log" | cut -c1-180
done
