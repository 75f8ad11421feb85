#!/bin/bash
# Kernel traces of the same engine step launched eagerly and replayed from a HIP graph
# (MULTIGRAD_GRAPH=0/1 pins the mode), headline size and the 8-GPU owner-shard proxy,
# then the per-kernel duration / gap / queue summary (tools/graph_trace_analyze.py).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/graph_trace
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
for cfg in "full:--steps 200 --warmup 10" "proxy:--params 1250000 --halos 16777216 --steps 600 --warmup 50"; do
  name=${cfg%%:*}; args=${cfg#*:}
  for g in 0 1; do
    MULTIGRAD_GRAPH=$g timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
      -d "$O/${name}_g$g" -o k -- python3 "$R/bench.py" $args --no-count-launches \
      > "$O/${name}_g$g.log" 2>&1 || exit $?
    grep -o '"ms_per_step": [0-9.]*' "$O/${name}_g$g.log" | sed "s/^/$name graph=$g /"
  done
done
cd "$R"
python3 tools/graph_trace_analyze.py $(ls "$O"/*/k_kernel_trace.csv "$O"/*/*/k_kernel_trace.csv 2>/dev/null) > "$O/summary.jsonl"
cat "$O/summary.jsonl"
