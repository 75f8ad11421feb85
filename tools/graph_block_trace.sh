#!/bin/bash
# Kernel trace of the fused 1-GPU step replayed one step per graph vs 16 steps per graph vs
# eager: per-kernel durations and the gaps between consecutive kernels (rocprofv3).
#   bash tools/graph_block_trace.sh [ROW]   (ROW: fused | owner_proxy)
set -u
export TMPDIR=/tmp
row=${1:-fused}
out=gpurun_out/gbt
mkdir -p $out
for mode in eager eager-dev graph-1 graph-K; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/$mode -o k -- \
    python3 -c "
import sys; sys.path.insert(0, '.')
import benchmarks.graph_modes as G
G.fused_row(*{'fused': (10_000_000, 1 << 27), 'owner_proxy': (1_250_000, 1 << 24)}['$row'], 64, 16, 16, '$mode')
" > $out/$mode.log 2>&1 || { echo "rocprof $mode failed"; exit 1; }
  t=$(find $out/$mode -name '*kernel_trace.csv' | head -1)
  python3 - "$t" "$mode" <<'PY'
import csv, sys, statistics
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
k = [r for r in rows if 'smf_' in r['Kernel_Name']][-64:]
dur = {}
gaps = []
prev = None
for r in k:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    name = r['Kernel_Name'].split('(')[0][-40:]
    dur.setdefault(name, []).append((e - s) / 1e3)
    if prev is not None:
        gaps.append((s - prev) / 1e3)
    prev = e
print(sys.argv[2], {n: round(statistics.median(v), 1) for n, v in dur.items()},
      "gap median %.2f us, max %.2f us, sum %.1f us over %d kernels" % (statistics.median(gaps), max(gaps), sum(gaps), len(k)))
# gap before each kernel, by (previous kernel -> kernel): where the idle time sits
pair = {}
for a, b, g in zip(k, k[1:], gaps):
    na = a['Kernel_Name'].split('(')[0].split('<')[0][-24:]
    nb = b['Kernel_Name'].split('(')[0].split('<')[0][-24:]
    pair.setdefault(na + ' -> ' + nb, []).append(g)
for n, v in sorted(pair.items()):
    print("   %-52s n=%2d median %6.2f us  max %6.2f us" % (n, len(v), statistics.median(v), max(v)))
PY
  find $out/$mode -type f -delete
done
