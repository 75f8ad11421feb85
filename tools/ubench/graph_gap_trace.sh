#!/bin/bash
# rocprofv3 kernel traces of tools/ubench/graph_gap.py per mode: median gap before each
# kernel by (previous kernel -> kernel), kernels labelled by grid size (A: 1 workgroup,
# B: chip-wide).   bash tools/ubench/graph_gap_trace.sh   -> gpurun_out/ggap/
set -u
export TMPDIR=/tmp
out=gpurun_out/ggap
mkdir -p $out
kind=${KIND:-mul}
timeout -k 10 120 python3 tools/ubench/graph_gap.py --kind $kind || exit 1
for mode in eager graph-1 graph-K; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $out/$mode -o k -- \
    python3 tools/ubench/graph_gap.py --kind $kind --only $mode --steps 64 --repeats 1 > $out/$mode.log 2>&1 || { echo "rocprof $mode failed"; exit 1; }
  t=$(find $out/$mode -name '*kernel_trace.csv' | head -1)
  python3 - "$t" "$mode" <<'PY'
import csv, sys, statistics
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
rows = [r for r in rows if 'at::' in r['Kernel_Name'] or 'elementwise' in r['Kernel_Name'] or 'reduce' in r['Kernel_Name'] or 'scan' in r['Kernel_Name']][-96:]
lab = lambda r: 'A' if int(r.get('Grid_Size', r.get('Grid_Size_X', 0)) or 0) <= 1024 else 'B'
dur, gap = {}, {}
for p, r in zip(rows, rows[1:]):
    g = (int(r['Start_Timestamp']) - int(p['End_Timestamp'])) / 1e3
    gap.setdefault(lab(p) + '->' + lab(r), []).append(g)
for r in rows:
    dur.setdefault(lab(r), []).append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
print(sys.argv[2], 'durations', {k: round(statistics.median(v), 2) for k, v in dur.items()},
      'gaps', {k: (round(statistics.median(v), 2), round(max(v), 2)) for k, v in gap.items()})
PY
  find $out/$mode -type f -delete
done
