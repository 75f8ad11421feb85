#!/bin/bash
# Generic-engine benchmarks on one MI355X (plain / randkey / 2-group population models,
# eager vs graph replay vs the auto policy), two sizes, then the headline bench twice.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/generic3
mkdir -p "$O"
cd "$R"
for size in "20000 400000" "100000 1000000"; do
  set -- $size
  for m in plain randkey group; do
    timeout -k 10 240 python -u benchmarks/generic_engine.py --params $1 --halos $2 --steps 60 \
      --model $m --repeats 5 >> "$O/generic.log" 2>&1 || { echo "generic $m $1 failed"; exit 1; }
  done
done
grep speedup "$O/generic.log"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench$i.log" 2>&1 || exit 1
  grep '^{' "$O/bench$i.log" | cut -c1-200
done
if [ -f variants/emonly/_C.so ]; then
  bash tools/archive/ab_script_so.sh emonly bench.py --steps 50 --warmup 5 --no-count-launches > "$O/ab_emonly.log" 2>&1
  cut -c1-160 "$O/ab_emonly.log"
fi
