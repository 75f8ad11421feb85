#!/bin/bash
# Round 5: lanes-forward grid size at the 8-GPU owner-shard size (MULTIGRAD_FWD_MAX_BLOCKS):
# 9766 groups over 4096 resident waves is 2 or 3 groups per wave; a grid of ceil(groups/12)
# workgroups gives every wave 3.  Per-wave trace and the proxy bench step, alternating.
set -o pipefail
O=gpurun_out/gridsweep; mkdir -p $O
for mb in 1024 814 700; do
  echo "== max blocks $mb" >> $O/trace.txt
  MULTIGRAD_FWD_MAX_BLOCKS=$mb PYTHONPATH=$PWD timeout -k 10 200 python -u tools/fwd_trace.py \
    --so variants/trace/_C.so --params 1250000 --halos 16777216 >> $O/trace.txt 2>> $O/err.txt \
    || { tail $O/err.txt; exit 1; }
done
cat $O/trace.txt
for rep in 1 2 3; do for mb in 1024 814 700 900; do
  MULTIGRAD_FWD_MAX_BLOCKS=$mb timeout -k 10 200 python -u bench.py --params 1250000 --halos 16777216 \
    --steps 300 --warmup 30 > $O/bench_${mb}_$rep.json 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
  echo "mb $mb rep $rep $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'])" $O/bench_${mb}_$rep.json)"
done; done
