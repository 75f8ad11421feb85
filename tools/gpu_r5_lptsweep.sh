#!/bin/bash
# Round 5: static LPT cost model at the 8-GPU owner-shard size (MULTIGRAD_LPT_OVERHEAD sweep):
# per-wave end times of one forward launch (trace variant) and the proxy bench step.
set -o pipefail
O=gpurun_out/lptsweep; mkdir -p $O
for ov in 3 8 16 32 10000; do
  echo "== overhead $ov" >> $O/trace.txt
  MULTIGRAD_LPT_OVERHEAD=$ov PYTHONPATH=$PWD timeout -k 10 200 python -u tools/fwd_trace.py \
    --so variants/trace/_C.so --params 1250000 --halos 16777216 >> $O/trace.txt 2>> $O/err.txt \
    || { tail $O/err.txt; exit 1; }
done
cat $O/trace.txt
for rep in 1 2; do for ov in 3 16 10000; do
  MULTIGRAD_LPT_OVERHEAD=$ov timeout -k 10 200 python -u bench.py --params 1250000 --halos 16777216 \
    --steps 200 --warmup 20 > $O/bench_${ov}_$rep.json 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
  echo "ov $ov rep $rep $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'])" $O/bench_${ov}_$rep.json)"
done; done
