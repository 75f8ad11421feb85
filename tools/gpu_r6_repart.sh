#!/bin/bash
# Round 6: peer all-to-all-v + engine re-partition on one MI355X: GPU tests, the 1-GPU
# headline, per-rank owner proxies at 1/2, 1/4, 1/8 of the catalog, and rehearsals of the
# multi-rank bench (hashed input -> re-partition vs dense) with N processes sharing the GPU.
set -o pipefail
O=gpurun_out/r6_repart
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_repartition_gpu.py \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_1gpu.json 2> $O/bench_1gpu.err || { tail -20 $O/bench_1gpu.err; exit 1; }
cat $O/bench_1gpu.json | cut -c1-300
for f in 2 4 8; do
  P=$((10000000 / f)); H=$((134217728 / f))
  timeout -k 10 300 python bench.py --params $P --halos $H --steps 400 --warmup 20 --no-count-launches \
    > $O/proxy_$f.json 2> $O/proxy_$f.err || { tail -20 $O/proxy_$f.err; exit 1; }
  python -c "import json;d=json.load(open('$O/proxy_$f.json'));print('proxy 1/$f', d['ms_per_step'])"
done
for n in 2 4; do
  NPROC=$n PLACEMENT=both timeout -k 10 900 bash tools/bench_2rank.sh --steps 20 --warmup 5 --no-count-launches \
    > $O/bench_n$n.json 2> $O/bench_n$n.err || { tail -30 $O/bench_n$n.err; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('$O/bench_n$n.json') if l.startswith('{')][-1])
print($n, 'value', d['value'], 'loss', d['loss_last'], 'dense', d['dense_steps_per_s'], d['dense_config']['loss_last'], 'setup', d['setup_s'])
print(json.dumps(d.get('repartition'))[:400])
print(json.dumps(d['peer_memory_selftest'].get('all-to-all'))[:400])"
done
NPROC=8 PLACEMENT=repartition timeout -k 10 900 bash tools/bench_2rank.sh --steps 20 --warmup 5 --no-count-launches \
  > $O/bench_n8.json 2> $O/bench_n8.err || { tail -30 $O/bench_n8.err; exit 1; }
python -c "
import json; d=json.loads([l for l in open('$O/bench_n8.json') if l.startswith('{')][-1])
print(8, 'value', d['value'], 'loss', d['loss_last'], 'setup', d['setup_s'])
print(json.dumps(d.get('repartition'))[:400])"
