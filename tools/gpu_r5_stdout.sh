#!/bin/bash
# bench.py on 2 and 4 ranks (sharing one GPU): stdout must hold exactly one line, the JSON record.
set -o pipefail
O=gpurun_out/r5_stdout
mkdir -p $O
for n in 2 4; do
  NPROC=$n timeout -k 10 600 bash tools/bench_2rank.sh --steps 10 --warmup 2 --params 2000000 --halos 16777216 \
    > $O/out_n$n.txt 2> $O/err_n$n.txt || { tail -20 $O/err_n$n.txt; exit 1; }
  echo "n=$n stdout lines: $(wc -l < $O/out_n$n.txt)"
  python3 -c "import json; d=json.loads(open('$O/out_n$n.txt').read()); print(d['n_gpus'], d['value'], d['owner_steps_per_s'])"
done
