#!/bin/bash
# Per-rank proxy of the 8-GPU owner-placement step on one GPU (1/8 of the parameters and
# halos) and the full 1-GPU bench, for each forward schedule (MULTIGRAD_LPT).
set -e
one() {  # label env... -- bench args
  local label=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" | tail -1 | \
    python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$label', d['ms_per_step'], d['value'])"
}
for mode in auto static dynamic; do
  one full_$mode MULTIGRAD_LPT=$mode -- --steps 50 --warmup 5
  one proxy_$mode MULTIGRAD_LPT=$mode -- --params 1250000 --halos 16777216 --steps 200 --warmup 20
done
