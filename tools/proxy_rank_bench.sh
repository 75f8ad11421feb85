#!/bin/bash
# Per-rank proxy of the 8-GPU owner-placement step on one GPU (1/8 of the parameters and
# halos), plus the full 1-GPU bench, each with and without the LPT forward schedule.
set -e
one() {  # label env... -- bench args
  local label=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python bench.py "$@" | tail -1 | \
    python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$label', d['ms_per_step'], d['value'])"
}
one full_lpt MULTIGRAD_LPT=1 -- --steps 50 --warmup 5
one full_rr MULTIGRAD_LPT=0 -- --steps 50 --warmup 5
one proxy_lpt MULTIGRAD_LPT=1 -- --params 1250000 --halos 16777216 --steps 200 --warmup 20
one proxy_rr MULTIGRAD_LPT=0 -- --params 1250000 --halos 16777216 --steps 200 --warmup 20
