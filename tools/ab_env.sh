#!/bin/bash
# Alternating same-box A/B of bench.py under different environment settings:
#   bash tools/ab_env.sh "<env A>" "<env B>" [...] -- [bench args]   (env "-" = none)
# prints "<env> ms_per_step" per run, three rounds.
set -u
envs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
[ $# -gt 0 ] && shift
for rep in 1 2 3; do
  for e in "${envs[@]}"; do
    if [ "$e" = "-" ]; then pre=""; else pre="$e"; fi
    ms=$(env $pre timeout -k 10 200 python3 bench.py "$@" 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || exit 1
    echo "$e $ms"
  done
done
