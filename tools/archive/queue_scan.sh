#!/bin/bash
# Headline bench over the number of dynamic forward work queues (MULTIGRAD_FWD_QUEUES),
# alternating values, two rounds: bash tools/archive/queue_scan.sh [bench args...]
set -u
for rep in 1 2; do
  for q in 64 128 256 512 1024; do
    ms=$(MULTIGRAD_FWD_QUEUES=$q timeout -k 10 200 python3 bench.py "$@" 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || exit 1
    echo "queues=$q $ms"
  done
done
