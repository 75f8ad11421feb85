#!/bin/bash
# A/B several variants/<name>/_C.so builds against the in-tree one on the same box, REPS
# rounds of (base, v1, v2, ...), printing each run's last output line:
#   REPS=2 bash tools/archive/ab_multi.sh "v1 v2" <script.py> [args...]
set -u
names=$1; shift
cp multigrad_amd/_C.so /tmp/_C_base.so
for rep in $(seq 1 ${REPS:-2}); do
  for v in base $names; do
    if [ $v = base ]; then cp /tmp/_C_base.so multigrad_amd/_C.so; else cp variants/$v/_C.so multigrad_amd/_C.so; fi
    line=$(timeout -k 10 200 python3 "$@" 2>/dev/null | tail -1) || { cp /tmp/_C_base.so multigrad_amd/_C.so; exit 1; }
    echo "$v $line"
  done
done
cp /tmp/_C_base.so multigrad_amd/_C.so
