#!/bin/bash
# A/B any timing script between the in-tree _C.so and variants/<name>/_C.so on the same box,
# alternating runs, printing each run's last output line:
#   bash tools/archive/ab_script_so.sh <name> <script.py> [args...]
set -u
name=$1; shift
cp multigrad_amd/_C.so /tmp/_C_base.so
for rep in 1 2 3; do
  for v in base $name; do
    if [ $v = base ]; then cp /tmp/_C_base.so multigrad_amd/_C.so; else cp variants/$v/_C.so multigrad_amd/_C.so; fi
    line=$(timeout -k 10 200 python3 "$@" 2>/dev/null | tail -1) || { cp /tmp/_C_base.so multigrad_amd/_C.so; exit 1; }
    echo "$v $line"
  done
done
cp /tmp/_C_base.so multigrad_amd/_C.so
