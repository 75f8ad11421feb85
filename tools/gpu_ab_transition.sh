#!/bin/bash
# Same-box A/B of the lanes-forward group transition: in-tree build vs variants/tr (next group's
# loads before the residual stores, split queue draw), each with the dynamic queues (default at
# the headline) and with the static LPT lists (no ticket atomics), alternating.
set -u
O=gpurun_out/ab_transition
mkdir -p $O
cp multigrad_amd/_C.so /tmp/_C_base.so
for rep in 1 2 3; do
  for v in base tr; do
    if [ $v = base ]; then cp /tmp/_C_base.so multigrad_amd/_C.so; else cp variants/tr/_C.so multigrad_amd/_C.so; fi
    for lpt in auto static; do
      ms=$(MULTIGRAD_LPT=$lpt timeout -k 10 200 python3 bench.py --steps 400 --warmup 20 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || exit 1
      echo "$v lpt=$lpt $ms" | tee -a $O/ab.log
    done
  done
done
cp /tmp/_C_base.so multigrad_amd/_C.so
