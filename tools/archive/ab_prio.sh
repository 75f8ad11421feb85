#!/bin/bash
# A/B of the static-list issue-priority feedback (MG_FWD_PRIO, variants/prio) against the
# in-tree build: forward kernel at the per-rank proxy size and at the headline size.
set -u
mkdir -p gpurun_out
out=gpurun_out/ab_prio.log
: > $out
kb() { timeout -k 10 300 python tools/kernel_bench.py "$@" --iters 50 >> $out 2>&1; }
P="--params 1250000 --halos 16777216"
H="--params 10000000 --halos 134217728"
MULTIGRAD_LPT=static kb --tag proxy_static_base $P || exit $?
MULTIGRAD_LPT=static kb --tag proxy_static_prio --so variants/prio/_C.so $P || exit $?
MULTIGRAD_LPT=dynamic kb --tag proxy_dynamic_base $P || exit $?
MULTIGRAD_LPT=static kb --tag head_static_base $H || exit $?
MULTIGRAD_LPT=static kb --tag head_static_prio --so variants/prio/_C.so $H || exit $?
MULTIGRAD_LPT=dynamic kb --tag head_dynamic_base $H || exit $?
grep tag $out
