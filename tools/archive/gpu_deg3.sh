#!/bin/bash
# Degree-3 Euler-Maclaurin correction below kEmH3Max: kernel tests, then the headline bench
# A/B against the build before the change (variants/pre_deg3).
set -u
O=gpurun_out/deg3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/kernels.log 2>&1 || { tail -5 $O/kernels.log; exit 1; }
tail -1 $O/kernels.log
bash tools/archive/ab_script_so.sh pre_deg3 bench.py --steps 300 --warmup 30 > $O/ab.log 2>&1 || exit 1
cat $O/ab.log | cut -c1-200
