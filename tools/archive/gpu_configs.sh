#!/bin/bash
# BASELINE configs on one GPU + the reference-anchor BFGS rate; each step time-limited.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python benchmarks/configs.py --which toy adam1e6 adam1e7 lbfgs > gpurun_out/configs.log 2>&1 || { echo "configs rc=$?"; tail -20 gpurun_out/configs.log; exit 1; }
cat gpurun_out/configs.log | grep '^{'
timeout -k 10 400 python benchmarks/configs.py --which adam1e8 --steps 10 > gpurun_out/configs8.log 2>&1 || { echo "1e8 rc=$?"; tail -20 gpurun_out/configs8.log; exit 1; }
grep '^{' gpurun_out/configs8.log
timeout -k 10 300 python benchmarks/bfgs_anchor.py > gpurun_out/anchor.log 2>&1 || { echo "anchor rc=$?"; tail -20 gpurun_out/anchor.log; exit 1; }
grep '^{' gpurun_out/anchor.log
timeout -k 10 300 python benchmarks/smf_gd_benchmark.py --num-halos 10000 --num-steps 200 | tail -2
timeout -k 10 300 python benchmarks/smf_gd_benchmark.py --num-halos 100000000 --num-steps 100 | tail -2
