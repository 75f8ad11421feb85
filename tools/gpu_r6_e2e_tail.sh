#!/bin/bash
# Round 6: run_adam end-to-end (first / repeated calls) and the per-wave tail fit.
set -o pipefail
O=gpurun_out/r6_e2e
mkdir -p $O
timeout -k 10 400 python -u benchmarks/run_adam_e2e.py > $O/e2e.log 2>&1 || { tail -30 $O/e2e.log; exit 1; }
grep '^{' $O/e2e.log > $O/run_adam_e2e.json
tail -1 $O/e2e.log
bash tools/gpu_r6_tailfit.sh
