#!/bin/bash
# Round 5: every BASELINE config on this tree (one GPU), plus kernel statistics of the 1e6 run.
set -o pipefail
O=gpurun_out/r5_configs
mkdir -p $O
timeout -k 10 900 python -u benchmarks/configs.py --which toy adam1e6 adam1e7 adam1e8 lbfgs lbfgsb --steps 200 \
  > $O/configs.log 2>&1 || { tail -30 $O/configs.log; exit 1; }
grep '^{' $O/configs.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof1e6 -o k -- \
  python -u $GRAFT_REPO_ROOT/benchmarks/configs.py --which adam1e6 --steps 200 > $GRAFT_REPO_ROOT/$O/prof1e6.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/$O/prof1e6.log; exit 1; }
head -4 $GRAFT_REPO_ROOT/$O/prof1e6/k_kernel_stats.csv | cut -c1-150
