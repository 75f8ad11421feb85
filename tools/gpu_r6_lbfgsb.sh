#!/bin/bash
# Round 6: where a device L-BFGS-B iteration goes at 1e7 parameters, plus kernel stats.
set -o pipefail
O=gpurun_out/r6_lbfgsb
mkdir -p $O
timeout -k 10 400 python -u tools/lbfgsb_breakdown.py > $O/breakdown.log 2>&1 || { tail -30 $O/breakdown.log; exit 1; }
tail -30 $O/breakdown.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o lbfgsb -- python benchmarks/configs.py --which lbfgsb > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec head -16 {} \;
