#!/bin/bash
set -o pipefail
O=gpurun_out/r5_relayoutcost
mkdir -p $O
PYTHONPATH=$PWD MULTIGRAD_PROGRESS=0 timeout -k 10 400 python -u tools/dbg/relayout_cost.py > $O/out.json 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
cat $O/out.json
