#!/bin/bash
set -o pipefail
O=gpurun_out/r5_epicost
mkdir -p $O
PYTHONPATH=$PWD timeout -k 10 300 python -u tools/ubench/epilogue_cost.py > $O/out.json 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
cat $O/out.json
