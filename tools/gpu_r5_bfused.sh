#!/bin/bash
# Round 5: bounded fused exchange (modes 2/3 carried by the tiles forward / recurrence VJP) --
# two-shot GPU tests.
set -o pipefail
O=gpurun_out/r5_bfused
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests/test_twoshot_gpu.py -m gpu -x -v \
  --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
