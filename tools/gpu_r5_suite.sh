#!/bin/bash
# Round 5: the whole GPU suite on the current tree.
set -o pipefail
O=gpurun_out/r5_suite
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
