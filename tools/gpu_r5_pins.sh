#!/bin/bash
# Round 5: generic engine / two-shot GPU tests after the hold-and-pin give-back change.
set -o pipefail
O=gpurun_out/r5_pins
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_generic_engine_gpu.py tests/test_twoshot_gpu.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
