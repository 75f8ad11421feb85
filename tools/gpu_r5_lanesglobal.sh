#!/bin/bash
# Round 5: hashed placement with the lanes layout in the global slot order (internal
# parameter order, residual VJP) on 2 ranks: two-shot vs RCCL/gloo bits.
set -o pipefail
O=gpurun_out/r5_lanesglobal
mkdir -p $O
timeout -k 10 900 python -u -m pytest "tests/test_twoshot_gpu.py::test_engine_hashed_twoshot_matches_rccl_path" -m gpu -x -v \
  --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
