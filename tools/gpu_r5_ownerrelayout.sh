#!/bin/bash
set -o pipefail
O=gpurun_out/r5_ownerrelayout
mkdir -p $O
timeout -k 10 900 python -u -m pytest "tests/test_twoshot_gpu.py::test_owner_relayout_two_ranks_matches_static_layout" -m gpu -x -v \
  --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
