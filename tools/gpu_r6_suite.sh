#!/bin/bash
# Round 6: the whole GPU suite + smoke on the current tree.
set -o pipefail
O=gpurun_out/r6_suite
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
grep -E "FAILED|ERROR" $O/pytest.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
