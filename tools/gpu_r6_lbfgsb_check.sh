#!/bin/bash
# Round 6: L-BFGS-B with one host copy per Cauchy scan batch: GPU tests, then the config.
set -o pipefail
O=gpurun_out/r6_lbfgsb_check
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_lbfgsb_gpu.py tests/test_lbfgs_comm_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
  timeout -k 10 400 python benchmarks/configs.py --which lbfgs lbfgsb > $O/configs_$rep.log 2>&1 || { tail -20 $O/configs_$rep.log; exit 1; }
  grep '^{' $O/configs_$rep.log | python -c 'import json,sys
for l in sys.stdin: d=json.loads(l); print(d["config"], round(d["value"],1), d.get("nfev"))'
done
