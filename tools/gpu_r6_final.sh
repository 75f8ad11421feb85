#!/bin/bash
# Round 6, final tree: the whole GPU suite + smoke, the GD benchmark at 1e6, the default bench.
set -o pipefail
O=gpurun_out/r6_final2
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
grep -E "FAILED|ERROR" $O/pytest.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for rep in 1 2; do
  timeout -k 10 300 python benchmarks/smf_gd_benchmark.py --num-halos 1000000 --num-steps 1000 > $O/gd_1e6_$rep.log 2>&1 || { tail -20 $O/gd_1e6_$rep.log; exit 1; }
  grep '^{' $O/gd_1e6_$rep.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print("gd 1e6", round(d["value"],1))'
done
timeout -k 10 300 python bench.py --steps 300 --warmup 10 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['value'], d['ms_per_step'])"
