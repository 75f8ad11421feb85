#!/bin/bash
# Round 5: hashed N=2 with the lanes layout chosen by bench.py (2 processes on one GPU):
# the autotune-fault tests, then the full-size bench with the auto layout and with tiles.
set -o pipefail
O=gpurun_out/r5_hashed2
mkdir -p $O
timeout -k 10 900 python -u -m pytest "tests/test_twoshot_gpu.py::test_autotune_drops_timed_out_candidate_and_bench_reports_it" \
  "tests/test_twoshot_gpu.py::test_autotune_falls_back_to_rccl_when_no_peer_schedule_survives" -m gpu -x -v \
  --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
export MULTIGRAD_DEVICE_COMM=0 MULTIGRAD_PROGRESS=0
for lay in auto tiles; do
  timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 \
    --master-port 29611 bench.py --gpus 2 --steps 50 --warmup 5 --placement hashed --layout $lay --no-count-launches \
    > $O/bench_$lay.json 2> $O/bench_$lay.err || { tail -30 $O/bench_$lay.err; exit 1; }
  python -c "import json; d=[json.loads(l) for l in open('$O/bench_$lay.json') if l.startswith('{')][-1]; c=d['config']; print('$lay', d['value'], d['ms_per_step'], c['layout'], c['grad_collective'], c.get('autotune',{}).get('chosen'))"
done
