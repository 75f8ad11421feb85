#!/bin/bash
# Round 6: reference anchors on this tree -- the GD benchmark (tests/smf_example/benchmark.py
# equivalent) at 1e4 / 1e6 / 1e8 halos (1 GPU, and 1e8 over 3 processes sharing the GPU),
# the quick-start L-BFGS-B at 1 and 3 ranks; rocprof kernel stats of the 1e8 GD run.
set -o pipefail
O=gpurun_out/r6_anchors
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_smf2_gpu.py tests/test_engine_cache_gpu.py \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for n in 10000 1000000 100000000; do
  for rep in 1 2; do
  timeout -k 10 300 python benchmarks/smf_gd_benchmark.py --num-halos $n --num-steps 1000 > $O/gd_${n}_$rep.log 2>&1 || { tail -20 $O/gd_${n}_$rep.log; exit 1; }
  echo "gd $n $rep $(grep '^{' $O/gd_${n}_$rep.log | cut -c1-110)"
  done
done
timeout -k 10 300 python benchmarks/smf_gd_benchmark.py --num-halos 100 --num-steps 100 > $O/gd_ref100.log 2>&1 || { tail -20 $O/gd_ref100.log; exit 1; }
timeout -k 10 300 python benchmarks/bfgs_anchor.py > $O/bfgs_1.log 2>&1 || { tail -20 $O/bfgs_1.log; exit 1; }
grep '^{' $O/bfgs_1.log | cut -c1-300
port=$(python3 -c "import socket;s=socket.socket();s.bind(('127.0.0.1',0));print(s.getsockname()[1])")
HSA_ENABLE_IPC_MODE_LEGACY=0 MULTIGRAD_DEVICE_COMM=0 OMP_NUM_THREADS=1 timeout -k 10 300 \
  python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=3 --master-addr 127.0.0.1 --master-port $port \
  benchmarks/bfgs_anchor.py > $O/bfgs_3.log 2>&1 || { tail -20 $O/bfgs_3.log; exit 1; }
grep '^{' $O/bfgs_3.log | cut -c1-300
port=$(python3 -c "import socket;s=socket.socket();s.bind(('127.0.0.1',0));print(s.getsockname()[1])")
HSA_ENABLE_IPC_MODE_LEGACY=0 MULTIGRAD_DEVICE_COMM=0 OMP_NUM_THREADS=1 timeout -k 10 300 \
  python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=3 --master-addr 127.0.0.1 --master-port $port \
  benchmarks/smf_gd_benchmark.py --num-halos 100000000 --num-steps 1000 > $O/gd_3ranks_1e8.log 2>&1 || { tail -20 $O/gd_3ranks_1e8.log; exit 1; }
grep '^{' $O/gd_3ranks_1e8.log | cut -c1-200
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_1e8 -o run -- python benchmarks/smf_gd_benchmark.py --num-halos 100000000 --num-steps 1000 > $O/prof_1e8.log 2>&1 || { tail -20 $O/prof_1e8.log; exit 1; }
find $O/prof_1e8 -name "*kernel_stats.csv" -exec head -4 {} \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_1e4 -o run -- python benchmarks/smf_gd_benchmark.py --num-halos 10000 --num-steps 1000 > $O/prof_1e4.log 2>&1 || { tail -20 $O/prof_1e4.log; exit 1; }
find $O/prof_1e4 -name "*kernel_stats.csv" -exec head -3 {} \;
