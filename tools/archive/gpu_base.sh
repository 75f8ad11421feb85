set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/base
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/base/bench.log 2>&1
timeout -k 10 300 python -u tools/uncached_theta_bench.py > gpurun_out/base/proxy8.log 2>&1
