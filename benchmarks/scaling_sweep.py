"""Scaling sweep of bench.py over 1, 2, 4, 8 GPUs of one node (the reference's
submit_benchmark_jobs.py submitted 1..10-node SLURM jobs; here one node, one process per
GPU over RCCL/xGMI).  Writes one JSON line per GPU count and the strong-scaling
efficiency value_N / (N * value_1).

    python benchmarks/scaling_sweep.py --gpus 1 2 4 8 --steps 50 --warmup 5 --out scale.jsonl
    python benchmarks/scaling_sweep.py --slurm --nodes 1 2 4 ...   (writes sbatch scripts only)
"""
import argparse
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run(n, steps, warmup, extra):
    if n == 1:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()),
               os.path.join(ROOT, "bench.py"), "--gpus", str(n)]
    cmd += ["--steps", str(steps), "--warmup", str(warmup)] + list(extra)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    p = subprocess.run(cmd, capture_output=True, text=True, env=env)
    for line in p.stdout.splitlines():
        if line.startswith("{"):
            return json.loads(line)
    raise RuntimeError(f"bench failed on {n} GPUs:\n{p.stdout[-2000:]}\n{p.stderr[-4000:]}")


def sbatch(nodes, gpus_per_node, steps, account, partition):
    return f"""#!/bin/bash
#SBATCH --job-name=multigrad_amd_{nodes}n
#SBATCH --nodes={nodes}
#SBATCH --ntasks-per-node={gpus_per_node}
#SBATCH --gpus-per-node={gpus_per_node}
#SBATCH --time=00:10:00
{f'#SBATCH --account={account}' if account else ''}
{f'#SBATCH --partition={partition}' if partition else ''}
export MASTER_ADDR=$(scontrol show hostnames $SLURM_NODELIST | head -n1)
export MASTER_PORT=29531 HSA_ENABLE_IPC_MODE_LEGACY=0
srun python {os.path.join(ROOT, 'bench.py')} --gpus $SLURM_NTASKS --steps {steps}
"""


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", nargs="+", type=int, default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--out", default=None)
    ap.add_argument("--slurm", action="store_true", help="write sbatch scripts instead of running")
    ap.add_argument("--nodes", nargs="+", type=int, default=[1, 2, 4])
    ap.add_argument("--account", default=None)
    ap.add_argument("--partition", default=None)
    a, extra = ap.parse_known_args(argv)
    if a.slurm:
        for n in a.nodes:
            path = f"multigrad_amd_scaling_{n}n.sbatch"
            with open(path, "w") as f:
                f.write(sbatch(n, 8, a.steps, a.account, a.partition))
            print(path)
        return
    base = None
    for n in a.gpus:
        r = run(n, a.steps, a.warmup, extra)
        base = r["value"] if n == 1 else base
        if base:
            r["strong_scaling_efficiency"] = r["value"] / (n * base)
        print(json.dumps(r), flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
