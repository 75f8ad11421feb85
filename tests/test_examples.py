"""Every example and benchmark script runs end to end on the CPU with small inputs (one
process; the 2-rank launches are covered by test_bench_contract.py)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [
    ("examples/hierarchical_groups.py", []),
    ("examples/parallel_sum_demo.py", []),
    ("examples/quickstart_bfgs.py", []),
    ("examples/smf_grad_descent.py", ["--num-halos", "2000", "--num-steps", "20"]),
    ("benchmarks/bfgs_anchor.py", []),
    ("benchmarks/smf_gd_benchmark.py", ["--num-halos", "2000", "--num-steps", "10"]),
    ("benchmarks/configs.py", ["--which", "toy", "--steps", "20"]),
    ("benchmarks/scaling_sweep.py", ["--slurm", "--out", "{tmp}"]),
]


@pytest.mark.parametrize("script,args", CASES, ids=[c[0] for c in CASES])
def test_script_runs(tmp_path, script, args):
    env = dict(os.environ, MULTIGRAD_PROGRESS="0", OMP_NUM_THREADS="2",
               HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="", MPLBACKEND="Agg")
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    args = [a.replace("{tmp}", str(tmp_path)) for a in args]
    r = subprocess.run([sys.executable, os.path.join(ROOT, script)] + args, cwd=str(tmp_path),
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
