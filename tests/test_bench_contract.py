"""The driver's bench.py contract on CPU: one JSON line with the required keys, at 1 rank
and at 2 gloo ranks launched by torch.distributed.run (owner and hashed placements)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
        "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"}
ARGS = ["--params", "2000", "--halos", "20000", "--steps", "3", "--warmup", "1"]


def _env():
    env = dict(os.environ, MULTIGRAD_PROGRESS="0", OMP_NUM_THREADS="1",
               MULTIGRAD_DEVICE_COMM="0", HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    return env


def _json_lines(out: str):
    return [json.loads(line) for line in out.splitlines() if line.startswith("{")]


def test_bench_single_rank_json():
    r = subprocess.run([sys.executable, "bench.py"] + ARGS + ["--profile-phases"], cwd=ROOT,
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    rec = lines[0]
    assert KEYS <= set(rec)
    assert rec["n_gpus"] == 1 and rec["steps"] == 3 and rec["warmup"] == 1
    assert rec["value"] > 0 and rec["higher_is_better"] is True
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(rec["config"])
    assert set(rec["phases_ms"]) >= {"forward", "loss", "vjp", "adam"}


@pytest.mark.parametrize("placement", ["owner", "hashed"])
def test_bench_two_ranks_json(placement):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(29400 + os.getpid() % 500),
           "bench.py", "--gpus", "2", "--placement", placement] + ARGS
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    rec = lines[0]
    assert KEYS <= set(rec) and rec["n_gpus"] == 2
    assert rec["config"]["placement"] == placement
    assert rec["config"]["optimizer_sharding"] == ("owner" if placement == "owner" else "zero1")


def test_extra_placement_failure_keeps_the_headline():
    """A failure of the extra (owner) placement is reported in the record's errors; a
    failure of the headline placement still ends the run."""
    import bench

    def timed(p):
        if p == "owner":
            raise MemoryError("out of device memory")
        return {"steps_per_s": 1.0}

    released = []
    res, errors = bench.run_placements(["hashed", "owner"], timed,
                                       on_error=lambda: released.append(True))
    assert res == {"hashed": {"steps_per_s": 1.0}}
    assert errors["owner"].startswith("MemoryError: out of device memory")
    assert released == [True]

    def broken(p):
        raise RuntimeError("headline failed")

    with pytest.raises(RuntimeError):
        bench.run_placements(["hashed", "owner"], broken)
