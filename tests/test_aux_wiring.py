"""The aux subsystems wired into the drivers: each environment
knob is set and its effect observed -- MULTIGRAD_CHECK_EVERY (bitwise rank agreement of
the parameters), MULTIGRAD_METRICS (JSONL per step from every driver),
MULTIGRAD_FINGERPRINT (collective signature cross-check), the sharded checkpoint commit
manifest, the 2-"node" split_subcomms_by_node, and bench.py's self-launch of N ranks."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import multigrad_amd as mg
from multigrad_amd.parallel import comm as C
from multigrad_amd.utils import checkpoint as ckpt
from multigrad_amd.utils import debug

from distributed import run_distributed

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ------------------------------------------------------------------ MULTIGRAD_CHECK_EVERY
def _check_every_body(rank, size, diverge):
    os.environ["MULTIGRAD_CHECK_EVERY"] = "2"
    from multigrad_amd.optim.adam import run_adam
    comm = mg.get_world_comm()
    target = torch.tensor([1.0, -2.0, 0.5])

    def lg(p, _):
        g = 2 * (p - target)
        if diverge and rank == 1:
            g = g * 1.5  # a rank whose gradient was never summed: parameters drift apart
        return ((p - target) ** 2).sum(), g

    try:
        run_adam(lg, torch.zeros(3), None, nsteps=6, learning_rate=0.1, comm=comm)
        return "ok"
    except debug.CollectiveMismatch as e:
        return "mismatch: " + str(e)[:40]


def test_check_every_detects_rank_divergence():
    ok = run_distributed(_check_every_body, 2, False)
    assert ok == ["ok", "ok"]
    bad = run_distributed(_check_every_body, 2, True)
    assert all(r.startswith("mismatch") and "after step 1" in r for r in bad), bad


# ------------------------------------------------------------------ MULTIGRAD_METRICS
def test_metrics_env_installs_logger_in_every_driver(tmp_path, monkeypatch):
    from multigrad_amd.models.toy import SumOfSquaresModel, make_toy_data
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    C.set_world_comm(None)
    path = tmp_path / "metrics.jsonl"
    monkeypatch.setenv("MULTIGRAD_METRICS", str(path))
    m = SumOfSquaresModel(aux_data=make_toy_data(ndim=3, npoints=20))
    m.run_adam(torch.zeros(3), nsteps=3, learning_rate=0.1)
    m.run_simple_grad_descent(torch.zeros(3), nsteps=2, learning_rate=0.01)
    m.run_bfgs(torch.zeros(3), maxsteps=3, method="device")
    n_generic = len(path.read_text().splitlines())
    data = make_population_data(400, 4000, seed=3, device=torch.device("cpu"))
    pm = PopulationSMFModel(aux_data=data)
    pm.set_target_from_truth()
    pm.run_adam(data["guess"], nsteps=2, learning_rate=1e-3)
    recs = [json.loads(line) for line in path.read_text().splitlines()]
    assert n_generic >= 3 + 2 + 1
    assert len(recs) == n_generic + 2
    assert all("step" in r and "loss" in r and "step_time_s" in r for r in recs)
    assert [r["step"] for r in recs[:3]] == [0, 1, 2]
    assert all(r["grad_norm"] > 0 for r in recs[:3])          # generic Adam
    assert all(r.get("comm_bytes") == 0 for r in recs[-2:])    # engine, one rank


def _engine_metrics(rank, size, path):
    os.environ["MULTIGRAD_METRICS"] = path
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    comm = mg.get_world_comm()
    data = make_population_data(400, 4000, seed=3, comm=comm, device=torch.device("cpu"))
    pm = PopulationSMFModel(aux_data=data, comm=comm)
    pm.set_target_from_truth()
    pm.run_adam(data["guess"], nsteps=3, learning_rate=1e-3)
    return rank


def test_engine_metrics_report_collective_bytes(tmp_path):
    """Two ranks, hashed placement (dense gradient): every record carries the bytes the
    rank sent through collectives in the step and the effective rate."""
    path = str(tmp_path / "m.jsonl")
    run_distributed(_engine_metrics, 2, path)
    recs = [json.loads(line) for line in open(path).read().splitlines()]
    assert len(recs) == 3
    # 10 sumstats + 2 (W-1)/W of the padded 400-vector, fp32
    assert all(r["comm_bytes"] >= 4 * (10 + 400) for r in recs)
    assert all(r["comm_GBps"] > 0 for r in recs)


# ------------------------------------------------------------------ MULTIGRAD_FINGERPRINT
def _fingerprint_body(rank, size):
    os.environ["MULTIGRAD_FINGERPRINT"] = "1"
    C.set_world_comm(C._wrap_default_group())
    comm = mg.get_world_comm()
    wrapped = isinstance(comm, debug.CollectiveFingerprint)
    t = torch.ones(2)
    comm.all_reduce(t)
    sub = comm.split(0)
    sub_wrapped = isinstance(sub, debug.CollectiveFingerprint)
    try:
        comm.all_reduce(torch.ones(2 + rank))
        caught = False
    except debug.CollectiveMismatch:
        caught = True
    return wrapped, sub_wrapped, float(t[0]), caught


def test_fingerprint_env_wraps_world():
    res = run_distributed(_fingerprint_body, 2)
    assert all(r == (True, True, 2.0, True) for r in res), res


# ------------------------------------------------------------------ checkpoint commit
def _ckpt_body(rank, size, path):
    import glob
    comm = mg.get_world_comm()
    ckpt.save_optimizer_state(path, {"step": 5, "size": size, "x": torch.ones(2) * rank},
                              comm=comm, sharded=True)
    st = ckpt.load_optimizer_state(path, rank=rank, sharded=True, comm=comm)
    ckpt.check_loaded_step(st["step"], comm)
    # an interrupted later checkpoint: rank 1 wrote its step-9 shard, the manifest was not
    # committed -- the committed step-5 shards are untouched and still load everywhere
    comm.barrier()
    if rank == 1:
        torch.save({"step": 9, "size": size}, ckpt.shard_path(path, 1, 9))
    comm.barrier()
    st2 = ckpt.load_optimizer_state(path, rank=rank, sharded=True, comm=comm)
    survived = st2["step"] == 5 and float(st2["x"][0]) == float(rank)
    # a committed step whose shard is damaged on rank 1 only: EVERY rank raises
    comm.barrier()
    ckpt.save_optimizer_state(path, {"step": 7, "size": size, "x": torch.ones(2) * rank},
                              comm=comm, sharded=True)
    old = sorted(glob.glob(path + f".step[59].rank{rank}"))  # superseded shards removed
    comm.barrier()
    if rank == 1:
        torch.save({"step": 6, "size": size}, ckpt.shard_path(path, 1, 7))
    comm.barrier()
    try:
        ckpt.load_optimizer_state(path, rank=rank, sharded=True, comm=comm)
        torn = False
    except ckpt.CheckpointMismatch as e:
        torn = "rank(s) [1]" in str(e)
    try:
        ckpt.check_loaded_step(5 + rank, comm)
        skew = False
    except ckpt.CheckpointMismatch:
        skew = True
    return float(st["x"][0]), survived, old, torn, skew


def test_sharded_checkpoint_manifest(tmp_path):
    path = str(tmp_path / "opt.pt")
    res = run_distributed(_ckpt_body, 2, path)
    for r, (x, survived, old, torn, skew) in enumerate(res):
        assert x == float(r) and survived and old == [] and torn and skew, res
    man = json.loads(open(ckpt.manifest_path(path)).read())
    assert man == {"step": 7, "size": 2, "sharded": True, "shards": "opt.pt.step7.rank{rank}"}


def _ckpt_broken_body(rank, size, path, kind):
    import pickle
    comm = mg.get_world_comm()
    ckpt.save_optimizer_state(path, {"step": 3, "size": size, "x": torch.ones(2)},
                              comm=comm, sharded=True)
    comm.barrier()
    if rank == 1:
        fn = ckpt.shard_path(path, 1, 3)
        if kind == "empty":  # truncated to zero bytes (EOFError / RuntimeError in torch.load)
            open(fn, "wb").close()
        else:  # a plain pickle of a non-weights object: weights_only refuses it
            with open(fn, "wb") as f:
                pickle.dump(_ckpt_broken_body, f)
    comm.barrier()
    try:
        ckpt.load_optimizer_state(path, rank=rank, sharded=True, comm=comm)
        return "loaded"
    except ckpt.CheckpointMismatch as e:
        return "rank(s) [1]" in str(e)


@pytest.mark.parametrize("kind", ["empty", "pickle"])
def test_sharded_checkpoint_broken_shard_raises_everywhere(tmp_path, kind):
    """Any failure of one rank's shard load (not only the anticipated exception types)
    reaches the collective verdict: every rank raises instead of the healthy ones hanging."""
    path = str(tmp_path / "opt.pt")
    res = run_distributed(_ckpt_broken_body, 2, path, kind, timeout=120)
    assert res == [True, True], res


# ------------------------------------------------------------------ two "nodes"
def _nodes_body(rank, size):
    os.environ["MULTIGRAD_NODE_NAME"] = "nodeB" if rank % 2 else "nodeA"
    sub, nnodes, node = mg.split_subcomms_by_node()
    t = torch.tensor([float(rank)])
    sub.all_reduce(t)
    return nnodes, node, sub.size, sub.rank, float(t[0]), sub.name


def test_split_subcomms_by_node_two_nodes():
    res = run_distributed(_nodes_body, 4)
    assert [r[:4] for r in res] == [(2, 0, 2, 0), (2, 1, 2, 0), (2, 0, 2, 1), (2, 1, 2, 1)]
    assert [r[4] for r in res] == [2.0, 4.0, 2.0, 4.0]  # ranks {0,2} on A, {1,3} on B


# ------------------------------------------------------------------ bench self-launch
def test_bench_self_launches_n_ranks():
    env = dict(os.environ, MULTIGRAD_PROGRESS="0", OMP_NUM_THREADS="1",
               MULTIGRAD_DEVICE_COMM="0", HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--params", "2000",
                        "--halos", "20000", "--steps", "3", "--warmup", "1"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = lines[0]
    assert rec["n_gpus"] == 2 and rec["value"] > 0
    # value: the hashed input re-partitioned by parameter owner at setup (one all-to-all-v)
    assert rec["config"]["placement"].startswith("owner (re-partitioned")
    assert rec["config"]["optimizer_sharding"] == "owner"
    assert rec["repartition"]["halos_after"] > 0 and rec["repartition"]["total_s"] >= 0
    # dense_steps_per_s: the same input, dense gradient summed across ranks every step
    assert rec["dense_steps_per_s"] > 0
    assert rec["dense_config"]["optimizer_sharding"] == "zero1"
    assert rec["dense_config"]["loss_last"] == pytest.approx(rec["loss_last"], rel=1e-4)


def test_bench_launcher_parent_is_gpu_free():
    """The parent that starts the ranks imports no torch (so it cannot initialise HIP) and
    counts GPUs from the environment / sysfs."""
    code = ("import sys, bench\n"
            "seen = []\n"
            "class R: returncode = 0\n"
            "bench.subprocess.run = lambda cmd, env=None: (seen.append(cmd), R)[1]\n"
            "rc = bench.main(['--gpus', '2', '--steps', '1'])\n"
            "assert rc == 0 and seen and 'torch.distributed.run' in seen[0], seen\n"
            "assert 'torch' not in sys.modules, 'launcher imported torch'\n"
            "import os\n"
            "os.environ['HIP_VISIBLE_DEVICES'] = '0,1,2'\n"
            "assert bench.visible_gpus() == 3\n"
            "print('ok')\n")
    env = dict(os.environ, HIP_VISIBLE_DEVICES="0,1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr[-2000:]
