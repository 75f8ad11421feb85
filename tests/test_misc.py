"""In-graph GD (mpi4jax variant), tree utilities, launcher, alias package, metrics,
profiling and the distributed debug aids."""
import json
import os

import numpy as np
import pytest
import torch

import multigrad_amd as mg
from multigrad_amd import ingraph
from multigrad_amd.parallel import comm as C
from multigrad_amd.utils import debug, metrics, profiling, tree, util

from distributed import run_distributed


def _lg(d, p):
    return ((p - d["t"]) ** 2).sum(), 2 * (p - d["t"])


def test_ingraph_gd_matches_simple_gd():
    C.set_world_comm(None)
    d = {"t": torch.tensor([1.0, -2.0, 0.5])}
    df = ingraph.simple_grad_descent(d, _lg, [0.0, 0.0, 0.0], learning_rate=0.1, nsteps=15)
    ref = util.simple_grad_descent(lambda p: ((p - d["t"]) ** 2).sum(), [0.0, 0.0, 0.0], 15, 0.1)
    assert list(df.columns) == ["loss", "params"] and len(df) == 15
    np.testing.assert_allclose(np.stack(df["params"].values), ref.params.numpy(), rtol=1e-6)
    np.testing.assert_allclose(df["loss"].values, ref.loss.numpy(), rtol=1e-6)


def _ingraph_body(rank, size):
    data = torch.arange(12.0)
    mine = ingraph.distribute_data(data)
    # partial loss sum_i (p - x_i)^2 over this rank's data; reduce_sum sums over ranks
    df = ingraph.simple_grad_descent(
        {"x": mine}, lambda d, p: (((p - d["x"]) ** 2).sum(), (2 * (p - d["x"])).sum().reshape(1)),
        [0.0], learning_rate=0.01, nsteps=50)
    return mine.tolist(), float(df["params"].values[-1][0]), float(ingraph.reduce_sum(torch.ones(2))[0])


def test_ingraph_multi_rank():
    res = run_distributed(_ingraph_body, 3)
    assert [r[0] for r in res] == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9, 10, 11]]
    assert all(r[1] == pytest.approx(res[0][1]) for r in res)
    assert res[0][1] == pytest.approx(5.5, abs=0.05)  # converging to the global mean
    assert all(r[2] == 3.0 for r in res)


def test_tree_utils():
    # forest: 0 <- 1 <- 2 <- 3 ; 4 <- 5 ; 6 (self roots: 0, 4, 6)
    parent = np.array([0, 0, 1, 2, 4, 4, 6])
    np.testing.assert_array_equal(tree.find_ultimate_top_indices(parent), [0, 0, 0, 0, 4, 4, 6])
    t = tree.find_ultimate_top_indices(torch.as_tensor(parent))
    assert isinstance(t, torch.Tensor)
    deep = np.arange(-1, 999)  # chain of depth 1000 rooted at 0
    deep[0] = 0
    assert (tree.find_ultimate_top_indices(deep) == 0).all()
    with pytest.raises(RecursionError):
        tree.find_ultimate_top_indices(deep, max_recursion=3)
    # sorting arrays by ultimate host keeps each forest contiguous and remaps indices
    dump = np.array([4, 0, 4, 1, 4, 0])
    vals = np.array([10, 11, 12, 13, 14, 15])
    (sv,), (ri,) = tree.sort_all_by_ultimate_top_dump(dump, [vals], [dump])
    tops = tree.find_ultimate_top_indices(dump)
    order = np.argsort(tops, kind="stable")
    np.testing.assert_array_equal(sv, vals[order])
    inv = np.argsort(order)
    np.testing.assert_array_equal(ri, inv[dump][order])


def test_launcher_command():
    from multigrad_amd import launch
    cmd = launch.build_command(8, "bench.py", ["--gpus", "8"], 29555)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "127.0.0.1" in cmd and cmd[-3:] == ["bench.py", "--gpus", "8"]


def test_multigrad_alias_package():
    import multigrad
    from multigrad.util import GradDescentResult, simple_grad_descent  # noqa: F401
    from multigrad.adam import run_adam, init_randkey  # noqa: F401
    from multigrad.bfgs import run_bfgs  # noqa: F401
    from multigrad.mpi4jax import distribute_data  # noqa: F401
    assert multigrad.OnePointModel is mg.OnePointModel
    assert multigrad.reduce_sum is mg.reduce_sum
    # the reference's per-module progress helpers (multigrad/adam.py:28-36, bfgs.py:21-29,
    # multigrad.py:37-45, util.py:39-47)
    import multigrad.adam as ma
    import multigrad.bfgs as mb
    import multigrad.multigrad as mm
    import multigrad.util as mu
    for mod, pick in ((ma, "adam_trange"), (mb, "bfgs_trange"), (mm, "trange"), (mu, "trange")):
        assert list(mod.trange_no_tqdm(3)) == [0, 1, 2]
        assert callable(mod.trange_with_tqdm)
        assert len(list(getattr(mod, pick)(4))) == 4
        assert (mod.RANK, mod.N_RANKS) == (mg.RANK, mg.N_RANKS)


def test_metrics_and_profiling(tmp_path):
    C.set_world_comm(None)
    path = str(tmp_path / "m.jsonl")
    cb = metrics.metrics_callback(path)
    from multigrad_amd.models.toy import SumOfSquaresModel, make_toy_data
    m = SumOfSquaresModel(aux_data=make_toy_data(ndim=3, npoints=20))
    m.run_adam(torch.zeros(3), nsteps=4, learning_rate=0.1, callback=cb)
    recs = [json.loads(l) for l in open(path)]
    assert [r["step"] for r in recs] == [0, 1, 2, 3] and all("loss" in r for r in recs)
    t = profiling.PhaseTimer(enabled=True)
    with t.phase("a"):
        torch.ones(10).sum()
    assert "a" in t.summary()


def _consistency_body(rank, size):
    comm = mg.get_world_comm()
    debug.check_consistent(torch.ones(3), comm)
    try:
        debug.check_consistent(torch.ones(3) * rank, comm)
        raised = False
    except debug.CollectiveMismatch:
        raised = True
    fp = debug.CollectiveFingerprint(comm)
    fp.all_reduce(torch.ones(2))
    try:
        fp.all_reduce(torch.ones(2 + rank))  # shape differs across ranks -> caught, no hang
        mismatch = False
    except debug.CollectiveMismatch:
        mismatch = True
    return raised, mismatch


def test_debug_aids_detect_divergence():
    res = run_distributed(_consistency_body, 2)
    assert all(r == (True, True) for r in res)


def test_stable_population_sort_chunked_matches_one_sort():
    """Shards beyond torch.sort's INT_MAX limit are sorted in chunks and placed by a stable
    counting sort: the same order, ids and counts as one stable sort."""
    from multigrad_amd.ops.smf import stable_population_sort
    g = torch.Generator().manual_seed(0)
    for n, npop, chunk in [(10000, 37, 1000), (12345, 5000, 999), (5000, 3, 5000), (7, 100, 2)]:
        pop = torch.randint(0, npop, (n,), generator=g, dtype=torch.int32)
        spop, order, counts = stable_population_sort(pop, npop, chunk=chunk)
        ref_s, ref_o = torch.sort(pop, stable=True)
        assert torch.equal(spop, ref_s) and torch.equal(order, ref_o)
        assert torch.equal(counts, torch.bincount(pop, minlength=npop))
