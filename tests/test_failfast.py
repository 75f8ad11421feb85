"""Fail-fast across ranks: an exception on one rank of a multi-rank fit ends
every rank promptly with an error instead of leaving the peers blocked in a collective
until the process-group timeout (reference worker loop multigrad/bfgs.py:96-106 only
guards against an unknown command).  Also: the device L-BFGS-B loop carries the per-step
hooks (MULTIGRAD_METRICS / MULTIGRAD_CHECK_EVERY)."""
import json
import os
import time

import numpy as np
import torch

import multigrad_amd as mg
from multigrad_amd.parallel import comm as C

from distributed import run_distributed


class _Quad(mg.OnePointModel):
    """Sum-of-squares model whose sumstats are all-reduced; rank ``fail_rank`` raises on its
    ``fail_at``-th evaluation (before the sumstat all-reduce, so the peers are inside it)."""

    def calc_partial_sumstats_from_params(self, params, randkey=None):
        d = self.aux_data
        d["n"] = d.get("n", 0) + 1
        if d.get("fail_rank") == self.comm.rank and d["n"] == d.get("fail_at"):
            raise ValueError(f"injected failure at evaluation {d['n']}")
        return (torch.as_tensor(params) - d["target"]) ** 2

    def calc_loss_from_sumstats(self, sumstats, sumstats_aux=None, randkey=None):
        return sumstats.sum()


def _fail_body(rank, size, method, fail_rank, fail_at):
    os.environ["MULTIGRAD_TIMEOUT"] = "600"
    m = _Quad(aux_data={"target": torch.tensor([1.0, -2.0, 0.5]), "fail_rank": fail_rank,
                        "fail_at": fail_at})
    t0 = time.perf_counter()
    try:
        if method == "adam":
            m.run_adam(torch.zeros(3), nsteps=50, learning_rate=0.05)
        else:
            m.run_bfgs(torch.zeros(3), maxsteps=50, method=method)
        return ("ok", "", time.perf_counter() - t0)
    except Exception as e:  # noqa: BLE001
        return (type(e).__name__, str(e)[:200], time.perf_counter() - t0)


def _check(res, fail_rank):
    for r, (kind, msg, dt) in enumerate(res):
        assert kind != "ok", res
        assert dt < 30.0, res
        if r == fail_rank:
            assert kind == "ValueError" and "injected failure at evaluation 3" in msg, res


def test_root_objective_failure_ends_every_rank_scipy():
    """Root-driven scipy L-BFGS-B: the root's objective raises at evaluation 3 while the
    workers are inside the sumstat all-reduce; both ranks end within 30 s with an error."""
    _check(run_distributed(_fail_body, 2, "scipy", 0, 3, timeout=120), 0)


def test_worker_objective_failure_ends_every_rank_scipy():
    _check(run_distributed(_fail_body, 2, "scipy", 1, 3, timeout=120), 1)


def test_objective_failure_ends_every_rank_device_lbfgs():
    _check(run_distributed(_fail_body, 2, "device", 1, 3, timeout=120), 1)


def test_objective_failure_ends_every_rank_adam():
    _check(run_distributed(_fail_body, 2, "adam", 0, 3, timeout=120), 0)


class _Boom(Exception):
    pass


def _abort_between_evals(rank, size):
    """The root fails between evaluations (in a scipy callback): the workers leave their
    command loop with RootAborted carrying the root's message."""
    from multigrad_amd.optim import bfgs as B
    comm = mg.get_world_comm()
    target = torch.tensor([1.0, 2.0])
    calls = [0]

    def lg(p):
        s = ((p - target) ** 2).clone()
        comm.all_reduce(s)
        return s.sum(), 2 * (p - target) * size

    orig = B.StepHooks

    class Hooks(orig):
        active = True

        def __call__(self, step, *a, **k):
            calls[0] += 1
            if calls[0] == 2:
                raise _Boom("callback failure")

    B.StepHooks = Hooks
    t0 = time.perf_counter()
    try:
        B.run_bfgs(lg, torch.zeros(2), maxsteps=20, comm=comm)
        return ("ok", "", 0.0)
    except Exception as e:  # noqa: BLE001
        return (type(e).__name__, str(e)[:200], time.perf_counter() - t0)
    finally:
        B.StepHooks = orig


def test_root_failure_between_evaluations_sends_abort():
    res = run_distributed(_abort_between_evals, 2, timeout=120)
    assert res[0][0] == "_Boom", res
    assert res[1][0] == "RootAborted" and "callback failure" in res[1][1], res
    assert all(dt < 30.0 for _, _, dt in res)


def test_device_lbfgsb_carries_step_hooks(tmp_path, monkeypatch):
    from multigrad_amd.optim import lbfgsb as LB
    C.set_world_comm(None)
    path = tmp_path / "m.jsonl"
    monkeypatch.setenv("MULTIGRAD_METRICS", str(path))
    monkeypatch.setenv("MULTIGRAD_CHECK_EVERY", "1")
    target = torch.tensor([0.3, -0.7, 2.0, 5.0])

    def lg(p):
        return ((p - target) ** 2).sum(), 2 * (p - target)

    res = LB.run_lbfgsb_device(lg, torch.zeros(4), maxsteps=20,
                               param_bounds=[(-1, 1), (-1, 1), (None, 1.5), (None, None)])
    np.testing.assert_allclose(res.x, [0.3, -0.7, 1.5, 5.0], atol=1e-5)
    recs = [json.loads(line) for line in path.read_text().splitlines()]
    assert len(recs) == res.nit and all("loss" in r and "nfev" in r for r in recs)
    assert [r["step"] for r in recs] == list(range(res.nit))
