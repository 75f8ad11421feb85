"""Fused step of the shared-parameter SMF models (csrc/smf.hip "shared-parameter fused
step", engine/smf2.py) on the MI355X, against fp64 PyTorch oracles of the same math and
the reference's golden values (reference tests/test_mpi.py,
docs/source/notebooks/intro.ipynb:209-214)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from distributed import run_distributed  # noqa: E402

DEV = torch.device("cuda", 0)


def _oracle(model, params, S_at=None):
    """fp64 oracle at ``params`` (PyTorch autograd over every halo): the loss, the sumstats
    and the gradient J^T dl/dS.  ``S_at``: the sumstats the cotangent dl/dS is evaluated at
    (default: the oracle's own) -- near the target the loss is a small difference of logs,
    so fp32 sumstats (whose far-tail bins carry the absolute error of a float32 erf, as the
    reference's do) move the cotangent; with the kernel's sumstats the VJP itself is checked
    tightly."""
    from multigrad_amd.ops.smf import logmse_loss, smf_sumstats_reference
    shard, bins = model._setup()
    x = shard.x.double().cpu()
    th = torch.tensor(params, dtype=torch.float64)
    J = torch.autograd.functional.jacobian(
        lambda t: smf_sumstats_reference(t, x, None, bins, model._log_sigma), th)
    S = smf_sumstats_reference(th, x, None, bins, model._log_sigma)
    Sc = (S if S_at is None else torch.as_tensor(S_at, dtype=torch.float64)).clone().requires_grad_(True)
    loss = logmse_loss(Sc, model._target.double().cpu(), model._loss_eps)
    (gS,) = torch.autograd.grad(loss, Sc)
    return float(loss.detach()), (gS @ J).numpy(), S.numpy()


def assert_close_bins(S, S64, rtol, atol, where):
    bad = np.abs(S - S64) > rtol * np.abs(S64) + atol
    assert not bad.any(), (where, S, S64)


@pytest.mark.parametrize("schedule", ["loop", "grid"])
@pytest.mark.parametrize("which", ["test", "docs"])
def test_fused_evaluation_matches_fp64_oracle_across_sigma(schedule, which, monkeypatch):
    """Loss, gradient and sumstats of one fused evaluation against fp64 autograd for sigma
    from 0.11 to 0.6 (bin width 0.1: h = 0.91 .. 0.17 -- both the per-edge fallback above
    h = 0.7 and the four-term Euler-Maclaurin path below it, including h = 0.67 and 0.5)."""
    monkeypatch.setenv("MULTIGRAD_SMF2_SCHEDULE", schedule)
    import multigrad_amd.parallel.comm as C
    from multigrad_amd.models.smf import DocsSMFModel, MySMFModel, make_docs_data, make_test_data
    C.set_world_comm(None)
    n = 30_000 if schedule == "loop" else 300_000
    if which == "test":
        model = MySMFModel(aux_data=make_test_data(n), device=DEV)
        pts = [(-2.0, s) for s in (0.11, 0.13, 0.15, 0.18, 0.2, 0.25, 0.35, 0.5, 0.6)] + [(-1.7, 0.3)]
    else:
        model = DocsSMFModel(aux_data=make_docs_data(n), device=DEV)
        pts = [(-2.0, float(np.log10(s))) for s in (0.11, 0.14, 0.15, 0.19, 0.21, 0.3, 0.45, 0.6)]
    eng = model.fused_step_engine()
    assert eng is not None and eng.schedule == schedule
    ev = eng.evaluator()
    for p in pts:
        loss, grad = ev(torch.tensor(p))
        S = eng.S[:10].cpu().double().numpy()
        l64, g64, S64 = _oracle(model, p)
        # sumstats: 2e-5 relative, plus the absolute contract of the per-halo tails
        # (~2e-7 of one halo's unit mass per edge, the float32-erf class) in each bin
        _, bins = model._setup()
        atol = 4e-7 * n * np.asarray(bins.scale)
        assert_close_bins(S, S64, 2e-5, atol, p)
        # loss and VJP at the kernel's own sumstats: bins whose mass is a far Gaussian tail
        # (S ~ the docs model's eps = 1e-10 at sigma = 0.15) carry the absolute error of
        # the float32 contract -- the reference's 0.5 (1 + erf) returns exactly 0 there --
        # which a log-MSE magnifies without bound, so the loss is checked for the epilogue's
        # arithmetic and the sumstats above for the forward's contract
        lk, gk, _ = _oracle(model, p, S_at=S)   # the VJP at the kernel's own sumstats
        assert float(loss) == pytest.approx(lk, rel=1e-4, abs=1e-8), p
        if (S64 > 1e3 * (model._loss_eps + 1e-30)).all() and (S64 > 1e-7 * S64.max()).all():
            assert float(loss) == pytest.approx(l64, rel=2e-3, abs=5e-8), p
        np.testing.assert_allclose(grad.cpu().double().numpy(), gk, rtol=2e-4,
                                   atol=1e-6 * np.abs(gk).max(), err_msg=str(p))


@pytest.mark.parametrize("schedule", ["loop", "grid"])
def test_fused_gd_matches_eager_chain_rule(schedule, monkeypatch):
    """run_simple_grad_descent on the fused step against the reference's eager loop
    (autograd chain rule per step) on the same model: GradDescentResult contract (loss[i]
    at params[i], the last update not recorded)."""
    monkeypatch.setenv("MULTIGRAD_SMF2_SCHEDULE", schedule)
    import multigrad_amd.parallel.comm as C
    from multigrad_amd.models.smf import MySMFModel, ParamTuple, make_test_data
    from multigrad_amd.utils import util
    C.set_world_comm(None)
    model = MySMFModel(aux_data=make_test_data(20_000 if schedule == "loop" else 200_000),
                       device=DEV)
    guess = torch.tensor([-1.0, 0.5], device=DEV)
    res = model.run_simple_grad_descent(ParamTuple(-1.0, 0.5), nsteps=60, learning_rate=1e-3)
    ref = util.simple_grad_descent(None, guess=guess, nsteps=60, learning_rate=1e-3,
                                   loss_and_grad_func=model.calc_loss_and_grad_from_params)
    assert res.loss.shape == (60,) and res.params.shape == (60, 2)
    torch.testing.assert_close(res.params[0].cpu(), guess.cpu())
    np.testing.assert_allclose(res.loss.cpu().numpy(), ref.loss.cpu().numpy(), rtol=5e-4)
    np.testing.assert_allclose(res.params.cpu().numpy(), ref.params.cpu().numpy(), rtol=2e-5,
                               atol=2e-6)


@pytest.mark.parametrize("bounded", [False, True])
def test_fused_adam_matches_generic(bounded):
    import multigrad_amd.parallel.comm as C
    from multigrad_amd.models.smf import DocsSMFModel, make_docs_data
    C.set_world_comm(None)
    model = DocsSMFModel(aux_data=make_docs_data(), device=DEV)
    guess = torch.tensor([-3.5, 0.2], device=DEV)
    bounds = [(-4.0, -1.0), (None, 0.5)] if bounded else None
    traj = model.run_adam(guess, nsteps=80, learning_rate=0.02, param_bounds=bounds)
    ref = model.run_adam(guess, nsteps=80, learning_rate=0.02, param_bounds=bounds,
                         use_engine=False)
    assert traj.shape == (81, 2)
    np.testing.assert_allclose(traj.cpu().numpy(), ref.cpu().numpy(), rtol=2e-4, atol=2e-5)
    if bounded:
        t = traj.cpu().numpy()
        assert (t[:, 0] > -4.0).all() and (t[:, 0] < -1.0).all() and (t[:, 1] < 0.5).all()


def test_reference_golden_values_on_fused_step():
    """Appendix A: the test model's sumstats at the truth equal the reference target; GD
    from the truth stays there; the docs model's loss and gradient at truth + 0.1
    (intro.ipynb:212-214: 0.44032094, [2.6187496, 4.2603974]) and at the truth (0, 0)."""
    import multigrad_amd.parallel.comm as C
    from multigrad_amd.models.smf import (DocsSMFModel, MySMFModel, ParamTuple, TARGET_SUMSTATS,
                                          make_docs_data, make_test_data)
    C.set_world_comm(None)
    data = make_test_data()
    model = MySMFModel(aux_data=data, device=DEV)
    ev = model.fused_step_engine().evaluator()
    ev(torch.tensor([-2.0, 0.2]))
    np.testing.assert_allclose(model.fused_step_engine().S[:10].cpu().numpy(), TARGET_SUMSTATS,
                               rtol=5e-5, atol=1e-9)
    data["target_sumstats"] = model.calc_sumstats_from_params(ParamTuple(-2.0, 0.2)).cpu().numpy()
    model = MySMFModel(aux_data=data, device=DEV)
    gd = model.run_simple_grad_descent(ParamTuple(-2.0, 0.2), nsteps=2)
    assert float(gd.loss.abs().max()) < 1e-9
    np.testing.assert_allclose(gd.params[-1].cpu().numpy(), [-2.0, 0.2], atol=1e-6)
    docs = DocsSMFModel(aux_data=make_docs_data(), device=DEV)
    ev = docs.fused_step_engine().evaluator()
    loss, grad = ev(torch.tensor([-1.9, -0.4]))
    assert float(loss) == pytest.approx(0.44032094, rel=2e-5)
    np.testing.assert_allclose(grad.cpu().numpy(), [2.6187496, 4.2603974], rtol=1e-4)
    loss, grad = ev(torch.tensor([-2.0, -0.5]))
    assert abs(float(loss)) < 1e-10 and float(grad.abs().max()) < 1e-4


def test_step_cache_second_call_captures_nothing(monkeypatch):
    """The engine is cached on the model: the second run reuses buffers and graphs (zero
    captures); new data (aux_data) rebuilds it."""
    monkeypatch.setenv("MULTIGRAD_SMF2_SCHEDULE", "grid")
    import multigrad_amd.parallel.comm as C
    from multigrad_amd.models.smf import MySMFModel, ParamTuple, make_test_data
    C.set_world_comm(None)
    model = MySMFModel(aux_data=make_test_data(100_000), device=DEV)
    r1 = model.run_simple_grad_descent(ParamTuple(-1.0, 0.5), nsteps=40, learning_rate=1e-3)
    eng = model.fused_step_engine()
    caps = eng.stats["captures"]
    assert caps >= 1
    r2 = model.run_simple_grad_descent(ParamTuple(-1.0, 0.5), nsteps=40, learning_rate=1e-3)
    assert model.fused_step_engine() is eng and eng.stats["captures"] == caps
    assert torch.equal(r1.params, r2.params) and torch.equal(r1.loss, r2.loss)


def test_scipy_bfgs_on_fused_evaluator():
    import multigrad_amd.parallel.comm as C
    from multigrad_amd.models.smf import DocsSMFModel, make_docs_data
    C.set_world_comm(None)
    model = DocsSMFModel(aux_data=make_docs_data(), device=DEV)
    res = model.run_bfgs(torch.tensor([-3.5, 0.2]), method="scipy")
    np.testing.assert_allclose(res.x, [-2.0, -0.5], atol=2e-3)
    assert res.fun < 1e-8


def _ranks(rank, size, schedule):
    os.environ["MULTIGRAD_SMF2_SCHEDULE"] = schedule
    import multigrad_amd as mg
    from multigrad_amd.models.smf import DocsSMFModel, MySMFModel, ParamTuple, make_docs_data, make_test_data
    comm = mg.get_world_comm()
    n = 30_000 if schedule == "loop" else 300_000
    model = MySMFModel(aux_data=make_test_data(n, comm=comm), comm=comm, device=DEV)
    gd = model.run_simple_grad_descent(ParamTuple(-1.0, 0.5), nsteps=50, learning_rate=1e-3)
    eng = model.fused_step_engine()
    docs = DocsSMFModel(aux_data=make_docs_data(comm=comm), comm=comm, device=DEV)
    loss, grad = docs.fused_step_engine().evaluator()(torch.tensor([-1.9, -0.4]))
    return (gd.loss.cpu().numpy(), gd.params.cpu().numpy(), eng.schedule, eng.oneshot is not None,
            float(loss), grad.cpu().numpy())


@pytest.mark.parametrize("size,schedule", [(2, "loop"), (3, "loop"), (2, "grid"), (3, "grid")])
def test_fused_step_ranks_one_gpu_match_single_rank(size, schedule):
    """Halos array_split over 2 / 3 processes sharing the GPU (the exchange is the one-shot
    peer kernel inside the step): the single-rank fit, identical bits on every rank, and the
    intro.ipynb values at 3 ranks (reference :495-514 ran them on 3 MPI ranks)."""
    import multigrad_amd.parallel.comm as C
    C.set_world_comm(None)
    one = _ranks(0, 1, schedule)
    res = run_distributed(_ranks, size, schedule, timeout=600)
    for loss, params, sched, peer, l2, g2 in res:
        assert sched == schedule and peer
        np.testing.assert_allclose(loss, one[0], rtol=2e-5, atol=1e-9)
        np.testing.assert_allclose(params, one[1], rtol=1e-5, atol=1e-6)
        assert l2 == pytest.approx(0.44032094, rel=2e-5)
        np.testing.assert_allclose(g2, [2.6187496, 4.2603974], rtol=1e-4)
    for r in res[1:]:
        np.testing.assert_array_equal(r[1], res[0][1])
