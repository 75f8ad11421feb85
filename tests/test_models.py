"""Model layer: the reference's pipeline test at several world sizes, the quick-start
notebook's numbers, aux plumbing, groups, LHS scans (SURVEY §4 "not tested" items)."""
from dataclasses import dataclass

import numpy as np
import pytest
import torch

import multigrad_amd as mg
from multigrad_amd.models.smf import (DocsSMFModel, MySMFModel, ParamTuple, TARGET_SUMSTATS,
                                      make_docs_data, make_test_data)
from multigrad_amd.models.toy import SumOfSquaresModel, make_toy_data
from multigrad_amd.parallel import comm as C

from distributed import run_distributed


def _pipeline(rank, size):
    data = make_test_data()
    model = MySMFModel(aux_data=data, device="cpu")
    truth = ParamTuple(log_shmrat=-2.0, sigma_logsm=0.2)
    s = model.calc_sumstats_from_params(truth)
    # against the reference's published float32 JAX target (partition invariant)
    np.testing.assert_allclose(s.numpy(), TARGET_SUMSTATS, rtol=5e-5, atol=1e-9)
    # reference assertions with a self-consistent target
    data["target_sumstats"] = s.numpy()
    model = MySMFModel(aux_data=data, device="cpu")
    gd = model.run_simple_grad_descent(guess=truth, nsteps=2)
    assert torch.isclose(gd.loss[-1], torch.tensor(0.0), atol=1e-8)
    assert torch.allclose(gd.params[-1], torch.tensor([*truth]))
    assert torch.allclose(model.calc_dloss_dparams(truth), torch.zeros(2), atol=1e-5)
    loss, grad = model.calc_loss_and_grad_from_params(truth)
    assert torch.allclose(loss, model.calc_loss_from_params(truth))
    assert torch.allclose(grad, model.calc_dloss_dparams(truth))
    off = model.calc_loss_and_grad_from_params([-1.9, 0.25])
    return s.numpy().tolist(), float(off[0]), off[1].numpy().tolist()


@pytest.mark.parametrize("size", [1, 2, 3])
def test_simple_grad_descent_pipeline(size):
    if size == 1:
        C.set_world_comm(None)
        res = [_pipeline(0, 1)]
    else:
        res = run_distributed(_pipeline, size)
    base = _pipeline_single()
    for s, loss, grad in res:
        np.testing.assert_allclose(s, base[0], rtol=2e-6)
        assert loss == pytest.approx(base[1], rel=1e-5)
        np.testing.assert_allclose(grad, base[2], rtol=1e-4)


def _pipeline_single():
    C.set_world_comm(None)
    return _pipeline(0, 1)


def _docs_loss_grad(rank, size):
    data = make_docs_data(comm=mg.get_world_comm(), device="cpu")
    model = DocsSMFModel(aux_data=data, device="cpu")
    loss, grad = model.calc_loss_and_grad_from_params(torch.tensor([-1.9, -0.4]))
    l0, g0 = model.calc_loss_and_grad_from_params(torch.tensor([-2.0, -0.5]))
    return float(loss), grad.tolist(), float(l0), g0.tolist()


@pytest.mark.parametrize("size", [1, 3])
def test_docs_notebook_loss_and_grad(size):
    """docs/source/notebooks/intro.ipynb:209-214: 0.44032094, [2.6187496, 4.2603974]."""
    if size == 1:
        C.set_world_comm(None)
        res = [_docs_loss_grad(0, 1)]
    else:
        res = run_distributed(_docs_loss_grad, size)
    for loss, grad, l0, g0 in res:
        assert loss == pytest.approx(0.44032094, rel=2e-5)
        np.testing.assert_allclose(grad, [2.6187496, 4.2603974], rtol=2e-4)
        assert l0 == pytest.approx(0.0, abs=1e-10)
        np.testing.assert_allclose(g0, [0, 0], atol=1e-5)


class AuxModel(mg.OnePointModel):
    """Both aux flags on: sumstats -> (s, aux), loss -> (loss, aux)."""

    def calc_partial_sumstats_from_params(self, params, randkey=None):
        x = self.aux_data["x"]
        s = torch.stack([(x * params[0]).sum(), (x ** 2 * params[1]).sum()])
        return s, {"n": x.numel(), "rk": randkey}

    def calc_loss_from_sumstats(self, sumstats, sumstats_aux=None, randkey=None):
        loss = ((sumstats - torch.tensor([3.0, 5.0])) ** 2).sum()
        return loss, {"seen_n": sumstats_aux["n"], "rk": randkey}


def _aux_body(rank, size):
    x = torch.arange(1.0, 7.0).tensor_split(size)[rank]
    m = AuxModel(aux_data={"x": x}, sumstats_func_has_aux=True, loss_func_has_aux=True)
    p = torch.tensor([0.3, 0.1])
    (loss, laux), grad = m.calc_loss_and_grad_from_params(p)
    s, saux = m.calc_sumstats_from_params(p)
    assert saux["n"] == x.numel() and laux["seen_n"] == x.numel()
    g, gaux = m.calc_dloss_dsumstats(s, saux)
    (l2, aux2) = m.calc_loss_from_params(p, randkey=7)
    assert aux2["rk"] == 7
    return float(loss), grad.tolist(), s.tolist(), g.tolist(), float(l2)


def test_has_aux_plumbing_matches_serial():
    C.set_world_comm(None)
    ref = _aux_body(0, 1)
    # hand computation: S = [sum(x)*p0, sum(x^2)*p1] = [6.3, 9.1]
    assert ref[2] == pytest.approx([21 * 0.3, 91 * 0.1])
    res = run_distributed(_aux_body, 2)
    for r in res:
        assert r[0] == pytest.approx(ref[0], rel=1e-6)
        np.testing.assert_allclose(r[1], ref[1], rtol=1e-6)
        np.testing.assert_allclose(r[3], ref[3], rtol=1e-6)


def _group_body(rank, size):
    sub, ng, g = mg.split_subcomms(num_groups=2)
    # group 0 fits one toy data set, group 1 another; each model sums over its sub-comm
    data = make_toy_data(ndim=3, npoints=40, seed=10 + g, comm=sub)
    model = SumOfSquaresModel(aux_data=data, comm=sub)
    group = mg.OnePointGroup(model, main_comm=mg.get_world_comm())
    p = torch.tensor([0.1, -0.2, 0.3])
    loss, grad = group.calc_loss_and_grad_from_params(p)
    res = group.run_bfgs([0.0, 0.0, 0.0], maxsteps=50)
    traj = group.run_adam([0.0, 0.0, 0.0], nsteps=5, learning_rate=0.1)
    gd = group.run_simple_grad_descent([0.0, 0.0, 0.0], nsteps=3, learning_rate=0.1)
    return float(loss), grad.tolist(), res.x.tolist(), traj.shape, traj[-1].tolist(), gd.params.shape


def test_onepointgroup_sums_subcomm_models():
    res = run_distributed(_group_body, 4)
    # serial oracle: the two data sets evaluated independently and summed
    C.set_world_comm(None)
    tot_l, tot_g, means = 0.0, np.zeros(3), []
    p = torch.tensor([0.1, -0.2, 0.3])
    for g in range(2):
        d = make_toy_data(ndim=3, npoints=40, seed=10 + g)
        m = SumOfSquaresModel(aux_data=d)
        l, gr = m.calc_loss_and_grad_from_params(p)
        tot_l += float(l)
        tot_g += gr.numpy()
        means.append(d["mean"])
    opt = (means[0] + means[1]) / 2  # minimiser of the summed loss
    for loss, grad, x, tshape, tlast, gshape in res:
        assert loss == pytest.approx(tot_l, rel=1e-5)
        np.testing.assert_allclose(grad, tot_g, rtol=1e-5)
        np.testing.assert_allclose(x, opt, atol=1e-4)
        assert tuple(tshape) == (6, 3) and tuple(gshape) == (3, 3)
    assert all(r[4] == res[0][4] for r in res)  # SPMD Adam: identical on all ranks


def _lhs_body(rank, size):
    m = SumOfSquaresModel(aux_data=make_toy_data(ndim=2, npoints=30, seed=1))
    params, sumstats, losses = m.run_lhs_param_scan([-1, -2], [1, 2], 2, 6, seed=None)
    # the scan's single batched all-reduce matches per-point evaluation
    for x, s, l in zip(params, sumstats, losses):
        np.testing.assert_allclose(s, m.calc_sumstats_from_params(x).numpy(), rtol=1e-6)
        assert l == pytest.approx(float(m.calc_loss_from_params(x)), rel=1e-6)
    return params.tolist(), sumstats.tolist(), losses.tolist()


def test_lhs_param_scan_consistent_across_ranks():
    res = run_distributed(_lhs_body, 3)
    params, sumstats, losses = res[0]
    assert np.asarray(params).shape == (6, 2) and np.asarray(sumstats).shape == (6, 2)
    p = np.asarray(params)
    assert (p[:, 0] >= -1).all() and (p[:, 0] <= 1).all() and (p[:, 1] >= -2).all()
    for r in res[1:]:
        assert r[0] == params and r[2] == pytest.approx(losses)


def test_lhs_param_scan_with_sumstats_aux():
    C.set_world_comm(None)
    m = AuxModel(aux_data={"x": torch.arange(1.0, 4.0)}, sumstats_func_has_aux=True,
                 loss_func_has_aux=True)
    params, sumstats, losses = m.run_lhs_param_scan(0, 1, 2, 4, seed=3)
    assert sumstats.shape == (4, 2) and losses.shape == (4,)


def test_model_identity_and_hash():
    C.set_world_comm(None)
    a = SumOfSquaresModel(aux_data=make_toy_data(ndim=2, npoints=5))
    b = SumOfSquaresModel(aux_data=a.aux_data)
    assert a == a and a != b
    assert hash(a) == hash(b)  # (comm name, loss function) as in the reference
    g = mg.OnePointGroup(a)
    assert g == g and isinstance(g.models, tuple) and len(g.models) == 1
    with pytest.raises(NotImplementedError):
        mg.OnePointModel().calc_partial_sumstats_from_params([1.0])


def test_toy_adam_converges_single_process():
    """BASELINE config 1: 10-parameter sum-of-squares, single-process Adam on CPU."""
    C.set_world_comm(None)
    d = make_toy_data(ndim=10, npoints=500, seed=2)
    m = SumOfSquaresModel(aux_data=d)
    traj = m.run_adam(torch.zeros(10), nsteps=400, learning_rate=0.05)
    assert traj.shape == (401, 10)
    np.testing.assert_allclose(traj[-1].numpy(), d["mean"], atol=2e-3)


def test_module_globals():
    C.set_world_comm(None)
    assert mg.RANK == 0 and mg.N_RANKS == 1 and mg.COMM.size == 1
    assert mg.__version__
