"""Device L-BFGS (compact representation, all-reduced dots): CPU/gloo coverage."""
import numpy as np
import pytest
import scipy.optimize
import torch

import multigrad_amd as mg
from multigrad_amd.models.population import PopulationSMFModel, make_population_data
from multigrad_amd.models.smf import DocsSMFModel, make_docs_data
from multigrad_amd.optim import lbfgs as L
from multigrad_amd.parallel import comm as C

from distributed import run_distributed


def _rosen(x):
    x = x.double()
    f = (100 * (x[1:] - x[:-1] ** 2) ** 2 + (1 - x[:-1]) ** 2).sum()
    return f


def _rosen_lg(x):
    xx = x.detach().double().requires_grad_(True)
    with torch.enable_grad():
        f = _rosen(xx)
        (g,) = torch.autograd.grad(f, xx)
    return f.detach(), g.float()


def test_lbfgs_rosenbrock_matches_scipy_minimum():
    res = L.run_lbfgs_device(_rosen_lg, torch.tensor([-1.2, 1.0, -0.5, 0.8]), maxsteps=500,
                             gtol=1e-6)
    assert res.success, res.message
    np.testing.assert_allclose(res.x.numpy(), np.ones(4), atol=2e-3)
    ref = scipy.optimize.minimize(lambda v: scipy.optimize.rosen(v), [-1.2, 1.0, -0.5, 0.8],
                                  jac=scipy.optimize.rosen_der, method="L-BFGS-B")
    assert res.fun < 1e-6 and abs(res.nit - ref.nit) < 60


def test_compact_direction_equals_two_loop():
    """The compact inverse-Hessian product equals the classical two-loop recursion."""
    rng = np.random.default_rng(0)
    n, m = 12, 5
    S = rng.normal(size=(m, n))
    Y = S + 0.3 * rng.normal(size=(m, n))  # s.y > 0
    g = rng.normal(size=n)
    order = [3, 0, 4, 1, 2]  # ring slots, oldest first
    SY, YY = S @ Y.T, Y @ Y.T
    gamma, a, b = L.compact_coefficients(SY, YY, S @ g, Y @ g, order)
    idx = np.array(order)
    Hg = gamma * g + S[idx].T @ a + gamma * (Y[idx].T @ b)
    # two-loop recursion, newest pair first
    q = g.copy()
    alphas = []
    for i in reversed(order):
        rho = 1.0 / (S[i] @ Y[i])
        al = rho * (S[i] @ q)
        alphas.append(al)
        q -= al * Y[i]
    r = gamma * q
    for i, al in zip(order, reversed(alphas)):
        rho = 1.0 / (S[i] @ Y[i])
        beta = rho * (Y[i] @ r)
        r += S[i] * (al - beta)
    np.testing.assert_allclose(Hg, r, rtol=1e-10, atol=1e-12)


def _docs_device(rank, size):
    data = make_docs_data(comm=mg.get_world_comm(), device="cpu")
    model = DocsSMFModel(aux_data=data, device="cpu")
    res = model.run_bfgs(torch.tensor([-3.5, 0.2]), method="device")
    return res.x.tolist(), float(res.fun), bool(res.success)


@pytest.mark.parametrize("size", [1, 2])
def test_device_lbfgs_docs_model(size):
    if size == 1:
        C.set_world_comm(None)
        res = [_docs_device(0, 1)]
    else:
        res = run_distributed(_docs_device, size)
    for x, fun, ok in res:
        np.testing.assert_allclose(x, [-2.0, -0.5], atol=5e-4)
        assert fun < 1e-7
    assert all(r == res[0] for r in res)


def _pop_lbfgs(rank, size, zero, placement="hashed"):
    comm = mg.get_world_comm()
    data = make_population_data(num_params=80, num_halos=3000, seed=3, comm=comm, device="cpu",
                                placement=placement)
    m = PopulationSMFModel(aux_data=data, comm=comm)
    m.set_target_from_truth()
    res = m.run_bfgs(data["guess"], maxsteps=30, method="device", zero=zero, chunks=3)
    return res.x.numpy(), float(res.fun), int(res.nit)


def test_sharded_lbfgs_matches_single_rank():
    C.set_world_comm(None)
    x1, f1, n1 = _pop_lbfgs(0, 1, False)
    res = run_distributed(_pop_lbfgs, 2, True)
    for x, f, nit in res:
        np.testing.assert_allclose(x, x1, rtol=1e-3, atol=1e-4)
        assert f == pytest.approx(f1, rel=1e-2, abs=1e-9)
    np.testing.assert_array_equal(res[0][0], res[1][0])


def test_sharded_lbfgs_owner_placement_matches_single_rank():
    C.set_world_comm(None)
    x1, f1, n1 = _pop_lbfgs(0, 1, False)
    res = run_distributed(_pop_lbfgs, 3, True, "owner")
    for x, f, nit in res:
        np.testing.assert_allclose(x, x1, rtol=1e-3, atol=1e-4)
        assert f == pytest.approx(f1, rel=1e-2, abs=1e-9)
    np.testing.assert_array_equal(res[0][0], res[1][0])
