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


def test_lbfgs_objective_returning_a_reused_buffer():
    """An objective that returns a view of one gradient buffer (as the engine objective
    does) must give the same iterates as one that returns fresh tensors."""
    buf = torch.zeros(4)

    class Fresh(L.GenericObjective):
        pass

    class Reused(L.GenericObjective):
        def __call__(self, u):
            f, g = super().__call__(u)
            buf.copy_(g)
            return f, buf

    x0 = torch.tensor([-1.2, 1.0, -0.5, 0.8])
    a = L.lbfgs_minimize(Fresh(_rosen_lg, x0), maxiter=30)
    b = L.lbfgs_minimize(Reused(_rosen_lg, x0), maxiter=30)
    assert a.nit == b.nit and a.nfev == b.nfev
    np.testing.assert_array_equal(a.x.numpy(), b.x.numpy())


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


# ---------------------------------------------------------------- device L-BFGS-B
from multigrad_amd.optim import lbfgsb as LB  # noqa: E402


def _bounded_problem(n, seed=0):
    rng = np.random.default_rng(seed)
    c = rng.normal(size=n)
    a = 0.5 + rng.random(n)
    lo = np.where(rng.random(n) < 0.5, c - 0.3 * rng.random(n), -np.inf)
    hi = np.where(rng.random(n) < 0.5, c + 0.3 * rng.random(n), np.inf)
    c2 = c + np.where(rng.random(n) < 0.3, 1.0, 0.0) * np.sign(rng.normal(size=n))

    def f_np(x):
        r = x - c2
        s = x.sum() / n
        g = 2 * a * r + 20 * s / n + 0.25 * (np.concatenate([[0], r[:-1]]) + np.concatenate([r[1:], [0]]))
        return float((a * r * r).sum() + 10 * s * s + 0.25 * (r[1:] * r[:-1]).sum()), g

    def lg(x):
        f, g = f_np(x.detach().double().cpu().numpy())
        return torch.tensor(f, dtype=torch.float64), torch.from_numpy(g).float()

    return lo, hi, f_np, lg


def test_lbfgsb_matches_scipy_on_bounded_1e4_problem():
    """1e4 coupled parameters, ~half with a bound, ~30% active at the optimum: x and f
    of scipy's L-BFGS-B (float64) reproduced by the device L-BFGS-B (float32)."""
    n = 10_000
    lo, hi, f_np, lg = _bounded_problem(n)
    x0 = np.clip(np.zeros(n), lo, hi)
    ref = scipy.optimize.minimize(f_np, x0, jac=True, method="L-BFGS-B",
                                  bounds=list(zip(lo, hi)), options=dict(maxiter=500))
    res = LB.run_lbfgsb_device(lg, torch.tensor(x0, dtype=torch.float32), maxsteps=500,
                               param_bounds=list(zip(lo, hi)))
    assert res.success, res.message
    assert res.fun == pytest.approx(ref.fun, rel=1e-7)
    np.testing.assert_allclose(res.x.numpy(), ref.x, atol=1e-4)
    x = res.x.numpy()
    assert (x >= lo.astype(np.float32)).all() and (x <= hi.astype(np.float32)).all()
    active = (np.abs(ref.x - lo) < 1e-9) | (np.abs(ref.x - hi) < 1e-9)
    assert active.mean() > 0.1
    assert abs(res.nit - ref.nit) <= 5


def test_lbfgsb_small_breakpoint_batches():
    """Breakpoint batches far smaller than the number of breakpoints before the Cauchy
    point (K=4: the scan carries its state across ~100 batches) give the same result."""
    n = 300
    lo, hi, f_np, lg = _bounded_problem(n, seed=2)
    x0 = torch.tensor(np.clip(np.zeros(n), lo, hi), dtype=torch.float32)
    obj = LB.BoxObjective(lg, x0)
    a = LB.lbfgsb_minimize(obj, torch.tensor(lo, dtype=torch.float32),
                           torch.tensor(hi, dtype=torch.float32), maxiter=200, K=4)
    b = LB.lbfgsb_minimize(obj, torch.tensor(lo, dtype=torch.float32),
                           torch.tensor(hi, dtype=torch.float32), maxiter=200)
    assert a.fun == pytest.approx(b.fun, rel=1e-7)
    np.testing.assert_allclose(a.x.numpy(), b.x.numpy(), atol=1e-6)


def _docs_bounded(rank, size, method):
    data = make_docs_data(comm=mg.get_world_comm(), device="cpu")
    model = DocsSMFModel(aux_data=data, device="cpu", dtype=torch.float64)
    bounds = [(-1.95, -1.0), (-1.0, 0.0)]          # the truth (-2, -0.5) is cut off in log_f
    res = model.run_bfgs(torch.tensor([-1.2, -0.1], dtype=torch.float64), param_bounds=bounds,
                         method=method)
    return np.asarray(res.x, dtype=np.float64).tolist(), float(res.fun), bool(res.success)


@pytest.mark.parametrize("size", [1, 2])
def test_lbfgsb_docs_model_bounded_matches_scipy(size):
    C.set_world_comm(None)
    ref = _docs_bounded(0, 1, "scipy")
    if size == 1:
        res = [_docs_bounded(0, 1, "device")]
    else:
        res = run_distributed(_docs_bounded, size, "device")
    for x, fun, ok in res:
        assert ok
        np.testing.assert_allclose(x, ref[0], atol=2e-4)
        assert x[0] == pytest.approx(-1.95, abs=1e-7)   # on the bound, as scipy
        assert fun == pytest.approx(ref[1], rel=1e-4)


def test_cauchy_scan_vectorised_matches_sequential():
    """The prefix-sum Cauchy-point scan against the sequential algorithm CP of Byrd et al.
    (1995), with a non-trivial compact matrix and many breakpoints, in batches."""
    import math
    rng = np.random.default_rng(3)
    n, k = 400, 3
    S = rng.normal(size=(k, n))
    Y = S + 0.2 * rng.normal(size=(k, n))
    theta = float((Y[-1] @ Y[-1]) / (S[-1] @ Y[-1]))
    sy = S @ Y.T
    D = np.diag(np.diag(sy))
    Lm = np.tril(sy, -1)
    M = np.linalg.inv(np.block([[-D, Lm.T], [Lm, theta * (S @ S.T)]]))
    Wrows = np.concatenate([Y, theta * S])          # rows of W' (2k x n)
    g = rng.normal(size=n)
    t = np.where(rng.random(n) < 0.7, rng.random(n) * 3, np.inf)
    d = np.where(t > 0, -g, 0.0)
    dd = float(d @ d)
    p0 = Wrows @ d
    # sequential reference
    fp, fpp = -dd, theta * dd - p0 @ M @ p0
    p, c, told = p0.copy(), np.zeros(2 * k), 0.0
    dtmin = -fp / fpp
    for j in np.argsort(t):
        if not np.isfinite(t[j]) or dtmin < t[j] - told:
            break
        dt, gb, wb = t[j] - told, g[j], Wrows[:, j]
        c = c + dt * p
        fp = fp + dt * fpp + gb * gb - theta * t[j] * gb * gb - gb * (wb @ M @ c)
        fpp = fpp - theta * gb * gb - 2 * gb * (wb @ M @ p) - gb * gb * (wb @ M @ wb)
        p = p + gb * wb
        dtmin = -fp / fpp
        told = t[j]
    dtmin = max(dtmin, 0.0)
    want_t, want_c = told + dtmin, c + dtmin * p
    HS = torch.tensor(np.concatenate([S, Y]), dtype=torch.float32)  # rows s_0..s_k-1, y_0..
    rows = np.concatenate([k + np.arange(k), np.arange(k)])
    fac = np.concatenate([np.ones(k), np.full(k, theta)])
    HSd = torch.tensor(np.concatenate([S, Y]), dtype=torch.float64)
    for K in (3, 50, 10_000):
        ts, cs = LB._cauchy_point(dd, p0, M, theta, torch.tensor(t), int(np.isfinite(t).sum()),
                                  torch.tensor(g), HSd, rows, fac, None, K)
        assert ts == pytest.approx(want_t, rel=1e-10)
        np.testing.assert_allclose(cs, want_c, rtol=1e-9, atol=1e-12)


def _pop_lbfgsb(rank, size, zero, placement="hashed"):
    comm = mg.get_world_comm()
    data = make_population_data(num_params=80, num_halos=3000, seed=3, comm=comm, device="cpu",
                                placement=placement)
    m = PopulationSMFModel(aux_data=data, comm=comm)
    m.set_target_from_truth()
    g = data["guess"].cpu().numpy()
    bounds = [(float(v) - 0.05, float(v) + 0.2) for v in g]
    res = m.run_bfgs(data["guess"], maxsteps=30, method="device", zero=zero, chunks=3,
                     param_bounds=bounds)
    return res.x.numpy(), float(res.fun), int(res.nit), np.asarray(bounds)


@pytest.mark.parametrize("placement", ["hashed", "owner"])
def test_sharded_lbfgsb_matches_single_rank(placement):
    """The engine-sharded L-BFGS-B (ZeRO slices / owner slices, breakpoints gathered
    across ranks) against one rank."""
    C.set_world_comm(None)
    x1, f1, n1, b = _pop_lbfgsb(0, 1, False)
    assert ((x1 >= b[:, 0] - 1e-6) & (x1 <= b[:, 1] + 1e-6)).all()
    res = run_distributed(_pop_lbfgsb, 2, True, placement)
    for x, f, nit, _ in res:
        np.testing.assert_allclose(x, x1, rtol=1e-3, atol=2e-4)
        assert f == pytest.approx(f1, rel=1e-2, abs=1e-9)
    np.testing.assert_array_equal(res[0][0], res[1][0])
