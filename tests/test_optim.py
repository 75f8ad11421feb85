"""Optimizers: exact JAX-Adam math, bound transforms, PRNG keys, L-BFGS-B (root-driven
protocol), checkpoint/resume, simple GD helpers."""
import math
import os

import numpy as np
import pytest
import torch

import multigrad_amd as mg
from multigrad_amd.models.smf import DocsSMFModel, make_docs_data
from multigrad_amd.models.toy import SumOfSquaresModel, make_toy_data
from multigrad_amd.optim import adam as A
from multigrad_amd.optim.transforms import Bounds
from multigrad_amd.parallel import comm as C
from multigrad_amd.utils import random as R
from multigrad_amd.utils import util

from distributed import run_distributed


def _jax_adam_reference(grad_fn, x0, nsteps, lr, b1=0.9, b2=0.999, eps=1e-8):
    """jax.example_libraries.optimizers.adam, transcribed in float32 numpy."""
    x = np.asarray(x0, np.float32).copy()
    m = np.zeros_like(x)
    v = np.zeros_like(x)
    traj = [x.copy()]
    for i in range(nsteps):
        g = grad_fn(x).astype(np.float32)
        m = (1 - b1) * g + b1 * m
        v = (1 - b2) * np.square(g) + b2 * v
        mhat = m / (1 - np.asarray(b1, np.float32) ** (i + 1))
        vhat = v / (1 - np.asarray(b2, np.float32) ** (i + 1))
        x = x - lr * mhat / (np.sqrt(vhat) + eps)
        traj.append(x.copy())
    return np.stack(traj)


def test_adam_matches_jax_adam_math():
    target = np.array([1.0, -2.0, 0.5, 3.0], np.float32)

    def fn(p, data):
        g = 2 * (p - torch.as_tensor(target)) * torch.arange(1, 5)
        return ((p - torch.as_tensor(target)) ** 2).sum(), g

    traj = A.run_adam(fn, [0.0, 0.0, 0.0, 0.0], None, nsteps=50, learning_rate=0.05)
    ref = _jax_adam_reference(lambda x: 2 * (x - target) * np.arange(1, 5), np.zeros(4), 50, 0.05)
    assert traj.shape == (51, 4)
    np.testing.assert_allclose(traj.numpy(), ref, rtol=1e-5, atol=1e-6)


def test_history_modes():
    fn = lambda p, d: (((p - 1) ** 2).sum(), 2 * (p - 1))  # noqa: E731
    t_full = A.run_adam(fn, [0.0, 0.0], None, nsteps=10, learning_rate=0.1)
    t_last = A.run_adam(fn, [0.0, 0.0], None, nsteps=10, learning_rate=0.1, history="last")
    t_k = A.run_adam(fn, [0.0, 0.0], None, nsteps=10, learning_rate=0.1, history=4)
    assert t_last.shape == (2, 2) and torch.equal(t_last[-1], t_full[-1])
    assert t_k.shape == (4, 2) and torch.equal(t_k[1], t_full[4]) and torch.equal(t_k[-1], t_full[-1])


@pytest.mark.parametrize("bounds", [(-1.0, 2.0), (0.5, None), (None, 3.0), None,
                                    (float("-inf"), float("inf"))])
def test_transform_roundtrip_and_jacobian(bounds):
    p = torch.tensor([0.9, 0.95, 1.2, 1.7], dtype=torch.float64)
    if bounds is not None and bounds[0] == 0.5:
        p = p + 0.0
    spec = [bounds] * 4
    b = Bounds.from_spec(spec, 4, dtype=torch.float64)
    u = b.forward(p)
    torch.testing.assert_close(b.inverse(u), p)
    # scalar helpers agree with the vectorised ones
    torch.testing.assert_close(A.apply_transforms(p, spec), u)
    torch.testing.assert_close(A.apply_inverse_transforms(u, spec), p)
    # diagonal Jacobian dp/du equals autograd of the inverse transform
    uu = u.clone().requires_grad_(True)
    (jac,) = torch.autograd.grad(b.inverse(uu).sum(), uu)
    torch.testing.assert_close(b.dpdu(u), jac)


def test_bounded_adam_stays_in_bounds_and_converges():
    # minimum of (p - 3)^2 lies outside [-1, 2]: Adam must approach the upper bound
    fn = lambda p, d: (((p - 3.0) ** 2).sum(), 2 * (p - 3.0))  # noqa: E731
    traj = A.run_adam(fn, [0.0, 0.0], None, nsteps=300, param_bounds=[(-1, 2), (None, 2.5)],
                      learning_rate=0.05)
    assert (traj[:, 0] < 2).all() and (traj[:, 0] > -1).all() and (traj[:, 1] < 2.5).all()
    assert traj[-1, 0] > 1.7 and traj[-1, 1] > 2.1
    assert (traj[1:, 0] >= traj[:-1, 0]).all()  # monotone approach to the active bound
    legacy = A.run_adam(fn, [0.0, 0.0], None, nsteps=300, param_bounds=[(-1, 2), (None, 2.5)],
                        learning_rate=0.05, legacy_bounds_jacobian=True)
    assert (legacy[:, 0] < 2).all() and legacy[-1, 0] > 1.5
    assert not torch.equal(legacy, traj)


def test_prng_keys():
    k = R.init_randkey(42)
    assert k == R.init_randkey(42) and k != R.init_randkey(43)
    a, b = k.split()
    assert a != b and R.gen_new_key(k) == k.split(1)[0]
    assert R.init_randkey(k) is k
    with pytest.raises(AssertionError):
        R.init_randkey("nope")
    g1 = torch.randn(3, generator=a.generator())
    g2 = torch.randn(3, generator=a.generator())
    assert torch.equal(g1, g2)


class NoisyQuadratic(mg.OnePointModel):
    """Sumstats depend on randkey (stochastic model)."""

    def calc_partial_sumstats_from_params(self, params, randkey=None):
        noise = torch.randn(2, generator=randkey.generator()) * 1e-3 if randkey is not None else 0
        self.aux_data.setdefault("keys", []).append(None if randkey is None else randkey.value)
        return (params - 1.0) ** 2 + noise

    def calc_loss_from_sumstats(self, sumstats, sumstats_aux=None, randkey=None):
        return sumstats.sum()


def _keys_body(rank, size):
    m = NoisyQuadratic(aux_data={})
    m.run_adam([0.0, 0.0], nsteps=4, learning_rate=0.1, randkey=5)
    per_step = list(m.aux_data["keys"])
    m.aux_data["keys"] = []
    m.run_adam([0.0, 0.0], nsteps=3, learning_rate=0.1, randkey=9, const_randkey=True)
    const = list(m.aux_data["keys"])
    return per_step, const


def test_randkey_per_step_and_const_identical_on_ranks():
    res = run_distributed(_keys_body, 2)
    per_step, const = res[0]
    assert len(set(per_step)) == 4 and None not in per_step
    assert len(set(const)) == 1
    assert res[1] == res[0]  # every rank sees the same key sequence (SURVEY Q3 fixed)
    k = R.init_randkey(5)
    expect = []
    for _ in range(4):
        k, ki = k.split(2)
        expect.append(ki.value)
    assert per_step == expect


def _bfgs_body(rank, size):
    data = make_docs_data(comm=mg.get_world_comm(), device="cpu")
    model = DocsSMFModel(aux_data=data, device="cpu")
    res = model.run_bfgs(torch.tensor([-3.5, 0.2]))
    return (res.x.tolist(), float(res.fun), bool(res.success), int(res.nit), int(res.nfev),
            sorted(res.keys()))


@pytest.mark.parametrize("size", [1, 3])
def test_bfgs_docs_notebook_converges(size):
    """intro.ipynb:265-280 / :499-514: converges to [-2, -0.5], fun ~ 5e-12."""
    if size == 1:
        C.set_world_comm(None)
        res = [_bfgs_body(0, 1)]
    else:
        res = run_distributed(_bfgs_body, size)
    for x, fun, success, nit, nfev, keys in res:
        np.testing.assert_allclose(x, [-2.0, -0.5], atol=2e-4)
        assert fun < 1e-8 and success
        for k in ("message", "success", "status", "fun", "x", "jac", "nfev", "njev", "nit", "hess_inv"):
            assert k in keys
    assert all(r[:5] == res[0][:5] for r in res)  # identical result on every rank


def test_bfgs_with_bounds_respects_them():
    C.set_world_comm(None)
    d = make_toy_data(ndim=3, npoints=50, seed=4)
    m = SumOfSquaresModel(aux_data=d)
    res = m.run_bfgs([0.0, 0.0, 0.0], param_bounds=[(-0.2, 0.2)] * 3)
    assert np.all(res.x <= 0.2 + 1e-12) and np.all(res.x >= -0.2 - 1e-12)


def test_checkpoint_resume_matches_uninterrupted(tmp_path):
    C.set_world_comm(None)
    d = make_toy_data(ndim=4, npoints=60, seed=5)
    m = SumOfSquaresModel(aux_data=d)
    full = m.run_adam(torch.zeros(4), nsteps=10, learning_rate=0.05, randkey=3)
    ck = str(tmp_path / "adam.pt")
    m.run_adam(torch.zeros(4), nsteps=6, learning_rate=0.05, randkey=3, checkpoint_path=ck,
               checkpoint_every=6)
    resumed = m.run_adam(torch.zeros(4), nsteps=10, learning_rate=0.05, randkey=3, resume_from=ck)
    torch.testing.assert_close(resumed, full, rtol=0, atol=0)


def test_simple_grad_descent_variants():
    f = lambda p: ((p - 2.0) ** 2).sum()  # noqa: E731
    r = util.simple_grad_descent(f, [0.0, 1.0], nsteps=20, learning_rate=0.1)
    assert r.loss.shape == (20,) and r.params.shape == (20, 2)
    assert torch.allclose(r.params[0], torch.tensor([0.0, 1.0]))  # params at each loss eval
    r2 = util.simple_grad_descent(f, [0.0, 1.0], 20, 0.1, grad_loss_func=lambda p: 2 * (p - 2.0))
    torch.testing.assert_close(r2.params, r.params)
    faux = lambda p: (((p - 2.0) ** 2).sum(), p.sum().detach())  # noqa: E731
    r3 = util.simple_grad_descent(faux, [0.0, 1.0], 5, 0.1, has_aux=True)
    assert r3.aux.shape == (5,)


def test_latin_hypercube_sampler():
    x = util.latin_hypercube_sampler([0, -1], [1, 1], 2, 10, seed=0)
    assert x.shape == (10, 2) and (x[:, 1] >= -1).all()
    # LHS: exactly one draw per stratum along each axis
    assert sorted(np.floor(x[:, 0] * 10).astype(int).tolist()) == list(range(10))


def test_bounds_from_numeric_array_equals_list_spec():
    """The vectorised (ndim, 2) numeric-array path of Bounds.from_spec (round 5: a 1e7-row
    Python loop took seconds) gives the same lo / hi / kind as the per-row list path,
    with non-finite entries marking an absent side."""
    rng = np.random.default_rng(3)
    n = 500
    lo = rng.normal(size=n)
    hi = lo + rng.random(n) + 0.1
    lo[rng.random(n) < 0.3] = -np.inf
    hi[rng.random(n) < 0.3] = np.inf
    lo[:5] = np.nan  # NaN: absent too
    arr = np.stack([lo, hi], 1)
    spec = [(None if not np.isfinite(a) else float(a), None if not np.isfinite(b) else float(b))
            for a, b in arr]
    b_arr = Bounds.from_spec(arr, n, dtype=torch.float64)
    b_lst = Bounds.from_spec(spec, n, dtype=torch.float64)
    torch.testing.assert_close(b_arr.lo, b_lst.lo)
    torch.testing.assert_close(b_arr.hi, b_lst.hi)
    assert torch.equal(b_arr.kind, b_lst.kind)
    b_t = Bounds.from_spec(torch.as_tensor(arr), n, dtype=torch.float64)
    assert torch.equal(b_t.kind, b_lst.kind)
