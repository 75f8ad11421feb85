"""Device L-BFGS-B on the MI355X (MultiDot / lincomb HIP kernels, topk breakpoints on the
device) against scipy's L-BFGS-B, and on the fused engine's objective."""
import numpy as np
import pytest
import scipy.optimize
import torch

from multigrad_amd.optim import lbfgsb as LB

pytestmark = pytest.mark.gpu


def test_lbfgsb_gpu_matches_scipy():
    from test_lbfgs import _bounded_problem
    n = 20_000
    lo, hi, f_np, _ = _bounded_problem(n, seed=5)

    def lg(x):
        f, g = f_np(x.detach().double().cpu().numpy())
        return torch.tensor(f, dtype=torch.float64), torch.from_numpy(g).float().cuda()

    x0 = np.clip(np.zeros(n), lo, hi)
    ref = scipy.optimize.minimize(f_np, x0, jac=True, method="L-BFGS-B",
                                  bounds=list(zip(lo, hi)), options=dict(maxiter=500))
    res = LB.run_lbfgsb_device(lg, torch.tensor(x0, dtype=torch.float32, device="cuda"),
                               maxsteps=500, param_bounds=list(zip(lo, hi)))
    assert res.success, res.message
    assert res.fun == pytest.approx(ref.fun, rel=1e-7)
    np.testing.assert_allclose(res.x.cpu().numpy(), ref.x, atol=1e-4)


def test_lbfgsb_gpu_population_engine():
    """Bounded fit of a population model through the engine objective: feasible, the loss
    decreases, and the lower bounds that cut off the truth end up active."""
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    data = make_population_data(num_params=20_000, num_halos=1_000_000, seed=4, device="cuda")
    m = PopulationSMFModel(aux_data=data)
    m.set_target_from_truth()
    g = data["guess"].cpu().numpy()
    # the truth is guess - 0.1: the lower bounds at guess - 0.05 are active at the solution
    bounds = list(zip((g - 0.05).tolist(), (g + 0.02).tolist()))
    res = m.run_bfgs(data["guess"], maxsteps=25, method="device", param_bounds=bounds)
    x = res.x.cpu().numpy()
    b = np.asarray(bounds, dtype=np.float32)
    assert (x >= b[:, 0]).all() and (x <= b[:, 1]).all()
    f0 = float(m.calc_loss_from_params(data["guess"]))
    assert res.fun < 0.8 * f0
    active = (np.abs(x - b[:, 0]) < 1e-7) | (np.abs(x - b[:, 1]) < 1e-7)
    assert active.mean() > 0.2
