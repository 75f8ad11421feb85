"""Generic (graph-capturable) Adam engine for any torch OnePointModel: CPU/gloo paths
against the eager distributed chain rule + run_adam."""
import numpy as np
import pytest
import torch

import multigrad_amd as mg
from multigrad_amd.engine.generic import GraphAdamEngine
from multigrad_amd.models.population import PopulationSMFModel, make_population_data
from multigrad_amd.models.toy import SumOfSquaresModel, make_toy_data
from multigrad_amd.models.torch_population import TorchPopulationSMFModel, torch_population_data
from multigrad_amd.parallel import comm as C

from distributed import run_distributed


def _torch_pop(comm=None, npar=400, nhalo=8000):
    data = make_population_data(npar, nhalo, seed=11, comm=comm, device="cpu")
    PopulationSMFModel(aux_data=data, comm=comm).set_target_from_truth()
    return TorchPopulationSMFModel(aux_data=torch_population_data(data), comm=comm), data["guess"]


def test_torch_population_model_matches_kernel_model():
    C.set_world_comm(None)
    data = make_population_data(400, 8000, seed=11, device="cpu")
    km = PopulationSMFModel(aux_data=data)
    km.set_target_from_truth()
    tm = TorchPopulationSMFModel(aux_data=torch_population_data(data))
    p = data["guess"]
    l1, g1 = km.calc_loss_and_grad_from_params(p)
    l2, g2 = tm.calc_loss_and_grad_from_params(p)
    assert float(l1) == pytest.approx(float(l2), rel=1e-4)
    torch.testing.assert_close(g1, g2, rtol=2e-3, atol=1e-3 * float(g1.abs().max()))


@pytest.mark.parametrize("bounded", [False, True])
@pytest.mark.parametrize("which", ["toy", "pop"])
def test_generic_engine_matches_eager_run_adam(which, bounded):
    C.set_world_comm(None)
    if which == "toy":
        m = SumOfSquaresModel(aux_data=make_toy_data(ndim=5, npoints=40))
        guess = torch.zeros(5)
    else:
        m, guess = _torch_pop()
    bounds = None
    if bounded:
        g = guess.numpy()
        bounds = np.stack([g - 0.3, g + 0.05], 1)
    ref = m.run_adam(guess, nsteps=6, learning_rate=0.05, param_bounds=bounds)
    eng = GraphAdamEngine(m)
    traj = eng.run_adam(guess, nsteps=6, learning_rate=0.05, param_bounds=bounds)
    assert traj.shape == ref.shape == (7,) + tuple(guess.shape)
    assert not eng.use_graph and eng.fallback_reason == "CPU tensors"
    torch.testing.assert_close(traj, ref, rtol=1e-6, atol=1e-7)


def _gloo(rank, size, history):
    comm = mg.get_world_comm()
    m, guess = _torch_pop(comm)
    eng = GraphAdamEngine(m)
    traj = eng.run_adam(guess, nsteps=4, learning_rate=0.02, history=history)
    return traj.numpy(), eng.fallback_reason


@pytest.mark.parametrize("history", ["full", "last"])
def test_generic_engine_gloo_ranks_match_single_rank(history):
    C.set_world_comm(None)
    m, guess = _torch_pop()
    ref = GraphAdamEngine(m).run_adam(guess, nsteps=4, learning_rate=0.02, history=history).numpy()
    res = run_distributed(_gloo, 2, history)
    for traj, why in res:
        assert "collectives" in why
        np.testing.assert_allclose(traj, ref, rtol=2e-5, atol=1e-6)
    np.testing.assert_array_equal(res[0][0], res[1][0])
