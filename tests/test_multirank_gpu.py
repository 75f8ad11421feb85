"""Two ranks sharing one MI355X (collectives staged through gloo): the HIP kernels under
the multi-rank engine schedules (ZeRO-1 chunks, sharded trajectory, sharded L-BFGS)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from distributed import run_distributed  # noqa: E402

NP, NH = 6000, 400_000


def _run(rank, size, zero, chunks, placement="hashed"):
    import multigrad_amd as mg
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    comm = mg.get_world_comm()
    dev = torch.device("cuda", 0)
    data = make_population_data(NP, NH, seed=21, comm=comm, device=dev, placement=placement)
    model = PopulationSMFModel(aux_data=data, comm=comm)
    model.set_target_from_truth()
    eng = FusedAdamEngine(model, zero=zero, chunks=chunks)
    traj = eng.run_adam(data["guess"], nsteps=5, learning_rate=1e-3)
    res = model.run_bfgs(data["guess"], maxsteps=8, method="device", zero=zero, chunks=chunks)
    return traj.cpu().numpy(), float(res.fun), res.x.cpu().numpy(), eng.owner or eng.zero


def test_two_ranks_one_gpu_match_single_rank():
    import multigrad_amd.parallel.comm as C
    C.set_world_comm(None)
    t1, f1, x1, _ = _run(0, 1, False, 1)
    res = run_distributed(_run, 2, True, 3, timeout=600)
    for traj, f, x, z in res:
        assert z
        np.testing.assert_allclose(traj, t1, rtol=2e-5, atol=2e-6)
        assert f == pytest.approx(f1, rel=1e-3)
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][2], res[1][2])


def test_two_ranks_one_gpu_owner_placement():
    """Population-owner placement on the HIP kernels: no gradient collective, same fit."""
    import multigrad_amd.parallel.comm as C
    C.set_world_comm(None)
    t1, f1, x1, _ = _run(0, 1, False, 1)
    res = run_distributed(_run, 2, True, 3, "owner", timeout=600)
    for traj, f, x, z in res:
        assert z
        np.testing.assert_allclose(traj, t1, rtol=2e-5, atol=2e-6)
        assert f == pytest.approx(f1, rel=1e-3)
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][2], res[1][2])
