"""Fused engine orchestration (chunking, ZeRO-1 reduce-scatter/all-gather, bounds,
trajectory) on the CPU/gloo path; the HIP path is covered in test_kernels_gpu.py."""
import numpy as np
import pytest
import torch

import multigrad_amd as mg
from multigrad_amd.engine.fused import FusedAdamEngine, plan_chunks
from multigrad_amd.models.population import PopulationSMFModel, make_population_data
from multigrad_amd.parallel import comm as C

from distributed import run_distributed

NP, NH = 120, 4000


def _model(comm=None):
    data = make_population_data(num_params=NP, num_halos=NH, seed=11, comm=comm, device="cpu")
    m = PopulationSMFModel(aux_data=data, comm=comm)
    m.set_target_from_truth()
    return m, data


def test_plan_chunks_alignment():
    for J, upp, W, C_ in [(61, 2, 4, 3), (5_000_000, 2, 8, 8), (7, 2, 1, 1), (100, 3, 2, 5)]:
        ub, pb, P_pad, lengths = plan_chunks(J, upp, W, C_)
        assert ub[0] == 0 and ub[-1] == J and pb == [u * upp for u in ub]
        assert sum(lengths) == P_pad >= J * upp and P_pad - J * upp < 4 * W
        assert all(L % (4 * W) == 0 and L > 0 for L in lengths)


def _generic_traj(nsteps, bounds=None):
    C.set_world_comm(None)
    m, data = _model()
    return m.run_adam(data["guess"], nsteps=nsteps, learning_rate=2e-3, param_bounds=bounds,
                      use_engine=False)


@pytest.mark.parametrize("chunks", [1, 3])
def test_engine_matches_generic_single_rank(chunks):
    ref = _generic_traj(5)
    C.set_world_comm(None)
    m, data = _model()
    eng = FusedAdamEngine(m, chunks=chunks)
    traj = eng.run_adam(data["guess"], nsteps=5, learning_rate=2e-3)
    assert traj.shape == (6, NP)
    torch.testing.assert_close(traj, ref, rtol=2e-5, atol=2e-6)


def test_engine_bounded_matches_generic():
    bounds = [(-2.3, -1.6) if i % 2 == 0 else (None, -0.2) for i in range(NP)]
    ref = _generic_traj(4, bounds)
    C.set_world_comm(None)
    m, data = _model()
    traj = FusedAdamEngine(m, chunks=2).run_adam(data["guess"], nsteps=4, learning_rate=2e-3,
                                                 param_bounds=bounds)
    torch.testing.assert_close(traj, ref, rtol=2e-5, atol=2e-6)


def _dist_engine(rank, size, zero, chunks, bounded):
    comm = mg.get_world_comm()
    m, data = _model(comm)
    bounds = [(-2.3, -1.6) if i % 2 == 0 else (None, -0.2) for i in range(NP)] if bounded else None
    eng = FusedAdamEngine(m, zero=zero, chunks=chunks)
    traj = eng.run_adam(data["guess"], nsteps=4, learning_rate=2e-3, param_bounds=bounds)
    return traj.numpy(), float(eng.loss[0]), eng.zero, eng.C


@pytest.mark.parametrize("size,zero,chunks,bounded", [(2, True, 3, False), (3, True, 4, False),
                                                      (2, False, 1, False), (2, True, 2, True)])
def test_engine_distributed_matches_single_rank(size, zero, chunks, bounded):
    res = run_distributed(_dist_engine, size, zero, chunks, bounded)
    bounds = [(-2.3, -1.6) if i % 2 == 0 else (None, -0.2) for i in range(NP)] if bounded else None
    ref = _generic_traj(4, bounds).numpy()
    for traj, loss, z, nc in res:
        assert z == zero
        np.testing.assert_allclose(traj, ref, rtol=3e-5, atol=3e-6)
        # every rank holds bitwise identical parameters (single owner per slice)
        np.testing.assert_array_equal(traj, res[0][0])


def _owner_model(comm, placement):
    data = make_population_data(num_params=NP, num_halos=NH, seed=11, comm=comm, device="cpu",
                                placement=placement)
    m = PopulationSMFModel(aux_data=data, comm=comm)
    m.set_target_from_truth()
    return m, data


def _dist_owner(rank, size, bounded, history):
    comm = mg.get_world_comm()
    m, data = _owner_model(comm, "owner")
    lo, hi = m.engine_support_units()
    ub = data["owner_units"]
    assert ub[rank] <= lo and hi <= ub[rank + 1]
    bounds = [(-2.3, -1.6) if i % 2 == 0 else (None, -0.2) for i in range(NP)] if bounded else None
    eng = FusedAdamEngine(m)
    traj = eng.run_adam(data["guess"], nsteps=4, learning_rate=2e-3, param_bounds=bounds,
                        history=history)
    return traj.numpy(), eng.params().numpy(), float(eng.loss[0]), eng.owner, ub


@pytest.mark.parametrize("size,bounded,history", [(2, False, "full"), (3, False, "full"),
                                                  (2, True, "full"), (3, False, "last")])
def test_engine_owner_placement_matches_single_rank(size, bounded, history):
    """Population-owner placement: same global catalog, no gradient collective; the
    trajectory equals the single-rank fit (the data set does not depend on placement)."""
    res = run_distributed(_dist_owner, size, bounded, history)
    bounds = [(-2.3, -1.6) if i % 2 == 0 else (None, -0.2) for i in range(NP)] if bounded else None
    ref = _generic_traj(4, bounds).numpy()
    if history == "last":
        ref = ref[[0, -1]]
    for traj, params, loss, owner, ub in res:
        assert owner and len(ub) == size + 1
        np.testing.assert_allclose(traj, ref, rtol=3e-5, atol=3e-6)
        np.testing.assert_array_equal(traj[-1], params)
        np.testing.assert_array_equal(traj, res[0][0])


def _dist_owner_fallback(rank, size):
    # hashed placement: every rank touches every population -> owner mode is refused
    # collectively and the engine runs the dense ZeRO schedule
    comm = mg.get_world_comm()
    m, data = _owner_model(comm, "hashed")
    m.aux_data["owner_units"] = [0, NP // 4, NP // 2][:size] + [NP // 2]
    eng = FusedAdamEngine(m, chunks=2)
    traj = eng.run_adam(data["guess"], nsteps=2, learning_rate=2e-3)
    return eng.owner, eng.zero, traj.numpy()


def test_engine_owner_mode_refused_for_dense_data():
    res = run_distributed(_dist_owner_fallback, 2)
    ref = _generic_traj(2).numpy()
    for owner, zero, traj in res:
        assert not owner and zero
        np.testing.assert_allclose(traj, ref, rtol=3e-5, atol=3e-6)


def test_owner_bounds_balanced():
    from multigrad_amd.models.population import owner_bounds
    J, N = 5000, 1 << 18
    for W in (2, 3, 8):
        ub = owner_bounds(N, J, 5, W, "cpu")
        assert ub[0] == 0 and ub[-1] == J and all(u % 2 == 0 for u in ub[:-1])
        assert all(a < b for a, b in zip(ub, ub[1:]))
        idx = torch.arange(N)
        from multigrad_amd.models.population import _global_pop
        cnt = torch.bincount(_global_pop(idx, 5, J), minlength=J)
        per = [int(cnt[a:b].sum()) for a, b in zip(ub, ub[1:])]
        assert sum(per) == N and max(per) - min(per) <= 3 * 80, per


def _resume_run(rank, size, placement, tmp, history, bounded):
    comm = mg.get_world_comm() if size > 1 else None
    if comm is None:
        C.set_world_comm(None)
    m, data = _owner_model(comm, placement)
    bounds = [(-2.3, -1.6) if i % 2 == 0 else (None, -0.2) for i in range(NP)] if bounded else None
    kw = dict(learning_rate=2e-3, param_bounds=bounds, history=history)
    full = FusedAdamEngine(m, chunks=2).run_adam(data["guess"], nsteps=6, **kw)
    ck = f"{tmp}/eng.ckpt"
    e1 = FusedAdamEngine(m, chunks=2)
    # a run of nsteps=6 interrupted after 4 steps, with its checkpoint from step 3
    e1.setup(data["guess"], 6, bounds, 2e-3, history=history)
    for i in range(4):
        e1.step()
        if i + 1 == 3:
            e1.save_checkpoint(ck)
    e2 = FusedAdamEngine(m, chunks=2)
    resumed = e2.run_adam(data["guess"], nsteps=6, resume_from=ck, **kw)
    mode = "owner" if e2.owner else "zero" if e2.zero else "replicated"
    return full.numpy(), resumed.numpy(), mode


@pytest.mark.parametrize("size,placement,history,bounded",
                         [(1, "hashed", "full", False), (1, "hashed", "last", True),
                          (2, "hashed", "full", True), (2, "owner", "full", False),
                          (3, "owner", "last", True)])
def test_engine_checkpoint_resume(tmp_path, size, placement, history, bounded):
    if size == 1:
        res = [_resume_run(0, 1, placement, str(tmp_path), history, bounded)]
    else:
        res = run_distributed(_resume_run, size, placement, str(tmp_path), history, bounded)
    for full, resumed, mode in res:
        assert mode == {("hashed", 1): "replicated", ("hashed", 2): "zero"}.get(
            (placement, size), "owner")
        np.testing.assert_array_equal(resumed, full)


def test_engine_rejects_unknown_options():
    C.set_world_comm(None)
    m, data = _model()
    with pytest.raises(TypeError):
        FusedAdamEngine(m).run_adam(data["guess"], nsteps=1, not_an_option=3)


def _zero_layout_resume(rank, size, tmp):
    comm = mg.get_world_comm()
    data = make_population_data(num_params=NP, num_halos=NH, seed=11, comm=comm, device="cpu",
                                layout="lanes")
    m = PopulationSMFModel(aux_data=data, comm=comm)
    m.set_target_from_truth()
    ck = f"{tmp}/zero.ckpt"
    e1 = FusedAdamEngine(m, zero=True, chunks=2)
    e1.setup(data["guess"], 4, None, 2e-3)
    e1.step()
    e1.save_checkpoint(ck)
    # another starting point: a third of the populations start narrow (bin width > 0.5
    # sigma), so the lanes are grouped differently and the internal order changes
    g2 = data["guess"].clone()
    g2[1::6] = -1.4
    e2 = FusedAdamEngine(m, zero=True, chunks=2)
    try:
        e2.run_adam(g2, nsteps=4, learning_rate=2e-3, resume_from=ck)
    except ValueError as exc:
        return "refused" if "different lanes layout" in str(exc) else str(exc)
    return "loaded"


def test_zero_checkpoint_with_another_lanes_layout_is_refused(tmp_path):
    """a ZeRO checkpoint loaded into an engine whose lanes layout differs is
    refused with a clear error (its slices would hold other parameters)."""
    res = run_distributed(_zero_layout_resume, 2, str(tmp_path))
    assert res == ["refused", "refused"], res
