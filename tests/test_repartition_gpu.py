"""Peer-memory all-to-all-v (csrc/xgmi.hip:xgmi_a2a_pull_kernel) and the engine's
setup-time re-partition by parameter owner, with several processes sharing one MI355X
(gloo for the host-side collectives: RCCL refuses two ranks on one GPU)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from distributed import run_distributed  # noqa: E402


def _a2a(rank, size, corrupt):
    import multigrad_amd as mg
    from multigrad_amd.parallel.xgmi import status
    if corrupt is not None:
        os.environ["MULTIGRAD_XGMI_SELFTEST_CORRUPT"] = str(corrupt)
    comm = mg.get_world_comm()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(77)
    counts = torch.randint(0, 300_000, (size, size), generator=g)
    counts[size - 1, 0] = 0
    sc = counts[rank].tolist()
    n = sum(sc)
    # row j of rank r: (r, j) as int32 pair + a float payload
    t = torch.stack([torch.full((n,), rank, dtype=torch.int32),
                     torch.arange(n, dtype=torch.int32)], 1).to(dev)
    got, rc = comm.all_to_all_v(t, sc)
    f = (torch.arange(n, dtype=torch.float32, device=dev) * 0.5 + rank)
    gotf, _ = comm.all_to_all_v(f, sc)
    torch.cuda.synchronize()
    return counts.numpy(), got.cpu().numpy(), gotf.cpu().numpy(), rc, status(comm).get("all-to-all")


def _want(counts, r):
    rows, fl = [], []
    for q in range(counts.shape[0]):
        start = int(counts[q, :r].sum())
        for j in range(start, start + int(counts[q, r])):
            rows.append((q, j))
            fl.append(j * 0.5 + q)
    return np.asarray(rows, dtype=np.int32).reshape(-1, 2), np.asarray(fl, dtype=np.float32)


@pytest.mark.parametrize("size", [2, 4])
def test_peer_all_to_all_v_procs_one_gpu(size):
    res = run_distributed(_a2a, size, None, timeout=300)
    for r, (counts, got, gotf, rc, st) in enumerate(res):
        w, wf = _want(counts, r)
        assert rc == [int(counts[q, r]) for q in range(size)]
        np.testing.assert_array_equal(got, w)
        np.testing.assert_array_equal(gotf, wf)
        assert st and all(e["path"] == "peer memory pull" and e["ok"] for e in st), st


def test_peer_all_to_all_v_checksum_mismatch_falls_back():
    res = run_distributed(_a2a, 2, 1, timeout=300)
    for r, (counts, got, gotf, rc, st) in enumerate(res):
        w, wf = _want(counts, r)
        np.testing.assert_array_equal(got, w)      # redone on the fallback path
        np.testing.assert_array_equal(gotf, wf)
        assert st[0]["ok"] is False and "checksum" in st[0]["fallback"], st
        assert st[1]["ok"] and st[1]["path"].startswith("gloo"), st


NP, NH = 6000, 400_000


def _fit(rank, size, repartition):
    import multigrad_amd as mg
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    from multigrad_amd.parallel.xgmi import status
    os.environ.pop("MULTIGRAD_REPARTITION", None)
    comm = mg.get_world_comm()
    dev = torch.device("cuda", 0)
    data = make_population_data(NP, NH, seed=21, comm=comm, device=dev)
    model = PopulationSMFModel(aux_data=data, comm=comm)
    model.set_target_from_truth()
    eng = FusedAdamEngine(model, repartition=repartition)
    traj = eng.run_adam(data["guess"], nsteps=6, learning_rate=1e-3)
    loss = eng.last_loss()
    return (traj.cpu().numpy(), loss, eng.owner, eng.grad_collective_name(),
            data["placement"], status(comm).get("all-to-all"))


@pytest.mark.parametrize("size", [2, 4])
def test_engine_repartition_procs_one_gpu_matches_single_rank(size):
    import multigrad_amd.parallel.comm as C
    C.set_world_comm(None)
    t1, l1, _, _, _, _ = _fit(0, 1, None)
    res = run_distributed(_fit, size, None, timeout=600)
    for traj, loss, owner, name, placement, st in res:
        assert owner and placement == "owner" and name.startswith("none"), name
        assert st and st[-1]["path"] == "peer memory pull", st
        np.testing.assert_allclose(traj, t1, rtol=2e-5, atol=2e-6)
        assert loss == pytest.approx(l1, rel=1e-5)
    for r in res[1:]:
        np.testing.assert_array_equal(r[0], res[0][0])
