"""All-to-all-v (``Comm.all_to_all_v``) and the engine's setup-time re-partition of a
data-parallel shard by parameter owner, on gloo ranks (CPU).

Reference behaviour kept: the user shards the catalog arbitrarily
(``np.array_split(...)[rank]``, reference tests/smf_example/smf_grad_descent.py:28) and the
fit is the same at any world size (partition invariance, reference tests/test_mpi.py).
"""
import os

import numpy as np
import pytest
import torch

import multigrad_amd as mg
from multigrad_amd.engine.fused import FusedAdamEngine
from multigrad_amd.models.population import (PopulationSMFModel, make_population_data,
                                             owner_bounds, owner_bounds_from_counts,
                                             repartition_by_owner)
from multigrad_amd.parallel import comm as C

from distributed import run_distributed

NP, NH = 120, 4000


def _a2a(rank, size, seed):
    comm = mg.get_world_comm()
    g = torch.Generator().manual_seed(seed)
    counts = torch.randint(0, 7, (size, size), generator=g)     # [src][dst], same on all ranks
    counts[0, size - 1] = 0                                        # an empty segment
    out = {}
    for dtype, row in ((torch.float32, ()), (torch.int32, (2,)), (torch.float64, (3,)),
                       (torch.int16, (2,))):
        sc = counts[rank].tolist()
        n = sum(sc)
        # row j of rank r: value r * 1000 + j (exact in every dtype used)
        base = (rank * 1000 + torch.arange(n, dtype=torch.float64)).reshape((n,) + (1,) * len(row))
        t = (base.expand((n,) + row) if row else base.reshape(n)).to(dtype).contiguous()
        got, rc = comm.all_to_all_v(t, sc)
        out[str(dtype)] = (got.double().numpy(), rc)
    return counts.numpy(), out


@pytest.mark.parametrize("size", [2, 3, 4, 8])
def test_all_to_all_v_gloo(size):
    res = run_distributed(_a2a, size, 5 + size, timeout=300)
    counts = res[0][0]
    for r, (cnt, out) in enumerate(res):
        np.testing.assert_array_equal(cnt, counts)
        for key, (got, rc) in out.items():
            assert rc == [int(counts[q, r]) for q in range(size)]
            want = []
            for q in range(size):
                start = int(counts[q, :r].sum())
                want.extend(q * 1000 + start + j for j in range(int(counts[q, r])))
            w = np.asarray(want, dtype=np.float64)
            flat = got.reshape(got.shape[0], -1)
            for c in range(flat.shape[1]):
                np.testing.assert_array_equal(flat[:, c], w, err_msg=f"{key} column {c}")


def test_all_to_all_v_serial_and_checks():
    comm = C.SerialComm()
    t = torch.arange(6.0).reshape(3, 2)
    got, rc = comm.all_to_all_v(t, [3])
    assert rc == [3] and torch.equal(got, t) and got.data_ptr() != t.data_ptr()
    with pytest.raises(ValueError):
        comm.all_to_all_v(t, [2])


def test_owner_bounds_from_counts_matches_generator():
    from multigrad_amd.models.population import _GEN_CHUNK, _global_pop  # noqa: F401
    for size in (1, 2, 3, 8):
        b1 = owner_bounds(NH, NP // 2, 11, size, "cpu")
        idx = torch.arange(NH, dtype=torch.int64)
        cnt = torch.bincount(_global_pop(idx, 11, NP // 2), minlength=NP // 2)
        assert owner_bounds_from_counts(cnt, size) == b1


def _repart(rank, size, mode):
    os.environ["MULTIGRAD_REPARTITION"] = mode
    comm = mg.get_world_comm()
    hashed = make_population_data(num_params=NP, num_halos=NH, seed=11, comm=comm, device="cpu")
    owner = make_population_data(num_params=NP, num_halos=NH, seed=11, comm=comm, device="cpu",
                                 placement="owner")
    assert hashed["placement"] == "hashed" and hashed["shard"].layout == "tiles"
    repartition_by_owner(hashed, comm)
    a, b = hashed["shard"], owner["shard"]
    same = (torch.equal(a.x, b.x) and torch.equal(a.pop, b.pop) and torch.equal(a.counts, b.counts)
            and hashed["owner_units"] == owner["owner_units"])
    rec = hashed["repartition"]
    return same, rec["halos_before"], rec["halos_after"], a.layout, a.lane_order


@pytest.mark.parametrize("size", [2, 3])
def test_repartition_gives_the_owner_placement_bitwise(size):
    res = run_distributed(_repart, size, "1", timeout=300)
    assert all(r[0] for r in res)
    assert sum(r[1] for r in res) == NH == sum(r[2] for r in res)
    assert all(r[3] == "lanes" and r[4] == "global" for r in res)


def _engine_default(rank, size, history):
    os.environ.pop("MULTIGRAD_REPARTITION", None)   # the library default
    comm = mg.get_world_comm()
    data = make_population_data(num_params=NP, num_halos=NH, seed=11, comm=comm, device="cpu")
    m = PopulationSMFModel(aux_data=data, comm=comm)
    m.set_target_from_truth()
    eng = FusedAdamEngine(m)
    traj = eng.run_adam(data["guess"], nsteps=4, learning_rate=2e-3, history=history)
    return (traj.numpy(), float(eng.loss[0]), eng.owner, eng.zero,
            eng.grad_collective_name(), dict(eng.repartitioned or {}))


@pytest.mark.parametrize("size,history", [(2, "full"), (3, "full"), (4, "last")])
def test_engine_repartitions_hashed_shards_by_default(size, history):
    C.set_world_comm(None)
    data = make_population_data(num_params=NP, num_halos=NH, seed=11, device="cpu")
    m = PopulationSMFModel(aux_data=data)
    m.set_target_from_truth()
    ref = FusedAdamEngine(m).run_adam(data["guess"], nsteps=4, learning_rate=2e-3,
                                       history=history).numpy()
    res = run_distributed(_engine_default, size, history, timeout=300)
    for traj, loss, owner, zero, name, rec in res:
        assert owner, "re-partitioned data must run in owner mode"
        assert name.startswith("none"), name          # no gradient collective per step
        assert rec["halos_after"] > 0 and sum(rec["sent_to"]) == rec["halos_before"]
        np.testing.assert_allclose(traj, ref, rtol=2e-5, atol=2e-6)
    for r in res[1:]:
        np.testing.assert_array_equal(r[0], res[0][0])   # replicated bits on every rank
    assert sum(r[5]["halos_after"] for r in res) == NH


def _engine_off(rank, size):
    os.environ.pop("MULTIGRAD_REPARTITION", None)   # the keyword decides
    comm = mg.get_world_comm()
    data = make_population_data(num_params=NP, num_halos=NH, seed=11, comm=comm, device="cpu")
    m = PopulationSMFModel(aux_data=data, comm=comm)
    m.set_target_from_truth()
    eng = FusedAdamEngine(m, repartition=False)
    eng.run_adam(data["guess"], nsteps=2, learning_rate=2e-3)
    return eng.owner, eng.zero, data["placement"]


def test_engine_repartition_can_be_turned_off():
    os.environ.pop("MULTIGRAD_REPARTITION", None)
    res = run_distributed(_engine_off, 2, timeout=300)
    assert all((not o) and z and p == "hashed" for o, z, p in res)


def _cached_after_repartition(rank, size):
    os.environ.pop("MULTIGRAD_REPARTITION", None)
    comm = mg.get_world_comm()
    data = make_population_data(num_params=NP, num_halos=NH, seed=11, comm=comm, device="cpu")
    m = PopulationSMFModel(aux_data=data, comm=comm)
    m.set_target_from_truth()
    e1 = m.fused_engine()
    e1.run_adam(data["guess"], nsteps=2, learning_rate=2e-3)
    hashed_id = id(e1._cache_shard)
    e2 = m.fused_engine()
    e2.run_adam(data["guess"], nsteps=2, learning_rate=2e-3)
    return (e1 is e2, data["placement"], len(m._engine_cache), e2.stats["setups"],
            id(data["shard"]) == hashed_id)


def test_cached_engine_survives_its_repartition():
    """The engine re-partitions the model's data at its first setup; the model's engine
    cache is re-keyed to the owner shard, so the next run_* call re-uses the same engine
    (one cache entry, a second setup of the same object)."""
    res = run_distributed(_cached_after_repartition, 2, timeout=300)
    for same, placement, entries, setups, pinned in res:
        assert same and placement == "owner" and entries == 1 and setups == 2 and pinned


def test_replaced_shard_drops_the_cached_engine():
    C.set_world_comm(None)
    data = make_population_data(num_params=NP, num_halos=NH, seed=11, device="cpu")
    m = PopulationSMFModel(aux_data=data)
    m.set_target_from_truth()
    e1 = m.fused_engine()
    m.aux_data["shard"] = make_population_data(num_params=NP, num_halos=NH, seed=12,
                                               device="cpu")["shard"]
    e2 = m.fused_engine()
    assert e2 is not e1 and len(m._engine_cache) == 1
    assert m.fused_engine() is e2
