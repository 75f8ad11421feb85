"""One-shot peer-memory all-reduce (csrc/xgmi.hip) with two processes sharing one MI355X:
IPC export/open of the uncached regions, the flag protocol over many back-to-back calls
(both slots reused), HIP-graph replay, and the engine with MULTIGRAD_ALLREDUCE=oneshot."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from distributed import run_distributed  # noqa: E402


def _protocol(rank, size, ncalls):
    import multigrad_amd as mg
    from multigrad_amd.parallel.xgmi import connect
    comm = mg.get_world_comm()
    dev = torch.device("cuda", 0)
    ar = connect(comm, timeout_s=10.0)
    assert ar is not None
    g = torch.Generator().manual_seed(100 + rank)
    vals = [torch.randn(int(n), generator=g) for n in np.arange(ncalls) % 64 + 1]
    outs = []
    for v in vals:
        t = v.to(dev)
        ar(t)
        outs.append(t.cpu())
    # graph replay: the sequence number lives in device memory
    t = torch.ones(16, device=dev) * (rank + 1)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph):
            ar(t)
    torch.cuda.current_stream().wait_stream(s)
    reps = []
    for _ in range(5):
        t.fill_(rank + 1.0)
        graph.replay()
        reps.append(t.cpu().clone())
    torch.cuda.synchronize()
    ok = ar.ok()
    ar.close()
    return [v.numpy() for v in vals], [o.numpy() for o in outs], [r.numpy() for r in reps], ok


def test_oneshot_protocol_two_procs_one_gpu():
    res = run_distributed(_protocol, 2, 200, timeout=300)
    (v0, o0, r0, ok0), (v1, o1, r1, ok1) = res
    assert ok0 and ok1
    for a, b, x, y in zip(v0, v1, o0, o1):
        np.testing.assert_array_equal(x, y)              # identical bits on every rank
        np.testing.assert_allclose(x, a + b, rtol=1e-6, atol=1e-6)
    for x, y in zip(r0, r1):
        np.testing.assert_array_equal(x, np.full(16, 3.0, dtype=np.float32))
        np.testing.assert_array_equal(y, x)


def _engine(rank, size, oneshot, graph=None):
    import os
    os.environ["MULTIGRAD_ALLREDUCE"] = "oneshot" if oneshot else "rccl"
    if graph is not None:
        os.environ["MULTIGRAD_GRAPH"] = "1" if graph else "0"
    import multigrad_amd as mg
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    comm = mg.get_world_comm()
    dev = torch.device("cuda", 0)
    data = make_population_data(6000, 400_000, seed=21, comm=comm, device=dev, placement="owner")
    model = PopulationSMFModel(aux_data=data, comm=comm)
    model.set_target_from_truth()
    eng = FusedAdamEngine(model)
    traj = eng.run_adam(data["guess"], nsteps=6, learning_rate=1e-3)
    used = bool(getattr(comm, "_oneshot", None))
    return traj.cpu().numpy(), used, bool(eng.use_graph and eng.graph is not None), eng.tuning


def test_owner_engine_graph_replay_matches_eager():
    """Owner placement, two ranks: the pipelined step (forward + fused update, one-shot
    epilogue) replayed from a HIP graph on every rank gives the eager trajectory bit for
    bit; the auto policy (setup-time timing of both, state restored) does too."""
    eager = run_distributed(_engine, 2, True, False, timeout=600)
    graph = run_distributed(_engine, 2, True, True, timeout=600)
    auto = run_distributed(_engine, 2, True, None, timeout=600)
    assert not eager[0][2] and graph[0][2] and graph[1][2]
    assert auto[0][3] is not None and auto[0][3]["chosen"] == auto[1][3]["chosen"]
    for r in range(2):
        np.testing.assert_array_equal(graph[r][0], eager[r][0])
        np.testing.assert_array_equal(auto[r][0], eager[r][0])


def test_engine_with_oneshot_sumstat_allreduce():
    ref = run_distributed(_engine, 2, False, timeout=600)
    res = run_distributed(_engine, 2, True, timeout=600)
    assert not ref[0][1] and res[0][1] and res[1][1]
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_allclose(res[0][0], ref[0][0], rtol=1e-5, atol=1e-6)


def _late_peer(rank, size):
    """Rank 1 reaches the exchange 1.5 s after rank 0 (timeout 0.3 s): rank 0's result
    must be NaN-poisoned and check() must raise -- never a silently partial sum; after a
    collective reset() the protocol works again."""
    import time
    import multigrad_amd as mg
    from multigrad_amd.parallel.xgmi import CollectiveTimeout, connect
    comm = mg.get_world_comm()
    dev = torch.device("cuda", 0)
    ar = connect(comm, timeout_s=0.3)
    assert ar is not None
    comm.barrier()
    if rank == 1:
        time.sleep(1.5)
    t = torch.full((8,), float(rank + 1), device=dev)
    ar(t)
    torch.cuda.synchronize()
    vals = t.cpu().numpy()
    try:
        ar.check("test")
        raised = ""
    except CollectiveTimeout as e:
        raised = str(e)
    ar.reset(comm)
    t2 = torch.full((4,), float(rank + 1), device=dev)
    ar(t2)
    after = t2.cpu().numpy()
    ok_after = ar.ok()
    ar.close()
    return vals, raised, after, ok_after


def test_oneshot_late_peer_fails_loudly():
    (v0, e0, a0, ok0), (v1, e1, a1, ok1) = run_distributed(_late_peer, 2, timeout=300)
    assert np.isnan(v0).all() and "timed out" in e0 and "rank 0/2" in e0
    np.testing.assert_array_equal(v1, np.full(8, 3.0, dtype=np.float32))  # the late rank
    assert e1 == ""                                                      # saw both values
    np.testing.assert_array_equal(a0, np.full(4, 3.0, dtype=np.float32))
    np.testing.assert_array_equal(a1, a0)
    assert ok0 and ok1


def _engine_err(rank, size):
    import multigrad_amd as mg
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    from multigrad_amd.parallel.xgmi import CollectiveTimeout
    comm = mg.get_world_comm()
    dev = torch.device("cuda", 0)
    data = make_population_data(4000, 200_000, seed=5, comm=comm, device=dev, placement="owner")
    model = PopulationSMFModel(aux_data=data, comm=comm)
    model.set_target_from_truth()
    eng = FusedAdamEngine(model)
    eng.setup(data["guess"], nsteps=4, learning_rate=1e-3)
    assert eng.oneshot is not None
    eng.step()
    eng.step()
    eng.params()  # clean so far
    if rank == 0:
        eng.oneshot.err.fill_(1)  # as a timed-out exchange leaves it
    out = []
    # local checks (last_loss, state_dict) raise on the failed rank only; the collective
    # ones (params, trajectory: they all-gather afterwards) raise on every rank together
    for fn in (eng.last_loss, eng.state_dict, eng.params, eng.trajectory):
        try:
            fn()
            out.append(False)
        except CollectiveTimeout:
            out.append(True)
    return out


def test_engine_raises_on_exchange_error():
    r0, r1 = run_distributed(_engine_err, 2, timeout=300)
    assert r0 == [True, True, True, True] and r1 == [False, False, True, True]


# ------------------------------------------------ connect-time stress self-tests (2 / 8 ranks)
def _stress(rank, size, corrupt):
    import os
    if corrupt:
        os.environ["MULTIGRAD_XGMI_SELFTEST_CORRUPT"] = "1"
    import multigrad_amd as mg
    from multigrad_amd.parallel.xgmi import STRESS_REPS, connect, connect_twoshot, status
    comm = mg.get_world_comm()
    one = connect(comm, timeout_s=20.0)
    two = connect_twoshot(comm, 4 * size * 4096, timeout_s=20.0)
    got = (one is not None, two is not None)
    for ctx in (one, two):
        if ctx is not None:
            ctx.close()
    torch.cuda.synchronize()
    return got, status(comm), STRESS_REPS


@pytest.mark.parametrize("size", [2, 8])
def test_stress_selftest_passes_and_corruption_falls_back(size):
    """The connect-time self-tests run 32 back-to-back device-only exchanges with
    step-unique values, one verification at the end: they pass on 2 and 8 processes
    sharing the GPU; a rank that corrupts its slice in one exchange (test hook) makes every
    rank fail them and fall back to RCCL, with the reason recorded."""
    ok = run_distributed(_stress, size, False, timeout=600)
    for got, st, reps in ok:
        assert got == (True, True), st
        assert st["one-shot"][-1]["ok"] and st["one-shot"][-1]["stress_exchanges"] == reps >= 32
        assert st["two-shot"][-1]["ok"] and st["two-shot"][-1]["stress_exchanges"] == reps
    bad = run_distributed(_stress, size, True, timeout=600)
    for got, st, reps in bad:
        assert got == (False, False), st
        for kind in ("one-shot", "two-shot"):
            e = st[kind][-1]
            assert not e["ok"] and "stress self-test failed" in e["fallback"] and "RCCL" in e["fallback"]
