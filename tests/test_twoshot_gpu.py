"""Two-shot peer-memory reduce-scatter -> Adam -> all-gather (csrc/xgmi.hip) with two
processes sharing one MI355X: the flag protocol and rank-order sum, graph replay, the Adam
modes against a PyTorch reference, the hashed-placement engine against the RCCL/gloo
gradient path (bitwise), and a late peer failing loudly."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from distributed import run_distributed  # noqa: E402


def _protocol(rank, size, numel, reps):
    import multigrad_amd as mg
    from multigrad_amd.parallel.xgmi import connect_twoshot
    comm = mg.get_world_comm()
    ts = connect_twoshot(comm, numel, timeout_s=10.0)
    assert ts is not None
    g = torch.Generator().manual_seed(7 + rank)
    grads, outs = [], []
    lo, n = ts.slice()
    for _ in range(reps):
        x = torch.randn(numel, generator=g)
        grads.append(x.numpy())
        ts.grad.copy_(x.cuda())
        ts.step(lo, n, 0)
        outs.append(ts.theta.cpu().numpy().copy())
    # graph replay: sequence number and flags live in device memory
    ts.grad.fill_(rank + 1.0)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph):
            ts.step(lo, n, 0)
    torch.cuda.current_stream().wait_stream(s)
    reps_out = []
    for _ in range(3):
        graph.replay()
        reps_out.append(ts.theta.cpu().numpy().copy())
    ok = ts.ok()
    ts.close()
    return grads, outs, reps_out, ok


def test_twoshot_protocol_two_procs_one_gpu():
    numel = 8 * 1000 + 8
    (g0, o0, r0, ok0), (g1, o1, r1, ok1) = run_distributed(_protocol, 2, numel, 6, timeout=300)
    assert ok0 and ok1
    for a, b, x, y in zip(g0, g1, o0, o1):
        np.testing.assert_array_equal(x, y)                       # same bits on every rank
        np.testing.assert_array_equal(x, (a + b).astype(np.float32))  # rank-order fp32 sum
    for x, y in zip(r0, r1):
        np.testing.assert_array_equal(x, np.full(numel, 3.0, dtype=np.float32))
        np.testing.assert_array_equal(y, x)


def _adam_modes(rank, size):
    import multigrad_amd as mg
    from multigrad_amd.optim.transforms import Bounds
    from multigrad_amd.parallel.xgmi import connect_twoshot
    comm = mg.get_world_comm()
    numel = 4096
    ts = connect_twoshot(comm, numel, timeout_s=10.0)
    lo, n = ts.slice()
    dev = ts.grad.device
    gen = torch.Generator().manual_seed(3)
    theta0 = torch.randn(numel, generator=gen)
    grads = [torch.randn(numel, generator=gen) for _ in range(2 * 3)]
    spec = [(-3.0, 3.0) if i % 3 == 0 else (-5.0, None) if i % 3 == 1 else (None, None)
            for i in range(numel)]
    bnd = Bounds.from_spec(spec, numel, device=dev)
    res = {}
    for mode in (1, 2):
        ts.theta.copy_(theta0.to(dev))
        m = torch.zeros(n, device=dev)
        v = torch.zeros(n, device=dev)
        bl = None if mode == 1 else Bounds(bnd.lo[lo:lo + n].contiguous(), bnd.hi[lo:lo + n].contiguous(),
                                          bnd.kind[lo:lo + n].contiguous())
        u = None if mode == 1 else bl.forward(ts.theta[lo:lo + n]).contiguous()
        traj = torch.zeros((4, n), device=dev)
        step = torch.zeros(2, dtype=torch.int32, device=dev)
        for k in range(3):
            ts.grad.copy_(grads[2 * k + rank].to(dev))
            ts.step(lo, n, mode, m=m, v=v, u=u, bounds=bl, traj=traj.reshape(-1), traj_stride=n,
                    step=step, lr=0.05)
        torch.cuda.synchronize()
        res[mode] = (ts.theta.cpu().numpy().copy(), traj.cpu().numpy(), int(step[0]))
    ok = ts.ok()
    ts.close()
    return res, ok, lo, n


def test_twoshot_adam_modes_match_reference():
    from multigrad_amd.ops.adam import adam_step_
    from multigrad_amd.optim.transforms import Bounds
    out = run_distributed(_adam_modes, 2, timeout=300)
    numel = 4096
    gen = torch.Generator().manual_seed(3)
    theta0 = torch.randn(numel, generator=gen)
    grads = [torch.randn(numel, generator=gen) for _ in range(6)]
    spec = [(-3.0, 3.0) if i % 3 == 0 else (-5.0, None) if i % 3 == 1 else (None, None)
            for i in range(numel)]
    bnd = Bounds.from_spec(spec, numel)
    for mode in (1, 2):
        p = theta0.clone()
        u = bnd.forward(p) if mode == 2 else p
        m = torch.zeros(numel)
        v = torch.zeros(numel)
        step = torch.zeros(2, dtype=torch.int32)
        for k in range(3):
            g = grads[2 * k] + grads[2 * k + 1]
            adam_step_(u, m, v, g, p if mode == 2 else None, step, 0.05, 0.9, 0.999, 1e-8,
                       bnd if mode == 2 else None)
        want = bnd.inverse(u) if mode == 2 else u
        for res, ok, lo, n in out:
            assert ok
            theta, traj, st = res[mode]
            assert st == 3
            np.testing.assert_allclose(theta, want.numpy(), rtol=1e-5, atol=2e-6)  # fp32 CPU vs GPU (fma)
            np.testing.assert_allclose(traj[3], want.numpy()[lo:lo + n], rtol=1e-5, atol=2e-6)
        np.testing.assert_array_equal(out[0][0][mode][0], out[1][0][mode][0])


def _engine_hashed(rank, size, twoshot, bounded, chunks, layout="auto", graph=None, side="auto",
                   legacy=False):
    lane_order = "local" if layout == "lanes" else None
    if layout == "lanes-global":  # global slot order: internal parameter order, residual VJP
        layout, lane_order = "lanes", "global"
    if graph is not None:
        os.environ["MULTIGRAD_GRAPH"] = "1" if graph else "0"
    os.environ["MULTIGRAD_TWOSHOT_SIDE_STREAM"] = side
    os.environ["MULTIGRAD_TWOSHOT"] = "1" if twoshot else "0"
    os.environ["MULTIGRAD_CHUNKS"] = str(chunks)
    import multigrad_amd as mg
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    comm = mg.get_world_comm()
    dev = torch.device("cuda", 0)
    data = make_population_data(6000, 300_000, seed=31, comm=comm, device=dev, placement="hashed",
                                layout=layout, lane_order=lane_order)
    model = PopulationSMFModel(aux_data=data, comm=comm)
    model.set_target_from_truth()
    eng = FusedAdamEngine(model)
    bounds = None
    if bounded:
        g = data["guess"].cpu()
        bounds = np.stack([g.numpy() - 0.5, g.numpy() + 0.7], 1)
        bounds[1::4, 1] = np.inf
    traj = eng.run_adam(data["guess"], nsteps=5, learning_rate=1e-3, param_bounds=bounds,
                        legacy_bounds_jacobian=legacy)
    sh = data["shard"]
    return (traj.cpu().numpy(), eng.twoshot is not None, eng.zero,
            f"{sh.layout}/{sh.lane_order}" if sh.layout == "lanes" else sh.layout,
            eng.grad_collective_name(), eng.C, eng.use_graph and eng.graph is not None,
            eng.ts_side, eng.tuning)


@pytest.mark.parametrize("bounded,chunks,layout,side", [
    (False, 1, "auto", "auto"), (True, 1, "auto", "auto"), (False, 3, "auto", "on"),
    (True, 4, "auto", "on"), (False, 3, "auto", "off"), (True, 2, "auto", "auto"),
    (False, 2, "lanes", "on"), (False, 2, "lanes-global", "auto"),
    (True, 2, "lanes-global", "off")])
def test_engine_hashed_twoshot_matches_rccl_path(bounded, chunks, layout, side):
    """One chunk, and several chunks whose exchanges run on the compute stream ("off"), on
    the side stream overlapping the next chunk's VJP and the next step's forward ("on"),
    or whichever the setup-time timing picked ("auto": the timing steps are undone): same
    bits as the RCCL/gloo path (the auto layout = tiles for hashed shards, and lanes in the
    local slot order with the recomputing VJP)."""
    ref = run_distributed(_engine_hashed, 2, False, bounded, chunks, layout, None, side,
                          timeout=600)
    res = run_distributed(_engine_hashed, 2, True, bounded, chunks, layout, None, side,
                          timeout=600)
    want = {"auto": "tiles", "lanes": "lanes/local", "lanes-global": "lanes/global"}[layout]
    assert all(r[2] and r[3] == want and r[5] == chunks for r in ref + res), ref[0][3]
    assert not ref[0][1] and res[0][1] and res[1][1], (ref[0][4], res[0][4])
    if chunks > 1:
        assert res[0][7] == res[1][7] and (res[0][7] if side == "on" else True)
        assert (res[0][8] is not None) == (side == "auto"), res[0][8]
        if side == "off":
            assert not res[0][7]
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(ref[0][0], ref[1][0])
    np.testing.assert_array_equal(res[0][0], ref[0][0])  # bitwise: same sums, same Adam bits


def _engine_hashed_rccl(rank, size, bounded):
    os.environ["MULTIGRAD_HASHED_EXCHANGE"] = "rccl"
    return _engine_hashed(rank, size, True, bounded, 2, "auto", None, "off")


@pytest.mark.parametrize("bounded", [False, True])
def test_engine_hashed_rccl_exchange_candidate(bounded):
    """The RCCL reduce-scatter / all-gather candidate of the hashed autotune, run on the
    two-shot context's buffers and shard layout (MULTIGRAD_HASHED_EXCHANGE=rccl): the
    same trajectory as the engine without a two-shot context."""
    ref = run_distributed(_engine_hashed, 2, False, bounded, 2, "auto", None, "off", timeout=600)
    res = run_distributed(_engine_hashed_rccl, 2, bounded, timeout=600)
    assert res[0][1] and "RCCL" in res[0][4], res[0][4]
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][0], ref[0][0])


@pytest.mark.parametrize("bounded", [False, True])
def test_engine_hashed_twoshot_graph_replay_matches_eager(bounded):
    """The whole hashed step (forward, one-shot epilogue, VJP, two-shot exchange) captured
    into one HIP graph per rank and replayed: the same trajectory bits as eager launches."""
    eager = run_distributed(_engine_hashed, 2, True, bounded, 1, "auto", False, timeout=600)
    graph = run_distributed(_engine_hashed, 2, True, bounded, 1, "auto", True, timeout=600)
    assert not eager[0][6] and graph[0][6] and graph[1][6]
    np.testing.assert_array_equal(graph[0][0], eager[0][0])
    np.testing.assert_array_equal(graph[1][0], eager[1][0])


def _late(rank, size):
    import time
    import multigrad_amd as mg
    from multigrad_amd.parallel.xgmi import CollectiveTimeout, connect_twoshot
    comm = mg.get_world_comm()
    ts = connect_twoshot(comm, 1024, timeout_s=0.3)
    comm.barrier()
    if rank == 1:
        time.sleep(1.5)
    ts.grad.fill_(1.0)
    lo, n = ts.slice()
    ts.step(lo, n, 0)
    torch.cuda.synchronize()
    nan_own = bool(torch.isnan(ts.theta[lo:lo + n]).all())
    try:
        ts.check("test")
        raised = False
    except CollectiveTimeout:
        raised = True
    ts.reset(comm)
    ts.grad.fill_(float(rank + 1))
    ts.step(lo, n, 0)
    torch.cuda.synchronize()
    after = ts.theta.cpu().numpy().copy()
    ok = ts.ok()
    ts.close()
    return nan_own, raised, after, ok


def test_twoshot_late_peer_fails_loudly():
    (n0, e0, a0, ok0), (n1, e1, a1, ok1) = run_distributed(_late, 2, timeout=300)
    assert n0 and e0             # rank 0 waited 0.3 s for rank 1's gradient: NaN + raise
    np.testing.assert_array_equal(a0, np.full(1024, 3.0, dtype=np.float32))
    np.testing.assert_array_equal(a1, a0)
    assert ok0 and ok1


def _ingraph(rank, size, graph):
    import multigrad_amd as mg
    from multigrad_amd import ingraph
    comm = mg.get_world_comm()
    if graph is False:  # the RCCL path for comparison
        os.environ["MULTIGRAD_TWOSHOT"] = "0"
    g = torch.Generator().manual_seed(11)
    x = torch.randn(4000, generator=g).cuda()
    data = dict(x=ingraph.distribute_data(x, comm))

    def loss_and_grad(d, p):  # sum over ranks of 0.5 * |x - p|^2 / N per coordinate
        r = d["x"][:, None] - p[None, :]
        return 0.5 * (r * r).sum() / x.numel(), -r.sum(0) / x.numel()

    guess = torch.tensor([0.5, -1.0, 2.0], device="cuda")
    df = ingraph.simple_grad_descent(data, loss_and_grad, guess, learning_rate=0.3,
                                     nsteps=20, comm=comm, graph=None)
    cached = getattr(comm, "_twoshot_ar", {})
    return (np.stack(df["params"].to_numpy()), np.asarray(df["loss"], dtype=np.float64),
            any(bool(v) for v in cached.values()))


def test_ingraph_descent_multirank_captured_matches_rccl():
    """ingraph.simple_grad_descent on two ranks: graph-captured with the two-shot all-reduce
    by default, matching the eager RCCL path and the closed-form descent."""
    out = run_distributed(_ingraph, 2, None, timeout=300)
    ref = run_distributed(_ingraph, 2, False, timeout=300)
    for (p, l, used), (pr, lr_, used_r) in zip(out, ref):
        assert used and not used_r
        np.testing.assert_allclose(p, pr, rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(l, lr_, rtol=1e-5, atol=1e-7)
    np.testing.assert_array_equal(out[0][0], out[1][0])  # same bits on both ranks
    # closed form: p_{k+1} = p_k - 0.3 (p_k - mean x)
    g = torch.Generator().manual_seed(11)
    mean = float(torch.randn(4000, generator=g).double().mean())
    p = np.array([0.5, -1.0, 2.0])
    for k in range(20):
        np.testing.assert_allclose(out[0][0][k], p, rtol=1e-4, atol=1e-5)
        p = p - 0.3 * (p - mean)


@pytest.mark.parametrize("size", [3, 4, 8])
def test_twoshot_protocol_more_ranks(size):
    """The flag protocol, the rank-order sum and graph replay with 3, 4 and 8 processes
    sharing one GPU (the driver's 8-GPU node runs 8): every rank ends with the same bits,
    equal to the fp32 sum in rank order."""
    numel = 4 * size * 257
    out = run_distributed(_protocol, size, numel, 3, timeout=600)
    grads = [o[0] for o in out]
    for rep in range(3):
        want = grads[0][rep].astype(np.float32)
        for r in range(1, size):
            want = (want + grads[r][rep]).astype(np.float32)
        for o in out:
            np.testing.assert_array_equal(o[1][rep], want)
    for o in out:
        assert o[3]
        for x in o[2]:
            np.testing.assert_array_equal(x, np.full(numel, size * (size + 1) / 2, dtype=np.float32))


@pytest.mark.parametrize("size", [4, 8])
def test_engine_hashed_twoshot_more_ranks(size):
    """The hashed engine step with 4 and 8 ranks on one GPU: the two-shot trajectory is the
    same on every rank and matches the RCCL/gloo path.  From 3 ranks on, the two paths add
    the W gradients in different orders (two-shot: fixed rank order; gloo: its ring/tree),
    so they agree to fp32 rounding rather than bitwise."""
    ref = run_distributed(_engine_hashed, size, False, False, 2, "auto", None, "on", timeout=900)
    res = run_distributed(_engine_hashed, size, True, False, 2, "auto", None, "on", timeout=900)
    assert all(r[1] for r in res) and not any(r[1] for r in ref)
    for r in range(size):
        np.testing.assert_array_equal(res[r][0], res[0][0])
        np.testing.assert_array_equal(ref[r][0], ref[0][0])
    np.testing.assert_allclose(res[0][0], ref[0][0], rtol=1e-6, atol=1e-7)


def _evict(rank, size):
    import multigrad_amd as mg
    from multigrad_amd import ingraph
    from multigrad_amd.parallel.xgmi import get_twoshot_allreduce, release_twoshot_allreduce
    comm = mg.get_world_comm()
    # a graph captured around the first size class (pins that context) ...
    x = torch.full((64,), float(rank + 1), device="cuda")
    ingraph.reduce_sum(x, comm)  # eager call: connects the size class before the capture
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g):
            y = ingraph.reduce_sum(x, comm)
    torch.cuda.current_stream().wait_stream(s)
    # ... an engine-style holder of the second ...
    held = get_twoshot_allreduce(comm, 4096, hold=True)
    # ... then five more size classes: the idle ones are evicted, the pinned / held stay
    for k in range(5):
        ingraph.reduce_sum(torch.ones(8192 * (k + 1), device="cuda"), comm)
    cache = comm._twoshot_ar
    first_alive = bool(cache[min(cache)]) and bool(cache[min(cache)].regions)
    held_alive = bool(held.regions)
    g.replay()
    torch.cuda.synchronize()
    out = y.cpu().numpy().copy()
    release_twoshot_allreduce(held)
    # a context closed by eviction raises on use instead of touching unmapped memory
    from multigrad_amd.parallel.xgmi import TwoShot
    closed = TwoShot.__new__(TwoShot)
    closed.regions = ()
    try:
        closed.step(0, 0, 0)
        raised = False
    except RuntimeError:
        raised = True
    n_live = sum(1 for t in cache.values() if t)
    return first_alive, held_alive, out, raised, n_live


def test_twoshot_allreduce_cache_keeps_pinned_and_held_contexts():
    """evicting the smallest cached all-reduce context must not close one a
    captured graph or an engine still uses.  Five more size classes are connected after a
    graph captured ingraph.reduce_sum on the first and an engine-style holder took the
    second; both survive, the replay sums correctly, idle contexts are evicted."""
    res = run_distributed(_evict, 2, timeout=300)
    for first_alive, held_alive, out, raised, n_live in res:
        assert first_alive and held_alive and raised
        np.testing.assert_array_equal(out, np.full(64, 3.0, dtype=np.float32))
        assert n_live <= 4 + 2  # at most _MAX_AR_CONTEXTS idle + the pinned + the held


def _bench_2rank(extra_env, *args):
    import json
    import socket
    import subprocess
    import sys
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # gloo for the device collectives: RCCL refuses two ranks on one GPU
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1",
               MULTIGRAD_PROGRESS="0", MULTIGRAD_DEVICE_COMM="0", **extra_env)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(repo, "bench.py"), "--gpus", "2", "--steps", "8", "--warmup", "2",
           "--params", "200000", "--halos", str(1 << 22), "--placement", "hashed",
           "--no-count-launches"] + list(args)
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400, cwd=repo)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return json.loads(lines[-1])


def test_autotune_drops_timed_out_candidate_and_bench_reports_it():
    """a candidate schedule whose peer-memory exchange times out during the
    setup autotune (test hook: rank 1 skips one exchange of the side-stream candidate) is
    dropped with its reason; the engine resets the protocol and keeps a surviving
    schedule, and bench.py still prints its line with the drop recorded."""
    rec = _bench_2rank({"MULTIGRAD_AUTOTUNE_FAULT": "ts_side=1:1",
                        "MULTIGRAD_ONESHOT_TIMEOUT": "1"})
    tun = rec["config"]["autotune"]
    assert rec["value"] > 0 and np.isfinite(rec["loss_last"])
    drops = tun.get("dropped", [])
    assert any(d["ts_side"] and "timed out" in d["reason"] for d in drops), tun
    assert not tun["chosen"]["ts_side"], tun


def test_autotune_falls_back_to_rccl_when_no_peer_schedule_survives():
    """Every two-shot candidate fails (rank 1 skips an exchange in each): the engine falls
    back to the RCCL reduce-scatter / all-gather on the same buffers."""
    rec = _bench_2rank({"MULTIGRAD_AUTOTUNE_FAULT": "rccl_exchange=0:1",
                        "MULTIGRAD_ONESHOT_TIMEOUT": "1"})
    tun = rec["config"]["autotune"]
    assert tun["chosen"]["rccl_exchange"], tun
    assert "RCCL" in rec["config"]["grad_collective"]
    assert np.isfinite(rec["loss_last"])


def _engine_hashed_fused(rank, size, fused, chunks, bounded=False, legacy=False):
    os.environ["MULTIGRAD_TWOSHOT_FUSED"] = "on" if fused else "off"
    os.environ["MULTIGRAD_TWOSHOT_SIDE_STREAM"] = "off"
    return _engine_hashed(rank, size, True, bounded, chunks, "auto", None, "off", legacy)


@pytest.mark.parametrize("size,chunks,bounded,legacy", [
    (2, 2, False, False), (2, 3, False, False), (4, 2, False, False), (8, 4, False, False),
    (2, 2, True, False), (4, 3, True, False), (2, 3, True, True)])
def test_engine_hashed_fused_exchange_matches_serial(size, chunks, bounded, legacy):
    """the fused exchange -- chunk c-1's two-shot exchange in the
    first workgroups of chunk c's VJP launch, the last chunk's in the next step's first
    forward launch (no side stream, no events) -- gives the same bits as the serial
    two-shot schedule (2, 4 and 8 processes on one GPU), and with 2 ranks as the RCCL/gloo
    path; unbounded (mode 1) and bounded (mode 2, mode 3 with the legacy Jacobian)."""
    ser = run_distributed(_engine_hashed_fused, size, False, chunks, bounded, legacy, timeout=900)
    fus = run_distributed(_engine_hashed_fused, size, True, chunks, bounded, legacy, timeout=900)
    assert all(r[1] and r[5] == chunks and "fused exchange" in r[4] for r in fus), fus[0][4]
    assert not any("fused exchange" in r[4] for r in ser)
    for r in range(size):
        np.testing.assert_array_equal(fus[r][0], fus[0][0])
        np.testing.assert_array_equal(fus[r][0], ser[r][0])
    if size == 2:
        ref = run_distributed(_engine_hashed, 2, False, bounded, chunks, "auto", None, "off",
                              legacy, timeout=600)
        np.testing.assert_array_equal(fus[0][0], ref[0][0])


def _load_midrun(rank, size):
    os.environ["MULTIGRAD_TWOSHOT_FUSED"] = "on"
    os.environ["MULTIGRAD_TWOSHOT_SIDE_STREAM"] = "off"
    os.environ["MULTIGRAD_CHUNKS"] = "2"
    import multigrad_amd as mg
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    comm = mg.get_world_comm()
    dev = torch.device("cuda", 0)
    data = make_population_data(6000, 300_000, seed=31, comm=comm, device=dev, placement="hashed")
    model = PopulationSMFModel(aux_data=data, comm=comm)
    model.set_target_from_truth()
    a = FusedAdamEngine(model)
    a.setup(data["guess"], nsteps=8, learning_rate=1e-3)
    assert a.ts_fused and a.C == 2
    a.steps(3)
    saved = a.state_dict()          # drains: the state after exactly 3 steps
    a.steps(2)                      # leaves the last chunk's exchange pending ...
    assert a._x_pending is not None
    a.load_state_dict(saved)        # ... which must not run on top of the loaded state
    a.steps(2)
    ta = a.trajectory()[:6].cpu().numpy()
    a.close()
    b = FusedAdamEngine(model)
    b.setup(data["guess"], nsteps=8, learning_rate=1e-3)
    b.load_state_dict(saved)
    b.steps(2)
    tb = b.trajectory()[:6].cpu().numpy()
    b.close()
    return ta, tb


def test_load_state_dict_mid_run_discards_nothing_pending():
    """loading a checkpoint into an engine with a pending fused exchange gives the
    same continuation as a fresh engine resumed from that checkpoint."""
    for ta, tb in run_distributed(_load_midrun, 2, timeout=600):
        np.testing.assert_array_equal(ta, tb)


def _owner_relayout(rank, size, relayout):
    os.environ["MULTIGRAD_RELAYOUT"] = "1" if relayout else "0"
    os.environ["MULTIGRAD_RELAYOUT_EVERY"] = "4"
    import multigrad_amd as mg
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    comm = mg.get_world_comm()
    dev = torch.device("cuda", 0)
    # 20% of the populations start wide and fit towards a narrow truth: they cross the
    # Euler-Maclaurin limit during the run
    data = make_population_data(6000, 300_000, seed=14, comm=comm, device=dev, placement="owner",
                                narrow_frac=0.2, narrow_guess_log_sigma=-0.6)
    model = PopulationSMFModel(aux_data=data, comm=comm)
    model.set_target_from_truth()
    eng = FusedAdamEngine(model, graph=False)
    traj = eng.run_adam(data["guess"], nsteps=40, learning_rate=2e-2)
    return traj.cpu().numpy(), eng.owner, [r["step"] for r in eng.relayouts]


def test_owner_relayout_two_ranks_matches_static_layout():
    """Re-layout under owner placement on 2 ranks: the ranks vote, re-lay out their own
    shards at the same step, and the trajectory equals the run without re-layout."""
    ref = run_distributed(_owner_relayout, 2, False, timeout=600)
    res = run_distributed(_owner_relayout, 2, True, timeout=600)
    assert all(r[1] for r in ref + res)
    assert not ref[0][2] and res[0][2], (ref[0][2], res[0][2])
    assert res[0][2] == res[1][2]  # the same steps on both ranks
    for r in range(2):
        np.testing.assert_allclose(res[r][0], ref[r][0], rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(res[0][0], res[1][0])
