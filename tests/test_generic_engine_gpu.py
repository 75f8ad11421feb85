"""Graph-captured generic Adam engine on the MI355X: one replayed HIP graph per step of a
plain-torch model against the eager chain rule + run_adam; capture fallback; two ranks
on one GPU with the one-shot + two-shot peer-memory collectives inside the graph."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from distributed import run_distributed  # noqa: E402

DEV = torch.device("cuda", 0)


def _torch_pop(comm=None, npar=20_000, nhalo=400_000, seed=11):
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    from multigrad_amd.models.torch_population import TorchPopulationSMFModel, torch_population_data
    data = make_population_data(npar, nhalo, seed=seed, comm=comm, device=DEV)
    PopulationSMFModel(aux_data=data, comm=comm).set_target_from_truth()
    return TorchPopulationSMFModel(aux_data=torch_population_data(data), comm=comm), data["guess"]


@pytest.mark.parametrize("bounded", [False, True])
def test_graph_engine_matches_eager(bounded):
    from multigrad_amd.engine.generic import GraphAdamEngine
    m, guess = _torch_pop()
    bounds = None
    if bounded:
        g = guess.cpu().numpy()
        bounds = np.stack([g - 0.3, g + 0.02], 1)
    ref = m.run_adam(guess, nsteps=6, learning_rate=1e-3, param_bounds=bounds, use_engine=False)
    eng = GraphAdamEngine(m, graph=True)
    traj = eng.run_adam(guess, nsteps=6, learning_rate=1e-3, param_bounds=bounds)
    assert eng.use_graph and eng.graph is not None, eng.fallback_reason
    torch.testing.assert_close(traj, ref, rtol=1e-5, atol=1e-6)
    # auto policy: warm-up, eager window, capture, replay window, then the faster mode --
    # same trajectory
    auto = GraphAdamEngine(m)
    n = 3 * GraphAdamEngine._TUNE + GraphAdamEngine._TUNE_WARM + 3
    t_auto = auto.run_adam(guess, nsteps=n, learning_rate=1e-3, param_bounds=bounds)
    assert auto.tuning is not None and {"eager_s", "graph_s", "graph"} <= set(auto.tuning)
    refn = m.run_adam(guess, nsteps=n, learning_rate=1e-3, param_bounds=bounds, use_engine=False)
    torch.testing.assert_close(t_auto, refn, rtol=1e-5, atol=1e-6)
    # the model front-end routes a GPU model without the fused protocol here
    t2 = m.run_adam(guess, nsteps=6, learning_rate=1e-3, param_bounds=bounds)
    torch.testing.assert_close(t2, traj, rtol=1e-6, atol=1e-7)


def test_graph_engine_falls_back_on_host_sync():
    from multigrad_amd.engine.generic import GraphAdamEngine
    from multigrad_amd.models.torch_population import TorchPopulationSMFModel

    class Syncing(TorchPopulationSMFModel):
        def calc_partial_sumstats_from_params(self, params, randkey=None):
            if float(params.sum()) != float(params.sum()):  # .item(): not capturable
                raise ValueError
            return super().calc_partial_sumstats_from_params(params)

    m, guess = _torch_pop()
    s = Syncing(aux_data=m.aux_data)
    ref = m.run_adam(guess, nsteps=4, learning_rate=1e-3, use_engine=False)
    eng = GraphAdamEngine(s)
    traj = eng.run_adam(guess, nsteps=4, learning_rate=1e-3)
    assert not eng.use_graph and "capture failed" in eng.fallback_reason
    torch.testing.assert_close(traj, ref, rtol=1e-5, atol=1e-6)


def _two_ranks(rank, size, graph):
    os.environ["MULTIGRAD_GRAPH"] = "1" if graph else "0"
    import multigrad_amd as mg
    from multigrad_amd.engine.generic import GraphAdamEngine
    comm = mg.get_world_comm()
    m, guess = _torch_pop(comm, npar=8000, nhalo=200_000)
    eng = GraphAdamEngine(m)
    traj = eng.run_adam(guess, nsteps=5, learning_rate=1e-3)
    return traj.cpu().numpy(), eng.use_graph, eng.grad_exchange == "two-shot", \
        eng.m_oneshot[0] is not None


def test_graph_engine_two_ranks_peer_memory_collectives():
    eager = run_distributed(_two_ranks, 2, False, timeout=600)
    graph = run_distributed(_two_ranks, 2, True, timeout=600)
    assert all(r[2] and r[3] for r in eager + graph)
    assert graph[0][1] and not eager[0][1]
    np.testing.assert_array_equal(graph[0][0], graph[1][0])
    np.testing.assert_array_equal(graph[0][0], eager[0][0])


def test_graph_simple_grad_descent_matches_eager(monkeypatch):
    """run_simple_grad_descent of a GPU model through one captured step per iteration:
    losses and the parameters they were evaluated at match the eager loop (the reference's
    GradDescentResult contract), in graph mode and under the auto policy."""
    from multigrad_amd.engine.generic import GraphAdamEngine
    m, guess = _torch_pop()
    monkeypatch.setenv("MULTIGRAD_GENERIC_ENGINE", "0")
    ref = m.run_simple_grad_descent(guess, nsteps=9, learning_rate=3e-3)
    monkeypatch.setenv("MULTIGRAD_GENERIC_ENGINE", "1")
    for graph in (True, None):
        eng = GraphAdamEngine(m, graph=graph)
        res = eng.run_simple_grad_descent(guess, nsteps=9, learning_rate=3e-3)
        assert eng.use_graph or graph is None
        assert res.params.shape == ref.params.shape and res.loss.shape == ref.loss.shape
        torch.testing.assert_close(res.params, ref.params, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(res.loss.float(), ref.loss.float(), rtol=1e-5, atol=1e-9)
    res2 = m.run_simple_grad_descent(guess, nsteps=9, learning_rate=3e-3)  # routed here
    torch.testing.assert_close(res2.params, ref.params, rtol=1e-5, atol=1e-6)


def _gd_two(rank, size, engine):
    os.environ["MULTIGRAD_GENERIC_ENGINE"] = "1" if engine else "0"
    import multigrad_amd as mg
    comm = mg.get_world_comm()
    m, guess = _torch_pop(comm=comm)
    res = m.run_simple_grad_descent(guess, nsteps=6, learning_rate=3e-3)
    return res.params.cpu().numpy(), res.loss.float().cpu().numpy()


def test_graph_simple_grad_descent_two_ranks():
    """Two ranks sharing one GPU: the gradient sum inside the captured GD step is the
    two-shot all-reduce (bitwise the same on both ranks), matching the eager gloo loop."""
    eng = run_distributed(_gd_two, 2, True, timeout=600)
    ref = run_distributed(_gd_two, 2, False, timeout=600)
    np.testing.assert_array_equal(eng[0][0], eng[1][0])
    np.testing.assert_allclose(eng[0][0], ref[0][0], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(eng[0][1], ref[0][1], rtol=1e-5, atol=1e-9)


def test_captured_evaluator_drives_scipy_bfgs(monkeypatch):
    """The root-driven scipy L-BFGS-B of a GPU model evaluates through one captured step:
    the same iterates as the eager chain rule (the same kernels run), and the docs fit
    converges to the reference's answer."""
    import multigrad_amd.parallel.comm as C
    from multigrad_amd.models.smf import DocsSMFModel, make_docs_data
    C.set_world_comm(None)
    data = make_docs_data()
    model = DocsSMFModel(aux_data=data)
    init = torch.tensor([-3.5, 0.2])
    monkeypatch.setenv("MULTIGRAD_SMF2", "0")  # the generic captured evaluator (not the fused step)
    monkeypatch.setenv("MULTIGRAD_GENERIC_ENGINE", "0")
    ref = model.run_bfgs(init, method="scipy")
    monkeypatch.setenv("MULTIGRAD_GENERIC_ENGINE", "1")
    res = model.run_bfgs(init, method="scipy")
    assert res.nit == ref.nit and res.nfev == ref.nfev
    np.testing.assert_allclose(res.x, ref.x, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(res.x, [-2.0, -0.5], atol=2e-3)


def _bfgs_two(rank, size, engine):
    os.environ["MULTIGRAD_GENERIC_ENGINE"] = "1" if engine else "0"
    os.environ["MULTIGRAD_SMF2"] = "0"  # the generic captured evaluator (not the fused step)
    import multigrad_amd as mg
    from multigrad_amd.models.smf import DocsSMFModel, make_docs_data
    comm = mg.get_world_comm()
    data = make_docs_data(comm=comm)
    model = DocsSMFModel(aux_data=data, comm=comm)
    res = model.run_bfgs(torch.tensor([-3.5, 0.2]), method="scipy")
    return np.asarray(res.x), int(res.nit), float(res.fun)


def test_captured_evaluator_two_ranks():
    """Root-driven scipy L-BFGS-B on two ranks sharing one GPU: the workers replay the
    captured evaluation (one-shot sumstats, two-shot gradient sum inside the graph) in the
    root's command loop; same result on both ranks, matching the eager path."""
    eng = run_distributed(_bfgs_two, 2, True, timeout=600)
    ref = run_distributed(_bfgs_two, 2, False, timeout=600)
    np.testing.assert_array_equal(eng[0][0], eng[1][0])
    np.testing.assert_allclose(eng[0][0], ref[0][0], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(eng[0][0], [-2.0, -0.5], atol=2e-3)


def _two_ranks_syncing(rank, size, mode):
    import multigrad_amd as mg
    from multigrad_amd.engine.generic import GraphAdamEngine
    from multigrad_amd.models.torch_population import TorchPopulationSMFModel

    class Syncing(TorchPopulationSMFModel):
        def calc_partial_sumstats_from_params(self, params, randkey=None):
            if rank == 1 and float(params.sum()) != float(params.sum()):  # rank 1 only
                raise ValueError
            return super().calc_partial_sumstats_from_params(params)

    comm = mg.get_world_comm()
    m, guess = _torch_pop(comm=comm)
    s = Syncing(aux_data=m.aux_data, comm=comm)
    eng = GraphAdamEngine(s)
    if mode == "adam":
        out = eng.run_adam(guess, nsteps=4, learning_rate=1e-3).cpu().numpy()
    else:
        out = eng.run_simple_grad_descent(guess, nsteps=4, learning_rate=3e-3).params.cpu().numpy()
    return out, eng.use_graph, eng.fallback_reason


@pytest.mark.parametrize("mode", ["adam", "sgd"])
def test_two_ranks_uncapturable_hooks_fall_back_together(mode):
    """Only rank 1's hooks synchronise with the host: the collective capture probe sends
    BOTH ranks down the eager path (no rank replays a graph whose collectives the other
    rank never issues), and the run completes with identical results."""
    res = run_distributed(_two_ranks_syncing, 2, mode, timeout=600)
    assert not res[0][1] and not res[1][1]
    assert "rank 1" in res[0][2] and "rank 1" in res[1][2]
    np.testing.assert_array_equal(res[0][0], res[1][0])


# ------------------------------------------------ per-step keys, sumstat aux, groups
def _stoch_pop(comm=None, npar=20_000, nhalo=400_000, seed=11):
    from multigrad_amd.models.torch_population import StochasticTorchPopulationSMFModel
    m, guess = _torch_pop(comm, npar, nhalo, seed)
    return StochasticTorchPopulationSMFModel(aux_data=m.aux_data, comm=comm), guess


@pytest.mark.parametrize("const", [False, True])
def test_graph_engine_randkey_replays_fresh_keys(const):
    """A stochastic model (halo-mass scatter drawn from randkey.generator(device)) through
    the captured step: the generators are registered with the graph and seeded with each
    step's key before its replay, so the trajectory equals the eager per-step-key loop's."""
    from multigrad_amd.engine.generic import GraphAdamEngine
    m, guess = _stoch_pop()
    ref = m.run_adam(guess, nsteps=6, learning_rate=1e-3, randkey=5, const_randkey=const,
                     use_engine=False)
    eng = GraphAdamEngine(m, graph=True)
    t = eng.run_adam(guess, nsteps=6, learning_rate=1e-3, randkey=5, const_randkey=const)
    assert eng.use_graph and eng.graph is not None, eng.fallback_reason
    torch.testing.assert_close(t, ref, rtol=1e-6, atol=1e-7)
    t2 = m.run_adam(guess, nsteps=6, learning_rate=1e-3, randkey=5, const_randkey=const)
    torch.testing.assert_close(t2, t, rtol=0, atol=0)      # the front-end routes here
    if not const:  # the keys really change per step: a constant key gives another path
        tc = m.run_adam(guess, nsteps=6, learning_rate=1e-3, randkey=5, const_randkey=True)
        assert not torch.equal(tc, t)


def test_graph_engine_host_key_use_falls_back():
    from multigrad_amd.engine.generic import GraphAdamEngine
    from multigrad_amd.models.torch_population import StochasticTorchPopulationSMFModel

    class HostKey(StochasticTorchPopulationSMFModel):
        def calc_partial_sumstats_from_params(self, params, randkey=None):
            _ = randkey.value  # a host integer: cannot be replayed with a fresh key
            return super().calc_partial_sumstats_from_params(params, randkey)

    m, guess = _stoch_pop()
    h = HostKey(aux_data=m.aux_data)
    ref = h.run_adam(guess, nsteps=4, learning_rate=1e-3, randkey=2, use_engine=False)
    eng = GraphAdamEngine(h)
    t = eng.run_adam(guess, nsteps=4, learning_rate=1e-3, randkey=2)
    assert not eng.use_graph and "randkey.value" in eng.fallback_reason
    torch.testing.assert_close(t, ref, rtol=1e-6, atol=1e-7)


def _keys_two(rank, size, engine):
    os.environ["MULTIGRAD_GENERIC_ENGINE"] = "1" if engine else "0"
    import multigrad_amd as mg
    from multigrad_amd.engine.generic import GraphAdamEngine
    comm = mg.get_world_comm()
    m, guess = _stoch_pop(comm, npar=8000, nhalo=200_000)
    if engine:
        eng = GraphAdamEngine(m, graph=True)
        t = eng.run_adam(guess, nsteps=5, learning_rate=1e-3, randkey=9)
        return t.cpu().numpy(), eng.use_graph
    return m.run_adam(guess, nsteps=5, learning_rate=1e-3, randkey=9).cpu().numpy(), False


def test_graph_engine_randkey_two_ranks_bitwise():
    """Two ranks on one GPU, per-step keys inside the captured step (one-shot sumstats,
    two-shot Adam exchange): bitwise the same trajectory on both ranks, equal to the
    eager two-rank loop."""
    eng = run_distributed(_keys_two, 2, True, timeout=600)
    ref = run_distributed(_keys_two, 2, False, timeout=600)
    assert eng[0][1] and eng[1][1]
    np.testing.assert_array_equal(eng[0][0], eng[1][0])
    np.testing.assert_allclose(eng[0][0], ref[0][0], rtol=1e-5, atol=1e-6)


def test_graph_engine_sumstats_aux():
    from multigrad_amd.engine.generic import GraphAdamEngine
    from multigrad_amd.models.torch_population import TorchPopulationSMFModel

    class WithAux(TorchPopulationSMFModel):
        def calc_partial_sumstats_from_params(self, params, randkey=None):
            s = super().calc_partial_sumstats_from_params(params)
            return s, self.aux_data["w"]

        def calc_loss_from_sumstats(self, sumstats, sumstats_aux=None, randkey=None):
            return super().calc_loss_from_sumstats(sumstats * sumstats_aux)

    m, guess = _torch_pop()
    aux = dict(m.aux_data, w=torch.linspace(0.8, 1.2, 10, device=DEV))
    w = WithAux(aux_data=aux, sumstats_func_has_aux=True)
    ref = w.run_adam(guess, nsteps=5, learning_rate=1e-3, use_engine=False)
    eng = GraphAdamEngine(w, graph=True)
    t = eng.run_adam(guess, nsteps=5, learning_rate=1e-3)
    assert eng.use_graph
    torch.testing.assert_close(t, ref, rtol=1e-6, atol=1e-7)


def _group_two(rank, size, engine):
    os.environ["MULTIGRAD_GENERIC_ENGINE"] = "1" if engine else "0"
    import multigrad_amd as mg
    from multigrad_amd.engine.generic import GraphAdamEngine
    comm = mg.get_world_comm()
    sub, ng, gidx = mg.split_subcomms(num_groups=2, comm=comm)
    m, guess = _torch_pop(sub, npar=8000, nhalo=150_000, seed=11 + gidx)
    guess = comm.bcast(guess.cpu(), root=0).to(DEV)  # the group shares ONE parameter vector
    grp = mg.OnePointGroup(m, main_comm=comm)
    if engine:
        eng = GraphAdamEngine(grp, graph=True)
        t = eng.run_adam(guess, nsteps=5, learning_rate=1e-3)
        return t.cpu().numpy(), eng.use_graph, eng.last_loss()
    t = grp.run_adam(guess, nsteps=5, learning_rate=1e-3)
    return t.cpu().numpy(), False, None


def test_graph_engine_group_two_groups():
    """A 2-group OnePointGroup (one population model per rank, each on its own
    sub-communicator) through ONE captured step per iteration: member chain rules, the
    group loss over a 1-float one-shot and the two-shot Adam exchange over the main
    communicator; same bits on both ranks, equal to the eager group loop."""
    eng = run_distributed(_group_two, 2, True, timeout=600)
    ref = run_distributed(_group_two, 2, False, timeout=600)
    assert eng[0][1] and eng[1][1]
    np.testing.assert_array_equal(eng[0][0], eng[1][0])
    assert eng[0][2] == eng[1][2]
    np.testing.assert_allclose(eng[0][0], ref[0][0], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("graph", [True, None])
def test_graph_engine_randkey_with_host_syncs(graph):
    """Keyed captured steps with a host synchronisation between replays (a user callback,
    and the auto policy's timing windows): the replays still equal the eager steps.
    Launched on the default stream right after a sync, a graph with an RNG op computed
    wrong sums downstream of it on this runtime; the engine replays keyed graphs on its
    own stream (GraphAdamEngine._replay)."""
    from multigrad_amd.engine.generic import GraphAdamEngine
    m, guess = _stoch_pop()
    n = 3 * GraphAdamEngine._TUNE + GraphAdamEngine._TUNE_WARM + 4  # the auto windows run
    ref = m.run_adam(guess, nsteps=n, learning_rate=1e-3, randkey=7, use_engine=False)

    def sync(i, loss, state):
        torch.cuda.synchronize()

    eng = GraphAdamEngine(m, graph=graph)
    t = eng.run_adam(guess, nsteps=n, learning_rate=1e-3, randkey=7, callback=sync)
    assert eng.use_graph or graph is None
    torch.testing.assert_close(t, ref, rtol=0, atol=0)


def test_graph_engine_block_replays_match_eager(monkeypatch):
    """The generic engine's unkeyed graph mode replays blocks of MULTIGRAD_GRAPH_STEPS
    steps after its one-step replays (Adam and gradient descent) with the eager results."""
    from multigrad_amd.engine.generic import GraphAdamEngine
    model, guess = _torch_pop()
    ref = GraphAdamEngine(model, graph=False).run_adam(guess, nsteps=13, learning_rate=1e-3)
    ref_gd = GraphAdamEngine(model, graph=False).run_simple_grad_descent(
        guess, nsteps=13, learning_rate=1e-3)
    monkeypatch.setenv("MULTIGRAD_GRAPH_STEPS", "5")
    eng = GraphAdamEngine(model, graph=True)
    t = eng.run_adam(guess, nsteps=13, learning_rate=1e-3)
    assert eng.use_graph and eng.graph_steps == 5
    torch.testing.assert_close(t, ref, rtol=1e-6, atol=1e-7)
    gd = GraphAdamEngine(model, graph=True).run_simple_grad_descent(
        guess, nsteps=13, learning_rate=1e-3)
    torch.testing.assert_close(gd.params, ref_gd.params, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(gd.loss, ref_gd.loss, rtol=1e-6, atol=1e-9)


def test_ingraph_descent_block_capture_matches_eager():
    """ingraph.simple_grad_descent with blocks of 4 steps and a remainder graph (11
    steps) matches the eager loop."""
    from multigrad_amd import ingraph
    g = torch.Generator().manual_seed(3)
    x = torch.randn(5000, generator=g).cuda()

    def loss_and_grad(d, p):
        r = d["x"][:, None] - p[None, :]
        return 0.5 * (r * r).mean(), -r.mean(0)

    guess = torch.tensor([0.5, -1.0], device="cuda")
    a = ingraph.simple_grad_descent(dict(x=x), loss_and_grad, guess, 0.3, nsteps=11,
                                    graph=True, block=4)
    b = ingraph.simple_grad_descent(dict(x=x), loss_and_grad, guess, 0.3, nsteps=11, graph=False)
    np.testing.assert_allclose(np.stack(a["params"].to_numpy()), np.stack(b["params"].to_numpy()),
                               rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(np.asarray(a["loss"], dtype=float), np.asarray(b["loss"], dtype=float),
                               rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("keyed", [False, True])
def test_graph_engine_replays_after_eager_steps_with_syncs(keyed):
    """Replays that follow eager steps, with a host synchronisation and a user kernel
    (inside engine.stream()) after every step -- the schedules that computed wrong results
    when the engine launched on the default stream (a HIP runtime defect reproduced with
    torch alone, tools/dbg/torch_replay_bisect.py).  Every launch of the engine now runs on
    its own stream, so the order eager / replay / eager / replay gives the eager trajectory."""
    from multigrad_amd.engine.generic import GraphAdamEngine
    m, guess = _stoch_pop() if keyed else _torch_pop()
    kw = dict(randkey=9) if keyed else {}
    sched = "eeeggggeeeggg"
    ref = m.run_adam(guess, nsteps=len(sched), learning_rate=1e-3, use_engine=False, **kw)
    eng = GraphAdamEngine(m, graph=True)
    eng.setup(guess, nsteps=len(sched), learning_rate=1e-3, **kw)
    eng.step_replay = True  # direct calls replay: the caller's kernels are in eng.stream()
    scratch = torch.zeros(1, device=DEV)
    for mode in sched:
        eng.use_graph = mode == "g"
        eng.step()
        with eng.stream():
            scratch.add_(1)
        torch.cuda.synchronize()
    assert eng.graph is not None
    torch.testing.assert_close(eng.trajectory(), ref, rtol=1e-6, atol=1e-7)


def test_engines_launch_on_their_own_stream():
    """Every public engine method runs on the engine's stream (never the legacy default
    stream; engine/_stream.py), user callbacks included, and hands the caller back a
    stream ordered after the engine's work."""
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.engine.generic import GraphAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    m, guess = _torch_pop(npar=2000, nhalo=40_000)
    seen = []

    def cb(i, loss, state):
        seen.append(torch.cuda.current_stream())

    eng = GraphAdamEngine(m, graph=True)
    t = eng.run_adam(guess, nsteps=4, learning_rate=1e-3, callback=cb)
    assert seen and all(s != torch.cuda.default_stream() for s in seen)
    assert all(s == eng._es for s in seen)
    assert torch.cuda.current_stream() == torch.cuda.default_stream()
    assert torch.isfinite(t).all()
    data = make_population_data(num_params=4000, num_halos=100_000, seed=3, device=DEV)
    model = PopulationSMFModel(aux_data=data)
    model.set_target_from_truth()
    seen.clear()
    feng = FusedAdamEngine(model, graph=False)
    tf = feng.run_adam(data["guess"], nsteps=4, learning_rate=1e-3, callback=cb)
    assert seen and all(s == feng._es for s in seen)
    assert torch.isfinite(tf).all()


@pytest.mark.parametrize("engine", ["generic", "fused"])
def test_direct_steps_with_default_stream_work_match_eager(engine):
    """a user loop of direct step() calls with its own kernels on the legacy default
    stream and a host synchronisation between the calls -- the schedule after which a graph
    replay computes garbage on this HIP runtime -- gives the eager trajectory bit for bit,
    because direct calls launch eagerly (step_replay off); steps() still replays."""
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.engine.generic import GraphAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    if engine == "generic":
        m, guess = _torch_pop()
        mk = lambda g: GraphAdamEngine(m, graph=g)  # noqa: E731
    else:
        data = make_population_data(num_params=4000, num_halos=100_000, seed=3, device=DEV)
        m = PopulationSMFModel(aux_data=data)
        m.set_target_from_truth()
        guess = data["guess"]
        mk = lambda g: FusedAdamEngine(m, graph=g)  # noqa: E731
    n = 12
    ref = mk(False)
    ref.setup(guess, nsteps=n, learning_rate=1e-3)
    ref.steps(n)
    want = ref.trajectory().cpu()
    eng = mk(True)
    eng.setup(guess, nsteps=n, learning_rate=1e-3)
    assert eng.use_graph and not eng.step_replay
    scratch = torch.zeros(1, device=DEV)
    eng.steps(4)                       # replays (a graph now exists)
    for _ in range(n - 4):
        eng.step()                     # direct calls: eager launches
        scratch.add_(1)                # the caller's own kernel on the default stream
        torch.cuda.synchronize()
    got = eng.trajectory().cpu()
    torch.testing.assert_close(got, want, rtol=1e-6, atol=1e-7)


def _ar_give_back(rank, size):
    import gc

    import multigrad_amd as mg
    from multigrad_amd.engine.generic import GraphAdamEngine
    comm = mg.get_world_comm()
    m, guess = _torch_pop(comm=comm, npar=2000, nhalo=40_000)
    # run_simple_grad_descent closes its engine: hold and pins given back
    eng = GraphAdamEngine(m)
    eng.run_simple_grad_descent(guess, nsteps=6, learning_rate=3e-3)
    ar = comm._twoshot_ar[min(comm._twoshot_ar)]
    after_run = (ar.holders, ar.pins)
    # an engine dropped without close(): the finalizer gives them back
    eng = GraphAdamEngine(m)
    eng.mode = "sgd"
    eng.setup(guess, 6, learning_rate=3e-3, history="last")
    eng.steps(6)
    torch.cuda.synchronize()
    during = (eng.ar.holders, eng.ar.pins, eng.use_graph)
    ar = eng.ar
    del eng
    gc.collect()
    return after_run, during, (ar.holders, ar.pins)


def test_allreduce_context_hold_and_pins_given_back():
    """the generic engine's hold on its two-shot all-reduce context and
    the pins of its captured graphs go back to the communicator's cache on close() and
    when the engine is dropped without it, so the cache can evict the context again."""
    res = run_distributed(_ar_give_back, 2, timeout=300)
    for after_run, during, dropped in res:
        assert after_run == (0, 0)
        assert during[0] == 1 and during[2] and during[1] >= 1
        assert dropped == (0, 0)
