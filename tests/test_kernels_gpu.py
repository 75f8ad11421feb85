"""HIP kernel numerics vs plain PyTorch fp64/fp32 references (run on an MI355X)."""
import numpy as np
import pytest
import torch

from multigrad_amd.ops import smf as S
from multigrad_amd.ops._schedule import build_tiles_py

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rand_shard(n, npop, seed=0, giant=None, device=DEV):
    g = torch.Generator().manual_seed(seed)
    x = 10.0 + torch.rand(n, generator=g, dtype=torch.float64)
    pop = torch.randint(0, npop, (n,), generator=g)
    if giant is not None:  # make one population huge (> tile) to exercise partial tiles
        pop[: n // 2] = giant
    return x, pop


def _theta(npop, seed=1, dtype=torch.float64):
    g = torch.Generator().manual_seed(seed)
    th = torch.empty(2 * npop, dtype=dtype)
    th[0::2] = -2.0 + 0.2 * (torch.rand(npop, generator=g, dtype=dtype) - 0.5)
    th[1::2] = -0.5 + 0.2 * (torch.rand(npop, generator=g, dtype=dtype) - 0.5)
    return th


@pytest.mark.parametrize("layout", ["lanes", "tiles"])
@pytest.mark.parametrize("nbins", [10, 7, 3])
@pytest.mark.parametrize("giant", [None, 3])
def test_population_forward_and_vjp_match_fp64(nbins, giant, layout):
    n, npop = 200_000, 300
    x, pop = _rand_shard(n, npop, giant=giant)
    theta64 = _theta(npop)
    bins = S.SmfBins.make(np.linspace(8.0, 9.6, nbins + 1), volume=1e4)
    shard = S.PopulationShard(x.float(), pop.int().to(DEV), npop, device=DEV, chunks=3,
                              layout=layout)
    assert shard.layout == layout
    # fp64 oracle on the same (float32-rounded) inputs
    xf = x.float().double()
    th_ref = theta64.float().double().requires_grad_(True)
    ref = S.smf_sumstats_reference(th_ref, xf, pop, bins, log_sigma=True)
    gS = torch.linspace(0.5, 1.5, nbins, dtype=torch.float64)
    (gref,) = torch.autograd.grad(ref, th_ref, gS)
    th = theta64.float().to(DEV).requires_grad_(True)
    out = S.smf_sumstats(th, shard, bins, log_sigma=True)
    (gk,) = torch.autograd.grad(out, th, gS.float().to(DEV))
    np.testing.assert_allclose(out.detach().cpu().double(), ref.detach(), rtol=2e-5, atol=1e-12)
    np.testing.assert_allclose(gk.cpu().double(), gref, rtol=2e-4,
                               atol=2e-5 * float(gref.abs().max()))


@pytest.mark.parametrize("logsig", [-0.4, -0.45, -0.55])
def test_em_forward_bin_width_ranges_vs_fp64(logsig):
    """Edges 0.1 apart and log10 sigma = logsig +- 0.1: bin widths in sigma units of
    0.20-0.32 (the headline guess), 0.22-0.35 and 0.28-0.45 on the Euler-Maclaurin path --
    forward and VJP against the fp64 oracle."""
    n, npop = 400_000, 2000
    x, pop = _rand_shard(n, npop, seed=7)  # x + a in [7.9, 9.1]: the bins 8.5..9.5 sit on it
    theta64 = _theta(npop, seed=8)
    theta64[1::2] += logsig + 0.5
    bins = S.SmfBins.make(np.linspace(8.5, 9.5, 11), volume=1e4)
    shard = S.PopulationShard(x.float(), pop.int().to(DEV), npop, device=DEV, chunks=2,
                              layout="lanes")
    xf = x.float().double()
    th_ref = theta64.float().double().requires_grad_(True)
    ref = S.smf_sumstats_reference(th_ref, xf, pop, bins, log_sigma=True)
    gS = torch.linspace(0.5, 1.5, 10, dtype=torch.float64)
    (gref,) = torch.autograd.grad(ref, th_ref, gS)
    th = theta64.float().to(DEV).requires_grad_(True)
    out = S.smf_sumstats(th, shard, bins, log_sigma=True)
    (gk,) = torch.autograd.grad(out, th, gS.float().to(DEV))
    np.testing.assert_allclose(out.detach().cpu().double(), ref.detach(), rtol=2e-5, atol=1e-12)
    np.testing.assert_allclose(gk.cpu().double(), gref, rtol=2e-4,
                               atol=2e-5 * float(gref.abs().max()))


@pytest.mark.parametrize("tail", ["relative", "absolute"])
@pytest.mark.parametrize("log_sigma", [False, True])
def test_shared_params_model_kernel(log_sigma, tail):
    # halos sit below the bins, so the upper bins are Gaussian-tail dominated
    n = 300_001
    x = 10.0 + 0.5 * torch.rand(n, dtype=torch.float64, generator=torch.Generator().manual_seed(3))
    bins = S.SmfBins.make(np.linspace(9, 10, 11), volume=10.0 * n, tail=tail)
    th64 = torch.tensor([-1.7, -0.6 if log_sigma else 0.25], dtype=torch.float64)
    shard = S.PopulationShard(x.float(), None, 1, device=DEV)
    thr = th64.clone().requires_grad_(True)
    ref = S.smf_sumstats_reference(thr, x.float().double(), None, bins, log_sigma)
    (gref,) = torch.autograd.grad(ref.sum(), thr)
    th = th64.float().to(DEV).requires_grad_(True)
    out = S.smf_sumstats(th, shard, bins, log_sigma)
    (gk,) = torch.autograd.grad(out.sum(), th)
    if tail == "relative":  # every bin, however deep in the tail, to ~1e-5 relative
        np.testing.assert_allclose(out.detach().cpu().double(), ref.detach(), rtol=2e-5)
    else:  # float32-erf contract: <= 1.1e-7 absolute per edge CDF per halo
        atol = 2.2e-7 * n * np.asarray(bins.scale)
        err = np.abs(out.detach().cpu().double().numpy() - ref.detach().numpy())
        assert (err <= atol + 2e-5 * np.abs(ref.detach().numpy())).all(), (err, atol)
    np.testing.assert_allclose(gk.cpu().double(), gref, rtol=5e-5)


@pytest.mark.parametrize("layout", ["lanes", "tiles"])
def test_forward_is_deterministic_and_chunks_sum(layout):
    n, npop = 100_000, 500
    x, pop = _rand_shard(n, npop, seed=5)
    shard = S.PopulationShard(x.float(), pop.int().to(DEV), npop, device=DEV, chunks=4,
                              layout=layout)
    th = _theta(npop).float().to(DEV)
    bins = S.SmfBins.make(np.linspace(8.0, 9.6, 11), volume=1e4)
    a = S.smf_sumstats(th, shard, bins)
    b = S.smf_sumstats(th, shard, bins)
    assert torch.equal(a, b)
    parts = torch.zeros(bins.nbp, device=DEV)
    for c in range(shard.nchunks):
        o = torch.zeros(bins.nbp, device=DEV)
        S.smf_forward_into(th, shard, bins, True, o, chunk=c)
        parts += o
    torch.testing.assert_close(parts[:10], a, rtol=1e-5, atol=0)
    # per-chunk VJPs write disjoint parameter ranges that reassemble the full VJP
    h = torch.randn(bins.nbp + 1, device=DEV)
    full = torch.zeros(2 * npop, device=DEV)
    S.smf_vjp_into(th, shard, bins, True, h, full)
    acc = torch.full((2 * npop,), float("nan"), device=DEV)
    for c in range(shard.nchunks):
        S.smf_vjp_into(th, shard, bins, True, h, acc, chunk=c)
    assert torch.equal(acc, full)


def test_tile_schedule_native_matches_python():
    from multigrad_amd.ops._ext import ext
    g = torch.Generator().manual_seed(0)
    counts = torch.randint(0, 40, (5000,), generator=g)
    counts[100] = 9000
    counts[4000] = 2049
    counts[200:260] = 0
    for breaks in ([], [1000, 2500], [100, 101, 4000]):
        a = ext().build_tiles(counts.long(), breaks, 2048, 2048)
        b = build_tiles_py(counts, breaks, 2048, 2048)
        for x, y in zip(a[:4], b[:4]):
            assert torch.equal(x.cpu(), y.cpu())
        assert a[4] == b[4]


def test_fused_adam_matches_reference():
    from multigrad_amd.ops.adam import adam_reference_, fused_adam_
    from multigrad_amd.optim.transforms import Bounds
    torch.manual_seed(0)
    n = 1_000_003  # odd size: vector body + scalar tail
    u = torch.randn(n, device=DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    ur, mr, vr = u.clone(), m.clone(), v.clone()
    step = torch.zeros(2, dtype=torch.int32, device=DEV)
    traj = torch.zeros(4, n, device=DEV)
    for i in range(3):
        g = torch.randn(n, device=DEV)
        fused_adam_(u, m, v, g, None, step, 1e-2, 0.9, 0.999, 1e-8, traj_base=traj.reshape(-1),
                    traj_stride=n)
        adam_reference_(ur, mr, vr, g, i, 1e-2, 0.9, 0.999, 1e-8)
    assert step.tolist() == [3, 0]
    torch.testing.assert_close(u, ur, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(m, mr, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(traj[3], u)
    # bounded variant vs the torch Adam implementation
    from multigrad_amd.optim.adam import Adam
    nb = 4097
    spec = [(-1.0, 2.0) if i % 4 == 0 else (0.0, None) if i % 4 == 1 else (None, 3.0)
            if i % 4 == 2 else None for i in range(nb)]
    p0 = torch.rand(nb, device=DEV) * 0.9 + 0.05
    for legacy in (False, True):
        b = Bounds.from_spec(spec, nb, device=DEV)
        fa = Adam(p0, 0.05, bounds=b, legacy_bounds_jacobian=legacy)
        ta = Adam(p0, 0.05, bounds=b, legacy_bounds_jacobian=legacy)
        ta.fused = False
        assert fa.fused
        for _ in range(5):
            g = torch.randn(nb, device=DEV)
            fa.update(g)
            ta.update(g)
        torch.testing.assert_close(fa.params(), ta.params(), rtol=2e-5, atol=2e-6)


def test_engine_matches_generic_adam():
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    data = make_population_data(num_params=4000, num_halos=200_000, seed=3, device=DEV)
    model = PopulationSMFModel(aux_data=data)
    model.set_target_from_truth()
    t_gen = model.run_adam(data["guess"], nsteps=4, learning_rate=1e-3, use_engine=False)
    for graph in (False, True):
        eng = model.fused_engine(graph=graph)
        t_eng = eng.run_adam(data["guess"], nsteps=4, learning_rate=1e-3)
        torch.testing.assert_close(t_eng, t_gen, rtol=1e-5, atol=1e-6)
    loss = model.calc_loss_from_params(t_gen[-1])
    loss0 = model.calc_loss_from_params(t_gen[0])
    assert float(loss) < float(loss0)


def test_engine_owner_schedule_single_rank():
    """The owner-mode schedule (own-chunk forward/VJP, owned-slice Adam with a strided
    trajectory, assembly) on the HIP kernels, forced on one rank: equals the replicated
    engine bitwise up to kernel-order effects."""
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    data = make_population_data(num_params=4000, num_halos=200_000, seed=3, device=DEV)
    model = PopulationSMFModel(aux_data=data)
    model.set_target_from_truth()
    ref = FusedAdamEngine(model, graph=False).run_adam(data["guess"], nsteps=4, learning_rate=1e-3)
    for graph in (False, True):
        eng = FusedAdamEngine(model, graph=graph, owner=True)
        t = eng.run_adam(data["guess"], nsteps=4, learning_rate=1e-3)
        assert eng.owner
        torch.testing.assert_close(t, ref, rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(eng.params(), t[-1], rtol=0, atol=0)


@pytest.mark.parametrize("owner,graph,history", [(False, True, "full"), (False, False, "last"),
                                                 (True, False, "full"), (True, True, "full")])
def test_fused_vjp_adam_matches_separate_kernels(owner, graph, history):
    """The fused VJP + Adam kernel (no gradient in HBM) against the VJP kernel followed by
    the fused Adam kernel."""
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    data = make_population_data(num_params=6000, num_halos=300_000, seed=5, device=DEV)
    model = PopulationSMFModel(aux_data=data)
    model.set_target_from_truth()
    sep = FusedAdamEngine(model, graph=graph, owner=owner)
    sep.fuse_vjp_adam = False
    ref = sep.run_adam(data["guess"], nsteps=5, learning_rate=1e-3, history=history)
    eng = FusedAdamEngine(model, graph=graph, owner=owner)
    assert eng.fuse_vjp_adam
    t = eng.run_adam(data["guess"], nsteps=5, learning_rate=1e-3, history=history)
    torch.testing.assert_close(t, ref, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(eng.m, sep.m, rtol=1e-5, atol=1e-9)


def test_reference_pipeline_on_gpu():
    """Reference tests/test_mpi.py::test_simple_grad_descent_pipeline on the HIP path."""
    from multigrad_amd.models.smf import MySMFModel, ParamTuple, TARGET_SUMSTATS, make_test_data
    data = make_test_data()
    model = MySMFModel(aux_data=data, device=DEV)
    truth = ParamTuple(-2.0, 0.2)
    s = model.calc_sumstats_from_params(truth)
    assert s.is_cuda
    np.testing.assert_allclose(s.cpu().numpy(), TARGET_SUMSTATS, rtol=5e-5, atol=1e-9)
    # self-consistent target (the reference target is itself a float32 JAX evaluation)
    data["target_sumstats"] = s.cpu().numpy()
    model = MySMFModel(aux_data=data, device=DEV)
    gd = model.run_simple_grad_descent(guess=truth, nsteps=2)
    assert abs(float(gd.loss[-1])) < 1e-10
    torch.testing.assert_close(gd.params[-1].cpu(), torch.tensor([*truth]), rtol=0, atol=1e-6)
    assert torch.allclose(model.calc_dloss_dparams(truth).cpu(), torch.zeros(2), atol=1e-5)
    loss, grad = model.calc_loss_and_grad_from_params(truth)
    assert torch.allclose(loss, model.calc_loss_from_params(truth))
    assert torch.allclose(grad, model.calc_dloss_dparams(truth))


def test_multi_dot_and_lincomb_kernels():
    from multigrad_amd.ops.lbfgs import MultiDot, lincomb_
    torch.manual_seed(1)
    n, r = 1_000_003, 20
    A = torch.randn(r, n, device=DEV)
    B = [torch.randn(n, device=DEV) for _ in range(3)]
    md = MultiDot(r, n, DEV)
    out = md(A, r, B).cpu()
    ref = (A.double() @ torch.stack(B).double().T).cpu()
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-3)
    assert torch.equal(md(A, r, B).cpu(), out)  # deterministic
    out1 = md(A, 7, B[:1]).cpu()
    torch.testing.assert_close(out1, ref[:7, :1], rtol=1e-5, atol=1e-3)
    # every row-count / vector-count instantiation (1-3 rows per thread; 2/4/6/8 rows per
    # wave; several row groups), float4 and scalar paths, against the fp64 product
    r2, n2 = 40, 1_000_000  # float4 path (rows 16-byte aligned)
    A2 = torch.randn(r2, n2, device=DEV)
    B2 = [torch.randn(n2, device=DEV) for _ in range(4)]
    ref2 = (A2.double() @ torch.stack(B2).double().T).cpu()
    md2 = MultiDot(r2, n2, DEV)
    for rows in (1, 2, 3, 4, 7, 8, 13, 16, 23, 24, 25, 32, 33, 40):
        for nc in (1, 2, 3, 4):
            got = md2(A2, rows, B2[:nc]).cpu()
            torch.testing.assert_close(got, ref2[:rows, :nc], rtol=1e-5, atol=1e-3)
    for rows in (1, 3, 13, 20):  # scalar path (n = 1_000_003: rows not 16-byte aligned)
        got = md(A, rows, B).cpu()
        torch.testing.assert_close(got, ref[:rows], rtol=1e-5, atol=1e-3)
    coef = torch.randn(r, device=DEV)
    y = torch.empty(n, device=DEV)
    lincomb_(A, r, coef, -0.5, B[0], y)
    torch.testing.assert_close(y, -0.5 * B[0] + coef @ A, rtol=1e-4, atol=1e-4)


def test_device_lbfgs_population_engine():
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    data = make_population_data(num_params=2000, num_halos=200_000, seed=9, device=DEV)
    model = PopulationSMFModel(aux_data=data)
    model.set_target_from_truth()
    f0 = float(model.calc_loss_from_params(data["guess"]))
    res = model.run_bfgs(data["guess"], maxsteps=40, method="device")
    assert res.x.is_cuda and res.x.shape == (2000,)
    assert res.fun < 1e-3 * f0
    # the generic (autograd + replicated-vector) device L-BFGS reaches a comparable loss
    from multigrad_amd.optim.lbfgs import run_lbfgs_device
    res2 = run_lbfgs_device(model.calc_loss_and_grad_from_params, data["guess"], maxsteps=40)
    assert res2.fun < 1e-3 * f0


def test_lanes_matches_tiles_and_residual_reuse():
    """The two layouts agree; the engine-style residual VJP equals the recomputing one;
    a stale-residual backward (another forward in between) is detected and recomputed."""
    n, npop = 150_000, 4000
    x, pop = _rand_shard(n, npop, seed=9, giant=7)
    th = _theta(npop).float().to(DEV)
    bins = S.SmfBins.make(np.linspace(8.0, 9.6, 11), volume=1e4)
    sl = S.PopulationShard(x.float(), pop.int().to(DEV), npop, device=DEV, layout="lanes",
                           lane_window=256, lane_lmax=1000)
    st = S.PopulationShard(x.float(), pop.int().to(DEV), npop, device=DEV, layout="tiles")
    assert sl.giant.shape[0] == 1  # the giant population is split into parts
    h = torch.randn(bins.nbp + 1, device=DEV)
    out_l = torch.zeros(bins.nbp, device=DEV)
    out_t = torch.zeros(bins.nbp, device=DEV)
    S.smf_forward_into(th, sl, bins, True, out_l, resid=True)
    S.smf_forward_into(th, st, bins, True, out_t)
    torch.testing.assert_close(out_l, out_t, rtol=2e-6, atol=0)
    g_ready = torch.zeros_like(th)
    S.smf_vjp_into(th, sl, bins, True, h, g_ready, residuals_ready=True)
    g_re = torch.zeros_like(th)
    S.smf_vjp_into(th, sl, bins, True, h, g_re)
    g_t = torch.zeros_like(th)
    S.smf_vjp_into(th, st, bins, True, h, g_t)
    assert torch.equal(g_ready, g_re)
    torch.testing.assert_close(g_ready, g_t, rtol=1e-4, atol=1e-5 * float(g_t.abs().max()))
    # stale residuals: forward at th, another residual forward at th2, backward at th
    thr = th.clone().requires_grad_(True)
    out = S.smf_sumstats(thr, sl, bins)
    S.smf_sumstats((th + 0.05).requires_grad_(True), sl, bins)
    (gk,) = torch.autograd.grad(out, thr, torch.ones_like(out))
    thr2 = th.clone().requires_grad_(True)
    (gk2,) = torch.autograd.grad(S.smf_sumstats(thr2, sl, bins), thr2, torch.ones_like(out))
    assert torch.equal(gk, gk2)


def test_forward_schedules_agree(monkeypatch):
    """Static LPT lists, dynamic work queues (run repeatedly: the kernel must leave its
    counters at zero) and plain grid-stride give the same sums and residual VJP."""
    from multigrad_amd.models.population import make_population_data
    from multigrad_amd.ops import smf as S
    data = make_population_data(num_params=40_000, num_halos=1_000_000, seed=9, device=DEV)
    shard, bins = data["shard"], data["bins"]
    th = data["guess"]
    h = torch.linspace(0.5, -0.5, bins.nbp + 1, device=DEV)
    res = {}
    for mode in ("static", "dynamic", "0"):
        monkeypatch.setenv("MULTIGRAD_LPT", mode)
        outs = []
        for _ in range(3):
            out = torch.zeros(bins.nbp, device=DEV)
            S.smf_forward_into(th, shard, bins, True, out, resid=True)
            grad = torch.zeros_like(th)
            S.smf_vjp_into(th, shard, bins, True, h, grad, residuals_ready=True)
            outs.append((out.clone(), grad.clone()))
        if mode == "dynamic":
            assert int(shard._queues.abs().sum()) == 0
        for o, g in outs[1:]:
            torch.testing.assert_close(o, outs[0][0], rtol=1e-6, atol=0)
            torch.testing.assert_close(g, outs[0][1], rtol=1e-6, atol=1e-12)
        res[mode] = outs[0]
    for mode in ("dynamic", "0"):
        torch.testing.assert_close(res[mode][0], res["static"][0], rtol=1e-6, atol=0)
        torch.testing.assert_close(res[mode][1], res["static"][1], rtol=1e-6, atol=1e-12)


@pytest.mark.parametrize("graph", [False, True])
def test_fused_epilogue_matches_separate_kernels(graph):
    """Slab reduction + loss + edge weights in one launch (single rank) against the
    separate reduce and loss kernels."""
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    data = make_population_data(num_params=6000, num_halos=300_000, seed=8, device=DEV)
    model = PopulationSMFModel(aux_data=data)
    model.set_target_from_truth()
    sep = FusedAdamEngine(model, graph=graph)
    sep.fuse_epilogue = False
    ref = sep.run_adam(data["guess"], nsteps=5, learning_rate=1e-3)
    eng = FusedAdamEngine(model, graph=graph)
    t = eng.run_adam(data["guess"], nsteps=5, learning_rate=1e-3)
    torch.testing.assert_close(t, ref, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(eng.loss, sep.loss, rtol=1e-6, atol=0)
    torch.testing.assert_close(eng.h, sep.h, rtol=1e-6, atol=1e-12)


@pytest.mark.parametrize("narrow", [False, True])
def test_folded_epilogue_matches_separate_launch(monkeypatch, narrow):
    """The sumstat epilogue passed to the forward's host call (MULTIGRAD_FOLD_EPILOGUE: the
    forward launches it right after the main kernel) against the engine's own epilogue
    launch, pipelined, with no narrow population and with narrow populations on the
    per-edge path."""
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    data = make_population_data(num_params=6000, num_halos=300_000, seed=21, device=DEV)
    model = PopulationSMFModel(aux_data=data)
    model.set_target_from_truth()
    guess = _narrow_guess(data, every=3) if narrow else data["guess"]
    out = {}
    for fold in ("0", "1"):
        monkeypatch.setenv("MULTIGRAD_FOLD_EPILOGUE", fold)
        eng = FusedAdamEngine(model, graph=False)
        out[fold] = (eng.run_adam(guess, nsteps=5, learning_rate=1e-3), eng.loss.clone(), eng.h.clone())
        assert eng.pipeline
    # the same kernels over the same slab rows in the same order: the same bits
    torch.testing.assert_close(out["1"][0], out["0"][0], rtol=0, atol=0)
    torch.testing.assert_close(out["1"][1], out["0"][1], rtol=0, atol=0)
    torch.testing.assert_close(out["1"][2], out["0"][2], rtol=0, atol=0)


@pytest.mark.parametrize("owner,graph,legacy,kind", [
    (False, False, False, "both"), (False, True, False, "both"), (True, False, False, "mixed"),
    (True, True, True, "both"), (False, False, True, "mixed")])
def test_bounded_pipelined_update_matches_unpipelined(monkeypatch, owner, graph, legacy, kind):
    """VERDICT r4 missing #2: bounded Adam (reference multigrad/adam.py:133-189) runs the
    pipelined two-launch step too -- Adam on u with the diagonal dp/du (at u, or at p with
    the legacy Jacobian), p = T^-1(u) -- and gives the unpipelined bounded trajectory
    (stand-alone bounded Adam kernel) in replicated, owner and graph modes."""
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    data = make_population_data(num_params=6000, num_halos=300_000, seed=12, device=DEV)
    model = PopulationSMFModel(aux_data=data)
    model.set_target_from_truth()
    g = data["guess"].detach().cpu()
    bounds = torch.stack([g - 0.3, g + 0.2], 1).numpy()
    if kind == "mixed":
        bounds[0::2, 1] = np.inf      # a: lower bound only
        bounds[1::4, 0] = -np.inf     # some log sigmas: upper bound only
    kw = dict(learning_rate=2e-2, param_bounds=bounds, legacy_bounds_jacobian=legacy)
    monkeypatch.setenv("MULTIGRAD_PIPELINE", "0")
    ref_eng = FusedAdamEngine(model, graph=graph, owner=owner)
    ref = ref_eng.run_adam(data["guess"], nsteps=8, **kw)
    assert not ref_eng.pipeline
    monkeypatch.setenv("MULTIGRAD_PIPELINE", "1")
    eng = FusedAdamEngine(model, graph=graph, owner=owner)
    t = eng.run_adam(data["guess"], nsteps=8, **kw)
    assert eng.pipeline and eng.bounds is not None
    torch.testing.assert_close(t, ref, rtol=2e-6, atol=2e-7)
    lo = torch.as_tensor(bounds[:, 0], dtype=torch.float32, device=DEV)
    hi = torch.as_tensor(bounds[:, 1], dtype=torch.float32, device=DEV)
    assert bool(((t >= lo) & (t <= hi)).all())
    assert float((t[-1] - t[0]).abs().max()) > 1e-3  # the fit moved


@pytest.mark.parametrize("owner,graph,history", [(False, True, "full"), (False, False, "full"),
                                                 (False, True, "last"), (True, False, "full"),
                                                 (True, True, 2)])
def test_pipelined_update_matches_unpipelined(monkeypatch, owner, graph, history):
    """VJP + Adam of step k fused into the forward of step k+1 (pending until the next
    step or drain) gives the trajectory of the step-by-step engine; stepping on after a
    drain (checkpoint) works."""
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    data = make_population_data(num_params=6000, num_halos=300_000, seed=12, device=DEV)
    model = PopulationSMFModel(aux_data=data)
    model.set_target_from_truth()
    monkeypatch.setenv("MULTIGRAD_PIPELINE", "0")
    ref_eng = FusedAdamEngine(model, graph=graph, owner=owner)
    ref = ref_eng.run_adam(data["guess"], nsteps=6, learning_rate=1e-3, history=history)
    assert not ref_eng.pipeline
    monkeypatch.setenv("MULTIGRAD_PIPELINE", "1")
    eng = FusedAdamEngine(model, graph=graph, owner=owner)
    eng.setup(data["guess"], 6, learning_rate=1e-3, history=history)
    eng.step_replay = True  # direct calls replay in graph mode (no default-stream work here)
    assert eng.pipeline
    for i in range(6):
        eng.step()
        if i == 2:
            eng.drain()  # e.g. a checkpoint in the middle
        assert np.isfinite(eng.last_loss())
    t = eng.trajectory()
    torch.testing.assert_close(t, ref, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(eng.params(), ref[-1], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("pipeline", ["1", "0"])
def test_setup_autotune_leaves_trajectory_unchanged(monkeypatch, pipeline):
    """One rank, auto graph policy: the setup-time eager-vs-replay timing runs steps (no
    trajectory rows) and restores the state; the trajectory equals a plain eager run's bit
    for bit (replayed and eager steps launch the same kernels), even when it is shorter
    than the tuning windows."""
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    monkeypatch.setenv("MULTIGRAD_PIPELINE", pipeline)
    data = make_population_data(num_params=6000, num_halos=300_000, seed=21, device=DEV)
    model = PopulationSMFModel(aux_data=data)
    model.set_target_from_truth()
    ref = FusedAdamEngine(model, graph=False).run_adam(data["guess"], nsteps=6, learning_rate=1e-3)
    eng = FusedAdamEngine(model)
    t = eng.run_adam(data["guess"], nsteps=6, learning_rate=1e-3)
    assert eng.tuning is not None and eng.use_graph == eng.tuning["chosen"]["use_graph"]
    assert eng.tuning["steps_per_window"] >= 8
    torch.testing.assert_close(t, ref, rtol=0, atol=0)
    monkeypatch.setenv("MULTIGRAD_AUTOTUNE", "0")
    off = FusedAdamEngine(model)
    off.setup(data["guess"], 4, learning_rate=1e-3)
    assert off.tuning is None


@pytest.mark.parametrize("giant", [None, 3])
def test_lanes_recompute_vjp_matches_residual_vjp(giant):
    """The recomputing lanes VJP (local slot order, hashed shards) against the residual
    VJP and the fp64 oracle, whole shard and per chunk, with split populations."""
    n, npop = 300_000, 700
    x, pop = _rand_shard(n, npop, seed=4, giant=giant)
    bins = S.SmfBins.make(np.linspace(8.0, 9.6, 11), volume=1e4)
    th = _theta(npop).float().to(DEV)
    loc = S.PopulationShard(x.float(), pop.int().to(DEV), npop, device=DEV, chunks=3,
                            layout="lanes", lane_order="local", lane_lmax=1024)
    ref = S.PopulationShard(x.float(), pop.int().to(DEV), npop, device=DEV, chunks=3,
                            layout="lanes", lane_lmax=1024)
    assert loc.vjp_recompute and not ref.vjp_recompute
    h = torch.linspace(0.7, -0.4, bins.nbp + 1, device=DEV)
    g_rc = torch.zeros_like(th)
    S.smf_vjp_into(th, loc, bins, True, h, g_rc, recompute=True)
    g_res = torch.zeros_like(th)
    S.smf_vjp_into(th, ref, bins, True, h, g_res)
    torch.testing.assert_close(g_rc, g_res, rtol=2e-5, atol=2e-6 * float(g_res.abs().max()))
    acc = torch.full_like(th, float("nan"))
    for c in range(loc.nchunks):
        S.smf_vjp_into(th, loc, bins, True, h, acc, chunk=c, recompute=True)
    assert torch.equal(acc, g_rc)
    # fp64 oracle: d/dtheta of sum_e h_e sqrt(2 pi) Phi(z_e)
    th64 = th.double().cpu().requires_grad_(True)
    hw = h[:bins.nb + 1].double().cpu() * np.sqrt(2 * np.pi)
    t2 = th64.reshape(-1, 2)
    mu = x.float().double() + t2[:, 0][pop]
    sig = torch.pow(10.0, t2[:, 1][pop])
    z = (torch.tensor(bins.edges, dtype=torch.float64)[None, :] - mu[:, None]) / sig[:, None]
    (g64,) = torch.autograd.grad((torch.special.ndtr(z) * hw[None, :]).sum(), th64)
    np.testing.assert_allclose(g_rc.cpu().double(), g64, rtol=2e-4, atol=2e-5 * float(g64.abs().max()))


@pytest.mark.parametrize("mode", ["static", "dynamic"])
def test_forward_schedules_at_eighth_shard_vs_fp64(monkeypatch, mode):
    """The headline forward at the size of one rank of the 8-GPU owner placement (1/8 of
    the parameters and halos): static LPT lists with the issue-priority feedback (the
    schedule `auto` picks there) and the dynamic queues, against a float64 PyTorch oracle
    of the same (float32-rounded) inputs; the residual VJP on a sub-sample of populations."""
    from multigrad_amd.models.population import make_population_data
    monkeypatch.setenv("MULTIGRAD_LPT", mode)
    data = make_population_data(num_params=1_250_000, num_halos=1 << 24, seed=1234, device=DEV)
    shard, bins = data["shard"], data["bins"]
    th = data["guess"]
    out = torch.zeros(bins.nbp, device=DEV)
    S.smf_forward_into(th, shard, bins, True, out, resid=True)
    # fp64 oracle on the device, in chunks of halos
    th64 = th.double()
    ref = torch.zeros(bins.nb, dtype=torch.float64, device=DEV)
    for a in range(0, shard.n, 1 << 22):
        ref += S.smf_sumstats_reference(th64, shard.x[a:a + (1 << 22)].double(),
                                        shard.pop[a:a + (1 << 22)], bins, True)
    np.testing.assert_allclose(out[:bins.nb].cpu().double(), ref.cpu(), rtol=2e-5)
    # VJP through the residuals against autograd of the oracle, populations [0, 2000)
    h = torch.linspace(0.6, -0.5, bins.nbp + 1, device=DEV)
    grad = torch.zeros_like(th)
    S.smf_vjp_into(th, shard, bins, True, h, grad, residuals_ready=True)
    npop_s = 2000
    sel = shard.pop < npop_s
    t64 = th64[:2 * npop_s].clone().requires_grad_(True)
    hw = h[:bins.nb + 1].double() * np.sqrt(2 * np.pi)
    t2 = t64.reshape(-1, 2)
    p = shard.pop[sel].long()
    mu = shard.x[sel].double() + t2[:, 0][p]
    sig = torch.pow(10.0, t2[:, 1][p])
    z = (torch.tensor(bins.edges, dtype=torch.float64, device=DEV)[None, :] - mu[:, None]) / sig[:, None]
    (g64,) = torch.autograd.grad((torch.special.ndtr(z) * hw[None, :]).sum(), t64)
    np.testing.assert_allclose(grad[:2 * npop_s].cpu().double(), g64.cpu(), rtol=2e-4,
                               atol=2e-5 * float(g64.abs().max()))


def _narrow_guess(data, every=2, logsig=-1.7):
    """The population guess with log10 sigma = ``logsig`` on every ``every``-th population:
    bin width / sigma = 5 there, far outside the Euler-Maclaurin path's kEmHMax = 0.5, so
    most lanes groups mix both kinds of lane and take the per-edge fallback."""
    g = data["guess"].clone()
    g[1::2 * every] = logsig
    return g


def test_em_forward_fallback_groups_vs_fp64():
    """Lanes forward with residuals where many groups must take the per-edge fallback
    (narrow populations) and the rest the Euler-Maclaurin path: sumstats against the fp64
    oracle, residual VJP against autograd of the oracle."""
    from multigrad_amd.models.population import make_population_data
    data = make_population_data(num_params=20_000, num_halos=600_000, seed=5, device=DEV)
    shard, bins = data["shard"], data["bins"]
    th = _narrow_guess(data)
    out = torch.zeros(bins.nbp, device=DEV)
    S.smf_forward_into(th, shard, bins, True, out, resid=True)
    # (the narrow groups went through the out-of-line per-edge call, LMODE 3)
    ref = S.smf_sumstats_reference(th.double(), shard.x.double(), shard.pop, bins, True)
    np.testing.assert_allclose(out[:bins.nb].cpu().double(), ref.cpu(), rtol=2e-5)
    h = torch.linspace(0.6, -0.5, bins.nbp + 1, device=DEV)
    grad = torch.zeros_like(th)
    S.smf_vjp_into(th, shard, bins, True, h, grad, residuals_ready=True)
    t64 = th.double().clone().requires_grad_(True)
    hw = h[:bins.nb + 1].double() * np.sqrt(2 * np.pi)
    t2 = t64.reshape(-1, 2)
    p = shard.pop.long()
    mu = shard.x.double() + t2[:, 0][p]
    sig = torch.pow(10.0, t2[:, 1][p])
    z = (torch.tensor(bins.edges, dtype=torch.float64, device=DEV)[None, :] - mu[:, None]) / sig[:, None]
    (g64,) = torch.autograd.grad((torch.special.ndtr(z) * hw[None, :]).sum(), t64)
    np.testing.assert_allclose(grad.cpu().double(), g64.cpu(), rtol=2e-4,
                               atol=2e-5 * float(g64.abs().max()))


def test_pipelined_update_with_fallback_groups_matches_unpipelined(monkeypatch):
    """The pipelined-update forward (Euler-Maclaurin + fallback groups in one launch) gives
    the step-by-step engine's trajectory."""
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    data = make_population_data(num_params=6000, num_halos=300_000, seed=12, device=DEV)
    model = PopulationSMFModel(aux_data=data)
    model.set_target_from_truth()
    guess = _narrow_guess(data, every=3)
    monkeypatch.setenv("MULTIGRAD_PIPELINE", "0")
    ref = FusedAdamEngine(model, graph=False).run_adam(guess, nsteps=5, learning_rate=1e-3)
    monkeypatch.setenv("MULTIGRAD_PIPELINE", "1")
    eng = FusedAdamEngine(model, graph=False)
    t = eng.run_adam(guess, nsteps=5, learning_rate=1e-3)
    assert eng.pipeline
    torch.testing.assert_close(t, ref, rtol=1e-6, atol=1e-7)


def test_headline_kernel_vs_fp64(monkeypatch):
    """The exact timed instantiation -- smf_fwd_lanes_kernel<10,true,false,true,true,3>, the
    pipelined forward with the fused VJP + Adam, at the headline size (1e7 parameters,
    1.34e8 halos) -- for 2 steps: S(theta_1) against the fp64 oracle (rtol 2e-5), and the
    step-0 gradient (read back from the first Adam moment, m = (1 - b1) g) on 2000
    populations against autograd of the fp64 loss (rtol 2e-4)."""
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    from multigrad_amd.ops.smf import logmse_loss
    monkeypatch.setenv("MULTIGRAD_PIPELINE", "1")
    monkeypatch.setenv("MULTIGRAD_AUTOTUNE", "0")
    data = make_population_data(num_params=10_000_000, num_halos=1 << 27, seed=1234, device=DEV)
    model = PopulationSMFModel(aux_data=data)
    model.set_target_from_truth()
    shard, bins = data["shard"], data["bins"]
    eng = FusedAdamEngine(model, graph=False)
    # more steps than are taken: the last step of a run drains its pending update
    eng.setup(data["guess"], nsteps=4, learning_rate=1e-3, history="last")
    assert eng.pipeline and shard.layout == "lanes"
    eng.step()
    eng.step()           # applies update 0 in the forward, evaluates S(theta_1)
    torch.cuda.synchronize()
    theta1 = eng.to_user(eng.theta[:eng.P]).clone()
    S1 = eng.S[:bins.nb].double().cpu()
    g0 = (eng.to_user(eng.m[:eng.P]) / (1.0 - eng.b1)).double()
    th0 = data["guess"].double()

    def oracle(th64, sel=None):
        tot = torch.zeros(bins.nb, dtype=torch.float64, device=DEV)
        for a in range(0, shard.n, 1 << 22):
            tot += S.smf_sumstats_reference(th64, shard.x[a:a + (1 << 22)].double(),
                                            shard.pop[a:a + (1 << 22)], bins, True)
        return tot

    ref1 = oracle(theta1.double())
    np.testing.assert_allclose(S1, ref1.cpu(), rtol=2e-5)
    # dL/dS at theta_0 from the fp64 sumstats, then the gradient of the populations < 2000
    S0 = oracle(th0).requires_grad_(True)
    t = data["target_sumstats"].double()
    (dLdS,) = torch.autograd.grad(logmse_loss(S0, t, data["loss_eps"]), S0)
    npop_s = 2000
    sel = shard.pop < npop_s
    t64 = th0[:2 * npop_s].clone().requires_grad_(True)
    part = S.smf_sumstats_reference(t64, shard.x[sel].double(), shard.pop[sel], bins, True)
    (gref,) = torch.autograd.grad(part, t64, dLdS)
    np.testing.assert_allclose(g0[:2 * npop_s].cpu(), gref.cpu(), rtol=2e-4,
                               atol=2e-5 * float(gref.abs().max()))


@pytest.mark.parametrize("pipeline,owner", [("1", False), ("0", False), ("1", True)])
def test_block_graph_replays_match_eager(monkeypatch, pipeline, owner):
    """Whole-loop capture in blocks: graph mode replays graphs of
    MULTIGRAD_GRAPH_STEPS unrolled steps (here 4, with a remainder of 3 single steps and a
    pipelined first step) and gives the eager trajectory."""
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    monkeypatch.setenv("MULTIGRAD_PIPELINE", pipeline)
    monkeypatch.setenv("MULTIGRAD_AUTOTUNE", "0")
    data = make_population_data(num_params=6000, num_halos=300_000, seed=14, device=DEV)
    model = PopulationSMFModel(aux_data=data)
    model.set_target_from_truth()
    ref = FusedAdamEngine(model, graph=False, owner=owner).run_adam(
        data["guess"], nsteps=11, learning_rate=1e-3)
    monkeypatch.setenv("MULTIGRAD_GRAPH_STEPS", "4")
    eng = FusedAdamEngine(model, graph=True, owner=owner)
    t = eng.run_adam(data["guess"], nsteps=11, learning_rate=1e-3)
    assert eng.use_graph and eng.graph_steps == 4 and eng._kgraph is not None
    torch.testing.assert_close(t, ref, rtol=1e-6, atol=1e-7)


def test_per_edge_kernel_mode_matches_em_kernel(monkeypatch):
    """LMODE 4 (the per-edge kernel for every group, chosen when most lane groups hold
    narrow populations): sumstats against the fp64 oracle, and the pipelined engine's
    trajectory against the Euler-Maclaurin kernel's with its out-of-line per-edge call."""
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    data = make_population_data(num_params=6000, num_halos=300_000, seed=17, device=DEV)
    shard, bins = data["shard"], data["bins"]
    model = PopulationSMFModel(aux_data=data)
    model.set_target_from_truth()
    guess = _narrow_guess(data, every=3)
    runs = {}
    for share in (2.0, 0.0):  # 2.0: never per-edge; 0.0: always
        monkeypatch.setattr(S, "PER_EDGE_SHARE", share)
        out = torch.zeros(bins.nbp, device=DEV)
        S.smf_forward_into(guess, shard, bins, True, out, resid=True)
        ref = S.smf_sumstats_reference(guess.double(), shard.x.double(), shard.pop, bins, True)
        np.testing.assert_allclose(out[:bins.nb].cpu().double(), ref.cpu(), rtol=2e-5)
        eng = FusedAdamEngine(model, graph=False)
        runs[share] = eng.run_adam(guess, nsteps=5, learning_rate=1e-3)
        assert eng.pipeline
    # two evaluation methods (Euler-Maclaurin vs per-edge tails, ~1e-6 apart in the bin
    # masses): Adam steps of lr 1e-3 on populations with near-zero gradients amplify that
    # to ~1e-5 in a few parameters (measured 1.04e-5 after 5 steps); a wrong kernel would
    # be off by whole steps
    torch.testing.assert_close(runs[0.0], runs[2.0], rtol=1e-5, atol=1e-4)


def test_narrow_populations_get_their_own_lane_groups():
    """The fused engine groups narrow populations (bin width > 0.5 sigma at the guess) into
    lane groups of their own: with 1% of populations narrow, about 1% of the groups take
    the per-edge path (without the layout hint, ~half of them would)."""
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    data = make_population_data(num_params=200_000, num_halos=2_700_000, seed=4, device=DEV,
                                narrow_frac=0.01)
    model = PopulationSMFModel(aux_data=data)
    model.set_target_from_truth()
    before = model.lane_fallback_groups(data["guess"])
    eng = FusedAdamEngine(model, graph=False)
    eng.setup(data["guess"], 3, learning_rate=1e-3)
    after = model.lane_fallback_groups(data["guess"])
    assert before[0] > 0.3 * before[1] and after[0] < 0.05 * after[1], (before, after)
    eng.steps(3)
    assert np.isfinite(eng.last_loss())


def _crossing_model(seed=14, npar=6000, nhalo=300_000):
    """20% of the populations start wide (log10 sigma -0.6, Euler-Maclaurin path) and fit
    towards a narrow truth (-1.1): they cross the limit (-0.70) during the run."""
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    data = make_population_data(num_params=npar, num_halos=nhalo, seed=seed, device=DEV,
                                narrow_frac=0.2, narrow_guess_log_sigma=-0.6)
    model = PopulationSMFModel(aux_data=data)
    model.set_target_from_truth()
    return model, data


@pytest.mark.parametrize("owner,graph,history", [(False, False, "full"), (False, True, "full"),
                                                 (True, False, "full"), (False, False, "last")])
def test_relayout_during_fit_matches_static_layout(monkeypatch, owner, graph, history):
    """populations crossing the Euler-Maclaurin limit mid-fit trigger a
    re-layout (device probe -> re-classification -> lanes rebuilt on the GPU, theta / m / v
    permuted); the trajectory equals the run that keeps its setup layout (rtol 1e-5)."""
    from multigrad_amd.engine.fused import FusedAdamEngine
    model, data = _crossing_model()
    kw = dict(nsteps=40, learning_rate=2e-2, history=history)
    monkeypatch.setenv("MULTIGRAD_RELAYOUT", "0")
    ref_eng = FusedAdamEngine(model, graph=graph, owner=owner)
    ref = ref_eng.run_adam(data["guess"], **kw)
    assert not ref_eng.relayouts
    monkeypatch.setenv("MULTIGRAD_RELAYOUT", "1")
    monkeypatch.setenv("MULTIGRAD_RELAYOUT_EVERY", "4")
    eng = FusedAdamEngine(model, graph=graph, owner=owner)
    t = eng.run_adam(data["guess"], **kw)
    assert eng.relayouts, "the crossing populations should have triggered a re-layout"
    r = eng.relayouts[-1]
    assert r["share_new"] < r["share_probe"]  # the narrow lanes are grouped again
    torch.testing.assert_close(t, ref, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(eng.params(), ref[-1], rtol=1e-5, atol=1e-6)


def test_relayout_checkpoint_resumes_in_setup_layout(tmp_path, monkeypatch):
    """A checkpoint written after a re-layout resumes in an engine laid out at the guess
    (the saved vectors carry their order) and continues the same trajectory."""
    from multigrad_amd.engine.fused import FusedAdamEngine
    model, data = _crossing_model(seed=15)
    monkeypatch.setenv("MULTIGRAD_RELAYOUT_EVERY", "4")
    a = FusedAdamEngine(model, graph=False)
    a.setup(data["guess"], nsteps=30, learning_rate=2e-2)
    a.steps(20)
    assert a.relayouts
    path = str(tmp_path / "ck.pt")
    a.save_checkpoint(path)
    a.steps(10)
    ta = a.trajectory()
    monkeypatch.setenv("MULTIGRAD_RELAYOUT", "0")
    b = FusedAdamEngine(model, graph=False)
    b.setup(data["guess"], nsteps=30, learning_rate=2e-2)
    assert b.load_checkpoint(path) == 20
    b.steps(10)
    torch.testing.assert_close(b.trajectory(), ta, rtol=1e-5, atol=1e-6)
