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


# ------------------------------------------------------------- keys, aux, groups (CPU)
class _Noisy(mg.OnePointModel):
    """Stochastic model: the sumstats draw noise from the step's randkey on the model's
    device (the engine's key contract: ``randkey.generator(device)``)."""

    def calc_partial_sumstats_from_params(self, params, randkey=None):
        t = self.aux_data["target"]
        noise = 0.0
        if randkey is not None:
            noise = 0.3 * torch.randn(t.shape, generator=randkey.generator(t.device),
                                      device=t.device)
        return (params - t) ** 2 * (1.0 + noise)

    def calc_loss_from_sumstats(self, sumstats, sumstats_aux=None, randkey=None):
        return sumstats.sum()


class _AuxModel(mg.OnePointModel):
    """sumstats_func_has_aux: the aux (a per-rank weight) reaches the loss, unreduced."""

    def calc_partial_sumstats_from_params(self, params, randkey=None):
        t = self.aux_data["target"]
        return (params - t) ** 2, self.aux_data["w"]

    def calc_loss_from_sumstats(self, sumstats, sumstats_aux=None, randkey=None):
        return (sumstats * sumstats_aux).sum()


@pytest.mark.parametrize("const", [False, True])
def test_generic_engine_randkey_matches_eager(const):
    C.set_world_comm(None)
    m = _Noisy(aux_data={"target": torch.tensor([1.0, -2.0, 0.5, 3.0])})
    g0 = torch.zeros(4)
    ref = m.run_adam(g0, nsteps=6, learning_rate=0.1, randkey=7, const_randkey=const,
                     use_engine=False)
    eng = GraphAdamEngine(m)
    t = eng.run_adam(g0, nsteps=6, learning_rate=0.1, randkey=7, const_randkey=const)
    torch.testing.assert_close(t, ref, rtol=0, atol=0)
    noiseless = m.run_adam(g0, nsteps=6, learning_rate=0.1, use_engine=False)
    assert not torch.equal(t, noiseless)


def test_generic_engine_sumstats_aux_matches_eager():
    C.set_world_comm(None)
    m = _AuxModel(aux_data={"target": torch.tensor([1.0, -2.0, 0.5]),
                            "w": torch.tensor([1.0, 2.0, 0.5])}, sumstats_func_has_aux=True)
    ref = m.run_adam(torch.zeros(3), nsteps=5, learning_rate=0.1, use_engine=False)
    t = GraphAdamEngine(m).run_adam(torch.zeros(3), nsteps=5, learning_rate=0.1)
    torch.testing.assert_close(t, ref, rtol=0, atol=0)


def _group_body(rank, size, engine):
    comm = mg.get_world_comm()
    sub, ngroups, gidx = mg.split_subcomms(num_groups=2, comm=comm)
    # (no coordinate whose gradient cancels exactly between the groups: Adam would turn
    # the summation-order residue of a zero into a full step)
    tgt = torch.tensor([1.0, -2.0, 0.5]) if gidx == 0 else torch.tensor([-1.5, 0.5, 2.0])
    m = _Noisy(aux_data={"target": tgt * (1 + sub.rank)}, comm=sub)
    grp = mg.OnePointGroup(m, main_comm=comm)
    if engine:
        t = GraphAdamEngine(grp).run_adam(torch.zeros(3), nsteps=5, learning_rate=0.1,
                                          randkey=3)
    else:
        t = grp.run_adam(torch.zeros(3), nsteps=5, learning_rate=0.1, randkey=3,
                         use_engine=False)
    lg = grp.calc_loss_and_grad_from_params(torch.tensor([0.1, 0.2, 0.3]))
    return t.numpy(), float(lg[0]), lg[1].numpy()


def test_generic_engine_group_matches_eager_group():
    """OnePointGroup through the engine (members' chain rule on their sub-communicators,
    one summed exchange on the main communicator) against the eager group path, 4 ranks
    in 2 groups, per-step keys."""
    eng = run_distributed(_group_body, 4, True)
    ref = run_distributed(_group_body, 4, False)
    for (t, l, g), (tr, lr, gr) in zip(eng, ref):
        np.testing.assert_allclose(t, tr, rtol=1e-5, atol=1e-6)
    for r in range(1, 4):
        np.testing.assert_array_equal(eng[r][0], eng[0][0])


def test_capture_key_attribute_probes_are_attribute_errors():
    """hasattr / getattr-with-default on the capture-time randkey behave like on
    any object without that attribute; using the attribute raises KeyNotCapturable (which
    sends the engine to the eager path)."""
    from multigrad_amd.engine.generic import KeyNotCapturable, _CaptureKey
    k = _CaptureKey(eng=None)
    assert not hasattr(k, "split")
    assert getattr(k, "seed", 7) == 7
    with pytest.raises(KeyNotCapturable):
        k.split(2)
    import copy
    with pytest.raises(Exception):
        copy.copy(k).split  # protocol probes fall through to plain AttributeErrors


def test_engine_stream_context_is_a_no_op_off_the_gpu():
    """engine/_stream.py on a CPU engine: no stream switch, tensors handed back untouched,
    and a decorated method's result passes through; nested contexts are fine."""
    from multigrad_amd.engine._stream import EngineStream, on_engine_stream

    class Owner:
        calls = 0

        def _engine_stream(self):
            Owner.calls += 1
            return None

        def _stream_wanted(self):
            return True

        @on_engine_stream
        def work(self, x):
            with EngineStream(self):
                return {"a": [x * 2, (x + 1,)], "b": self}

    o = Owner()
    x = torch.ones(3)
    out = o.work(x)
    assert torch.equal(out["a"][0], 2 * x) and out["b"] is o
    assert Owner.calls == 2
    ctx = EngineStream(o)
    with ctx as s:
        assert s is None
    ctx.hand_over([out, out])  # cycles and repeats are fine
