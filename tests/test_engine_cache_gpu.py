"""The fused engines are cached per model: a repeated run_adam / run_simple_grad_descent
re-uses buffers, layout, autotune verdict and captured graphs (zero trial steps, zero
captures) -- the analogue of the jit cache the reference's benchmark warms once
(tests/smf_example/benchmark.py:41-46)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _budgeted_autotune(monkeypatch):
    monkeypatch.setenv("MULTIGRAD_AUTOTUNE", "auto")   # the library default


def _model(npar=20_000, nhalo=400_000):
    import multigrad_amd.parallel.comm as C
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    C.set_world_comm(None)
    data = make_population_data(npar, nhalo, seed=3, device=DEV)
    m = PopulationSMFModel(aux_data=data)
    m.set_target_from_truth()
    return m, data


@pytest.mark.parametrize("history", ["full", "last"])
def test_second_run_adam_makes_no_captures_and_no_trial_steps(history):
    m, data = _model()
    t1 = m.run_adam(data["guess"], nsteps=3000, learning_rate=1e-3, history=history)
    eng = m.fused_engine()
    s1 = dict(eng.stats)
    assert eng.tuning is not None and not eng.tuning.get("budget_skipped"), eng.tuning
    assert s1["trial_steps"] > 0
    t2 = m.run_adam(data["guess"], nsteps=3000, learning_rate=1e-3, history=history)
    assert m.fused_engine() is eng and eng.tuning.get("cached")
    s2 = eng.stats
    assert s2["trial_steps"] == s1["trial_steps"], (s1, s2)
    assert s2["captures"] == s1["captures"], (s1, s2)
    assert s2["layouts"] == s1["layouts"], (s1, s2)
    assert torch.equal(t1, t2)   # the same schedule, bit for bit
    # the first trajectory is the caller's: the second run did not overwrite it
    assert t1.data_ptr() != t2.data_ptr()


def test_short_first_run_keeps_the_tuning_within_budget():
    """A run too short for the minimum autotune windows keeps the default schedule: the
    trial steps stay within ~10 % of the requested steps (plus the 4-step probe)."""
    m, data = _model()
    m.run_adam(data["guess"], nsteps=100, learning_rate=1e-3)
    eng = m.fused_engine()
    assert eng.tuning.get("budget_skipped"), eng.tuning
    assert eng.stats["trial_steps"] <= 4 + 10 + 1, eng.stats
    n = eng.stats["trial_steps"]
    m.run_adam(data["guess"], nsteps=100, learning_rate=1e-3)   # the same short run again
    assert eng.tuning.get("cached") and eng.stats["trial_steps"] == n, eng.stats


def test_new_data_rebuilds_the_cached_engine():
    from multigrad_amd.models.population import make_population_data
    m, data = _model()
    m.run_adam(data["guess"], nsteps=20, learning_rate=1e-3)
    eng = m.fused_engine()
    m.aux_data["shard"] = make_population_data(20_000, 300_000, seed=4, device=DEV)["shard"]
    assert m.fused_engine() is not eng


def test_smf2_second_gd_call_captures_nothing():
    import multigrad_amd.parallel.comm as C
    from multigrad_amd.models.smf import MySMFModel, ParamTuple, make_test_data
    C.set_world_comm(None)
    model = MySMFModel(aux_data=make_test_data(1_000_000), device=DEV)
    model.run_simple_grad_descent(ParamTuple(-1.0, 0.5), nsteps=1, learning_rate=1e-3)  # warm-up
    eng = model.fused_step_engine()
    caps = eng.stats["captures"]
    r = model.run_simple_grad_descent(ParamTuple(-1.0, 0.5), nsteps=100, learning_rate=1e-3)
    assert eng.stats["captures"] == caps and r.loss.shape == (100,)
