"""Run-to-run reproducibility of the fused Adam step at a size where every forward wave
processes many lane groups (the headline's regime).  Until round 5 the forward drew its
groups from device work queues there, so which wave summed which group -- and with it the
last bits of the bin sums -- changed from run to run; the static LPT lists (the default at
every size since round 6, ``ops/smf.py:PopulationShard.fwd_schedule``) fix the order."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _trajectory(data, nsteps=6):
    from multigrad_amd.models.population import PopulationSMFModel
    m = PopulationSMFModel(aux_data=data)
    m.set_target_from_truth()
    eng = m.fused_engine(cache=False, graph=False)
    eng.setup(data["guess"], nsteps=nsteps, learning_rate=1e-3, history="full")
    eng.steps(nsteps)
    traj = eng.trajectory()
    loss = eng.last_loss()
    eng.close()
    return traj, loss


def test_default_schedule_is_bitwise_reproducible(monkeypatch):
    import multigrad_amd.parallel.comm as C
    from multigrad_amd.models.population import make_population_data
    monkeypatch.delenv("MULTIGRAD_LPT", raising=False)
    monkeypatch.setenv("MULTIGRAD_AUTOTUNE", "off")
    C.set_world_comm(None)
    # 2.4e6 populations (~37.5k lane groups) over 4096 forward waves: > 8 groups per wave
    data = make_population_data(4_800_000, 1 << 26, seed=11, device=DEV)
    shard = data["shard"]
    assert shard.ngroups >= 8 * 4096, shard.ngroups
    t1, l1 = _trajectory(data)
    t2, l2 = _trajectory(data)
    assert torch.equal(t1, t2)
    assert l1 == l2
