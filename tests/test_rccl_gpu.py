"""RCCL communicator path on one MI355X (a 1-rank RCCL communicator built exactly like
the multi-GPU ones), and the ZeRO-1 engine running its reduce-scatter / all-gather
schedule through it."""
import datetime
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _store():
    from torch._C._distributed_c10d import TCPStore
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    return TCPStore("127.0.0.1", port, 1, True, timeout=datetime.timedelta(seconds=60))


def _rccl_comm():
    from multigrad_amd.parallel.comm import TorchComm
    return TorchComm(_store(), 0, 1, "WORLD", "w-test", [0], use_device=True)


def test_rccl_collectives_single_rank(monkeypatch):
    monkeypatch.setenv("MULTIGRAD_ALLREDUCE", "rccl")  # tiny all-reduces would go one-shot
    comm = _rccl_comm()
    dev = torch.device("cuda", 0)
    x = torch.arange(8.0, device=dev)
    comm.all_reduce(x)
    assert torch.equal(x, torch.arange(8.0, device=dev))
    assert comm._dev is not None  # the device backend (RCCL) was used
    out = torch.empty(8, device=dev)
    w = comm.reduce_scatter_tensor(out, torch.arange(8.0, device=dev), async_op=True)
    w.wait()
    torch.cuda.synchronize()
    assert torch.equal(out, torch.arange(8.0, device=dev))
    full = torch.zeros(8, device=dev)
    full[:4] = 5.0
    w = comm.all_gather_into_tensor(full[:8], full[:8], async_op=True)
    w.wait()
    torch.cuda.synchronize()
    assert float(full[:4].sum()) == 20.0
    b = torch.full((3,), 2.0, device=dev)
    comm.broadcast(b, root=0)
    assert comm.bcast({"k": 1}) == {"k": 1}


def test_zero_engine_schedule_over_rccl():
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    dev = torch.device("cuda", 0)
    data = make_population_data(num_params=4002, num_halos=300_000, seed=5, device=dev)
    model = PopulationSMFModel(aux_data=data)
    model.set_target_from_truth()
    ref = model.run_adam(data["guess"], nsteps=4, learning_rate=1e-3, use_engine=False)
    eng = FusedAdamEngine(model, comm=_rccl_comm(), chunks=3, graph=False)
    eng.zero = True  # force the sharded schedule on a 1-rank communicator
    traj = eng.run_adam(data["guess"], nsteps=4, learning_rate=1e-3)
    assert eng.C == 3 and eng.P_pad >= 4002
    torch.testing.assert_close(traj, ref, rtol=1e-5, atol=1e-6)


def test_onepoint_group_on_rccl_subcommunicators(monkeypatch):
    """OnePointGroup with each model on its own RCCL-backed communicator and the group sum
    over a third one, on the GPU (1 rank each: the communicators short-circuit their
    collectives at size 1, so this pins the group plumbing on device tensors; the
    multi-rank sums are covered on gloo by test_models.py)."""
    monkeypatch.setenv("MULTIGRAD_ALLREDUCE", "rccl")
    import multigrad_amd as mg
    from multigrad_amd.models.smf import DocsSMFModel, make_docs_data
    dev = torch.device("cuda", 0)
    sub_a, sub_b, main = _rccl_comm(), _rccl_comm(), _rccl_comm()
    ma = DocsSMFModel(aux_data=make_docs_data(20_000, device=dev), comm=sub_a, device=dev)
    mb = DocsSMFModel(aux_data=make_docs_data(30_000, true_params=(-1.9, -0.6), device=dev),
                      comm=sub_b, device=dev)
    grp = mg.OnePointGroup(models=(ma, mb), main_comm=main)
    p = torch.tensor([-1.9, -0.4], device=dev)
    loss, grad = grp.calc_loss_and_grad_from_params(p)
    la, ga = ma.calc_loss_and_grad_from_params(p)
    lb, gb = mb.calc_loss_and_grad_from_params(p)
    torch.testing.assert_close(loss, la + lb)
    torch.testing.assert_close(grad, ga + gb)
    assert grad.is_cuda and loss.is_cuda
    res = grp.run_bfgs(p, maxsteps=30)
    assert res.success or res.nit > 0
    # the group's GD / Adam front-ends keep the eager loop (the captured engine takes
    # single models only)
    gd = grp.run_simple_grad_descent(p, nsteps=3, learning_rate=1e-3)
    assert gd.params.shape == (3, 2) and torch.isfinite(gd.loss).all()
    traj = grp.run_adam(p, nsteps=3, learning_rate=1e-3)
    assert tuple(traj.shape) == (4, 2)
