"""Device-side collectives of the device L-BFGS(-B) (BASELINE config 4), with several
processes sharing one MI355X:

* the wide one-shot fp64 all-reduce (sum + max parts, bitwise identical on every rank);
* the two-shot reduce-scatter (mode 4) and all-gather (mode 5) of the sharded evaluation,
  and the raw-bit peer all-gather;
* the device L-BFGS on the fused engine at 2, 4 and 8 ranks: the same iterate as one rank
  after 10 iterations, and ZERO host (gloo) collectives in the iterations -- every
  reduction of the loop runs on the GPU (reference multigrad/bfgs.py:32-113 broadcasts
  every trial point from the root instead).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from distributed import run_distributed  # noqa: E402


def _values(r, i, n):
    g = torch.Generator().manual_seed(1000 * i + r)
    return torch.randn(n, generator=g, dtype=torch.float64)


def _wide(rank, size, ncalls):
    import multigrad_amd as mg
    from multigrad_amd.parallel.xgmi import get_wide_oneshot
    comm = mg.get_world_comm()
    dev = torch.device("cuda", 0)
    ar = get_wide_oneshot(comm)
    assert ar is not None, "wide one-shot context did not connect"
    outs = []
    for i in range(ncalls):
        n = 1 + (37 * i) % 1024
        nmax = i % 5
        nmax = min(nmax, n)
        t = _values(rank, i, n).to(dev)
        ar(t, n - nmax, nmax)
        outs.append(t)
    got = [o.cpu().numpy() for o in outs]
    torch.cuda.synchronize()
    return got, ar.ok()


@pytest.mark.parametrize("size", [2, 4])
def test_wide_oneshot_sum_and_max(size):
    res = run_distributed(_wide, size, 60, timeout=300)
    ncalls = 60
    for r in range(size):
        assert res[r][1]
    for i in range(ncalls):
        n = 1 + (37 * i) % 1024
        nmax = min(i % 5, n)
        vals = [_values(r, i, n).numpy() for r in range(size)]
        want = vals[0].copy()
        for r in range(1, size):  # rank order, fp64: the kernel's order
            want[:n - nmax] += vals[r][:n - nmax]
            want[n - nmax:] = np.where(vals[r][n - nmax:] > want[n - nmax:],
                                       vals[r][n - nmax:], want[n - nmax:])
        for r in range(size):
            np.testing.assert_array_equal(res[r][0][i], want)


def _modes45(rank, size):
    import multigrad_amd as mg
    from multigrad_amd.parallel.xgmi import connect_twoshot, peer_all_gather
    comm = mg.get_world_comm()
    dev = torch.device("cuda", 0)
    numel = 4 * size * 1000
    ts = connect_twoshot(comm, numel)
    assert ts is not None
    out = []
    for rep in range(3):
        # every rank's gradient region: distinct values; mode 4 sums this rank's slice
        idx = torch.arange(numel, device=dev, dtype=torch.float32)
        ts.grad.copy_(torch.remainder(idx * (rank + 2), 251.0) + rep)
        lo, n = ts.slice()
        red = torch.empty(n, device=dev)
        ts.reduce_scatter_(red, lo, n)
        # mode 5: this rank's slice -> every rank's parameter region
        src = torch.full((n,), float(rank + 10 * rep), device=dev)
        ts.all_gather_(src, lo, n)
        out.append((red.cpu().numpy(), ts.theta.cpu().numpy().copy()))
    x = torch.arange(7, dtype=torch.float64, device=dev) + 1000.0 * rank + 0.1
    g = torch.empty((size, 7), dtype=torch.float64, device=dev)
    ok_gather = peer_all_gather(comm, g, x)
    torch.cuda.synchronize()
    ok = ts.ok()
    ts.close()
    return out, g.cpu().numpy(), ok_gather, ok


@pytest.mark.parametrize("size", [2, 4])
def test_twoshot_reduce_scatter_and_all_gather_modes(size):
    res = run_distributed(_modes45, size, timeout=300)
    numel = 4 * size * 1000
    n = numel // size
    idx = np.arange(numel, dtype=np.float32)
    for rep in range(3):
        grads = [np.remainder(idx * (r + 2), np.float32(251.0)).astype(np.float32) + rep
                 for r in range(size)]
        total = grads[0].copy()
        for r in range(1, size):
            total = total + grads[r]
        gathered = np.concatenate([np.full(n, r + 10 * rep, dtype=np.float32)
                                   for r in range(size)])
        for r in range(size):
            red, theta = res[r][0][rep]
            np.testing.assert_array_equal(red, total[r * n:(r + 1) * n])
            np.testing.assert_array_equal(theta, gathered)
    for r in range(size):
        out, g, ok_gather, ok = res[r]
        assert ok_gather and ok
        want = np.stack([np.arange(7) + 1000.0 * q + 0.1 for q in range(size)])
        np.testing.assert_array_equal(g, want)


NP, NH = 6000, 400_000


def _lbfgs(rank, size, placement, bounded=False, iters=10):
    import multigrad_amd as mg
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    comm = mg.get_world_comm()
    dev = torch.device("cuda", 0)
    data = make_population_data(NP, NH, seed=21, comm=comm, device=dev, placement=placement)
    model = PopulationSMFModel(aux_data=data, comm=comm)
    model.set_target_from_truth()
    kw = {}
    if bounded:
        g = data["guess"].cpu()
        kw["param_bounds"] = torch.stack([g - 0.05, g + 0.3], 1).numpy()
    res = model.run_bfgs(data["guess"], maxsteps=iters, method="device", **kw)
    return (res.x.cpu().numpy(), float(res.fun), int(res.nit), int(res.nfev),
            int(getattr(res, "host_collectives", -1)), getattr(res, "reduction", None))


@pytest.mark.parametrize("placement,size", [("hashed", 2), ("hashed", 4), ("hashed", 8),
                                            ("owner", 2), ("owner", 4)])
def test_device_lbfgs_multirank_one_gpu_no_host_collectives(placement, size):
    import multigrad_amd.parallel.comm as C
    C.set_world_comm(None)
    x1, f1, nit1, nfev1, _, _ = _lbfgs(0, 1, placement)
    res = run_distributed(_lbfgs, size, placement, timeout=900)
    for x, f, nit, nfev, host, how in res:
        assert host == 0, f"{host} host collectives in the L-BFGS iterations ({how})"
        assert how == "xgmi wide one-shot"
        assert nit == nit1
        assert f == pytest.approx(f1, rel=2e-4, abs=1e-9)
        np.testing.assert_allclose(x, x1, rtol=2e-4, atol=2e-5)
    for r in range(1, size):  # the SPMD iterate is bitwise identical on every rank
        np.testing.assert_array_equal(res[r][0], res[0][0])


def test_device_lbfgsb_two_ranks_one_gpu_no_host_collectives():
    import multigrad_amd.parallel.comm as C
    C.set_world_comm(None)
    x1, f1, nit1, _, _, _ = _lbfgs(0, 1, "hashed", True)
    res = run_distributed(_lbfgs, 2, "hashed", True, timeout=900)
    for x, f, nit, nfev, host, how in res:
        assert host == 0, f"{host} host collectives in the L-BFGS-B iterations ({how})"
        assert nit == nit1
        assert f == pytest.approx(f1, rel=2e-4, abs=1e-9)
        np.testing.assert_allclose(x, x1, rtol=2e-4, atol=2e-5)
    np.testing.assert_array_equal(res[1][0], res[0][0])


def _lbfgs_fault(rank, size):
    import os
    os.environ["MULTIGRAD_ONESHOT_TIMEOUT"] = "1"
    os.environ["MULTIGRAD_LBFGS_FAULT"] = "1:3"   # rank 1 skips the 3rd evaluation
    from multigrad_amd.parallel.xgmi import CollectiveTimeout
    try:
        _lbfgs(rank, size, "hashed", iters=6)
    except CollectiveTimeout as exc:
        return "raised", str(exc)[:200]
    return "returned", ""


def test_device_lbfgs_zero_exchange_timeout_raises_on_every_rank():
    """A peer that skips the ZeRO evaluation's two-shot exchanges makes the others' bounded
    waits time out: the run must raise CollectiveTimeout on every rank (checked at the end of
    the optimizer), not return a NaN iterate with an ordinary status."""
    res = run_distributed(_lbfgs_fault, 2, timeout=600)
    assert [r[0] for r in res] == ["raised", "raised"], res
