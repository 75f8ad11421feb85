"""Where a device L-BFGS-B iteration goes at 1e7 parameters (one GPU): CUDA-event timing
of the Cauchy-point pieces (breakpoint sort, batch scans) and where the Cauchy point
lands in the sorted breakpoints."""
import sys
import time

import torch

sys.path.insert(0, ".")
import multigrad_amd.optim.lbfgsb as LB  # noqa: E402
from multigrad_amd.models.population import PopulationSMFModel, make_population_data  # noqa: E402

data = make_population_data(10_000_000, 1 << 27, seed=1234, device=torch.device("cuda", 0))
m = PopulationSMFModel(aux_data=data)
m.set_target_from_truth()
g = data["guess"].detach().cpu().numpy()
bounds = __import__("numpy").stack([g - 0.15, g + 0.05], 1)
stats = {"scan_calls": 0, "scan_ms": 0.0, "cp_ms": 0.0, "cp_calls": 0, "batchN": []}
orig_scan, orig_cp = LB._scan_batch, LB._cauchy_point


def ev():
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


def scan(st, t, gg, W, M, theta):
    e0 = ev()
    r = orig_scan(st, t, gg, W, M, theta)
    e1 = ev()
    torch.cuda.synchronize()
    stats["scan_calls"] += 1
    stats["scan_ms"] += e0.elapsed_time(e1)
    stats["batchN"].append(int(t.numel()))
    return r


def cp(*a, **k):
    e0 = ev()
    r = orig_cp(*a, **k)
    e1 = ev()
    torch.cuda.synchronize()
    stats["cp_calls"] += 1
    stats["cp_ms"] += e0.elapsed_time(e1)
    return r


LB._scan_batch, LB._cauchy_point = scan, cp


def run(n):
    obj = m.fused_engine().lbfgs_objective(data["guess"])
    lo, hi = obj.local_box(bounds)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = LB.lbfgsb_minimize(obj, lo, hi, maxiter=n, pgtol=0.0, factr=0.0)
    torch.cuda.synchronize()
    return res, time.perf_counter() - t0


run(2)
for k in stats:
    stats[k] = [] if k == "batchN" else 0
res, dt = run(10)
tc = torch.rand(10_000_000, device="cuda")
torch.cuda.synchronize()
e0 = ev()
for _ in range(5):
    torch.argsort(tc)
e1 = ev()
torch.cuda.synchronize()
print({"iters": res.nit, "nfev": res.nfev, "s_per_iter_ms": 1e3 * dt / res.nit,
       "cauchy_ms_per_iter": stats["cp_ms"] / res.nit, "scan_ms_per_iter": stats["scan_ms"] / res.nit,
       "scans_per_iter": stats["scan_calls"] / res.nit, "batch_sizes": stats["batchN"][:12],
       "argsort_1e7_ms": e0.elapsed_time(e1) / 5})
