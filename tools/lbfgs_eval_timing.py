"""Where a device L-BFGS evaluation's wall time goes at 1e7 parameters (one GPU): the
same evaluation sequence the line search issues (x + a d, engine device_call, the g.d dot,
one reduction copy), timed (a) with the per-evaluation host copy the line search needs,
(b) launched back to back with one sync at the end (GPU-bound time), and (c) host issue
time alone.  The difference (a) - (b) is the GPU idle time a synchronous line search pays
per evaluation."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MULTIGRAD_AUTOTUNE", "off")


def main():
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    from multigrad_amd.optim._reduce import DeviceReducer
    from multigrad_amd.ops.lbfgs import MultiDot
    dev = torch.device("cuda", 0)
    data = make_population_data(10_000_000, 1 << 27, seed=1234, device=dev)
    m = PopulationSMFModel(aux_data=data)
    m.set_target_from_truth()
    obj = m.fused_engine().lbfgs_objective(data["guess"])
    x = obj.x0().contiguous()
    d = torch.randn_like(x) * 1e-4
    xt = torch.empty_like(x)
    red = DeviceReducer(obj.comm, obj.sharded, dev)
    dot1 = MultiDot(1, x.numel(), dev)

    def one(sync: bool):
        torch.add(x, d, alpha=0.5, out=xt)
        lt, ga = obj.device_call(xt)
        ga = ga.clone()
        if sync:
            red.reduce(sums=[dot1(ga.view(1, -1), 1, [d])], local=[lt.reshape(1)])
        else:
            dot1(ga.view(1, -1), 1, [d])

    for _ in range(5):
        one(True)
    torch.cuda.synchronize()
    n = 40
    t0 = time.perf_counter()
    for _ in range(n):
        one(True)
    torch.cuda.synchronize()
    t_sync = (time.perf_counter() - t0) / n
    t0 = time.perf_counter()
    for _ in range(n):
        one(False)
    t_issue = (time.perf_counter() - t0) / n
    torch.cuda.synchronize()
    t_async = (time.perf_counter() - t0) / n
    rec = {"eval_ms_with_copy": round(1e3 * t_sync, 4), "eval_ms_back_to_back": round(1e3 * t_async, 4),
           "host_issue_ms": round(1e3 * t_issue, 4),
           "idle_ms_per_eval": round(1e3 * (t_sync - t_async), 4)}
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
