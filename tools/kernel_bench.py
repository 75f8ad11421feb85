"""Micro-benchmark of the SMF forward / VJP kernels and fused Adam (one process, events).

Usage: python tools/kernel_bench.py [--so path/to/_C.so] [--halos N] [--params P]
"""
import argparse
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--so", default=None)
    ap.add_argument("--halos", type=int, default=1 << 27)
    ap.add_argument("--params", type=int, default=10_000_000)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tag", default="")
    ap.add_argument("--tail", default="absolute", choices=["relative", "absolute"])
    ap.add_argument("--layout", default="lanes", choices=["lanes", "tiles"])
    a = ap.parse_args()
    import torch
    if a.so:
        spec = importlib.util.spec_from_file_location("multigrad_amd._C", a.so)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        sys.modules["multigrad_amd._C"] = mod
    from multigrad_amd.models.population import make_population_data, PopulationSMFModel
    from multigrad_amd.ops import smf as S
    from multigrad_amd.ops.adam import fused_adam_
    dev = torch.device("cuda", 0)
    data = make_population_data(a.params, a.halos, seed=1, device=dev, tail=a.tail,
                                layout=a.layout)
    model = PopulationSMFModel(aux_data=data)
    model.set_target_from_truth()
    shard, bins = data["shard"], data["bins"]
    th = data["guess"]
    out = torch.zeros(bins.nbp, device=dev)
    nblk = shard.fwd_rows(shard.n, bins.nb, True, bins.rel_tail, resid=True)
    slab = torch.zeros(nblk * bins.nbp, device=dev)
    h = torch.zeros(bins.nbp + 1, device=dev)
    loss = torch.zeros(1, device=dev)
    grad = torch.zeros_like(th)
    m = torch.zeros_like(th); v = torch.zeros_like(th); u = th.clone()
    step = torch.zeros(2, dtype=torch.int32, device=dev)

    def timeit(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.iters

    # as in the engine step: the forward keeps the VJP residuals (lanes layout)
    t_fwd = timeit(lambda: S.smf_forward_into(th, shard, bins, True, out, slab=slab, resid=True))
    t_fwd_nores = timeit(lambda: S.smf_forward_into(th, shard, bins, True, out, slab=slab))
    model.engine_loss_into(out, loss, h)
    S.smf_forward_into(th, shard, bins, True, out, slab=slab, resid=True)
    t_vjp = timeit(lambda: S.smf_vjp_into(th, shard, bins, True, h, grad, residuals_ready=True))
    t_vjp_int = t_fwd_int = None
    if shard.layout == "lanes":  # the engine's internal (slot) parameter order
        thi = th.reshape(-1, 2)[shard.perm].reshape(-1).contiguous()
        S.smf_forward_into(thi, shard, bins, True, out, slab=slab, resid=True, order="internal")
        t_fwd_int = round(timeit(lambda: S.smf_forward_into(thi, shard, bins, True, out, slab=slab,
                                                            resid=True, order="internal")), 1)
        t_vjp_int = round(timeit(lambda: S.smf_vjp_into(thi, shard, bins, True, h, grad,
                                                        residuals_ready=True,
                                                        order="internal")), 1)
    t_adam = timeit(lambda: fused_adam_(u, m, v, grad, None, step, 1e-3, 0.9, 0.999, 1e-8))
    res = {"tag": a.tag, "halos": shard.n, "params": th.numel(), "layout": shard.layout,
           "fwd_us": round(t_fwd, 1), "fwd_noresid_us": round(t_fwd_nores, 1),
           "vjp_us": round(t_vjp, 1), "vjp_internal_us": t_vjp_int, "fwd_internal_us": t_fwd_int, "adam_us": round(t_adam, 1), "fwd_blocks": nblk,
           "ntiles": int(shard.tiles.shape[0]) if shard.layout == "tiles" else shard.ngroups,
           "fwd_Ghalo_s": round(shard.n / t_fwd / 1e3, 2), "vjp_Ghalo_s": round(shard.n / t_vjp / 1e3, 2),
           "S": [float(f"{v:.7e}") for v in out[:bins.nb].tolist()],
           "grad_l1": float(f"{grad.double().abs().sum().item():.9e}")}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
