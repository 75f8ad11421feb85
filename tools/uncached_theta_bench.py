"""Cost of reading the parameters from (and writing the gradient to) the two-shot exchange's
uncached peer-memory regions, measured on one GPU.

In the hashed multi-rank engine the forward and the VJP work directly on the two-shot
buffers (``TwoShot.theta`` / ``TwoShot.grad``, allocated ``hipDeviceMallocUncached``), so
every per-halo parameter gather bypasses L2.  This times the per-rank kernels of the hashed
8-GPU step (1e7 parameters, 1/8 of the 1.34e8 halos, tiles layout) with cached buffers and
with uncached ones.  Usage: python tools/uncached_theta_bench.py [--halos N] [--iters K]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from multigrad_amd.models.population import PopulationSMFModel, make_population_data  # noqa: E402
from multigrad_amd.ops._ext import ext  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return 1e3 * a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=10_000_000)
    ap.add_argument("--halos", type=int, default=(1 << 27) // 8)
    ap.add_argument("--layout", default="tiles")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    data = make_population_data(args.params, args.halos, seed=1234, device=dev,
                                layout=args.layout)
    md = PopulationSMFModel(aux_data=data)
    md.set_target_from_truth()
    eng = md.fused_engine(graph=False)
    eng.setup(data["guess"], nsteps=4, learning_rate=1e-3)
    eng.step()
    eng.drain()
    torch.cuda.synchronize()
    E = ext()
    n = eng.theta.numel()
    regions = [E.xgmi_alloc(4 * n), E.xgmi_alloc(4 * n)]
    th_uc = E.xgmi_tensor(regions[0], n)
    gr_uc = E.xgmi_tensor(regions[1], n)
    th_uc.copy_(eng.theta)
    gr_c = torch.zeros_like(eng.theta)
    slab, h = eng.slab, eng.h
    out = {}
    for name, th, gr in (("cached", eng.theta, gr_c), ("uncached", th_uc, gr_uc),
                         ("cached", eng.theta, gr_c), ("uncached", th_uc, gr_uc)):
        fwd = timeit(lambda: md.engine_forward_chunk(th, slab, None), args.iters)
        vjp = timeit(lambda: md.engine_vjp_into(th, h, gr, None), args.iters)
        copy = timeit(lambda: eng.theta.copy_(th_uc), args.iters)
        out.setdefault(name, []).append({"forward_us": round(fwd, 1), "vjp_us": round(vjp, 1),
                                         "copy_from_uncached_us": round(copy, 1)})
    torch.cuda.synchronize()
    assert torch.equal(gr_c, gr_uc), "uncached gradient differs"
    print(json.dumps({"params": args.params, "halos": args.halos, "layout": args.layout,
                      "results": out}), flush=True)
    del th_uc, gr_uc
    torch.cuda.synchronize()
    for r in regions:
        E.xgmi_free(r)


if __name__ == "__main__":
    main()
