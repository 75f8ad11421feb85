"""BASELINE.json configurations 1-5 (one JSON line each).

  1  toy      -- sum-of-squares, 10 params, single-process Adam on CPU
  2  adam1e6  -- population SMF model, 1e6 params, Adam, this node's ranks (1 GPU: config 2)
  3            (same as 2 launched on 8 ranks: config 3)
  4  lbfgs    -- device L-BFGS with all-reduced dot products (ZeRO-sharded on >1 rank)
     lbfgsb   -- the same with every parameter boxed (device L-BFGS-B)
  5  adam1e8  -- 1e8-param model, fused Adam (history="last": a full 1e8 x steps trajectory
               would not be a meaningful benchmark)

    python benchmarks/configs.py --which toy adam1e6 lbfgs
    python -m multigrad_amd.launch -n 8 benchmarks/configs.py --which adam1e6 lbfgs adam1e8
"""
import argparse

import numpy as np
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MULTIGRAD_PROGRESS", "0")


PLACEMENT = "hashed"


def _sync():
    import torch
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def toy(comm, steps):
    import torch
    from multigrad_amd.models.toy import SumOfSquaresModel, make_toy_data
    from multigrad_amd.parallel.comm import SerialComm
    m = SumOfSquaresModel(aux_data=make_toy_data(ndim=10, npoints=1000, comm=SerialComm()),
                          comm=SerialComm())
    m.run_adam(torch.zeros(10), nsteps=5, learning_rate=0.05)
    t0 = time.perf_counter()
    traj = m.run_adam(torch.zeros(10), nsteps=steps, learning_rate=0.05)
    dt = time.perf_counter() - t0
    return {"config": "toy-10param-adam-cpu", "value": steps / dt, "unit": "steps/s",
            "n_ranks": 1, "final_dist_to_mean": float((traj[-1] - torch.as_tensor(m.aux_data["mean"])).abs().max())}


def adam(comm, steps, params, halos, history):
    import torch
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    dev = torch.device("cuda", torch.cuda.current_device())
    data = make_population_data(params, halos, seed=1234, comm=comm, device=dev,
                                placement=PLACEMENT)
    m = PopulationSMFModel(aux_data=data, comm=comm)
    m.set_target_from_truth()
    eng = m.fused_engine()
    eng.setup(data["guess"], nsteps=steps + 3, learning_rate=1e-3, history=history)
    eng.steps(3)
    eng.drain()
    _sync(); comm.barrier(); _sync()
    t0 = time.perf_counter()
    eng.steps(steps)
    eng.drain()
    _sync(); comm.barrier()
    dt = time.perf_counter() - t0
    return {"config": f"adam-{params:.0e}param", "value": steps / dt, "unit": "steps/s",
            "ms_per_step": 1e3 * dt / steps, "n_ranks": comm.size, "halos": halos,
            "history": history, "zero": eng.zero, "chunks": eng.C, "pipelined": eng.pipeline,
            "graph": bool(eng.use_graph), "loss": eng.last_loss()}


def lbfgs(comm, iters, params, halos):
    import torch
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    from multigrad_amd.optim.lbfgs import lbfgs_minimize
    dev = torch.device("cuda", torch.cuda.current_device())
    data = make_population_data(params, halos, seed=1234, comm=comm, device=dev,
                                placement=PLACEMENT)
    m = PopulationSMFModel(aux_data=data, comm=comm)
    m.set_target_from_truth()
    # warm-up run (first kernel launches load code objects), then a fresh objective
    lbfgs_minimize(m.fused_engine().lbfgs_objective(data["guess"]), maxiter=2, gtol=0.0, ftol=0.0)
    obj = m.fused_engine().lbfgs_objective(data["guess"])
    _sync(); comm.barrier()
    t0 = time.perf_counter()
    res = lbfgs_minimize(obj, maxiter=iters, gtol=0.0, ftol=0.0)
    _sync(); comm.barrier()
    dt = time.perf_counter() - t0
    return {"config": f"lbfgs-{params:.0e}param", "value": res.nit / dt, "unit": "iterations/s",
            "fevals_per_s": res.nfev / dt, "n_ranks": comm.size, "nit": int(res.nit),
            "nfev": int(res.nfev), "fun": float(res.fun), "sharded": bool(obj.sharded),
            "reduction": res.get("reduction"), "host_collectives": res.get("host_collectives")}


def lbfgsb(comm, iters, params, halos):
    """Device L-BFGS-B with a box around the starting point (every parameter bounded;
    a fraction active at the solution): Cauchy point + subspace step + projected search."""
    import torch
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    from multigrad_amd.optim.lbfgsb import lbfgsb_minimize
    dev = torch.device("cuda", torch.cuda.current_device())
    data = make_population_data(params, halos, seed=1234, comm=comm, device=dev,
                                placement=PLACEMENT)
    m = PopulationSMFModel(aux_data=data, comm=comm)
    m.set_target_from_truth()
    g = data["guess"].detach().cpu().numpy()
    bounds = np.stack([g - 0.15, g + 0.05], 1)  # (P, 2) array: the truth (g - 0.1) inside

    def prep():
        obj = m.fused_engine().lbfgs_objective(data["guess"])
        return (obj,) + tuple(obj.local_box(bounds))

    obj, lo, hi = prep()
    lbfgsb_minimize(obj, lo, hi, maxiter=2, pgtol=0.0, factr=0.0)  # warm-up (kernel loading)
    obj, lo, hi = prep()
    _sync(); comm.barrier()
    t0 = time.perf_counter()
    res = lbfgsb_minimize(obj, lo, hi, maxiter=iters, pgtol=0.0, factr=0.0)
    _sync(); comm.barrier()
    dt = time.perf_counter() - t0
    return {"config": f"lbfgsb-{params:.0e}param", "value": res.nit / dt, "unit": "iterations/s",
            "fevals_per_s": res.nfev / dt, "n_ranks": comm.size, "nit": int(res.nit),
            "nfev": int(res.nfev), "fun": float(res.fun), "sharded": bool(obj.sharded),
            "reduction": res.get("reduction"), "host_collectives": res.get("host_collectives")}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--which", nargs="+", default=["toy", "adam1e6", "lbfgs"])
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--halos", type=int, default=1 << 27)
    ap.add_argument("--placement", default="hashed", choices=["hashed", "owner"],
                    help="multi-rank data placement: 'hashed' (dense gradient: the data-parallel "
                         "RCCL configs 3-5) or 'owner' (population-owner shards)")
    args = ap.parse_args(argv)
    global PLACEMENT
    PLACEMENT = args.placement
    import torch
    import multigrad_amd as mg
    comm = mg.init_distributed() if int(os.environ.get("WORLD_SIZE", "1")) > 1 else mg.get_world_comm()
    if torch.cuda.is_available():
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    out = []
    for w in args.which:
        if w == "toy":
            r = toy(comm, 200) if comm.rank == 0 else None
        elif w == "adam1e6":
            r = adam(comm, args.steps, 1_000_000, args.halos, "full")
        elif w == "adam1e7":
            r = adam(comm, args.steps, 10_000_000, args.halos, "full")
        elif w == "adam1e8":
            r = adam(comm, args.steps, 100_000_000, args.halos * 4, "last")
        elif w == "lbfgs":
            r = lbfgs(comm, 20, 10_000_000, args.halos)
        elif w == "lbfgsb":
            r = lbfgsb(comm, 20, 10_000_000, args.halos)
        else:
            raise SystemExit(f"unknown config {w}")
        if comm.rank == 0 and r is not None:
            print(json.dumps(r), flush=True)
            out.append(r)


if __name__ == "__main__":
    main()
