"""Eager launches vs one-step graph replays vs replays of blocks of K unrolled steps, one
process on one MI355X (one same-box table for every engine).

Rows: the fused engine's 1-GPU headline step (1e7 parameters, 1.34e8 halos), the per-rank
proxy of the 8-GPU owner step (1/8 of both), the generic engine on the plain-torch
population model (small: launch bound; large: GPU bound), and ingraph.simple_grad_descent
(the reference's mpi4jax lax.scan variant, multigrad/mpi4jax/multigrad.py:57-58).  Each
(row, mode) runs ``--warm`` untimed steps, then ``--steps`` timed steps between two
synchronisations, ``--repeats`` times alternating the modes; the table reports the median
ms/step.  Usage: python benchmarks/graph_modes.py [--steps 200] [--K 16]
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MULTIGRAD_PROGRESS", "0")
os.environ["MULTIGRAD_AUTOTUNE"] = "0"   # the mode is pinned per run, not tuned


def fused_row(params, halos, steps, warm, K, mode):
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    key = (params, halos)
    if key not in _CACHE:
        data = make_population_data(params, halos, seed=1234, device=torch.device("cuda", 0))
        model = PopulationSMFModel(aux_data=data)
        model.set_target_from_truth()
        _CACHE[key] = (data, model)
    data, model = _CACHE[key]
    eng = FusedAdamEngine(model, graph=not mode.startswith("eager"))
    eng.device_step = mode == "eager-dev"
    eng.graph_steps = K if mode == "graph-K" else 1
    eng.setup(data["guess"], warm + steps + 1, learning_rate=1e-3)
    eng.steps(warm)
    eng.drain()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.steps(steps)
    eng.drain()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    assert eng.use_graph == (not mode.startswith("eager"))
    eng.close()
    return dt


def generic_row(params, halos, steps, warm, K, mode):
    from multigrad_amd.engine.generic import GraphAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    from multigrad_amd.models.torch_population import TorchPopulationSMFModel, torch_population_data
    key = ("g", params, halos)
    if key not in _CACHE:
        data = make_population_data(params, halos, seed=5, device=torch.device("cuda", 0))
        PopulationSMFModel(aux_data=data).set_target_from_truth()
        _CACHE[key] = (TorchPopulationSMFModel(aux_data=torch_population_data(data)), data["guess"])
    m, guess = _CACHE[key]
    eng = GraphAdamEngine(m, graph=not mode.startswith("eager"))
    eng.graph_steps = K if mode == "graph-K" else 1
    eng.setup(guess, warm + steps, learning_rate=1e-3)
    eng.steps(warm)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.steps(steps)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    eng.close()
    return dt


def ingraph_row(params, halos, steps, warm, K, mode):
    from multigrad_amd import ingraph
    g = torch.Generator().manual_seed(3)
    x = torch.randn(halos, generator=g).cuda()

    def loss_and_grad(d, p):
        r = d["x"][:, None] - p[None, :]
        return 0.5 * (r * r).mean(), -r.mean(0)

    guess = torch.zeros(params, device="cuda")
    kw = dict(graph=not mode.startswith("eager"), block=K if mode == "graph-K" else 1)
    ingraph.simple_grad_descent(dict(x=x), loss_and_grad, guess, 0.1, nsteps=warm, **kw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ingraph.simple_grad_descent(dict(x=x), loss_and_grad, guess, 0.1, nsteps=steps, **kw)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps   # includes the capture and the host copy


_CACHE = {}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warm", type=int, default=40)
    ap.add_argument("--K", type=int, default=16)
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--modes", default="eager,graph-1,graph-K",
                    help="eager, eager-dev (fused rows: eager launches on the device step "
                         "counter), graph-1, graph-K")
    ap.add_argument("--rows", default="fused,owner_proxy,generic_small,generic_large,ingraph")
    a = ap.parse_args(argv)
    rows = {
        "fused": (fused_row, 10_000_000, 1 << 27),
        "owner_proxy": (fused_row, 1_250_000, 1 << 24),
        "generic_small": (generic_row, 2_000, 40_000),
        "generic_large": (generic_row, 200_000, 4_000_000),
        "ingraph": (ingraph_row, 3, 20_000),
    }
    modes = tuple(a.modes.split(","))
    res = {}
    for name in a.rows.split(","):
        fn, params, halos = rows[name]
        times = {m: [] for m in modes}
        for _ in range(a.repeats):
            for mode in modes:
                times[mode].append(1e3 * fn(params, halos, a.steps, a.warm, a.K, mode))
        res[name] = {m: round(statistics.median(v), 4) for m, v in times.items()}
        res[name]["all_ms"] = {m: [round(t, 4) for t in v] for m, v in times.items()}
        print(json.dumps({name: res[name]}), flush=True)
    print("| row | " + " | ".join(f"{m} ms/step" for m in modes) + " | K-step / eager |")
    print("|---" * (len(modes) + 2) + "|")
    for name, r in res.items():
        ratio = (f"{r['eager'] / r['graph-K']:.3f}x" if "eager" in r and "graph-K" in r else "-")
        print(f"| {name} | " + " | ".join(f"{r[m]:.4f}" for m in modes) + f" | {ratio} |")

if __name__ == "__main__":
    main()
