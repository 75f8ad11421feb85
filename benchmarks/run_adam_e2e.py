"""End-to-end wall time of ``model.run_adam(guess, nsteps)`` on the headline model, first
and repeated calls, against the engine's steady step time.

The first call sets the engine up (layout, peer memory, budgeted autotune: at most
MULTIGRAD_TUNE_BUDGET = 10 % of the run's estimated time); repeated calls re-use the model's
cached engine (no trial steps, no captures).  Prints one JSON line.

    python benchmarks/run_adam_e2e.py [--params 1e7] [--halos 2**27] [--nsteps 100]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MULTIGRAD_PROGRESS", "0")


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--params", type=int, default=10_000_000)
    ap.add_argument("--halos", type=int, default=1 << 27)
    ap.add_argument("--nsteps", type=int, default=100)
    ap.add_argument("--calls", type=int, default=3)
    ap.add_argument("--history", default="full")
    a = ap.parse_args(argv)
    import torch
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    dev = torch.device("cuda", 0)
    data = make_population_data(a.params, a.halos, seed=1234, device=dev)
    model = PopulationSMFModel(aux_data=data)
    model.set_target_from_truth()
    torch.cuda.synchronize()
    calls = []
    for i in range(a.calls):
        t0 = time.perf_counter()
        traj = model.run_adam(data["guess"], nsteps=a.nsteps, learning_rate=1e-3,
                              history=a.history)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        eng = model.fused_engine()
        calls.append({"call": i + 1, "wall_s": round(dt, 5), "stats": dict(eng.stats),
                      "tuning": {k: v for k, v in (eng.tuning or {}).items()
                                 if k in ("chosen", "budget_skipped", "cached", "budget_ms",
                                          "step_ms_probe")}})
        del traj
    # steady step time on the same engine: a long timed block after a warm block
    eng = model.fused_engine()
    eng.setup(data["guess"], 2200, learning_rate=1e-3, history="last")
    eng.steps(200)
    eng.drain()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.steps(2000)
    eng.drain()
    torch.cuda.synchronize()
    step_s = (time.perf_counter() - t0) / 2000
    ideal = a.nsteps * step_s
    rec = {"metric": "run_adam end-to-end wall time", "nsteps": a.nsteps, "params": a.params,
           "halos": a.halos, "history": a.history, "step_ms": round(1e3 * step_s, 4),
           "ideal_s": round(ideal, 5), "calls": calls,
           "ratio_first": round(calls[0]["wall_s"] / ideal, 3),
           "ratio_repeat": [round(c["wall_s"] / ideal, 3) for c in calls[1:]]}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
