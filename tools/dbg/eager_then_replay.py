"""Generic engine: graph replays that FOLLOW eager steps (e.g. an auto-policy order eager /
replay / eager / replay).  Prints, per schedule and replay stream, the largest trajectory
deviation from the eager reference, with and without a host synchronisation after each
step.  Usage (one GPU): python tools/dbg/eager_then_replay.py"""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from multigrad_amd.engine.generic import GraphAdamEngine  # noqa: E402
from multigrad_amd.models.population import PopulationSMFModel, make_population_data  # noqa: E402
from multigrad_amd.models.torch_population import (TorchPopulationSMFModel,  # noqa: E402
                                                   torch_population_data)

dev = torch.device("cuda", 0)
data = make_population_data(20000, 400000, seed=5, device=dev)
PopulationSMFModel(aux_data=data).set_target_from_truth()
g = data["guess"]
m = TorchPopulationSMFModel(aux_data=torch_population_data(data))
N = 20
ref = m.run_adam(g, nsteps=N, learning_rate=1e-3, use_engine=False)


def run(schedule, side, sync):
    eng = GraphAdamEngine(m, graph=True)
    eng.setup(g, nsteps=N, learning_rate=1e-3)
    prev = None
    for k, mode in enumerate(schedule):
        if mode == "g":
            if eng.graph is None or prev == "e":
                eng.step_dev[0] = k
            if eng.graph is None:
                eng.graph = eng._capture()
            if side:
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    eng.graph.replay()
                torch.cuda.current_stream().wait_stream(s)
            else:
                eng.graph.replay()
        else:
            eng._body(k, None)
        eng.step_host += 1
        if sync:
            torch.cuda.synchronize()
        prev = mode
    t = eng.trajectory()
    d = (t - ref).abs().amax(dim=1)
    bad = [i for i in range(d.numel()) if float(d[i]) > 1e-5]
    return "%.1e first_bad_row=%s" % (float(d.max()), bad[0] if bad else None)


for sched in ("eeeeeggggggggggggggg", "eeeeeggggggeeeeegggg", "eeeeeggggggeeeeeeeee"):
    for side in (False, True):
        for sync in (False, True):
            print(sched, "side" if side else "default", "sync" if sync else "nosync",
                  run(sched, side, sync), flush=True)
