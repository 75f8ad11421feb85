"""Generic engine: graph replays that FOLLOW eager steps (an order eager / replay / eager /
replay), through the engine's public API (``use_graph`` switched between ``step()`` calls).
Prints, per schedule, the largest trajectory deviation from the eager reference, with and
without a host synchronisation after each step, and with a user kernel between the steps
issued inside ``engine.stream()``.  Every line should read 0.0e+00.

The last section shows the one schedule the engine cannot protect: user work launched on
the legacy DEFAULT stream between direct ``step()`` calls, with host synchronisations
(the HIP runtime defect of tools/dbg/torch_replay_bisect.py, case user_null; see
docs/design.md "Graph replays and the default stream").
Usage (one GPU): python tools/dbg/eager_then_replay.py"""
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
scratch = torch.zeros(1, device=dev)


def run(schedule, sync, user=None, replay=True):
    eng = GraphAdamEngine(m, graph=True)
    eng.setup(g, nsteps=N, learning_rate=1e-3)
    eng.step_replay = replay
    for mode in schedule:
        eng.use_graph = mode == "g"
        eng.step()
        if user == "engine_stream":
            with eng.stream():
                scratch.add_(1)
        elif user == "default_stream":
            scratch.add_(1)
        if sync:
            torch.cuda.synchronize()
    t = eng.trajectory()
    torch.cuda.synchronize()
    d = (t - ref).abs().amax(dim=1)
    bad = [i for i in range(d.numel()) if not float(d[i]) <= 1e-5]
    return "%.1e first_bad_row=%s" % (float(d.max()), bad[0] if bad else None)


for sched in ("eeeeeggggggggggggggg", "eeeeeggggggeeeeegggg", "eeeeeggggggeeeeeeeee",
              "gggggggggggggggggggg"):
    for sync in (False, True):
        for user in (None, "engine_stream"):
            print(sched, "sync" if sync else "nosync", user or "-", run(sched, sync, user),
                  flush=True)
print("-- user kernels on the default stream between direct step() calls:")
for sched in ("eeeeeggggggeeeeegggg", "gggggggggggggggggggg"):
    # default (round 5): direct step() calls launch eagerly -> exact
    print(sched, "sync default_stream", run(sched, True, "default_stream", replay=False),
          flush=True)
    # opting in to replays of direct calls (step_replay) exposes the runtime defect
    print(sched, "sync default_stream step_replay", run(sched, True, "default_stream"),
          flush=True)
