"""Host time per eager engine step: how long ``engine.step()`` takes to ENQUEUE its launches
(timed without synchronising, while the GPU works through the queue), against the GPU time
per step.  A host cost near the GPU time would starve the GPU on small per-rank shards.
Usage (one GPU): python tools/host_step_cost.py [--params 1250000 --halos 16777216]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MULTIGRAD_PROGRESS", "0")
os.environ["MULTIGRAD_AUTOTUNE"] = "0"

from multigrad_amd.engine.fused import FusedAdamEngine  # noqa: E402
from multigrad_amd.models.population import PopulationSMFModel, make_population_data  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--params", type=int, default=1_250_000)
ap.add_argument("--halos", type=int, default=1 << 24)
ap.add_argument("--steps", type=int, default=200)
a = ap.parse_args()
data = make_population_data(a.params, a.halos, seed=1234, device=torch.device("cuda", 0))
model = PopulationSMFModel(aux_data=data)
model.set_target_from_truth()
eng = FusedAdamEngine(model, graph=False)
eng.setup(data["guess"], 3 * a.steps + 10, learning_rate=1e-3)
eng.steps(10)
eng.drain()
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.step()
    t1 = time.perf_counter()
    eng.drain()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host enqueue {1e6 * (t1 - t0) / a.steps:.1f} us/step, wall {1e6 * (t2 - t0) / a.steps:.1f} us/step",
          flush=True)
