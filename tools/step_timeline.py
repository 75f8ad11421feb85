"""Per-step GPU time of the headline engine step (CUDA events around every step), to see
where the fixed cost of a short timed window goes: python tools/step_timeline.py [steps]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from multigrad_amd.models.population import PopulationSMFModel, make_population_data  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 30
data = make_population_data(10_000_000, 1 << 27, seed=1234, device=torch.device("cuda", 0))
model = PopulationSMFModel(aux_data=data)
model.set_target_from_truth()
eng = model.fused_engine()
eng.setup(data["guess"], nsteps=5 + K + 1, learning_rate=1e-3)
for _ in range(5):
    eng.step()
eng.last_loss()
torch.cuda.synchronize()
evs = [torch.cuda.Event(enable_timing=True) for _ in range(K + 2)]
t0 = time.perf_counter()
evs[0].record()
for i in range(K):
    eng.step()
    evs[i + 1].record()
eng.drain()
evs[K + 1].record()
torch.cuda.synchronize()
wall = time.perf_counter() - t0
ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(K + 1)]
print("per-step ms:", " ".join(f"{v:.3f}" for v in ms[:K]))
print(f"drain ms: {ms[K]:.3f}  sum {sum(ms):.3f}  wall {1e3 * wall:.3f}")
