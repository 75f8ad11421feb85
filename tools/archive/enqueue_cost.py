"""Host-side enqueue cost of one eager engine step (no HIP graph) vs its GPU time, at the
per-rank proxy size of the 8-GPU owner run.  Usage: python tools/enqueue_cost.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MULTIGRAD_PROGRESS", "0")


def main():
    import torch
    from multigrad_amd.engine.fused import FusedAdamEngine
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    dev = torch.device("cuda", 0)
    data = make_population_data(1_250_000, 1 << 24, seed=1234, device=dev)
    m = PopulationSMFModel(aux_data=data)
    m.set_target_from_truth()
    eng = FusedAdamEngine(m, graph=False, owner=True)
    n = 300
    eng.setup(data["guess"], nsteps=n + 20, learning_rate=1e-3)
    for _ in range(10):
        eng.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        eng.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"enqueue {1e6 * (t1 - t0) / n:.1f} us/step, wall {1e6 * (t2 - t0) / n:.1f} us/step")


if __name__ == "__main__":
    main()
