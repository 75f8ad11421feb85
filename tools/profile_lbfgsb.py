"""cProfile of the device L-BFGS-B at 1e7 parameters (one GPU): where an iteration goes."""
import cProfile
import pstats
import sys
import time

import torch

sys.path.insert(0, ".")
from multigrad_amd.models.population import PopulationSMFModel, make_population_data  # noqa: E402
from multigrad_amd.optim.lbfgsb import lbfgsb_minimize  # noqa: E402

data = make_population_data(10_000_000, 1 << 27, seed=1234, device=torch.device("cuda", 0))
m = PopulationSMFModel(aux_data=data)
m.set_target_from_truth()
g = data["guess"].detach().cpu().numpy()
bounds = __import__("numpy").stack([g - 0.15, g + 0.05], 1)


def run(n):
    obj = m.fused_engine().lbfgs_objective(data["guess"])
    lo, hi = obj.local_box(bounds)
    return lbfgsb_minimize(obj, lo, hi, maxiter=n, pgtol=0.0, factr=0.0)


run(2)
torch.cuda.synchronize()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
res = run(6)
torch.cuda.synchronize()
pr.disable()
print("iterations", res.nit, "nfev", res.nfev, "s", time.perf_counter() - t0, res.message)
pstats.Stats(pr).sort_stats("cumulative").print_stats(30)
