import os, sys, torch
sys.path.insert(0, os.getcwd())
from multigrad_amd.engine.generic import GraphAdamEngine
from multigrad_amd.models.population import PopulationSMFModel, make_population_data
from multigrad_amd.models.torch_population import StochasticTorchPopulationSMFModel, torch_population_data
dev = torch.device("cuda", 0)
data = make_population_data(20000, 400000, seed=5, device=dev)
PopulationSMFModel(aux_data=data).set_target_from_truth()
g = data["guess"]
m = StochasticTorchPopulationSMFModel(aux_data=torch_population_data(data))
rec = {}
def mk(name, sync):
    def cb(i, loss, state):
        if sync: torch.cuda.synchronize()
        rec.setdefault(name, []).append((float(torch.as_tensor(loss).reshape(-1)[0]), state.m[:40000].clone()))
    return cb
m.run_adam(g, nsteps=4, learning_rate=1e-3, use_engine=False, randkey=7, callback=mk("eager", False))
for s in (False, True):
    GraphAdamEngine(m, graph=True).run_adam(g, nsteps=4, learning_rate=1e-3, randkey=7, callback=mk(f"graph_sync{s}", s))
for name in rec:
    if name == "eager": continue
    print(name, [(round(a[0]-b[0], 9), float((a[1]-b[1]).abs().max())) for a, b in zip(rec[name], rec["eager"])], flush=True)
