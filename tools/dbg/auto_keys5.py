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
def cb(i, loss, state): torch.cuda.synchronize()
runs = {}
for name, fn in (("eager", lambda c: m.run_adam(g, nsteps=6, learning_rate=1e-3, randkey=7, use_engine=False, callback=c)),
                 ("graph", lambda c: GraphAdamEngine(m, graph=True).run_adam(g, nsteps=6, learning_rate=1e-3, randkey=7, callback=c))):
    for sync in (False, True, False, True):
        runs.setdefault(name, []).append(fn(cb if sync else None))
base = runs["eager"][0]
for name, ts in runs.items():
    print(name, ["%.1e" % float((t - base).abs().max()) for t in ts], flush=True)
