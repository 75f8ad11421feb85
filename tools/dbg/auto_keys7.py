import os, sys, torch
sys.path.insert(0, os.getcwd())
from multigrad_amd.engine.generic import GraphAdamEngine
from multigrad_amd.models.population import PopulationSMFModel, make_population_data
from multigrad_amd.models.torch_population import StochasticTorchPopulationSMFModel, torch_population_data
dev = torch.device("cuda", 0)
data = make_population_data(20000, 400000, seed=5, device=dev)
PopulationSMFModel(aux_data=data).set_target_from_truth()
g = data["guess"]
m = StochasticTorchPopulationSMFModel(aux_data=torch_population_data(data), scatter=0.0)
for sync in (False, True):
    eng = GraphAdamEngine(m, graph=True)
    eng.mode = "adam"
    eng.setup(g, 6, learning_rate=1e-3, randkey=7)
    steps = []
    for i in range(6):
        eng.step()
        if sync: torch.cuda.synchronize()
        steps.append(eng.step_dev.clone())
    torch.cuda.synchronize()
    gen = eng._gens[0] if eng._gens else None
    print("sync", sync, "step_dev after each step", [s.tolist() for s in steps], flush=True)
    print("   m sum", float(eng.m.double().abs().sum()), "v sum", float(eng.v.double().abs().sum()), flush=True)
    eng.close()
