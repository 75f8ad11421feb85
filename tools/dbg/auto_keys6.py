import os, sys, torch
sys.path.insert(0, os.getcwd())
from multigrad_amd.engine.generic import GraphAdamEngine
from multigrad_amd.models.population import PopulationSMFModel, make_population_data
from multigrad_amd.models.torch_population import StochasticTorchPopulationSMFModel, torch_population_data
dev = torch.device("cuda", 0)
data = make_population_data(20000, 400000, seed=5, device=dev)
PopulationSMFModel(aux_data=data).set_target_from_truth()
g = data["guess"]
def cb(i, loss, state): torch.cuda.synchronize()
for scatter in (0.02, 0.0):
    m = StochasticTorchPopulationSMFModel(aux_data=torch_population_data(data), scatter=scatter)
    for const in (False, True):
        ref = m.run_adam(g, nsteps=6, learning_rate=1e-3, randkey=7, const_randkey=const, use_engine=False)
        out = []
        for c in (None, cb):
            t = GraphAdamEngine(m, graph=True).run_adam(g, nsteps=6, learning_rate=1e-3, randkey=7, const_randkey=const, callback=c)
            out.append("%.1e" % float((t - ref).abs().max()))
        print("scatter", scatter, "const", const, "nosync/sync diffs", out, flush=True)
