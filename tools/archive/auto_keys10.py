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
m = StochasticTorchPopulationSMFModel(aux_data=torch_population_data(data))
ref = m.run_adam(g, nsteps=6, learning_rate=1e-3, randkey=7, use_engine=False)
for mode in ("", "side", "pre_sync"):
    os.environ["MULTIGRAD_DBG_REPLAY"] = mode
    out = []
    for c in (None, cb):
        t = GraphAdamEngine(m, graph=True).run_adam(g, nsteps=6, learning_rate=1e-3, randkey=7, callback=c)
        out.append("%.1e" % float((t - ref).abs().max()))
    print("replay mode", repr(mode), "[nosync, sync]", out, flush=True)
