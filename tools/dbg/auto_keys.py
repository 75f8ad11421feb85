import os, sys, torch
sys.path.insert(0, os.getcwd())
from multigrad_amd.engine.generic import GraphAdamEngine
from multigrad_amd.models.population import PopulationSMFModel, make_population_data
from multigrad_amd.models.torch_population import StochasticTorchPopulationSMFModel, torch_population_data
dev = torch.device("cuda", 0)
data = make_population_data(20000, 400000, seed=5, device=dev)
PopulationSMFModel(aux_data=data).set_target_from_truth()
m = StochasticTorchPopulationSMFModel(aux_data=torch_population_data(data))
g = data["guess"]
ref = m.run_adam(g, nsteps=10, learning_rate=1e-3, randkey=7, use_engine=False)
def sync_cb(i, loss, state):
    torch.cuda.synchronize()
for gr, cb in ((True, None), (True, sync_cb), (None, None), (None, sync_cb)):
    eng = GraphAdamEngine(m, graph=gr)
    t = eng.run_adam(g, nsteps=10, learning_rate=1e-3, randkey=7, callback=cb)
    d = (t - ref).abs().amax(1)
    print("graph_req", gr, "sync", cb is not None, "tuning", eng.tuning is not None, "rows", [f"{x:.1e}" for x in d.tolist()], flush=True)
