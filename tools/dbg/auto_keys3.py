import os, sys, torch
sys.path.insert(0, os.getcwd())
from multigrad_amd.engine.generic import GraphAdamEngine
from multigrad_amd.models.population import PopulationSMFModel, make_population_data
from multigrad_amd.models.torch_population import StochasticTorchPopulationSMFModel, TorchPopulationSMFModel, torch_population_data
dev = torch.device("cuda", 0)
data = make_population_data(20000, 400000, seed=5, device=dev)
PopulationSMFModel(aux_data=data).set_target_from_truth()
g = data["guess"]
def cb(i, loss, state):
    torch.cuda.synchronize()
def cb_nosync(i, loss, state):
    pass
for cls, kw in ((TorchPopulationSMFModel, {}), (StochasticTorchPopulationSMFModel, {"randkey": 7})):
    m = cls(aux_data=torch_population_data(data))
    ref = m.run_adam(g, nsteps=6, learning_rate=1e-3, use_engine=False, **kw)
    for c in (None, cb_nosync, cb):
        eng = GraphAdamEngine(m, graph=True)
        t = eng.run_adam(g, nsteps=6, learning_rate=1e-3, callback=c, **kw)
        d = (t - ref).abs().amax(1)
        print(cls.__name__[:10], "cb", None if c is None else c.__name__, [f"{x:.1e}" for x in d.tolist()], flush=True)
