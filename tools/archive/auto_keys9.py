import os, sys, torch
sys.path.insert(0, os.getcwd())
import multigrad_amd.engine.generic as G
from multigrad_amd.engine.generic import GraphAdamEngine
from multigrad_amd.models.population import PopulationSMFModel, make_population_data
from multigrad_amd.models.torch_population import StochasticTorchPopulationSMFModel, torch_population_data
dev = torch.device("cuda", 0)
data = make_population_data(20000, 400000, seed=5, device=dev)
PopulationSMFModel(aux_data=data).set_target_from_truth()
g = data["guess"]
K = 6
rec = {"S": torch.zeros(K, 10, device=dev), "g": torch.zeros(K, 20000, device=dev), "x": torch.zeros(K, 64, device=dev)}
class M(StochasticTorchPopulationSMFModel):
    def calc_partial_sumstats_from_params(self, params, randkey=None):
        x = self.aux_data["x"]
        n = torch.randn(x.shape, generator=randkey.generator(x.device), device=x.device, dtype=x.dtype)
        xs = x + self.scatter * n
        S = self._sumstats(params, xs)
        i = self._eng.step_dev[:1].long() if hasattr(self._eng, 'step_dev') else torch.zeros(1, dtype=torch.long, device=x.device)
        rec["x"].index_copy_(0, i, xs[:64].reshape(1, 64))
        rec["S"].index_copy_(0, i, S.detach().reshape(1, 10))
        return S
m = M(aux_data=torch_population_data(data))
# grad recording: wrap the engine's adam step input
orig = G.adam_step_
def spy(u, mm, v, grad, *a, **k):
    rec["g"].index_copy_(0, m._eng.step_dev[:1].long(), grad.reshape(1, -1))
    return orig(u, mm, v, grad, *a, **k)
G.adam_step_ = spy
def cb(i, loss, state): torch.cuda.synchronize()
res = {}
for name, c in (("nosync", None), ("sync", cb)):
    for t in rec.values(): t.zero_()
    eng = GraphAdamEngine(m, graph=True)
    m._eng = eng
    eng.run_adam(g, nsteps=K, learning_rate=1e-3, randkey=7, callback=c)
    torch.cuda.synchronize()
    res[name] = {k: v.clone() for k, v in rec.items()}
for k in ("x", "S", "g"):
    print(k, "per-step maxdiff sync vs nosync:", ["%.1e" % float((res["sync"][k][i] - res["nosync"][k][i]).abs().max()) for i in range(K)], flush=True)
