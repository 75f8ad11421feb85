import os, torch, numpy as np
os.environ["MULTIGRAD_AUTOTUNE"]="0"; os.environ["MULTIGRAD_PIPELINE"]="1"
from multigrad_amd.engine.fused import FusedAdamEngine
from multigrad_amd.models.population import PopulationSMFModel, make_population_data
from multigrad_amd.ops import smf as S
DEV="cuda"
import sys
npar=int(sys.argv[1]) if len(sys.argv)>1 else 10_000_000
nh=int(sys.argv[2]) if len(sys.argv)>2 else 1<<27
data = make_population_data(num_params=npar, num_halos=nh, seed=1234, device=DEV)
model = PopulationSMFModel(aux_data=data); model.set_target_from_truth()
shard, bins = data["shard"], data["bins"]
def oracle(th64):
    tot = torch.zeros(bins.nb, dtype=torch.float64, device=DEV)
    for a in range(0, shard.n, 1 << 22):
        tot += S.smf_sumstats_reference(th64, shard.x[a:a + (1 << 22)].double(), shard.pop[a:a + (1 << 22)], bins, True)
    return tot.cpu().numpy()
def kern(th, resid):
    out = torch.zeros(bins.nbp, device=DEV); S.smf_forward_into(th, shard, bins, True, out, resid=resid); return out[:bins.nb].double().cpu().numpy()
eng = FusedAdamEngine(model, graph=False)
eng.setup(data["guess"], nsteps=3, learning_rate=1e-3, history="last")
eng.step(); torch.cuda.synchronize(); S_a = eng.S[:bins.nb].double().cpu().numpy(); th_a = eng.to_user(eng.theta[:eng.P]).clone()
eng.step(); torch.cuda.synchronize(); S_b = eng.S[:bins.nb].double().cpu().numpy(); th_b = eng.to_user(eng.theta[:eng.P]).clone()
g0=data["guess"]
print("th_a==guess", bool(torch.equal(th_a, g0)), "max|th_b-th_a|", float((th_b-th_a).abs().max()))
o0=oracle(g0.double()); o1=oracle(th_b.double())
np.set_printoptions(precision=7)
print("S_a/o0", S_a/o0); print("S_b/o1", S_b/o1); print("S_b/o0", S_b/o0)
print("kern resid th0 / o0", kern(g0,True)/o0); print("kern nores th0 / o0", kern(g0,False)/o0); print("kern resid th1 / o1", kern(th_b,True)/o1)
