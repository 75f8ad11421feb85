"""How fast do the narrow populations of ``--narrow-guess`` cross the Euler-Maclaurin limit
in the headline fit?  Prints quantiles of their log10 sigma every 100 steps."""
import math
import sys, os
sys.path.insert(0, os.getcwd())
import torch
from multigrad_amd.models.population import PopulationSMFModel, make_population_data, hash_uniform

P = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
H = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 24
lr = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-3
dev = torch.device("cuda", 0)
data = make_population_data(P, H, seed=1234, device=dev, narrow_frac=0.01, narrow_guess_log_sigma=-0.6)
m = PopulationSMFModel(aux_data=data)
m.set_target_from_truth()
npop = P // 2
narrow = (hash_uniform(torch.arange(npop, device=dev), 1234 + 4) < 0.01)
eng = m.fused_engine()
eng.setup(data["guess"], nsteps=2000, learning_rate=lr, history="last")
thr = math.log10(0.2)
for k in range(20):
    eng.steps(100)
    p = eng.params()
    s = p[1::2][narrow]
    q = torch.quantile(s.float(), torch.tensor([0.05, 0.5, 0.95], device=dev))
    print(k * 100 + 100, "narrow s q05/50/95", [round(float(x), 4) for x in q],
          "frac crossed", round(float((s < thr).float().mean()), 4), "loss", eng.last_loss(),
          "relayouts", len(eng.relayouts), flush=True)
