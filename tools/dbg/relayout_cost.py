"""Where a re-layout's time goes (engine.relayout at the headline size): every model /
shard method it calls is wrapped with a synchronising timer.  The synchronisation itself
adds a little; the point is the split.  Usage: python tools/dbg/relayout_cost.py"""
import functools
import json
import time

import torch

from multigrad_amd.engine.fused import FusedAdamEngine
from multigrad_amd.models.population import PopulationSMFModel, make_population_data

dev = torch.device("cuda", 0)
data = make_population_data(10_000_000, 1 << 27, seed=1234, device=dev, narrow_frac=0.01,
                            narrow_guess_log_sigma=-0.64)
model = PopulationSMFModel(aux_data=data)
model.set_target_from_truth()
eng = FusedAdamEngine(model, graph=False)
eng.setup(data["guess"], nsteps=1000, learning_rate=1e-3)
eng.steps(200)
torch.cuda.synchronize()
before = []
for _ in range(6):
    t1 = time.perf_counter()
    eng.step()
    torch.cuda.synchronize()
    before.append(round((time.perf_counter() - t1) * 1e3, 3))


def batch_ms(n=200):
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    eng.steps(n)
    torch.cuda.synchronize()
    return round((time.perf_counter() - t1) * 1e3 / n, 4)


print(json.dumps({"steps_before_ms": before, "batch_before_ms": batch_ms()}))

times = {}


def timed(obj, name, label=None):
    fn = getattr(obj, name)

    @functools.wraps(fn)
    def w(*a, **k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn(*a, **k)
        torch.cuda.synchronize()
        times[label or name] = times.get(label or name, 0.0) + (time.perf_counter() - t0) * 1e3
        return r
    setattr(obj, name, w)


sh = data["shard"]
timed(model, "engine_layout_hint")
timed(model, "engine_set_chunks")
timed(sh, "_build_lanes")
timed(sh, "set_lane_classes")
timed(eng, "_probe_now")
timed(eng, "drain")
timed(model, "engine_fwd_rows")
torch.cuda.synchronize()
t0 = time.perf_counter()
changed = eng.relayout(reason={"forced": True})
torch.cuda.synchronize()
total = (time.perf_counter() - t0) * 1e3
times = {k: round(v, 2) for k, v in times.items()}


def step_times(n):
    out = []
    for _ in range(n):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        eng.step()
        torch.cuda.synchronize()
        out.append(round((time.perf_counter() - t1) * 1e3, 3))
    return out


after = step_times(12)
print(json.dumps({"changed": changed, "total_ms": round(total, 2), "parts_ms": times,
                  "steps_after_ms": after, "steps_later_ms": step_times(6),
                  "batch_after_ms": [batch_ms(), batch_ms()],
                  "record": eng.relayouts[-1] if eng.relayouts else None}))
