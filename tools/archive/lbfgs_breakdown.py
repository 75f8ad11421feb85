"""Where the device L-BFGS iteration time goes (1e7 params, one GPU): objective
evaluations vs everything else, synchronised wall times."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MULTIGRAD_PROGRESS", "0")


def main():
    import torch
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    from multigrad_amd.optim.lbfgs import lbfgs_minimize
    dev = torch.device("cuda", 0)
    data = make_population_data(10_000_000, 1 << 27, seed=1234, device=dev)
    m = PopulationSMFModel(aux_data=data)
    m.set_target_from_truth()
    obj = m.fused_engine().lbfgs_objective(data["guess"])
    x = obj.x0()
    for _ in range(3):
        obj(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        obj(x)
    torch.cuda.synchronize()
    t_eval = (time.perf_counter() - t0) / 10
    stats = {"evals": 0, "t": 0.0}
    real_call = type(obj).__call__

    def timed(self, u):
        torch.cuda.synchronize()
        a = time.perf_counter()
        r = real_call(self, u)
        torch.cuda.synchronize()
        stats["t"] += time.perf_counter() - a
        stats["evals"] += 1
        return r
    type(obj).__call__ = timed
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = lbfgs_minimize(obj, maxiter=20, gtol=0.0, ftol=0.0)
    torch.cuda.synchronize()
    tt = time.perf_counter() - t0
    print(f"eval {1e3 * t_eval:.3f} ms; lbfgs {1e3 * tt / res.nit:.3f} ms/it, "
          f"{stats['evals'] / res.nit:.2f} evals/it taking {1e3 * stats['t'] / res.nit:.3f} ms/it")


if __name__ == "__main__":
    main()
