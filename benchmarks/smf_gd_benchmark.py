"""Speed test of the SMF gradient-descent pipeline (reference tests/smf_example/benchmark.py).

Prints "Grad descent iterations/sec" for ``run_simple_grad_descent`` on the test-suite
SMF model (2 parameters, ``--num-halos`` power-law halos sharded over the ranks) and
optionally appends a result dict to ``--save``.  The reference calls a non-existent
``run_grad_descent``; this harness calls ``run_simple_grad_descent``.

    python benchmarks/smf_gd_benchmark.py --num-halos 1000000
    python -m multigrad_amd.launch -n 8 benchmarks/smf_gd_benchmark.py --num-halos 100000000
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MULTIGRAD_PROGRESS", "0")


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--num-halos", type=int, default=10_000)
    ap.add_argument("--num-steps", type=int, default=100)
    ap.add_argument("--learning-rate", type=float, default=1e-3)
    ap.add_argument("--device", default=None)
    ap.add_argument("--save", type=str, default=None)
    args = ap.parse_args(argv)
    import torch
    import multigrad_amd as mg
    from multigrad_amd.models.smf import MySMFModel, ParamTuple, make_test_data
    comm = mg.init_distributed() if int(os.environ.get("WORLD_SIZE", "1")) > 1 else mg.get_world_comm()
    data = make_test_data(args.num_halos, comm=comm)
    model = MySMFModel(aux_data=data, comm=comm, device=args.device)
    guess = ParamTuple(log_shmrat=-1, sigma_logsm=0.5)
    model.run_simple_grad_descent(guess, nsteps=1, learning_rate=args.learning_rate)  # warm-up
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    res = model.run_simple_grad_descent(guess, nsteps=args.num_steps, learning_rate=args.learning_rate)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    comm.barrier()
    t = time.perf_counter() - t0
    if comm.rank == 0:
        ips = args.num_steps / t
        eng = getattr(model, "fused_step_engine", lambda: None)()
        rec = dict(metric="Grad descent iterations/sec", value=ips, num_halos=args.num_halos,
                   num_steps=args.num_steps, num_processes=comm.size,
                   engine=None if eng is None else dict(schedule=eng.schedule,
                                                        graph=eng.use_graph, stats=eng.stats),
                   final_params=res.params[-1].tolist(), final_loss=float(res.loss[-1]))
        print(json.dumps(rec), flush=True)
        print(f"Benchmark with {comm.size} processes {vars(args)}")
        print("=" * 70)
        print(f"Grad descent iterations/sec = {ips}")
        print(f"final params = {res.params[-1].tolist()}")
        if args.save:
            with open(args.save, "a") as f:
                f.write(json.dumps(dict(calls_per_sec=ips, num_processes=comm.size,
                                        num_halos=args.num_halos, num_steps=args.num_steps,
                                        learning_rate=args.learning_rate)) + "\n")


if __name__ == "__main__":
    main()
