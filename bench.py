"""Headline benchmark: Adam steps/sec (whole node) on the 1e7-parameter summed-loss model.

BASELINE.json metric: "Adam steps/sec (whole node), 1e7-param summed-loss model at
1/2/4/8 MI355X".  The model is the population SMF model (``multigrad_amd.models.population``):
5e6 populations x (a, log10 sigma) = 1e7 fp32 parameters, synthetic halos generated on
each GPU from a hash of the global halo index (strong scaling: the global data set is
fixed, each of N ranks owns 1/N of it), random-init truth parameters.

Every timed step does the full work of the reference's Adam step
(multigrad/adam.py:59-66 + multigrad/multigrad.py:508-538): forward over all halos,
all-reduce of the sumstats, loss + cotangent, VJP over all halos, the cross-rank
gradient sum, the Adam update of all 1e7 parameters, and the trajectory write of the new
parameters.  On one GPU the step is two eager launches (pipelined update + epilogue).  On N GPUs (one process per
GPU, RCCL) the default ``--placement owner`` splits the global catalog by population:
each rank's gradient is then complete on the populations it owns and zero elsewhere, so
the per-step collective is the 10-float sumstat all-reduce and every rank updates (and
records the trajectory of) only its own parameters.  ``--placement hashed`` splits the
catalog by halo index instead: every rank's gradient is dense and the engine runs a
chunked RCCL reduce-scatter (overlapped with the VJP), Adam on each rank's 1/N slice and
an in-place all-gather (ZeRO-1) -- the same bytes as one all-reduce.  Both placements
hold the same global data set and give the same trajectory (tests/test_engine.py).

Usage: ``python bench.py [--gpus N] [--steps K] [--warmup W]``; for N>1 launch with
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ.setdefault("MULTIGRAD_PROGRESS", "0")


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--params", type=int, default=10_000_000)
    ap.add_argument("--halos", type=int, default=1 << 27,
                    help="global number of halos (fixed across GPU counts: strong scaling)")
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--history", default="full", help="trajectory: full | last | <stride>")
    ap.add_argument("--placement", default="owner", choices=["owner", "hashed"],
                    help="halo -> rank placement for N > 1: 'owner' splits the catalog by "
                         "population (gradient shards complete on their owner, no gradient "
                         "collective); 'hashed' splits it by halo index (dense gradient, "
                         "ZeRO reduce-scatter + all-gather every step)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--profile-phases", action="store_true")
    args = ap.parse_args(argv)

    import torch
    import multigrad_amd as mg
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        comm = mg.init_distributed()
    else:
        comm = mg.get_world_comm()
    if torch.cuda.is_available():
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    # CPU fallback (PyTorch reference math) only so the JSON contract is testable without a
    # GPU; every measured number comes from the HIP path
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
        else torch.device("cpu")

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    t_setup = time.perf_counter()
    data = make_population_data(args.params, args.halos, seed=1234, comm=comm, device=dev,
                                placement=args.placement if comm.size > 1 else "hashed")
    model = PopulationSMFModel(aux_data=data, comm=comm)
    model.set_target_from_truth()
    history = args.history if args.history in ("full", "last") else int(args.history)
    engine = model.fused_engine(graph=False if (args.no_graph or args.profile_phases) else None)
    if args.profile_phases:  # HIP-event timing per phase (eager launches; stderr summary)
        from multigrad_amd.utils.profiling import PhaseTimer
        engine.timer = PhaseTimer(True)
    engine.setup(data["guess"], nsteps=args.warmup + args.steps, learning_rate=args.lr,
                 history=history)
    sync()
    setup_s = time.perf_counter() - t_setup

    for _ in range(args.warmup):
        engine.step()
    loss0 = engine.last_loss()
    sync()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        engine.step()
    engine.drain()  # last all-gathers joined into the compute stream
    sync()
    comm.barrier()
    elapsed = time.perf_counter() - t0
    loss1 = engine.last_loss()
    if comm.size > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        comm.all_reduce(t, op="max")
        elapsed = float(t.item())

    sps = args.steps / elapsed
    rec = {
        "metric": "Adam steps/sec (whole node), 1e7-param summed-loss model",
        "value": round(sps, 3),
        "unit": "steps/s",
        "n_gpus": comm.size,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic",
        "config": {
            "model": f"population-SMF summed-loss model, {args.params:.0e} params "
                     f"({args.params // 2} populations x (a, log10 sigma)), 10 bins, log-MSE",
            "global_batch": args.halos,
            "seq_len": 10,
            "parallelism": f"dp{comm.size}" + ("-owner" if engine.owner else ""),
            "params": args.params,
            "halos_global": args.halos,
            "optimizer": "Adam (fused HIP kernel), full trajectory" if history == "full"
                         else f"Adam (fused HIP kernel), history={history}",
            "graph": bool(engine.use_graph),
            "optimizer_sharding": ("owner" if engine.owner else "zero1" if engine.zero
                                   else "replicated"),
            "placement": data["placement"],
            "grad_collective": ("none: owner-local gradients, sumstat all-reduce only"
                                if engine.owner else "RCCL reduce-scatter + all-gather"
                                if engine.zero else "RCCL all-reduce" if comm.size > 1
                                else "none (1 rank)"),
            "sumstat_allreduce": ("xGMI one-shot kernel (self-tested)"
                                  if getattr(comm, "_oneshot", None) else
                                  "RCCL" if comm.size > 1 else "none (1 rank)"),
            "chunks": engine.C,
        },
        "loss_first_timed": loss0,
        "loss_last": loss1,
        "setup_s": round(setup_s, 2),
    }
    if args.profile_phases:
        rec["phases_ms"] = {k: round(v, 4) for k, v in engine.timer.summary().items()}
    if comm.rank == 0:
        print(json.dumps(rec), flush=True)
    if comm.size > 1:
        comm.barrier()
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
