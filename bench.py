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
parameters.

On N > 1 GPUs (one process per GPU) every rank starts from the reference's data
parallelism: a contiguous block of halo indices (``np.array_split`` of the catalog,
reference tests/smf_example/smf_grad_descent.py:28), so every rank touches every
population.  Two schedules of that same input are timed back to back in one run:

* ``value`` -- the engine's default: at setup it **re-partitions** the halos by parameter
  owner with one all-to-all-v (``Comm.all_to_all_v``: xGMI peer pulls, RCCL fallback;
  ``models.population.repartition_by_owner``), after which each rank's gradient is
  complete on the populations it owns and the only per-step collective is the 10-float
  sumstat all-reduce.  ``setup_s`` includes the re-partition (``repartition`` in the
  record has its own timing).
* ``dense_steps_per_s`` -- the data-parallel schedule kept as it is (BASELINE config 3,
  reference multigrad/multigrad.py:522,531-532): the dense 1e7-float gradient is summed
  across ranks every step (reduce-scatter -> Adam on the owned 1/N slice -> all-gather,
  ZeRO-1, the same bytes as one all-reduce) by the two-shot xGMI exchange or RCCL.

Usage: ``python bench.py [--gpus N] [--steps K] [--warmup W]``.  With ``--gpus N > 1`` and no
launcher environment the script starts ``torch.distributed.run`` with N ranks itself
(before any GPU call in this process) and relays rank 0's JSON line; under a launcher
(``WORLD_SIZE`` set) it runs as one rank.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

os.environ.setdefault("MULTIGRAD_PROGRESS", "0")
# the benchmark measures the steady state: the full setup autotune and settle steps (not the
# library default's budget of 10 % of the requested run), outside the timed region
os.environ.setdefault("MULTIGRAD_AUTOTUNE", "on")


def _args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--params", type=int, default=10_000_000)
    ap.add_argument("--halos", type=int, default=1 << 27,
                    help="global number of halos (fixed across GPU counts: strong scaling)")
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--history", default="full", help="trajectory: full | last | <stride>")
    ap.add_argument("--placement", default="both",
                    choices=["both", "repartition", "hashed", "owner"],
                    help="schedule timed for N > 1: 'repartition' (hashed input re-partitioned "
                         "by parameter owner at setup: the headline value), 'hashed' (dense "
                         "gradient summed across ranks every step), 'owner' (catalog generated "
                         "split by population), or 'both' (default: repartition is 'value', "
                         "hashed is 'dense_steps_per_s')")
    ap.add_argument("--layout", default="auto", choices=["auto", "lanes", "tiles"],
                    help="device layout of the halo shards (auto: lanes for one rank and the "
                         "owner placement, tiles for hashed shards on several ranks)")
    ap.add_argument("--lane-order", default="auto", choices=["auto", "global", "local"],
                    help="lanes layout slot order (auto: local for hashed shards on several "
                         "ranks, global otherwise)")
    ap.add_argument("--narrow-frac", type=float, default=0.0,
                    help="fraction of populations (scattered by a hash) with a narrow true "
                         "sigma (bin width > 0.5 sigma: outside the Euler-Maclaurin forward's "
                         "range, evaluated by the per-edge path); the headline is 0")
    ap.add_argument("--narrow-guess", type=float, default=None,
                    help="starting log10 sigma of the narrow populations (default: truth + 0.1); "
                         "a wide start (e.g. -0.6) makes the fit cross the Euler-Maclaurin limit "
                         "mid-run (the engine re-lays the lanes out)")
    ap.add_argument("--phase-steps", type=int, default=0,
                    help="also report the step rate of every window of this many timed steps "
                         "(a host sync per window)")
    ap.add_argument("--bounds", default="none", choices=["none", "both", "mixed"],
                    help="box constraints (reference run_adam(param_bounds=...)): 'both' boxes "
                         "every parameter around the start (truth inside), 'mixed' gives the "
                         "a's a lower bound only and the log sigmas both bounds; the headline "
                         "is unbounded")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--profile-phases", action="store_true")
    ap.add_argument("--no-count-launches", dest="count_launches", action="store_false",
                    help="skip counting the device operations of one step (torch.profiler, "
                         "after the timed region)")
    return ap.parse_args(argv)


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def visible_gpus() -> int:
    """GPUs this process could use, counted without touching the GPU runtime (no torch, no
    HIP call): the first ``*_VISIBLE_DEVICES`` list that is set, else the KFD topology nodes
    with a non-zero ``gpu_id`` (CPU nodes have 0).  0 if nothing is visible."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([d for d in v.split(",") if d.strip() not in ("", "-1")])
    base = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        for node in os.listdir(base):
            try:
                with open(os.path.join(base, node, "gpu_id")) as f:
                    n += int(f.read().strip() or 0) != 0
            except (OSError, ValueError):
                pass
    except OSError:
        return 0
    return n


def launch(args, argv) -> int:
    """Start ``args.gpus`` ranks with torch.distributed.run and relay their output.

    GPU-free by construction: this parent process imports no torch and makes no HIP call
    (GPUs are counted from the environment / sysfs), and it starts the ranks as children
    -- never exec."""
    ndev = visible_gpus()
    if 0 < ndev < args.gpus:
        print(f"bench.py: --gpus {args.gpus} requested but only {ndev} GPU(s) are visible",
              file=sys.stderr, flush=True)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


def bench_bounds(args, data):
    """``(P, 2)`` box constraints for ``--bounds`` (None: unbounded), around the start."""
    if args.bounds == "none":
        return None
    import torch
    g = data["guess"].detach()
    pb = torch.stack([g - 1.0, g + 0.5], 1)
    if args.bounds == "mixed":
        pb[0::2, 1] = float("inf")  # a: lower bound only
    return pb


def time_placement(placement, args, comm, dev, sync):
    """Build the data and engine for one placement, warm up, time ``args.steps`` steps.

    Returns the per-rank record (elapsed is the MAX over ranks)."""
    import torch
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    from multigrad_amd.utils.trace import trace

    trace(f"bench: {placement}: data")
    t_setup = time.perf_counter()
    gen = "owner" if placement == "owner" and comm.size > 1 else "hashed"
    data = make_population_data(args.params, args.halos, seed=1234, comm=comm, device=dev,
                                placement=gen,
                                layout=args.layout,
                                lane_order=None if args.lane_order == "auto" else args.lane_order,
                                narrow_frac=args.narrow_frac,
                                narrow_guess_log_sigma=args.narrow_guess)
    model = PopulationSMFModel(aux_data=data, comm=comm)
    model.set_target_from_truth()
    history = args.history if args.history in ("full", "last") else int(args.history)
    engine = model.fused_engine(graph=False if (args.no_graph or args.profile_phases) else None,
                                repartition=placement == "repartition")
    if args.profile_phases:  # HIP-event timing per phase (eager launches)
        from multigrad_amd.utils.profiling import PhaseTimer
        engine.timer = PhaseTimer(True)
    count = args.count_launches and dev.type == "cuda"
    engine.setup(data["guess"], nsteps=args.warmup + args.steps + (2 if count else 0),
                 learning_rate=args.lr, history=history, param_bounds=bench_bounds(args, data))
    sync()
    setup_s = time.perf_counter() - t_setup

    trace(f"bench: {placement}: warmup")
    engine.steps(args.warmup)
    # the last warmup step's pending (pipelined) update is applied before the clock starts,
    # so the timed region holds exactly K forwards and K updates (the K-th one in drain())
    engine.drain()
    loss0 = engine.last_loss()
    sync()
    comm.barrier()
    sync()
    trace(f"bench: {placement}: timed steps")
    t0 = time.perf_counter()
    phases = []
    if args.phase_steps > 0:
        done = 0
        while done < args.steps:
            w = min(args.phase_steps, args.steps - done)
            tw = time.perf_counter()
            nrel = len(getattr(engine, "relayouts", []))
            engine.steps(w)
            sync()
            phases.append({"first_step": done, "steps": w,
                           "ms_per_step": round(1e3 * (time.perf_counter() - tw) / w, 4),
                           "relayouts": len(getattr(engine, "relayouts", [])) - nrel,
                           "per_edge_share": round(model.engine_layout_share(
                               comm.rank if engine.owner else None), 4)})
            done += w
    else:
        engine.steps(args.steps)  # graph mode: blocks of engine.graph_steps steps per replay
    engine.drain()  # the pipelined last update / last all-gathers are inside the timing
    sync()
    comm.barrier()
    elapsed = time.perf_counter() - t0
    trace(f"bench: {placement}: timed {elapsed:.4f} s")
    engine.check()  # a failed peer exchange raises here instead of reporting wrong numbers
    loss1 = engine.last_loss()
    fb = model.lane_fallback_groups(data["guess"])  # lane groups on the per-edge path
    ops = {}
    if count:  # after the timing: device operations of one steady-state step
        from multigrad_amd.utils.profiling import count_device_ops
        ops = count_device_ops(engine.step, 2)
        engine.drain()
        engine.check()
    if comm.size > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        comm.all_reduce(t, op="max")
        elapsed = float(t.item())
    info = {
        "elapsed": elapsed,
        "steps_per_s": args.steps / elapsed,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "parallelism": f"dp{comm.size}" + ("-owner" if engine.owner else ""),
        "graph": bool(engine.use_graph),
        "graph_steps": int(engine.graph_steps) if engine.use_graph else 0,
        "pipelined": bool(engine.pipeline),
        "optimizer_sharding": ("owner" if engine.owner else "zero1" if engine.zero
                               else "replicated"),
        "placement": data["placement"] + (" (re-partitioned from hashed at setup)"
                                          if engine.repartitioned else ""),
        "repartition": engine.repartitioned or None,
        "grad_collective": engine.grad_collective_name(),
        "sumstat_allreduce": engine.sumstat_collective_name(),
        "chunks": engine.C,
        "layout": data["shard"].layout + ("/" + data["shard"].lane_order
                                          if data["shard"].layout == "lanes" else ""),
        "loss_first_timed": loss0,
        "loss_last": loss1,
        "setup_s": round(setup_s, 2),
        "fallback_groups": list(fb),
        "history": history,
        "device_ops_per_step": ops or None,
        "autotune": getattr(engine, "tuning", None),
        "relayouts": list(getattr(engine, "relayouts", [])),
        "phases": phases or None,
    }
    if args.profile_phases:
        info["phases_ms"] = {k: round(v, 4) for k, v in engine.timer.summary().items()}
    engine.close()  # the two-shot context goes back to the communicator's pool
    del engine, model, data
    if dev.type == "cuda":
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    return info


def run_placements(order, timed, on_error=None):
    """Time each placement in ``order`` with ``timed(placement)``.  The first one is the
    headline and its failure ends the run; a failure of a later (extra) placement that every
    rank sees (e.g. out of memory) is returned in ``errors`` instead, so it does not cost the
    headline line."""
    res, errors = {}, {}
    for i, p in enumerate(order):
        if i == 0:
            res[p] = timed(p)
            continue
        try:
            res[p] = timed(p)
        except Exception as exc:  # noqa: BLE001
            errors[p] = f"{type(exc).__name__}: {exc}"[:300]
            print(f"bench.py: {p} placement failed: {errors[p]}", file=sys.stderr, flush=True)
            if on_error is not None:
                on_error()
    return res, errors


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = _args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch(args, argv)

    import torch
    import multigrad_amd as mg

    world = int(os.environ.get("WORLD_SIZE", "1"))
    json_fd = None
    if world > 1:
        # every rank's fd 1 goes to stderr while it runs (gloo prints its connection
        # messages to stdout), so rank 0's JSON record is the only line on stdout
        sys.stdout.flush()
        json_fd = os.dup(1)
        os.dup2(2, 1)
    comm = mg.init_distributed() if world > 1 else mg.get_world_comm()
    if comm.size != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started "
                         f"{comm.size} rank(s)")
    if torch.cuda.is_available():
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    # CPU fallback (PyTorch reference math) only so the JSON contract is testable without a
    # GPU; every measured number comes from the HIP path
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
        else torch.device("cpu")

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    if comm.size == 1:
        order = ["hashed"]  # one rank: the placements coincide
    elif args.placement == "both":
        order = ["repartition", "hashed"]
    else:
        order = [args.placement]
    def release():
        if dev.type == "cuda":
            torch.cuda.synchronize()
            torch.cuda.empty_cache()

    res, errors = run_placements(order, lambda p: time_placement(p, args, comm, dev, sync),
                                 on_error=release)
    head = res[order[0]]
    dense = res.get("hashed", head if comm.size == 1 else None)
    history = head["history"]
    rec = {
        "metric": "Adam steps/sec (whole node), 1e7-param summed-loss model",
        "value": round(head["steps_per_s"], 3),
        "unit": "steps/s",
        "n_gpus": comm.size,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(head["ms_per_step"], 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (counter-hash halo catalog, random-init truth parameters)",
        "config": {
            "model": f"population-SMF summed-loss model, {args.params:.0e} params "
                     f"({args.params // 2} populations x (a, log10 sigma)), 10 bins, log-MSE",
            "global_batch": args.halos,
            "seq_len": 10,
            "parallelism": head["parallelism"],
            "params": args.params,
            "halos_global": args.halos,
            "optimizer": "Adam (fused HIP kernel), full trajectory" if history == "full"
                         else f"Adam (fused HIP kernel), history={history}",
            "graph": head["graph"],
            "graph_steps": head["graph_steps"],
            "pipelined": head["pipelined"],
            "optimizer_sharding": head["optimizer_sharding"],
            "placement": head["placement"],
            "grad_collective": head["grad_collective"],
            "sumstat_allreduce": head["sumstat_allreduce"],
            "chunks": head["chunks"],
            "layout": head["layout"],
            "narrow_frac": args.narrow_frac,
            "bounds": args.bounds,
            "narrow_guess": args.narrow_guess,
            "relayouts": head["relayouts"],
            "per_edge_groups": head["fallback_groups"],
            "device_ops_per_step": head["device_ops_per_step"],
            "autotune": head["autotune"],
        },
        "dense_steps_per_s": None if dense is None else round(dense["steps_per_s"], 3),
        "dense_ms_per_step": None if dense is None else round(dense["ms_per_step"], 4),
        "loss_first_timed": head["loss_first_timed"],
        "loss_last": head["loss_last"],
        "setup_s": head["setup_s"],
    }
    if head["repartition"]:
        rec["repartition"] = head["repartition"]
    if head["phases"]:
        rec["phases"] = head["phases"]
    if comm.size > 1:
        # connect-time verdicts of the peer-memory collectives: stress self-test passed
        # (back-to-back device-only exchanges) or the RCCL fallback and why
        from multigrad_amd.parallel.xgmi import status
        rec["peer_memory_selftest"] = status(comm)
    if errors:
        rec["errors"] = errors
    if dense is not None and dense is not head:
        rec["dense_config"] = {k: dense[k] for k in ("parallelism", "optimizer_sharding",
                                                     "grad_collective", "sumstat_allreduce",
                                                     "chunks", "pipelined", "layout",
                                                     "device_ops_per_step", "autotune", "graph",
                                                     "loss_last", "setup_s")}
    if args.profile_phases:
        rec["phases_ms"] = head["phases_ms"]
        if dense is not None and dense is not head:
            rec["dense_phases_ms"] = dense["phases_ms"]
    if comm.rank == 0:
        if json_fd is not None:
            sys.stdout.flush()
            os.write(json_fd, (json.dumps(rec) + "\n").encode())
        else:
            print(json.dumps(rec), flush=True)
    if comm.size > 1:
        comm.barrier()
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
