"""Multi-process test harness: spawn N ranks on the gloo backend (127.0.0.1).

Each rank initialises torch.distributed, builds the multigrad_amd world communicator
and runs ``fn(rank, size, *args)``.  Return values are collected; an exception on any
rank fails the test with that rank's traceback.
"""
import os
import socket
import traceback

import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, size, port, fn, args, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(size), "LOCAL_RANK": str(rank),
                       "MULTIGRAD_DEVICE_COMM": "0", "MULTIGRAD_PROGRESS": "0",
                       "OMP_NUM_THREADS": "1"})
    # the engines' setup-time re-partition by parameter owner is on by default for several
    # ranks; tests of the data-parallel (hashed) schedules keep their placement, the
    # re-partition tests turn it back on (tests/test_repartition.py)
    os.environ.setdefault("MULTIGRAD_REPARTITION", "0")
    try:
        import torch
        torch.set_num_threads(1)
        import multigrad_amd.parallel.comm as C
        C.set_world_comm(None)
        C.init_distributed(backend="gloo")
        res = fn(rank, size, *args)
        q.put((rank, "ok", res))
    except BaseException:  # noqa: BLE001
        q.put((rank, "err", traceback.format_exc()))
    finally:
        try:
            import torch.distributed as dist
            if dist.is_initialized():
                dist.destroy_process_group()
        except Exception:
            pass


def run_distributed(fn, size: int, *args, timeout: float = 240.0):
    """Run ``fn(rank, size, *args)`` on ``size`` gloo ranks; return the per-rank results."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, size, port, fn, args, q)) for r in range(size)]
    for p in procs:
        p.start()
    results, errors = {}, []
    try:
        for _ in range(size):
            rank, status, payload = q.get(timeout=timeout)
            if status == "ok":
                results[rank] = payload
            else:
                errors.append(f"rank {rank}:\n{payload}")
                break
    finally:
        for p in procs:
            p.join(timeout=5 if errors else 30)
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join()
    if errors:
        raise AssertionError("\n".join(errors))
    return [results[r] for r in range(size)]
