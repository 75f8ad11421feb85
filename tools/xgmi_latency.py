"""Latency of the one-shot all-reduce (csrc/xgmi.hip) for a 16-float vector: two
processes sharing one GPU (the only multi-process setup this pool offers), back-to-back
calls timed with events.  Usage: python tools/xgmi_latency.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _run(rank, size, n):
    import torch
    import multigrad_amd as mg
    from multigrad_amd.parallel.xgmi import connect
    comm = mg.get_world_comm()
    ar = connect(comm)
    t = torch.ones(16, device="cuda:0")
    for _ in range(50):
        ar(t)
    torch.cuda.synchronize()
    comm.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        ar(t)
    e1.record()
    torch.cuda.synchronize()
    ok = ar.ok()
    ar.close()
    return 1e3 * e0.elapsed_time(e1) / n, ok


def main():
    from distributed import run_distributed
    res = run_distributed(_run, 2, 2000, timeout=300)
    for r, (us, ok) in enumerate(res):
        print(f"rank {r}: one-shot all-reduce of 16 floats, 2 ranks on one GPU: {us:.2f} us/call ok={ok}")


if __name__ == "__main__":
    main()
