"""HIP graph dispatch cost with torch kernels only: a step of a one-workgroup kernel (A) and
a chip-wide kernel (B, ~60 us of HBM traffic), run eagerly, as one-step graph replays and
as 16-step graphs.  Prints ms per step per mode (median of alternating repeats); run under
``rocprofv3 --kernel-trace`` to see the gaps.  Separates the runtime's graph dispatch cost
from anything in multigrad's kernels (docs/design.md "Graph replay vs eager launches").
Usage (one GPU): python tools/ubench/graph_gap.py [--steps 512] [--K 16]"""
import argparse
import statistics
import time

import torch

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=512)
ap.add_argument("--K", type=int, default=16)
ap.add_argument("--repeats", type=int, default=5)
ap.add_argument("--kind", default="mul", choices=["mul", "sum", "cumsum"],
                help="kernel B: elementwise (no LDS), row reduction or scan (LDS)")
ap.add_argument("--only", default=None, help="run one mode (for a profiler trace)")
ap.add_argument("--mb", type=int, default=256, help="bytes moved by kernel B, MiB (read+write)")
a = ap.parse_args()

dev = torch.device("cuda", 0)
n = a.mb * 2 ** 20 // 8
big = torch.ones(n, device=dev)
small = torch.zeros(64, device=dev)
rows = big.view(-1, 4096)
red = torch.zeros(rows.shape[0], device=dev)


def step():
    small[:1].add_(1.0)      # A: one workgroup
    if a.kind == "mul":
        big.mul_(1.0000001)  # B: every CU, HBM bound
    elif a.kind == "sum":
        torch.sum(rows, dim=1, out=red)
    else:
        torch.cumsum(rows, dim=1, out=rows)


def capture(k):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(k):
            step()
    return g


graphs = {1: capture(1), a.K: capture(a.K)}


def run(mode):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if mode == "eager":
        for _ in range(a.steps):
            step()
    else:
        k = 1 if mode == "graph-1" else a.K
        for _ in range(a.steps // k):
            graphs[k].replay()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / a.steps


modes = ("eager", "graph-1", "graph-K") if a.only is None else (a.only,)
for m in modes:
    run(m)  # warm
res = {m: [] for m in modes}
for _ in range(a.repeats):
    for m in modes:
        res[m].append(run(m))
print({m: round(statistics.median(v), 4) for m, v in res.items()}, "ms/step, K =", a.K,
      "B moves", a.mb, "MiB", flush=True)
