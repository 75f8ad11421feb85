"""Where the sumstat epilogue's time goes: the stand-alone epilogue kernel timed over
back-to-back launches (HIP events) for slab sizes 1 .. 4096 rows, plus an empty kernel for
the launch floor.  Usage: python tools/ubench/epilogue_cost.py"""
import json

import torch

from multigrad_amd.ops._ext import ext

dev = torch.device("cuda", 0)
nb = 10
edges = [9.0 + 0.1 * i for i in range(nb + 1)]
scale = [1.0] * nb
target = torch.full((nb,), 1e3, device=dev)
S = torch.zeros(16, device=dev)
loss = torch.zeros(1, device=dev)
h = torch.zeros(16, device=dev)
seq = torch.zeros(1, dtype=torch.int32, device=dev)
err = torch.zeros(1, dtype=torch.int32, device=dev)
E = ext()
out = {}


def timeit(fn, reps=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps  # us per launch


for rows in (1, 64, 256, 1024, 2048, 4096):
    slab = torch.rand(rows * 16, device=dev)
    out[f"epilogue_rows_{rows}"] = round(timeit(lambda: E.smf_epilogue(
        slab, rows, edges, scale, target, 1e-10, S, loss, h, [], 0, seq, err, 5.0)), 2)
z = torch.zeros(1, device=dev)
out["torch_fill_1"] = round(timeit(lambda: z.fill_(1.0)), 2)
print(json.dumps(out))
