"""Host cost of launching one HIP graph vs the eager launches it replaces, and the device
gap between back-to-back graph launches: python tools/graph_launch_cost.py"""
import json
import time

import torch

x = torch.zeros(1 << 20, device="cuda")
for nk in (1, 2, 8):
    def body():
        for _ in range(nk):
            x.add_(1.0)
    body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    res = {"kernels_per_step": nk}
    for mode, fn in (("eager", body), ("graph", g.replay)):
        for _ in range(50):
            fn()
        torch.cuda.synchronize()
        n = 2000
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        host = (time.perf_counter() - t0) / n
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / n
        res[mode] = {"host_us_per_step": round(1e6 * host, 2), "wall_us_per_step": round(1e6 * wall, 2)}
    print(json.dumps(res), flush=True)
