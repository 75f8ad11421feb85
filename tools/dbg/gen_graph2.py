import torch
dev = torch.device("cuda", 0)
N = 400000
x = torch.rand(N, device=dev)
g = torch.Generator(device=dev)
out = torch.zeros(4, device=dev)
def body(gen):
    n = torch.randn(N, generator=gen, device=dev)
    y = x + 0.02 * n
    out.copy_(torch.stack([y.sum(), y[0], y[N // 2], (y * y).sum()]))
s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    body(g)
torch.cuda.current_stream().wait_stream(s)
gr = torch.cuda.CUDAGraph()
gr.register_generator_state(g)
with torch.cuda.graph(gr):
    body(g)
def ref(seed):
    r = torch.Generator(device=dev); r.manual_seed(seed); body(r); return out.clone()
seeds = [101, 202, 303, 404, 505, 606]
exp = [ref(sd) for sd in seeds]
for mode in ("nosync", "sync", "sync+dummy"):
    outs = []
    for sd in seeds:
        if mode == "sync+dummy": x.add_(0)
        g.manual_seed(sd)
        gr.replay()
        if mode.startswith("sync"): torch.cuda.synchronize()
        outs.append(out.clone())
    torch.cuda.synchronize()
    print(mode, [bool(torch.equal(o, e)) for o, e in zip(outs, exp)], flush=True)
