import torch
dev = torch.device("cuda", 0)
N = 400000
x = torch.rand(N, device=dev)
x0 = x.clone()
g = torch.Generator(device=dev)
out = torch.zeros(4, device=dev)
nbuf = torch.zeros(N, device=dev)
ybuf = torch.zeros(N, device=dev)
def body(gen):
    n = torch.randn(N, generator=gen, device=dev)
    nbuf.copy_(n)
    y = x + 0.02 * n
    ybuf.copy_(y)
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
    r = torch.Generator(device=dev); r.manual_seed(seed); body(r); return out.clone(), nbuf.clone(), ybuf.clone()
seeds = [101, 202, 303]
exp = [ref(sd) for sd in seeds]
for mode in ("nosync", "sync"):
    res = []
    for sd in seeds:
        g.manual_seed(sd)
        gr.replay()
        if mode == "sync": torch.cuda.synchronize()
        res.append((out.clone(), nbuf.clone(), ybuf.clone()))
    torch.cuda.synchronize()
    print(mode, "out/n/y ok:", [(bool(torch.equal(a[0], b[0])), bool(torch.equal(a[1], b[1])), bool(torch.equal(a[2], b[2]))) for a, b in zip(res, exp)],
          "x intact:", bool(torch.equal(x, x0)), flush=True)
    if mode == "sync":
        a, b = res[0], exp[0]
        print("  out got", a[0].tolist(), "exp", b[0].tolist())
        d = (a[2] - b[2]).abs(); print("  y maxdiff", float(d.max()), "n maxdiff", float((a[1]-b[1]).abs().max()))
