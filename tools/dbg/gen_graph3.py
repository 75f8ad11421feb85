import torch
dev = torch.device("cuda", 0)
N = 400000
g = torch.Generator(device=dev)
out = torch.zeros(N, device=dev)
def body(gen):
    out.copy_(torch.randn(N, generator=gen, device=dev))
s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    body(g)
torch.cuda.current_stream().wait_stream(s)
gr = torch.cuda.CUDAGraph()
gr.register_generator_state(g)
with torch.cuda.graph(gr):
    body(g)
def ref(seed, offset_calls=0):
    r = torch.Generator(device=dev); r.manual_seed(seed)
    for _ in range(offset_calls): torch.randn(N, generator=r, device=dev)
    return torch.randn(N, generator=r, device=dev)
seeds = [101, 202, 303, 404]
cands = {(sd, oc): ref(sd, oc) for sd in seeds for oc in range(3)}
def which(o):
    for k, v in cands.items():
        if torch.equal(o, v): return k
    return None
for mode in ("nosync", "sync", "nosync"):
    res = []
    for sd in seeds:
        g.manual_seed(sd)
        gr.replay()
        if mode == "sync": torch.cuda.synchronize()
        res.append(out.clone())
    torch.cuda.synchronize()
    print(mode, [which(o) for o in res], "gen offset", g.get_offset() if hasattr(g, "get_offset") else "?", flush=True)
