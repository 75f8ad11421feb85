import torch
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
y = torch.empty(4, device=dev)
s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    y.copy_(torch.randn(4, generator=g, device=dev))
torch.cuda.current_stream().wait_stream(s)
gr = torch.cuda.CUDAGraph()
gr.register_generator_state(g)
with torch.cuda.graph(gr):
    y.copy_(torch.randn(4, generator=g, device=dev))
def ref(seed):
    r = torch.Generator(device=dev); r.manual_seed(seed); return torch.randn(4, generator=r, device=dev)
for mode in ("nosync", "sync", "sync_before_seed"):
    outs = []
    for i, seed in enumerate([11, 22, 33, 44]):
        if mode == "sync_before_seed": torch.cuda.synchronize()
        g.manual_seed(seed)
        gr.replay()
        if mode == "sync": torch.cuda.synchronize()
        outs.append(y.clone())
    torch.cuda.synchronize()
    print(mode, [bool(torch.equal(o, ref(sd))) for o, sd in zip(outs, [11, 22, 33, 44])], flush=True)
# alternative: set_state of a freshly seeded generator
outs=[]
for seed in [11, 22, 33, 44]:
    r = torch.Generator(device=dev); r.manual_seed(seed)
    g.graphsafe_set_state(r.graphsafe_get_state()) if hasattr(g, "graphsafe_set_state") else None
    gr.replay(); torch.cuda.synchronize(); outs.append(y.clone())
print("graphsafe_set_state", [bool(torch.equal(o, ref(sd))) for o, sd in zip(outs, [11, 22, 33, 44])])
