import torch
dev = torch.device("cuda", 0)
N = 400000
x = torch.rand(N, device=dev)
out = torch.zeros(2, device=dev)
def make(with_gen, reps=30):
    g = torch.Generator(device=dev) if with_gen else None
    def body():
        if with_gen:
            n = torch.randn(N, generator=g, device=dev)
            y = x + 0.0 * n
        else:
            y = x * 1.0 + 0.0
        out[:1].copy_(y.sum().reshape(1))
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s): body()
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    if with_gen: gr.register_generator_state(g)
    with torch.cuda.graph(gr): body()
    torch.cuda.synchronize()
    body(); torch.cuda.synchronize(); expect = out[:1].clone()
    res = {}
    for mode in ("nosync", "sync"):
        bad = 0
        outs = []
        for k in range(reps):
            if with_gen: g.manual_seed(100 + k)
            gr.replay()
            if mode == "sync": torch.cuda.synchronize()
            outs.append(out[:1].clone())
        torch.cuda.synchronize()
        res[mode] = sum(int(not torch.equal(o, expect)) for o in outs)
    return res
for wg in (False, True):
    print("with_gen", wg, "wrong sums:", make(wg), flush=True)
