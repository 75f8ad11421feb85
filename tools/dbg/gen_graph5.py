import torch
dev = torch.device("cuda", 0)
N = 400000
x = torch.rand(N, device=dev)
out = torch.zeros(2, device=dev)
def make(with_gen, use_rng, pre_fill):
    g = torch.Generator(device=dev) if with_gen else None
    def body():
        if use_rng:
            nb = torch.randn(16, generator=g, device=dev)
            out[1:2].copy_(nb[:1])
        out[:1].copy_(x.sum().reshape(1))
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s): body()
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    if with_gen: gr.register_generator_state(g)
    with torch.cuda.graph(gr): body()
    torch.cuda.synchronize()
    expect = x.sum()
    bad = 0
    for k in range(20):
        if pre_fill: x.mul_(1.0)
        if with_gen: g.manual_seed(100 + k)
        gr.replay()
        torch.cuda.synchronize()
        bad += int(not torch.equal(out[:1], expect.reshape(1)))
    return bad
for cfg in [(False, False, False), (False, False, True), (True, False, False), (True, True, False), (True, True, True)]:
    print("with_gen, use_rng, pre_fill =", cfg, "-> wrong sums:", make(*cfg), "of 20", flush=True)
