"""Is work enqueued on a stream right before hipGraphLaunch ordered before the graph?"""
import torch
dev = torch.device("cuda", 0)
N = 1 << 22
x = torch.zeros(N, device=dev)
y = torch.zeros(N, device=dev)
gr = torch.cuda.CUDAGraph()
s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    torch.mul(x, 2.0, out=y)
torch.cuda.current_stream().wait_stream(s)
with torch.cuda.graph(gr):
    torch.mul(x, 2.0, out=y)
def check(mode, reps=20):
    bad = 0
    for k in range(1, reps + 1):
        torch.cuda.synchronize()
        x.fill_(float(k))
        if mode == "event":
            ev = torch.cuda.Event(); ev.record(); torch.cuda.current_stream().wait_event(ev)
        if mode == "side":
            st = torch.cuda.Stream(); st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                gr.replay()
            torch.cuda.current_stream().wait_stream(st)
        else:
            gr.replay()
        torch.cuda.synchronize()
        bad += int(not bool((y[::4096] == 2.0 * k).all()))
    return bad
for mode in ("plain", "event", "side"):
    print(mode, "stale replays:", check(mode), "of 20", flush=True)
# back-to-back without host sync: fill k then replay, collect y[0] after each
outs = []
for k in range(1, 21):
    x.fill_(float(k)); gr.replay(); outs.append(y[:1].clone())
torch.cuda.synchronize()
print("nosync stale:", sum(int(float(o[0]) != 2.0 * k) for k, o in zip(range(1, 21), outs)))
