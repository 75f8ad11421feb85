"""Torch-only reproductions (no multigrad code) of the two graph-replay anomalies seen in the
generic engine (docs/design.md "Graph replay vs eager launches"), VERDICT r3 #4:

  A. a captured optimizer step replayed after eager steps, with a host synchronisation
     after every step ("eeeeeggggggeeeeegggg"), deviates from the eager trajectory;
  B. a step with an RNG op on a graph-registered generator, replayed on the default stream
     right after a host synchronisation, computes wrong sums downstream of the RNG op.

The step mimics the engine's: autograd VJP of a sum-of-erf model, Adam with the step index
from a device counter (graph) or a host int (eager), the trajectory row written at the
device step.  Before a replay that follows eager steps the device counter is set from the
host, once with a Python item assignment (pageable host-to-device copy, as the engine did)
and once with an in-stream fill kernel.  Prints the largest deviation from the all-eager
trajectory per schedule.  Usage (one GPU): python tools/dbg/torch_replay_repro.py
"""
import os

import torch

dev = torch.device("cuda", 0)
N, H, STEPS = 4096, 200_000, 20
g0 = torch.Generator(device="cpu").manual_seed(0)
x = torch.randn(H, generator=g0).to(dev)
pop = torch.randint(0, N, (H,), generator=g0).to(dev)
edges = torch.linspace(-2.0, 2.0, 11, device=dev)
target = torch.rand(10, generator=g0).to(dev) * H / 10
b1, b2, eps, lr = 0.9, 0.999, 1e-8, 1e-3
b1t, b2t = torch.tensor(b1, device=dev), torch.tensor(b2, device=dev)  # (no copies in a capture)


class State:
    def __init__(self):
        self.p = (0.1 * torch.randn(N, generator=torch.Generator().manual_seed(1))).to(dev)
        self.m = torch.zeros(N, device=dev)
        self.v = torch.zeros(N, device=dev)
        self.step = torch.zeros(1, dtype=torch.int64, device=dev)
        self.traj = torch.zeros(STEPS + 1, N, device=dev)
        self.traj[0] = self.p


def body(s: State, host_step, gen=None):
    leaf = s.p.detach().requires_grad_(True)
    with torch.enable_grad():
        xs = x if gen is None else x + 0.01 * torch.randn(x.shape, generator=gen, device=dev)
        z = (edges[None, :] - xs[:, None] - leaf[pop][:, None]) * 2.0
        cdf = 0.5 * (1.0 + torch.erf(z))
        S = (cdf[:, 1:] - cdf[:, :-1]).sum(0)
        loss = ((S - target) ** 2).mean()
        (g,) = torch.autograd.grad(loss, leaf)
    st = (s.step.to(torch.float32) if host_step is None
          else torch.full((1,), float(host_step), device=dev))  # fill kernel, no copy
    s.m.mul_(b1).add_(g, alpha=1 - b1)
    s.v.mul_(b2).addcmul_(g, g, value=1 - b2)
    bc1 = 1 - torch.pow(b1t, st + 1)
    bc2 = 1 - torch.pow(b2t, st + 1)
    s.p.sub_(lr * (s.m / bc1) / (torch.sqrt(s.v / bc2) + eps))
    row = (st.to(torch.int64) + 1) if host_step is None else \
        torch.full((1,), host_step + 1, dtype=torch.int64, device=dev)
    s.traj.index_copy_(0, row, s.p.reshape(1, N))
    if host_step is None:
        s.step.add_(1)


def capture(s: State, gen=None):
    saved = [t.clone() for t in (s.p, s.m, s.v, s.step, s.traj)]
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        body(s, None, gen)  # warm-up
    torch.cuda.current_stream().wait_stream(side)
    for t, v in zip((s.p, s.m, s.v, s.step, s.traj), saved):
        t.copy_(v)
    graph = torch.cuda.CUDAGraph()
    if gen is not None:
        graph.register_generator_state(gen)
    with torch.cuda.graph(graph):
        body(s, None, gen)
    return graph


def run(schedule, sync, set_step="item", keyed=False, replay_stream="default"):
    s = State()
    gen = torch.Generator(device=dev) if keyed else None
    graph, prev = None, None
    for k, mode in enumerate(schedule):
        if gen is not None:
            gen.manual_seed(1000 + k)  # one key per step (the engine's per-step keys)
        if mode == "g":
            if graph is None or prev == "e":
                if set_step == "item":
                    s.step[0] = k                 # pageable host-to-device copy
                else:
                    s.step.fill_(k)               # a kernel on the current stream
            if graph is None:
                graph = capture(s, gen)
                if gen is not None:
                    gen.manual_seed(1000 + k)
            if replay_stream == "side":
                st = torch.cuda.Stream()
                st.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(st):
                    graph.replay()
                torch.cuda.current_stream().wait_stream(st)
            else:
                graph.replay()
        else:
            body(s, k, gen)
        if sync:
            if os.environ.get("REPRO_SYNC", "device") == "stream":
                torch.cuda.current_stream().synchronize()
            else:
                torch.cuda.synchronize()
        prev = mode
    torch.cuda.synchronize()
    return s.traj


def report(name, ref, t):
    d = (t - ref).abs().amax(dim=1)
    bad = [i for i in range(d.numel()) if float(d[i]) > 1e-6]
    print(f"{name:52s} max {float(d.max()):.1e}  first_bad_row={bad[0] if bad else None}",
          flush=True)


ref = run("e" * STEPS, False)
for sched in ("eeeeeggggggggggggggg", "eeeeeggggggeeeeegggg"):
    for sync in (False, True):
        for set_step in ("item", "fill"):
            for rs in ("default", "side"):
                if os.environ.get("REPRO_QUICK") and not (sync and sched[-1] == "g" and "e" in sched[6:]):
                    continue
                report(f"A {sched} {'sync' if sync else 'nosync'} {set_step} {rs}", ref,
                       run(sched, sync, set_step, replay_stream=rs))
refk = run("e" * STEPS, False, keyed=True)
for sched in ("eeeeeggggggggggggggg", "gggggggggggggggggggg"):
    for sync in ((True,) if os.environ.get("REPRO_QUICK") else (False, True)):
        for rs in ("default", "side"):
            report(f"B {sched} {'sync' if sync else 'nosync'} {rs}", refk,
                   run(sched, sync, "fill", keyed=True, replay_stream=rs))
