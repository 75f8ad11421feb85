"""Bisection of the two torch-only replay anomalies of tools/dbg/torch_replay_repro.py.

The captured step also records, per trajectory row, what it READ: the step index it used,
the sums of p / m / v at its start, the gradient sum and (keyed runs) the sum of its noise
draw.  Comparing these with the eager run's records at the first wrong row says which input
the replay saw stale.  Each anomaly is re-run with one change before the replay:

  none        as in the repro
  sync_pre    a host synchronisation between the pre-replay work and the replay
  dummy       a one-element kernel on the current stream right before the replay
  persist     the replay on one persistent non-default stream (event-ordered both ways)
  *_nosync    the same without the host synchronisation after every step
  all_stream  every launch of the run (eager steps, fills, capture, replays) on one
              persistent non-default stream: nothing on the default stream
  user_null   all_stream, plus one kernel on the default stream after every step's host
              synchronisation (user code between the engine's steps)
  split       eager steps and fills on one non-default stream, replays on another
              (event-ordered), nothing on the default stream
  capture_side  the capture issued from a non-default stream, everything else as in none

Usage (one GPU): python tools/dbg/torch_replay_bisect.py
"""
import torch

dev = torch.device("cuda", 0)
N, H, STEPS = 4096, 200_000, 20
g0 = torch.Generator(device="cpu").manual_seed(0)
x = torch.randn(H, generator=g0).to(dev)
pop = torch.randint(0, N, (H,), generator=g0).to(dev)
edges = torch.linspace(-2.0, 2.0, 11, device=dev)
target = torch.rand(10, generator=g0).to(dev) * H / 10
b1, b2, eps, lr = 0.9, 0.999, 1e-8, 1e-3
b1t, b2t = torch.tensor(b1, device=dev), torch.tensor(b2, device=dev)
DIAG = ("step", "p_sum", "m_sum", "v_sum", "g_sum", "noise_sum")


class State:
    def __init__(self):
        self.p = (0.1 * torch.randn(N, generator=torch.Generator().manual_seed(1))).to(dev)
        self.m = torch.zeros(N, device=dev)
        self.v = torch.zeros(N, device=dev)
        self.step = torch.zeros(1, dtype=torch.int64, device=dev)
        self.traj = torch.zeros(STEPS + 1, N, device=dev)
        self.traj[0] = self.p
        self.diag = torch.zeros(STEPS + 1, len(DIAG), dtype=torch.float64, device=dev)


def body(s, host_step, gen=None):
    st = (s.step.to(torch.float32) if host_step is None
          else torch.full((1,), float(host_step), device=dev))
    row = (st.to(torch.int64) + 1) if host_step is None else \
        torch.full((1,), host_step + 1, dtype=torch.int64, device=dev)
    rec = [st.double(), s.p.double().sum().reshape(1), s.m.double().sum().reshape(1),
           s.v.double().sum().reshape(1)]
    leaf = s.p.detach().requires_grad_(True)
    noise = None
    with torch.enable_grad():
        if gen is None:
            xs = x
        else:
            noise = torch.randn(x.shape, generator=gen, device=dev)
            xs = x + 0.01 * noise
        z = (edges[None, :] - xs[:, None] - leaf[pop][:, None]) * 2.0
        cdf = 0.5 * (1.0 + torch.erf(z))
        S = (cdf[:, 1:] - cdf[:, :-1]).sum(0)
        loss = ((S - target) ** 2).mean()
        (g,) = torch.autograd.grad(loss, leaf)
    rec.append(g.double().sum().reshape(1))
    rec.append(noise.double().sum().reshape(1) if noise is not None
               else torch.zeros(1, dtype=torch.float64, device=dev))
    s.diag.index_copy_(0, row, torch.cat(rec).reshape(1, -1))
    s.m.mul_(b1).add_(g, alpha=1 - b1)
    s.v.mul_(b2).addcmul_(g, g, value=1 - b2)
    bc1 = 1 - torch.pow(b1t, st + 1)
    bc2 = 1 - torch.pow(b2t, st + 1)
    s.p.sub_(lr * (s.m / bc1) / (torch.sqrt(s.v / bc2) + eps))
    s.traj.index_copy_(0, row, s.p.reshape(1, N))
    if host_step is None:
        s.step.add_(1)


def capture(s, gen=None):
    saved = [t.clone() for t in (s.p, s.m, s.v, s.step, s.traj, s.diag)]
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        body(s, None, gen)
    torch.cuda.current_stream().wait_stream(side)
    for t, v in zip((s.p, s.m, s.v, s.step, s.traj, s.diag), saved):
        t.copy_(v)
    graph = torch.cuda.CUDAGraph()
    if gen is not None:
        graph.register_generator_state(gen)
    with torch.cuda.graph(graph):
        body(s, None, gen)
    return graph


_persist = None


def replay(graph, how):
    global _persist
    if how == "sync_pre":
        torch.cuda.synchronize()
    elif how.startswith("dummy"):
        torch.cuda.current_stream()  # noqa: B018 (the launch below is the point)
        _dummy.add_(1)
    if how == "persist":
        if _persist is None:
            _persist = torch.cuda.Stream()
        _persist.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(_persist):
            graph.replay()
        torch.cuda.current_stream().wait_stream(_persist)
    else:
        graph.replay()


_dummy = torch.zeros(1, device=dev)


def run(schedule, how, keyed):
    if how in ("all_stream", "user_null", "split"):
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            out = run(schedule, {"all_stream": "none", "user_null": "_user_null",
                                 "split": "persist"}[how], keyed)
        torch.cuda.current_stream().wait_stream(st)
        torch.cuda.synchronize()
        return out
    s = State()
    gen = torch.Generator(device=dev) if keyed else None
    graph, prev = None, None
    for k, mode in enumerate(schedule):
        if gen is not None:
            gen.manual_seed(1000 + k)
        if mode == "g":
            if graph is None or prev == "e":
                s.step.fill_(k)
            if graph is None:
                if how == "capture_side":
                    cs = torch.cuda.Stream()
                    cs.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(cs):
                        graph = capture(s, gen)
                    torch.cuda.current_stream().wait_stream(cs)
                else:
                    graph = capture(s, gen)
                if gen is not None:
                    gen.manual_seed(1000 + k)
            replay(graph, how)
        else:
            body(s, k, gen)
        if not how.endswith("_nosync"):
            torch.cuda.synchronize()
        if how == "_user_null":
            with torch.cuda.stream(torch.cuda.default_stream()):
                _dummy.add_(1)
        prev = mode
    torch.cuda.synchronize()
    return s


def report(name, ref, s):
    d = (s.traj - ref.traj).abs().amax(dim=1)
    bad = [i for i in range(d.numel()) if float(d[i]) > 1e-6]
    line = f"{name:34s} max {float(d.max()):.1e} first_bad_row={bad[0] if bad else None}"
    if bad:
        r = bad[0]
        got, want = s.diag[r].tolist(), ref.diag[r].tolist()
        diffs = [f"{n}: {g:.6g} vs {w:.6g}" for n, g, w in zip(DIAG, got, want)
                 if abs(g - w) > 1e-9 * max(1.0, abs(w))]
        line += "  inputs that differ at that row: " + ("; ".join(diffs) or "none")
        # did the wrong replay see an older row's inputs?
        for name_, j in (("p_sum", 1), ("noise_sum", 5)):
            for rr in range(1, ref.diag.shape[0]):
                if rr != r and abs(got[j] - ref.diag[rr, j].item()) <= 1e-9 * max(1.0, abs(got[j])) \
                        and abs(got[j] - want[j]) > 1e-9 * max(1.0, abs(want[j])):
                    line += f"  [{name_} equals eager row {rr}'s]"
                    break
    print(line, flush=True)


ref = run("e" * STEPS, "none", False)
refk = run("e" * STEPS, "none", True)
HOWS = ("none", "none_nosync", "sync_pre", "dummy", "dummy_nosync", "persist", "all_stream",
        "user_null", "split", "capture_side")
for how in HOWS:
    report(f"A eeeeeggggggeeeeegggg {how}", ref, run("eeeeeggggggeeeeegggg", how, False))
for how in HOWS:
    report(f"B gggggggggggggggggggg {how}", refk, run("g" * STEPS, how, True))
