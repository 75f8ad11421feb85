"""Narrowing probe for tools/dbg/torch_replay_repro.py case A (torch only): per step, which
state tensor first leaves the eager reference, and whether a host synchronisation between
the step-counter fill and the replay changes the outcome."""
import importlib.util
import os
import sys

import torch

spec = importlib.util.spec_from_file_location(
    "rep", os.path.join(os.path.dirname(os.path.abspath(__file__)), "torch_replay_repro.py"))
src = open(spec.origin).read().split("\nref = run(")[0]  # definitions only
rep = {}
exec(compile(src, spec.origin, "exec"), rep)
State, body, capture, STEPS = rep["State"], rep["body"], rep["capture"], rep["STEPS"]


def run(schedule, sync, sync_before_replay=False, snap=True):
    s = State()
    graph, prev, snaps = None, None, []
    for k, mode in enumerate(schedule):
        if mode == "g":
            if graph is None or prev == "e":
                s.step.fill_(k)
                if sync_before_replay:
                    torch.cuda.synchronize()
            if graph is None:
                graph = capture(s)
            graph.replay()
        else:
            body(s, k)
        if sync:
            torch.cuda.synchronize()
        if snap:
            snaps.append([t.clone() for t in (s.p, s.m, s.v, s.step)])
        prev = mode
    torch.cuda.synchronize()
    return snaps


ref = run("e" * STEPS, False)
for sched, sync, sbr in (("eeeeeggggggeeeeegggg", True, False), ("eeeeeggggggeeeeegggg", True, True),
                         ("eeeeeggggggeeeeegggg", False, False), ("ggggggggggeeeeegggg", True, False)):
    out = run(sched, sync, sbr)
    first = None
    for k, (a, b) in enumerate(zip(out, ref)):
        d = [float((x - y).abs().max()) for x, y in zip(a[:3], b[:3])]
        if max(d) > 1e-6 and first is None:
            first = (k, sched[k], ["%.1e" % v for v in d], int(a[3]), int(b[3]) if sched[k] == "g" else None)
    print(f"{sched} sync={sync} sync_before_replay={sbr}: first deviating step {first}", flush=True)
