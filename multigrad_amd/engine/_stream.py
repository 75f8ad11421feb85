"""The engines' own HIP stream.

Every public method of :class:`~multigrad_amd.engine.fused.FusedAdamEngine` and
:class:`~multigrad_amd.engine.generic.GraphAdamEngine` runs its GPU work -- eager launches,
graph captures and replays, collectives, and the user hooks and callbacks it calls -- on
a stream of the engine's own, never on the legacy default stream.

Why: on this ROCm runtime a graph replay that follows a host synchronisation AND any
launch on the default stream since the graph's previous replay computes garbage in the
graph's intermediates (its inputs read right), while the same schedules with nothing
launched on the default stream match eager launches bit for bit.  Reproduced with torch
alone (tools/dbg/torch_replay_repro.py, tools/dbg/torch_replay_bisect.py; the cases and
logs are in docs/design.md "Graph replays and the default stream" and
profiles/replay_anomaly/).

The engine stream is ordered after the caller's current stream on entry and before it on
exit with events (an event record / wait on the caller's stream is not a launch and does
not trigger the defect: case "persist" of the bisection).  Tensors handed back to the
caller are marked as used on the caller's stream (``record_stream``) so the caching
allocator does not give their memory to later engine work too early.
"""
from __future__ import annotations

import functools

import torch

__all__ = ["EngineStream", "on_engine_stream"]


class EngineStream:
    """Context: the current stream becomes ``owner._engine_stream()`` (a no-op when that is
    None, i.e. on the CPU, or when it is already current, i.e. nested engine calls).

    ``always=False``: only while the owner may replay graphs (``owner._stream_wanted()``).
    An engine that runs eager launches only keeps them on the caller's stream: it replays no
    graph, and entering the engine stream costs a cross-queue event round trip per call:
    direct ``step()`` calls on the owner-shard proxy measured 86-90 us/step of wall time and
    49-54 us of host time with it, 64-67 and 19-21 us without (`tools/host_step_cost.py`)."""

    def __init__(self, owner, always: bool = True):
        self.owner = owner
        self.always = always
        self._ctx = None
        self._cur = None
        self._es = None

    def __enter__(self):
        if not self.always and not self.owner._stream_wanted():
            return None
        es = self.owner._engine_stream()
        if es is None:
            return None
        cur = torch.cuda.current_stream(es.device)
        if cur == es:
            return es
        es.wait_stream(cur)
        self._cur, self._es = cur, es
        self._ctx = torch.cuda.stream(es)
        self._ctx.__enter__()
        return es

    def __exit__(self, *exc):
        if self._ctx is not None:
            self._ctx.__exit__(*exc)
            self._cur.wait_stream(self._es)
            self._ctx = None
        return False

    def hand_over(self, out) -> None:
        """Record the caller's stream on the CUDA tensors in ``out`` (a tensor, or lists /
        tuples / dicts of them, e.g. a GradDescentResult)."""
        if self._ctx is None:
            return
        todo, seen = [out], set()
        while todo:
            o = todo.pop()
            if id(o) in seen:
                continue
            seen.add(id(o))
            if isinstance(o, torch.Tensor):
                if o.is_cuda:
                    o.record_stream(self._cur)
            elif isinstance(o, (list, tuple)):
                todo.extend(o)
            elif isinstance(o, dict):
                todo.extend(o.values())


def on_engine_stream(fn=None, *, always: bool = False):
    """Decorator: run an engine method inside :class:`EngineStream` of its engine --
    whenever the engine may replay graphs, or (``always=True``: setup and the run drivers,
    which capture and time graphs themselves) on every call."""
    def deco(f):
        @functools.wraps(f)
        def wrapper(self, *args, **kw):
            ctx = EngineStream(self, always=always)
            with ctx:
                out = f(self, *args, **kw)
                ctx.hand_over(out)
            return out
        return wrapper
    return deco(fn) if fn is not None else deco


def make_engine_stream(current, device):
    """The engine stream for ``device`` (``current``: the engine's stream so far, reused
    when it is on that device); None off the GPU."""
    dev = torch.device(device)
    if dev.type != "cuda":
        return None
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    if current is not None and current.device == dev:
        return current
    return torch.cuda.Stream(device=dev)
