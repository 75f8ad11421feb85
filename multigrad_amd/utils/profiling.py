"""Phase timing with HIP events (``MULTIGRAD_PROFILE=1``) and torch.profiler hooks.

``PhaseTimer`` records start/stop events per named phase on the current stream without
host synchronisation; ``summary()`` synchronises once and returns mean milliseconds per
phase.  Kernel-level profiles come from ``rocprofv3 --kernel-trace --stats`` (see
``tools/profile_bench.sh``); ``torch_profile(...)`` wraps ``torch.profiler`` for
operator-level traces.
"""
from __future__ import annotations

import collections
import contextlib
import os
import time

import torch

__all__ = ["PhaseTimer", "profiling_enabled", "torch_profile"]


def profiling_enabled() -> bool:
    return os.environ.get("MULTIGRAD_PROFILE", "0").lower() in ("1", "true", "on", "yes")


class PhaseTimer:
    def __init__(self, enabled=None):
        self.enabled = profiling_enabled() if enabled is None else bool(enabled)
        self._ev = collections.defaultdict(list)
        self._cpu = collections.defaultdict(list)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            yield
            b.record()
            self._ev[name].append((a, b))
        else:
            t = time.perf_counter()
            yield
            self._cpu[name].append(1e3 * (time.perf_counter() - t))

    def summary(self) -> dict:
        out = {}
        if self._ev:
            torch.cuda.synchronize()
        for k, v in self._ev.items():
            out[k] = sum(a.elapsed_time(b) for a, b in v) / len(v)
        for k, v in self._cpu.items():
            out[k] = sum(v) / len(v)
        return out


@contextlib.contextmanager
def torch_profile(path: str = "gpurun_out/torch_trace.json", **kw):
    """``torch.profiler`` trace of the enclosed region, exported as a Chrome trace."""
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts, **kw) as prof:
        yield prof
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    prof.export_chrome_trace(path)


def count_device_ops(fn, reps: int = 2) -> dict:
    """Device operations per call of ``fn`` (kernels, copies, fills), counted with
    ``torch.profiler`` over ``reps`` calls -- graph replays included, since the tracer sees
    each dispatched kernel.  Returns ``{"kernels": k, "memcpy": c, "memset": s}`` per call,
    or ``{}`` when the profiler cannot trace the device."""
    if not torch.cuda.is_available():
        return {}
    torch.cuda.synchronize()
    try:
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
        counts = collections.Counter()
        for e in prof.events():
            if e.device_type != torch.autograd.DeviceType.CUDA:
                continue
            name = e.name.lower()
            kind = ("memcpy" if "memcpy" in name or "copy" in name and "kernel" not in name
                    else "memset" if "memset" in name or "fill_buffer" in name else "kernels")
            counts[kind] += 1
    except Exception:  # noqa: BLE001 -- a tracer problem must not fail the caller
        return {}
    return {k: round(counts[k] / reps, 2) for k in ("kernels", "memcpy", "memset")}
