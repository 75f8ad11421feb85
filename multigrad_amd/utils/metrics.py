"""Structured per-step metrics (JSONL sink, rank 0) -- SURVEY §5.5.

``MetricsLogger(path)`` appends one JSON object per record; set ``MULTIGRAD_METRICS`` to
a path to have the optimizers' ``callback`` hook log loss / step time automatically via
:func:`metrics_callback`.
"""
from __future__ import annotations

import json
import os
import time
from typing import Optional

import torch

__all__ = ["MetricsLogger", "metrics_callback"]


class MetricsLogger:
    def __init__(self, path: str, comm=None, every: int = 1):
        self.path = path
        self.rank = 0 if comm is None else comm.rank
        self.every = max(1, int(every))
        self._t = time.perf_counter()
        if self.rank == 0:
            d = os.path.dirname(os.path.abspath(path))
            os.makedirs(d, exist_ok=True)

    def log(self, **rec) -> None:
        if self.rank != 0:
            return
        rec.setdefault("time", time.time())
        with open(self.path, "a") as f:
            f.write(json.dumps({k: _jsonable(v) for k, v in rec.items()}) + "\n")

    def step(self, step: int, loss=None, **extra) -> None:
        if step % self.every:
            return
        lossf = None if loss is None else float(torch.as_tensor(loss).reshape(-1)[0])  # syncs
        now = time.perf_counter()
        dt, self._t = now - self._t, now
        per = dt / self.every
        if extra.get("comm_bytes") and per > 0:
            extra["comm_GBps"] = float(f"{float(extra['comm_bytes']) / per / 1e9:.4g}")
        self.log(step=step, loss=lossf, step_time_s=per, **extra)


def _jsonable(v):
    if isinstance(v, torch.Tensor):
        return v.detach().cpu().tolist()
    if hasattr(v, "tolist"):
        return v.tolist()
    return v


def metrics_callback(path: Optional[str] = None, comm=None, every: int = 1):
    """An optimizer ``callback(step, loss, state)`` that writes JSONL records."""
    path = path or os.environ.get("MULTIGRAD_METRICS")
    if not path:
        return None
    logger = MetricsLogger(path, comm=comm, every=every)

    def cb(step, loss, state=None, **extra):
        logger.step(step, loss, **extra)

    return cb
