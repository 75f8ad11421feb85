"""Per-step driver hooks: the aux subsystems of SURVEY §5.2/§5.3/§5.5 wired into the
optimizer loops -- Adam, the fused and generic engines, simple GD, in-graph GD (eager
steps), device L-BFGS and device L-BFGS-B (metrics also on the root of the scipy
L-BFGS-B; its workers run no loop of their own).

Environment knobs (read when a driver starts):

``MULTIGRAD_CHECK_EVERY=k``
    every k steps, all-gather a digest of the replicated parameters and raise
    :class:`~multigrad_amd.utils.debug.CollectiveMismatch` unless every rank holds the
    same bits (the SPMD optimizers keep them identical by construction; this verifies it).
``MULTIGRAD_METRICS=path``
    append one JSON record per step to ``path`` on rank 0: step, loss, step time, and
    what the driver knows besides -- the gradient norm (generic Adam), the bytes this
    rank sent through collectives in the step and the resulting effective rate
    (``comm_bytes``, ``comm_GBps``: the engines).
``MULTIGRAD_METRICS_EVERY=k``
    log every k-th step only (default 1).

The reference's only guard is ``ValueError`` on an unknown command
(multigrad/adam.py:125-126, multigrad/bfgs.py:105-106).
"""
from __future__ import annotations

import contextlib
import os
from typing import Callable, Optional

__all__ = ["StepHooks", "driver_guard"]


def _int_env(name: str, default: int = 0) -> int:
    try:
        return int(os.environ.get(name, default) or default)
    except ValueError:
        return default


class StepHooks:
    """``hooks(step, loss, state, params_fn)`` after every optimizer step.

    ``params_fn`` returns the replicated parameter tensor to verify (called only on a
    check step, so a sharded engine can assemble it lazily)."""

    def __init__(self, comm=None, callback: Optional[Callable] = None, what: str = "params"):
        from .metrics import metrics_callback
        self.comm = comm
        self.callback = callback
        self.what = what
        self.check_every = _int_env("MULTIGRAD_CHECK_EVERY")
        self.metrics = metrics_callback(comm=comm, every=max(1, _int_env("MULTIGRAD_METRICS_EVERY", 1)))
        self.n_checks = 0

    @property
    def active(self) -> bool:
        return bool(self.callback or self.metrics or self.check_every)

    def __call__(self, step: int, loss, state=None, params_fn: Optional[Callable] = None,
                 **extra) -> None:
        """``extra``: additional metrics fields (values or zero-argument callables, which
        are only evaluated when a metrics record is written)."""
        if self.callback is not None:
            self.callback(step, loss, state)
        if self.metrics is not None:
            self.metrics(step, loss, state,
                         **{k: (v() if callable(v) else v) for k, v in extra.items()})
        if self.check_every and params_fn is not None and (step + 1) % self.check_every == 0:
            from .debug import check_consistent
            check_consistent(params_fn(), self.comm, f"{self.what} after step {step}")
            self.n_checks += 1


@contextlib.contextmanager
def driver_guard(comm=None):
    """Fail fast across ranks: an exception escaping an optimizer loop on a multi-rank
    communicator tears the process group down (``abort_on_error``) so the peers error
    out of their next collective instead of blocking until the process-group timeout."""
    if comm is None or getattr(comm, "size", 1) == 1:
        yield
        return
    from .debug import abort_on_error
    with abort_on_error(comm):
        yield
