"""Distributed debugging aids.

* ``check_consistent(tensor, comm)`` -- assert a replicated tensor is bitwise identical
  on every rank (hash all-gather); the SPMD optimizers keep parameters identical by
  construction, this verifies it (``MULTIGRAD_CHECK_EVERY=k`` in the drivers).
* ``CollectiveFingerprint`` -- wraps a communicator and all-gathers an
  ``(op, shape, dtype, seq)`` fingerprint before every collective, raising on the first
  mismatch instead of hanging (the classic "ranks disagree on the collective sequence"
  bug, e.g. a rank-dependent LHS draw -- reference quirk Q8).
* ``abort_on_error(comm)`` -- context manager that destroys the process group when an
  exception escapes, so peers fail fast instead of blocking in a collective.
"""
from __future__ import annotations

import contextlib
import hashlib

import numpy as np
import torch

__all__ = ["tensor_digest", "check_consistent", "CollectiveFingerprint", "abort_on_error",
           "CollectiveMismatch"]


class CollectiveMismatch(RuntimeError):
    pass


def tensor_digest(t: torch.Tensor) -> str:
    a = t.detach().contiguous().cpu()
    return hashlib.sha1(a.view(torch.uint8).numpy().tobytes() if a.numel() else b"").hexdigest()


def check_consistent(t: torch.Tensor, comm, what: str = "tensor") -> None:
    if comm is None or comm.size == 1:
        return
    digests = comm.allgather(tensor_digest(t))
    if len(set(digests)) != 1:
        raise CollectiveMismatch(f"{what} differs across ranks: {digests}")


class CollectiveFingerprint:
    """Communicator proxy that cross-checks every collective's signature."""

    _CHECKED = {"all_reduce", "reduce", "broadcast", "all_gather_into_tensor",
                "reduce_scatter_tensor", "bcast", "allgather", "barrier", "split"}

    def __init__(self, comm):
        self._comm = comm
        self._seq = 0

    def __getattr__(self, name):
        attr = getattr(self._comm, name)
        if name not in self._CHECKED or not callable(attr):
            return attr

        def wrapped(*args, **kw):
            t = next((a for a in args if isinstance(a, torch.Tensor)), None)
            sig = (name, self._seq, None if t is None else (tuple(t.shape), str(t.dtype)))
            self._seq += 1
            sigs = self._comm.allgather(sig)
            if any(s != sigs[0] for s in sigs):
                raise CollectiveMismatch(f"collective #{sig[1]} mismatch across ranks: {sigs}")
            return attr(*args, **kw)

        return wrapped


@contextlib.contextmanager
def abort_on_error(comm=None):
    try:
        yield
    except BaseException:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass
        raise
