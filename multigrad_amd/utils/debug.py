"""Distributed debugging aids.

* ``check_consistent(tensor, comm)`` -- assert a replicated tensor is bitwise identical
  on every rank (hash all-gather); the SPMD optimizers keep parameters identical by
  construction, this verifies it (``MULTIGRAD_CHECK_EVERY=k`` in every optimizer loop, utils/hooks.py).
* ``CollectiveFingerprint`` -- wraps a communicator and all-gathers an
  ``(op, shape, dtype, seq)`` fingerprint before every collective, raising on the first
  mismatch instead of hanging (the classic "ranks disagree on the collective sequence"
  bug, e.g. a rank-dependent LHS draw -- reference quirk Q8); ``MULTIGRAD_FINGERPRINT=1``
  wraps the world communicator.
* ``abort_on_error(comm)`` -- context manager that destroys the process group when an
  exception escapes, so peers fail fast instead of blocking in a collective.
"""
from __future__ import annotations

import contextlib
import hashlib

import os

import torch

from ..parallel.comm import Comm

__all__ = ["tensor_digest", "check_consistent", "CollectiveFingerprint", "abort_on_error",
           "CollectiveMismatch", "maybe_fingerprint"]


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


def _fingerprinted(name):
    def method(self, *args, **kw):
        t = next((a for a in list(args) + list(kw.values()) if isinstance(a, torch.Tensor)), None)
        sig = (name, self._seq, None if t is None else (tuple(t.shape), str(t.dtype)))
        self._seq += 1
        sigs = self._comm.allgather(sig)
        if any(s != sigs[0] for s in sigs):
            raise CollectiveMismatch(f"collective #{sig[1]} mismatch across ranks: {sigs}")
        out = getattr(self._comm, name)(*args, **kw)
        if name == "split" and out is not None:
            out = CollectiveFingerprint(out)
        return out
    method.__name__ = name
    return method


class CollectiveFingerprint(Comm):
    """Communicator proxy that cross-checks every collective's signature
    ``(op, sequence number, shape, dtype)`` with an all-gather before running it, so
    ranks that disagree on the collective sequence raise :class:`CollectiveMismatch`
    instead of hanging or silently mixing buffers.  ``MULTIGRAD_FINGERPRINT=1`` wraps
    the world communicator (and every communicator split from it)."""

    _CHECKED = ("all_reduce", "reduce", "broadcast", "all_gather_into_tensor",
                "reduce_scatter_tensor", "bcast", "allgather", "barrier", "split", "scatter",
                "all_to_all_v")

    def __init__(self, comm):
        object.__setattr__(self, "_comm", comm)
        object.__setattr__(self, "_seq", 0)

    rank = property(lambda self: self._comm.rank)
    size = property(lambda self: self._comm.size)
    uid = property(lambda self: self._comm.uid)
    global_ranks = property(lambda self: self._comm.global_ranks)

    @property
    def name(self):
        return self._comm.name

    @name.setter
    def name(self, v):
        self._comm.name = v

    def send(self, obj, dest, tag=0):
        return self._comm.send(obj, dest, tag)

    def recv(self, buf=None, source=0, tag=0):
        return self._comm.recv(buf, source, tag)

    def __getattr__(self, name):
        return getattr(object.__getattribute__(self, "_comm"), name)

    def __setattr__(self, name, value):
        if name == "_seq":
            object.__setattr__(self, name, value)
        else:
            setattr(self._comm, name, value)


for _n in CollectiveFingerprint._CHECKED:
    setattr(CollectiveFingerprint, _n, _fingerprinted(_n))


def maybe_fingerprint(comm):
    """Wrap ``comm`` in :class:`CollectiveFingerprint` when ``MULTIGRAD_FINGERPRINT`` is set."""
    if comm is None or isinstance(comm, CollectiveFingerprint):
        return comm
    if os.environ.get("MULTIGRAD_FINGERPRINT", "0").lower() in ("", "0", "false", "off", "no"):
        return comm
    return CollectiveFingerprint(comm)


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
