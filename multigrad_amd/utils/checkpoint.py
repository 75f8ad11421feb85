"""Resumable optimizer checkpoints (new: the reference persists no optimizer state,
SURVEY §5.4).

Files are plain ``torch.save`` dictionaries of tensors and Python scalars written
atomically (``tmp`` + ``os.replace``) and loaded with ``weights_only=True``, so loading
executes nothing from the file.

Sharded optimizer state (owner / ZeRO engine) is written one file per rank with a
``.rank<r>`` suffix, then committed: after every rank's shard is on disk (barrier) rank 0
atomically writes ``<path>.manifest.json`` holding the step and the number of ranks.  A
crash between the shard writes and the manifest leaves the previous manifest in place,
so :func:`load_optimizer_state` refuses a shard whose step disagrees with the manifest,
and :func:`check_loaded_step` verifies collectively that every rank resumes from the
same step (otherwise the ranks' collectives would no longer line up).
"""
from __future__ import annotations

import json
import os
from typing import Optional

import torch

__all__ = ["save_optimizer_state", "load_optimizer_state", "shard_path", "manifest_path",
           "check_loaded_step", "CheckpointMismatch"]


class CheckpointMismatch(RuntimeError):
    pass


def shard_path(path: str, rank: int) -> str:
    return f"{path}.rank{rank}"


def manifest_path(path: str) -> str:
    return f"{path}.manifest.json"


def _atomic_write(path: str, write) -> None:
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = f"{path}.tmp{os.getpid()}"
    write(tmp)
    os.replace(tmp, path)


def save_optimizer_state(path: str, state: dict, comm=None, sharded: bool = False) -> None:
    rank = 0 if comm is None else comm.rank
    size = 1 if comm is None else comm.size
    if sharded:
        _atomic_write(shard_path(path, rank), lambda t: torch.save(state, t))
        if comm is not None:
            comm.barrier()  # every shard is on disk before the manifest commits them
        if rank == 0:
            man = {"step": int(state.get("step", -1)), "size": size, "sharded": True}
            _atomic_write(manifest_path(path),
                          lambda t: open(t, "w").write(json.dumps(man)))
        if comm is not None:
            comm.barrier()
        return
    if rank == 0:
        _atomic_write(path, lambda t: torch.save(state, t))
    if comm is not None:
        comm.barrier()


def load_optimizer_state(path: str, map_location="cpu", rank: Optional[int] = None,
                         sharded: bool = False) -> dict:
    if not sharded:
        return torch.load(path, map_location=map_location, weights_only=True)
    st = torch.load(shard_path(path, 0 if rank is None else rank), map_location=map_location,
                    weights_only=True)
    mp = manifest_path(path)
    if not os.path.exists(mp):
        raise CheckpointMismatch(f"{mp} missing: the sharded checkpoint was never committed")
    with open(mp) as f:
        man = json.load(f)
    if int(st.get("step", -1)) != int(man["step"]):
        raise CheckpointMismatch(
            f"shard {shard_path(path, rank or 0)} holds step {st.get('step')} but the "
            f"manifest commits step {man['step']} (interrupted checkpoint write)")
    if "size" in st and int(st["size"]) != int(man["size"]):
        raise CheckpointMismatch(f"shard written by {st['size']} ranks, manifest says "
                                 f"{man['size']}")
    return st


def check_loaded_step(step: int, comm) -> None:
    """Collective: raise on every rank unless all ranks resume from the same step."""
    if comm is None or comm.size == 1:
        return
    t = torch.tensor([int(step), -int(step)], dtype=torch.int64)
    comm.all_reduce(t, op="max")
    if int(t[0]) != -int(t[1]):
        raise CheckpointMismatch(f"ranks resume from different steps ({-int(t[1])}..{int(t[0])})")
