"""Resumable optimizer checkpoints (new: the reference persists no optimizer state,
SURVEY §5.4).

Files are plain ``torch.save`` dictionaries of tensors and Python scalars written
atomically by rank 0 (``tmp`` + ``os.replace``) and loaded with ``weights_only=True``, so
loading executes nothing from the file.  Sharded optimizer state (ZeRO-style engine) is
written one file per rank with a ``.rank<r>`` suffix.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

__all__ = ["save_optimizer_state", "load_optimizer_state", "shard_path"]


def shard_path(path: str, rank: int) -> str:
    return f"{path}.rank{rank}"


def save_optimizer_state(path: str, state: dict, comm=None, sharded: bool = False) -> None:
    rank = 0 if comm is None else comm.rank
    if sharded:
        path = shard_path(path, rank)
    elif rank != 0:
        if comm is not None:
            comm.barrier()
        return
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = f"{path}.tmp{os.getpid()}"
    torch.save(state, tmp)
    os.replace(tmp, path)
    if comm is not None and not sharded:
        comm.barrier()


def load_optimizer_state(path: str, map_location="cpu", rank: Optional[int] = None,
                         sharded: bool = False) -> dict:
    if sharded:
        path = shard_path(path, 0 if rank is None else rank)
    return torch.load(path, map_location=map_location, weights_only=True)
