"""Resumable optimizer checkpoints (new: the reference persists no optimizer state,
SURVEY §5.4).

Files are plain ``torch.save`` dictionaries of tensors and Python scalars written
atomically (``tmp`` + ``os.replace``) and loaded with ``weights_only=True``, so loading
executes nothing from the file.

Sharded optimizer state (owner / ZeRO engine) is written one file per rank, named by the
step: ``<path>.step<k>.rank<r>``.  After every rank's shard is on disk (barrier) rank 0
atomically writes ``<path>.manifest.json`` naming the committed step, the number of ranks
and the shard pattern; only then (second barrier) does each rank delete its shards of
older steps.  A crash anywhere in a save therefore leaves the previous checkpoint complete
and committed: its shards are never overwritten, and the manifest still names them.

Loading reads the manifest first and the shards it names.  With a communicator the
verdict is collective: every rank reports whether its shard loaded and agrees with the
manifest, and if any rank failed, every rank raises :class:`CheckpointMismatch` (no rank is
left waiting in a later collective for a peer that gave up).
"""
from __future__ import annotations

import glob
import json
import os
import re
from typing import Optional

import torch

__all__ = ["save_optimizer_state", "load_optimizer_state", "shard_path", "manifest_path",
           "check_loaded_step", "CheckpointMismatch"]


class CheckpointMismatch(RuntimeError):
    pass


def shard_path(path: str, rank: int, step: Optional[int] = None) -> str:
    """Shard file of ``rank``; ``step=None`` is the pre-round-3 unversioned name."""
    if step is None:
        return f"{path}.rank{rank}"
    return f"{path}.step{int(step)}.rank{rank}"


def manifest_path(path: str) -> str:
    return f"{path}.manifest.json"


def _atomic_write(path: str, write) -> None:
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = f"{path}.tmp{os.getpid()}"
    write(tmp)
    os.replace(tmp, path)


def _write_json(obj):
    def w(t):
        with open(t, "w") as f:
            f.write(json.dumps(obj))
    return w


def _old_shards(path: str, rank: int, keep_step: int):
    pat = re.compile(re.escape(os.path.basename(path)) + r"\.step(\d+)\.rank" + str(rank) + "$")
    for f in glob.glob(f"{glob.escape(path)}.step*.rank{rank}"):
        m = pat.search(os.path.basename(f))
        if m and int(m.group(1)) != keep_step:
            yield f
    legacy = shard_path(path, rank)
    if os.path.exists(legacy):
        yield legacy


def save_optimizer_state(path: str, state: dict, comm=None, sharded: bool = False) -> None:
    rank = 0 if comm is None else comm.rank
    size = 1 if comm is None else comm.size
    if sharded:
        step = int(state.get("step", -1))
        _atomic_write(shard_path(path, rank, step), lambda t: torch.save(state, t))
        if comm is not None:
            comm.barrier()  # every shard is on disk before the manifest commits them
        if rank == 0:
            _atomic_write(manifest_path(path), _write_json(
                {"step": step, "size": size, "sharded": True,
                 "shards": os.path.basename(path) + f".step{step}.rank{{rank}}"}))
        if comm is not None:
            comm.barrier()  # committed everywhere: the previous step's shards can go
        for f in _old_shards(path, rank, step):
            try:
                os.remove(f)
            except OSError:
                pass
        return
    if rank == 0:
        _atomic_write(path, lambda t: torch.save(state, t))
    if comm is not None:
        comm.barrier()


def _load_shard(path: str, rank: int, map_location) -> dict:
    mp = manifest_path(path)
    if not os.path.exists(mp):
        raise CheckpointMismatch(f"{mp} missing: the sharded checkpoint was never committed")
    with open(mp) as f:
        man = json.load(f)
    if "shards" in man:
        fn = os.path.join(os.path.dirname(os.path.abspath(path)),
                          man["shards"].format(rank=rank))
    else:  # a manifest from before step-named shards
        fn = shard_path(path, rank)
    if not os.path.exists(fn):
        raise CheckpointMismatch(f"shard {fn} named by {mp} is missing")
    st = torch.load(fn, map_location=map_location, weights_only=True)
    if int(st.get("step", -1)) != int(man["step"]):
        raise CheckpointMismatch(
            f"shard {fn} holds step {st.get('step')} but the manifest commits step "
            f"{man['step']} (interrupted checkpoint write)")
    if "size" in st and int(st["size"]) != int(man["size"]):
        raise CheckpointMismatch(f"shard written by {st['size']} ranks, manifest says "
                                 f"{man['size']}")
    return st


def load_optimizer_state(path: str, map_location="cpu", rank: Optional[int] = None,
                         sharded: bool = False, comm=None) -> dict:
    """Load a checkpoint written by :func:`save_optimizer_state`.  ``comm`` (sharded
    state): the verdict is collective -- if any rank's shard is missing or disagrees with
    the manifest, every rank raises :class:`CheckpointMismatch`."""
    if not sharded:
        return torch.load(path, map_location=map_location, weights_only=True)
    r = (comm.rank if comm is not None else 0) if rank is None else rank
    st, err = None, None
    try:
        st = _load_shard(path, r, map_location)
    except Exception as exc:  # noqa: BLE001 -- every failure must reach the collective
        # verdict (an unpickling error, EOFError of a truncated file, KeyError of a broken
        # manifest ...): a rank that raised here alone would leave its peers in allgather
        err = f"{type(exc).__name__}: {exc}"
    if comm is not None and comm.size > 1:
        errs = comm.allgather(err)
        bad = [(i, e) for i, e in enumerate(errs) if e is not None]
        if bad:
            raise CheckpointMismatch(f"checkpoint {path} unusable on rank(s) "
                                     f"{[i for i, _ in bad]}: rank {bad[0][0]}: {bad[0][1]}")
    elif err is not None:
        raise CheckpointMismatch(err)
    return st


def check_loaded_step(step: int, comm) -> None:
    """Collective: raise on every rank unless all ranks resume from the same step."""
    if comm is None or comm.size == 1:
        return
    t = torch.tensor([int(step), -int(step)], dtype=torch.int64)
    comm.all_reduce(t, op="max")
    if int(t[0]) != -int(t[1]):
        raise CheckpointMismatch(f"ranks resume from different steps ({-int(t[1])}..{int(t[0])})")
