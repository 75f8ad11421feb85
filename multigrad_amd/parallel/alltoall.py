"""All-to-all-v of device (or host) rows: ``Comm.all_to_all_v``.

Used once per fit, at engine setup, to move every data point of an arbitrary
data-parallel shard (the reference's ``np.array_split(...)[rank]``,
tests/smf_example/smf_grad_descent.py:28) to the rank that owns its parameters
(:func:`multigrad_amd.models.population.repartition_by_owner`).  After that the per-step
collective of a population model is the 10-float sumstat all-reduce instead of the
P-float gradient all-reduce of reference multigrad/multigrad.py:531-532.

Paths, chosen collectively (every rank takes the same branch):

* **peer memory** (device tensors, 2..8 ranks, ``MULTIGRAD_ALLTOALL`` auto/peer): every rank
  exports an uncached region holding its send rows packed by destination, the IPC handles
  and the count matrix go over the object channel once, and each rank pulls its W-1
  incoming segments at once over the W-1 xGMI links (``csrc/xgmi.hip:xgmi_a2a_pull_kernel``).
  A ring would push every byte through one link per hop.  Each segment carries a
  position-weighted checksum computed by its sender; a mismatch on any rank rejects the
  result on every rank and the exchange is redone on RCCL (``status(comm)['all-to-all']``
  records which path ran and why).
* **RCCL** ``alltoall_base`` on the device tensors (one process per GPU).
* **gloo** ``alltoall_base`` on host tensors (CPU tests; device tensors staged through host
  when no device backend exists, e.g. several ranks sharing one GPU).

Rows are the first dimension; any dtype whose row size is a multiple of 4 bytes moves
bit-exactly (the data are copied, never reduced).
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import torch

__all__ = ["all_to_all_v", "exchange_counts", "alltoall_mode", "segment_checksums"]


def alltoall_mode() -> str:
    """``MULTIGRAD_ALLTOALL``: ``auto`` (default: peer memory when it is available, else
    RCCL / gloo), ``peer`` (same, named explicitly), ``rccl`` (never peer memory)."""
    m = os.environ.get("MULTIGRAD_ALLTOALL", "auto").strip().lower()
    return m if m in ("auto", "peer", "rccl") else "auto"


def exchange_counts(comm, send_counts: Sequence[int]) -> List[List[int]]:
    """Collective: the full ``[src][dst]`` row-count matrix (one object all-gather)."""
    sc = [int(c) for c in send_counts]
    if len(sc) != comm.size:
        raise ValueError(f"all_to_all_v: {len(sc)} send counts for {comm.size} ranks")
    if any(c < 0 for c in sc):
        raise ValueError("all_to_all_v: negative send count")
    return [list(r) for r in comm.allgather(sc)] if comm.size > 1 else [sc]


def _words(t: torch.Tensor) -> torch.Tensor:
    """Flat 32-bit word view of a contiguous tensor (row bytes a multiple of 4)."""
    flat = t.contiguous().reshape(-1)
    if flat.numel() == 0:
        return torch.zeros(0, dtype=torch.int32, device=t.device)
    return flat.view(torch.uint8).view(torch.int32)


_CK_CHUNK = 1 << 24


def segment_checksums(words: torch.Tensor, counts: Sequence[int]) -> List[int]:
    """Per segment of consecutive ``counts`` words: ``sum_i w_i * (1 + i mod 8191)`` in int64
    (wrapping), ``i`` relative to the segment start -- a lost, stale or shifted word changes
    it.  Computed where ``words`` lives (chunks of 2^24 words)."""
    out, off = [], 0
    for n in counts:
        n = int(n)
        s = torch.zeros((), dtype=torch.int64, device=words.device)
        for a in range(0, n, _CK_CHUNK):
            b = min(n, a + _CK_CHUNK)
            w = words[off + a:off + b].to(torch.int64)
            wt = torch.remainder(torch.arange(a, b, dtype=torch.int64, device=words.device), 8191) + 1
            s += (w * wt).sum()
        out.append(s)
        off += n
    return [int(v) for v in (torch.stack(out).cpu().tolist() if out else [])]


def _record(comm, **info) -> None:
    from .xgmi import _record as rec
    rec(comm, "all-to-all", **info)


def all_to_all_v(comm, tensor: torch.Tensor, send_counts: Sequence[int],
                 counts: Optional[List[List[int]]] = None) -> Tuple[torch.Tensor, List[int]]:
    """Collective: rows ``tensor[sdispl[d] : sdispl[d] + send_counts[d]]`` go to rank ``d``;
    returns ``(received rows concatenated in source-rank order, recv_counts)``.
    ``counts``: the ``[src][dst]`` matrix when the caller already has it (else one object
    all-gather builds it)."""
    sc = [int(c) for c in send_counts]
    if sum(sc) != tensor.shape[0]:
        raise ValueError(f"all_to_all_v: send counts sum to {sum(sc)}, tensor has "
                         f"{tensor.shape[0]} rows")
    if comm is None or comm.size == 1:
        return tensor.clone(), sc
    C = exchange_counts(comm, sc) if counts is None else counts
    rc = [C[q][comm.rank] for q in range(comm.size)]
    row_shape = tuple(tensor.shape[1:])
    out = torch.empty((sum(rc),) + row_shape, dtype=tensor.dtype, device=tensor.device)
    row_bytes = tensor[:1].numel() * tensor.element_size() if tensor.shape[0] else \
        int(torch.Size(row_shape).numel()) * tensor.element_size()
    if tensor.is_cuda and alltoall_mode() != "rccl" and row_bytes % 4 == 0:
        from .xgmi import MAX_RANKS
        if comm.size <= MAX_RANKS and _peer(comm, tensor, out, C, row_bytes // 4):
            return out, rc
    # the backends move bytes: any dtype (gloo has no int16 / bool all-to-all) and row shape
    src = tensor.contiguous().reshape(-1).view(torch.uint8).reshape(tensor.shape[0], row_bytes)
    dst = out.reshape(-1).view(torch.uint8).reshape(out.shape[0], row_bytes)
    path = comm._all_to_all_base(dst, src, rc, sc)
    if tensor.is_cuda:
        _record(comm, ok=True, path=path, rows=int(tensor.shape[0]), fallback=None)
    return out, rc


def _peer(comm, tensor, out, C, wpr: int) -> bool:
    """The peer-memory path (see the module docstring); False when any rank cannot map
    peer memory or a checksum failed on any rank (the caller then uses RCCL / gloo)."""
    W, r = comm.size, comm.rank
    E, base, handle = None, 0, None
    send = _words(tensor)
    nwords = send.numel()
    try:
        from ..ops._ext import ext
        E = ext()
        base = E.xgmi_alloc(max(16, 4 * nwords))
        handle = bytes(E.xgmi_handle(base))
        if nwords:
            E.xgmi_tensor(base, nwords).view(torch.int32).copy_(send)
    except Exception as exc:  # noqa: BLE001  (no extension / no IPC on this rank)
        from .xgmi import _debug
        _debug(exc)
        handle = None
    sw = [C[r][d] * wpr for d in range(W)]
    sums = segment_checksums(send, sw) if handle is not None else None
    from .xgmi import _corrupt_rank
    if sums is not None and _corrupt_rank() == r:
        # test hook (MULTIGRAD_XGMI_SELFTEST_CORRUPT=<rank>): this rank announces a wrong
        # checksum for every segment, so every rank must reject the peer result
        sums = [v + 1 for v in sums]
    if handle is not None:
        torch.cuda.synchronize()  # the packed rows are in memory before any peer reads them
    info = comm.allgather((handle, sums))
    peers, ok = [], all(h is not None for h, _ in info)
    if ok:
        try:
            peers = [base if q == r else E.xgmi_open(info[q][0]) for q in range(W)]
        except Exception as exc:  # noqa: BLE001
            from .xgmi import _debug
            _debug(exc)
            ok = False
    good = False
    mapped = all(comm.allgather(ok))
    if mapped:
        rw = [C[q][r] * wpr for q in range(W)]
        srcs, doff, off = [], [], 0
        for q in range(W):
            sdis = sum(C[q][d] for d in range(r)) * wpr   # q's send displacement of r
            srcs.append(peers[q] + 4 * sdis)
            doff.append(off)
            off += rw[q]
        recv = _words(out) if out.numel() else torch.zeros(0, dtype=torch.int32, device=out.device)
        try:  # a rank that fails here must still reach the verdict all-gather below
            if off:
                E.xgmi_a2a_pull(srcs, rw, doff, recv)
            got = segment_checksums(recv, rw)
            want = [info[q][1][r] for q in range(W)]
            good = got == want
            torch.cuda.synchronize()
        except Exception as exc:  # noqa: BLE001
            from .xgmi import _debug
            _debug(exc)
            good = False
    verdicts = comm.allgather(bool(good))   # also: no rank frees its region before all pulled
    if E is not None:
        for q, p in enumerate(peers):
            if q != r and p:
                E.xgmi_close(p)
        if base:
            E.xgmi_free(base)
    if all(verdicts):
        _record(comm, ok=True, path="peer memory pull", rows=int(tensor.shape[0]), fallback=None)
        return True
    bad = [q for q, v in enumerate(verdicts) if not v]
    _record(comm, ok=False, path="peer memory pull", rows=int(tensor.shape[0]),
            fallback=("RCCL/gloo: peer memory unavailable on some rank" if not mapped else
                      f"RCCL/gloo: checksum mismatch on rank(s) {bad}"))
    return False
