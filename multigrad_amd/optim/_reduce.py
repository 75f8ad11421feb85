"""Cross-rank reductions of the SPMD device optimizers (device L-BFGS / L-BFGS-B).

The reference's BFGS (``multigrad/bfgs.py:32-113``) runs scipy on the root rank and
broadcasts every trial point; the SPMD optimizers here instead take every decision on
scalars that are reduced across the ranks, so all ranks take the same branch.  Those
scalars are the inner products of an iteration (compact-form dot block, max|g|) and the
directional derivative of every line-search point.

:class:`DeviceReducer` reduces them **on the devices** and brings the result to the host in
**one** device->host copy per call:

* peer memory (the wide one-shot kernel, ``csrc/xgmi.hip``: every rank pushes its values into
  every peer's inbox and sums / max-reduces the inboxes in rank order -- one single-workgroup
  launch, bitwise identical on all ranks), when the ranks share an xGMI node (or a GPU) and
  the connect-time self-test passed;
* else RCCL all-reduces of the device buffer (a sum and a max launch);
* else (CPU tensors, gloo-only worlds) the host all-reduce of the copied values.

Every path returns the same layout: ``[summed values, max-reduced values, local values]``
as one fp64 numpy vector.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

__all__ = ["DeviceReducer"]


def _flat64(parts: Sequence, device) -> list:
    out = []
    for p in parts:
        t = torch.as_tensor(p)
        if t.device != device:
            t = t.to(device)
        out.append(t.reshape(-1).to(torch.float64))
    return out


class DeviceReducer:
    """Reductions for an optimizer whose vectors are ``sharded`` over ``comm`` (replicated
    vectors need none: every rank already holds the full inner products).

    Construction is collective (it may connect the wide one-shot context)."""

    def __init__(self, comm, sharded: bool, device):
        self.device = torch.device(device)
        self.comm = comm if (comm is not None and comm.size > 1 and sharded) else None
        self.wide = None
        self.rccl = False
        self.path = "local"
        if self.comm is None:
            return
        if self.device.type == "cuda":
            from ..parallel.xgmi import get_wide_oneshot
            self.wide = get_wide_oneshot(self.comm)  # collective
            if self.wide is not None:
                self.path = "xgmi wide one-shot"
            else:
                fn = getattr(self.comm, "device_collectives", None)
                self.rccl = bool(fn()) if fn is not None else False
                self.path = "rccl" if self.rccl else "host"
        else:
            self.path = "host"

    # ------------------------------------------------------------------ reductions
    def reduce(self, sums: Sequence = (), maxes: Sequence = (), local: Sequence = ()) -> np.ndarray:
        """``[sum over ranks of sums..., max over ranks of maxes..., local...]`` (each part
        flattened, fp64) on the host, after one device->host copy."""
        dev = self.device
        s = _flat64(sums, dev)
        m = _flat64(maxes, dev)
        lo = _flat64(local, dev)
        parts = s + m + lo
        if not parts:
            return np.zeros(0)
        buf = torch.cat(parts) if len(parts) > 1 else parts[0].clone()
        ns = sum(int(t.numel()) for t in s)
        nm = sum(int(t.numel()) for t in m)
        comm = self.comm
        if comm is None or ns + nm == 0:
            return buf.cpu().numpy()
        if self.wide is not None:
            from ..parallel.xgmi import MAX_WIDE
            # sum part then max part, in pieces of at most MAX_WIDE values per launch
            for a0, b0, is_max in ((0, ns, False), (ns, ns + nm, True)):
                for a in range(a0, b0, MAX_WIDE):
                    k = min(MAX_WIDE, b0 - a)
                    piece = buf[a:a + k]
                    self.wide(piece, 0 if is_max else k, k if is_max else 0)
            return buf.cpu().numpy()
        if self.rccl and buf.is_cuda:
            if ns:
                comm.all_reduce(buf[:ns])
            if nm:
                comm.all_reduce(buf[ns:ns + nm], op="max")
            return buf.cpu().numpy()
        host = buf.cpu()
        if ns:
            t = host[:ns].contiguous()
            comm.all_reduce(t)
            host[:ns] = t
        if nm:
            t = host[ns:ns + nm].contiguous()
            comm.all_reduce(t, op="max")
            host[ns:ns + nm] = t
        return host.numpy()

    def check(self, where: str = "") -> None:
        """Raise :class:`~multigrad_amd.parallel.xgmi.CollectiveTimeout` if a peer-memory
        reduction timed out (its values are NaN-poisoned; a host sync)."""
        if self.wide is not None:
            self.wide.check(where or "optimizer reduction")

    # ------------------------------------------------------------------ all-gather
    def reserve_gather(self, nbytes: int) -> None:
        """Collective: connect the peer-memory context that :meth:`all_gather` will use for
        pieces of up to ``nbytes`` per rank now, outside the optimizer's iterations
        (connecting is a host-synchronising collective)."""
        if self.comm is None or self.device.type != "cuda" or self.wide is None:
            return
        from ..parallel.xgmi import get_twoshot_allreduce
        floats = -(-int(nbytes) // 4)
        n = -(-floats // 4) * 4  # float4-aligned piece per rank (as peer_all_gather sizes it)
        get_twoshot_allreduce(self.comm, n * self.comm.size)

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """``[W, *t.shape]``: every rank's ``t`` (same shape on all ranks) in rank order --
        peer memory when available, else the communicator's all-gather."""
        comm = self.comm
        if comm is None:
            return t.reshape((1,) + tuple(t.shape)).clone()
        out = torch.empty((comm.size,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        if t.is_cuda:
            from ..parallel.xgmi import peer_all_gather
            if peer_all_gather(comm, out, t.contiguous()):
                return out
        comm.all_gather_into_tensor(out.reshape(-1), t.contiguous().reshape(-1))
        return out

    def describe(self) -> Optional[str]:
        return None if self.comm is None else self.path
