"""Fused Adam op (``csrc/adam.hip``) with a PyTorch reference for CPU tensors."""
from __future__ import annotations

from typing import Optional

import torch

from ._ext import ext

__all__ = ["fused_adam_", "adam_reference_", "adam_step_"]


def fused_adam_(u: torch.Tensor, m: torch.Tensor, v: torch.Tensor, g: torch.Tensor,
                p: Optional[torch.Tensor], step: torch.Tensor, lr: float, b1: float, b2: float,
                eps: float, bounds=None, legacy: bool = False,
                traj_row: Optional[torch.Tensor] = None, traj_base: Optional[torch.Tensor] = None,
                traj_stride: int = 0, host_step: Optional[int] = None) -> None:
    """One in-place Adam step on device.

    ``step`` is a ``[2]`` int32 device tensor ``[step, ticket]``; the kernel reads the
    0-based step for bias correction and advances it.  Either ``traj_row`` (eager: the
    row for this step) or ``traj_base``/``traj_stride`` (graph-replayable: row
    ``step+1`` is computed on the device) may be given.  ``host_step`` (eager callers
    only, never inside a graph capture) supplies the 0-based step directly; the device
    counter is then neither read nor advanced.
    """
    if traj_row is not None:
        # express the eager row through the device-step formula: base = row - (step+1)*stride
        # is not available without a host sync, so pass the row with stride 0 and let the
        # kernel add (step+1)*0.
        traj_base, traj_stride = traj_row, 0
    if bounds is not None:
        ext().fused_adam(u, m, v, g, p, bounds.lo, bounds.hi, bounds.kind, step, float(lr),
                         float(b1), float(b2), float(eps), bool(legacy), traj_base,
                         int(traj_stride), -1 if host_step is None else int(host_step))
    else:
        ext().fused_adam(u, m, v, g, None, None, None, None, step, float(lr), float(b1),
                         float(b2), float(eps), False, traj_base, int(traj_stride),
                         -1 if host_step is None else int(host_step))


def adam_reference_(u, m, v, g, step: int, lr, b1, b2, eps):
    """fp32 PyTorch reference of the same update (0-based ``step``)."""
    m.mul_(b1).add_((1 - b1) * g)
    v.mul_(b2).add_((1 - b2) * g * g)
    mhat = m / (1 - b1 ** (step + 1))
    vhat = v / (1 - b2 ** (step + 1))
    u.sub_(lr * mhat / (torch.sqrt(vhat) + eps))


def adam_step_(u, m, v, g, p, step: torch.Tensor, lr, b1, b2, eps, bounds=None,
               legacy: bool = False, traj_base=None, traj_stride: int = 0,
               host_step: Optional[int] = None) -> None:
    """Device-agnostic in-place Adam step: the fused HIP kernel on GPU tensors, the same
    arithmetic in PyTorch on CPU tensors (``step`` is then a CPU ``[2]`` int tensor).
    ``host_step``: see :func:`fused_adam_` (the CPU path then leaves ``step`` alone)."""
    if u.device.type == "cuda":
        fused_adam_(u, m, v, g, p, step, lr, b1, b2, eps, bounds, legacy,
                    traj_base=traj_base, traj_stride=traj_stride, host_step=host_step)
        return
    i = int(step[0]) if host_step is None else int(host_step)
    gg = g
    if bounds is not None:
        at = p if legacy else u
        gg = g * bounds.dpdu(at)
    m.mul_(b1).add_((1 - b1) * gg)
    v.mul_(b2).add_((1 - b2) * gg * gg)
    mhat = m / (1 - b1 ** (i + 1))
    vhat = v / (1 - b2 ** (i + 1))
    u.sub_(lr * mhat / (torch.sqrt(vhat) + eps))
    newp = bounds.inverse(u) if bounds is not None else u
    if bounds is not None:
        p.copy_(newp)
    if traj_base is not None:
        n = u.numel()
        traj_base[(i + 1) * traj_stride:(i + 1) * traj_stride + n].copy_(newp)
    if host_step is None:
        step[0] = i + 1
