"""Box-constraint reparameterisation for Adam (reference ``multigrad/adam.py:192-239``).

Each bounded parameter ``p`` is optimised in an unbounded coordinate ``u = T(p)``:

=================  ===========================  ==============================  =====================
bounds             u = T(p)                     p = T^-1(u)                     dp/du
=================  ===========================  ==============================  =====================
both finite        s tan((p - mid)/s)           mid + s atan(u/s)               1/(1 + (u/s)^2)
low only           p - lo + 1/(lo - p)          (2 lo + u + sqrt(u^2+4))/2      (1 + u/sqrt(u^2+4))/2
high only          p - hi + 1/(hi - p)          (2 hi + u - sqrt(u^2+4))/2      (1 - u/sqrt(u^2+4))/2
none               p                            u                               1
=================  ===========================  ==============================  =====================

with ``mid = (lo+hi)/2`` and ``s = (hi-lo)/pi``.  The reference builds a dense
``P x P`` ``jax.jacobian`` of the inverse transform and evaluates it at the *bounded*
parameters; the Jacobian is diagonal, so here it is the elementwise
``dp/du`` evaluated at ``u`` (``legacy=True`` evaluates it at ``p`` for bit-parity).
The device path fuses these formulas into the Adam kernel (``csrc/adam.hip``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np
import torch

__all__ = ["Bounds", "transform", "inverse_transform", "apply_transforms",
           "apply_inverse_transforms", "dparams_duparams"]

# per-parameter bound kinds (shared with the HIP kernel)
KIND_NONE, KIND_BOTH, KIND_LOW, KIND_HIGH = 0, 1, 2, 3


def _finite(x) -> bool:
    return x is not None and np.isfinite(x)


def _bound_pair(b):
    if b is None:
        return (None, None)
    lo, hi = b
    return (float(lo) if _finite(lo) else None, float(hi) if _finite(hi) else None)


@dataclass
class Bounds:
    """Vectorised per-parameter bounds: ``lo``/``hi`` tensors (+-inf where absent)."""

    lo: torch.Tensor
    hi: torch.Tensor
    kind: torch.Tensor  # int8 KIND_* per parameter

    @staticmethod
    def from_spec(param_bounds, ndim: int, device=None, dtype=torch.float32) -> Optional["Bounds"]:
        if param_bounds is None:
            return None
        if isinstance(param_bounds, (np.ndarray, torch.Tensor)) and \
                param_bounds.dtype not in (object, np.object_) and tuple(param_bounds.shape) == (ndim, 2):
            # numeric (ndim, 2) array: vectorised (a 1e7-row Python loop takes seconds);
            # non-finite entries mark an absent side, as in the list form
            arr = torch.as_tensor(param_bounds).to(device=device, dtype=torch.float64)
            lo_t, hi_t = arr[:, 0], arr[:, 1]
            fl, fh = torch.isfinite(lo_t), torch.isfinite(hi_t)
            kind = torch.where(fl & fh, KIND_BOTH, torch.where(fl, KIND_LOW, torch.where(
                fh, KIND_HIGH, KIND_NONE))).to(torch.int8)
            return Bounds(torch.where(fl, lo_t, -math.inf).to(dtype),
                          torch.where(fh, hi_t, math.inf).to(dtype), kind)
        if hasattr(param_bounds, "tolist"):
            param_bounds = param_bounds.tolist()
        pb = list(param_bounds)
        assert len(pb) == ndim, "param_bounds must have shape (ndim, 2)"
        lo = np.full(ndim, -np.inf)
        hi = np.full(ndim, np.inf)
        kind = np.zeros(ndim, dtype=np.int8)
        for i, b in enumerate(pb):
            l, h = _bound_pair(b)
            if l is not None:
                lo[i] = l
            if h is not None:
                hi[i] = h
            kind[i] = (KIND_BOTH if (l is not None and h is not None) else
                       KIND_LOW if l is not None else KIND_HIGH if h is not None else KIND_NONE)
        return Bounds(torch.as_tensor(lo, dtype=dtype, device=device),
                      torch.as_tensor(hi, dtype=dtype, device=device),
                      torch.as_tensor(kind, device=device))

    def to(self, device=None, dtype=None) -> "Bounds":
        return Bounds(self.lo.to(device=device, dtype=dtype), self.hi.to(device=device, dtype=dtype),
                      self.kind.to(device=device))

    # ------------------------------------------------------------- vectorised maps
    def _safe(self, like: torch.Tensor):
        """Bounds with absent sides replaced by finite dummies, so the branches that
        ``torch.where`` discards never produce inf/NaN (which would poison gradients)."""
        k = self.kind.to(like.device)
        lo = torch.where(torch.isfinite(self.lo), self.lo, torch.zeros_like(self.lo)).to(like)
        hi = torch.where(torch.isfinite(self.hi), self.hi, torch.ones_like(self.hi)).to(like)
        both = k == KIND_BOTH
        mid = torch.where(both, (hi + lo) / 2, torch.zeros_like(lo))
        s = torch.where(both, (hi - lo) / math.pi, torch.ones_like(lo))
        return k, lo, hi, mid, s

    def forward(self, p: torch.Tensor) -> torch.Tensor:
        k, lo, hi, mid, s = self._safe(p)
        both = torch.where(k == KIND_BOTH, s * torch.tan((p - mid) / s), p)
        dl = torch.where(k == KIND_LOW, lo - p, torch.ones_like(p))
        low = torch.where(k == KIND_LOW, p - lo + 1.0 / dl, both)
        dh = torch.where(k == KIND_HIGH, hi - p, torch.ones_like(p))
        return torch.where(k == KIND_HIGH, p - hi + 1.0 / dh, low)

    def inverse(self, u: torch.Tensor) -> torch.Tensor:
        k, lo, hi, mid, s = self._safe(u)
        r = torch.sqrt(u * u + 4)
        both = torch.where(k == KIND_BOTH, mid + s * torch.atan(u / s), u)
        low = torch.where(k == KIND_LOW, 0.5 * (2 * lo + u + r), both)
        return torch.where(k == KIND_HIGH, 0.5 * (2 * hi + u - r), low)

    def dpdu(self, u: torch.Tensor) -> torch.Tensor:
        k, lo, hi, mid, s = self._safe(u)
        r = torch.sqrt(u * u + 4)
        one = torch.ones_like(u)
        both = torch.where(k == KIND_BOTH, 1.0 / (1.0 + (u / s) ** 2), one)
        low = torch.where(k == KIND_LOW, 0.5 * (1 + u / r), both)
        return torch.where(k == KIND_HIGH, 0.5 * (1 - u / r), low)


def transform(param, bounds):
    """Transform one bounded parameter into its unbounded coordinate."""
    lo, hi = _bound_pair(bounds)
    p = torch.as_tensor(param, dtype=torch.float32) if not isinstance(param, torch.Tensor) else param
    if lo is not None and hi is not None:
        mid, s = (hi + lo) / 2.0, (hi - lo) / math.pi
        return s * torch.tan((p - mid) / s)
    if lo is not None:
        return p - lo + 1.0 / (lo - p)
    if hi is not None:
        return p - hi + 1.0 / (hi - p)
    return p


def inverse_transform(uparam, bounds):
    """Map one unbounded coordinate back into its bounded parameter."""
    lo, hi = _bound_pair(bounds)
    u = torch.as_tensor(uparam, dtype=torch.float32) if not isinstance(uparam, torch.Tensor) else uparam
    if lo is not None and hi is not None:
        mid, s = (hi + lo) / 2.0, (hi - lo) / math.pi
        return mid + s * torch.atan(u / s)
    if lo is not None:
        return 0.5 * (2.0 * lo + u + torch.sqrt(u ** 2 + 4))
    if hi is not None:
        return 0.5 * (2.0 * hi + u - torch.sqrt(u ** 2 + 4))
    return u


def apply_transforms(params, bounds: Sequence):
    return torch.stack([torch.as_tensor(transform(p, b)) for p, b in zip(params, bounds)])


def apply_inverse_transforms(uparams, bounds: Sequence):
    return torch.stack([torch.as_tensor(inverse_transform(u, b)) for u, b in zip(uparams, bounds)])


def dparams_duparams(uparams: torch.Tensor, bounds: Bounds) -> torch.Tensor:
    """Diagonal of the Jacobian dp/du (the reference's dense ``jax.jacobian``)."""
    return bounds.dpdu(uparams)
