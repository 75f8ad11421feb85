"""L-BFGS vector ops (``csrc/lbfgs.hip``) with PyTorch fallbacks for CPU tensors."""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from ._ext import ext

__all__ = ["MultiDot", "lincomb_"]


class MultiDot:
    """``out[r, c] = A[r, :n] . B_c[:n]`` for up to 4 right-hand vectors, fp64 results,
    deterministic fixed-order reduction.  Workspace is allocated once."""

    def __init__(self, nrows_max: int, n: int, device):
        self.n = int(n)
        self.device = torch.device(device)
        self.out = torch.zeros(nrows_max * 4, dtype=torch.float64, device=self.device)
        if self.device.type == "cuda":
            ws = ext().multi_dot_workspace(nrows_max, self.n)
            self.ws = torch.zeros(ws, dtype=torch.float64, device=self.device)

    def __call__(self, A: torch.Tensor, nrows: int, B: Sequence[torch.Tensor]) -> torch.Tensor:
        nc = len(B)
        if self.device.type == "cuda":
            ext().multi_dot(A, int(nrows), list(B), self.n, self.out, self.ws)
            return self.out[:nrows * nc].view(nrows, nc)
        Bm = torch.stack([b[:self.n] for b in B]).double()
        res = A[:nrows, :self.n].double() @ Bm.T
        self.out[:nrows * nc] = res.reshape(-1)
        return self.out[:nrows * nc].view(nrows, nc)


def lincomb_(H: torch.Tensor, nrows: int, coef: torch.Tensor, alpha: float,
             x: Optional[torch.Tensor], y: torch.Tensor) -> torch.Tensor:
    """``y = alpha * x + sum_i coef[i] * H[i]`` (one fused pass on the GPU)."""
    n = y.numel()
    if y.device.type == "cuda":
        ext().lincomb(H, int(nrows), coef, float(alpha), x, n, y)
        return y
    acc = torch.zeros(n, dtype=torch.float64)
    if x is not None:
        acc += alpha * x[:n].double()
    if nrows:
        acc += coef[:nrows].double() @ H[:nrows, :n].double()
    y.copy_(acc.to(y.dtype))
    return y
