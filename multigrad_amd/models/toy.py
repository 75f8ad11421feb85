"""Sum-of-squares toy model (BASELINE.json config 1: 10-parameter plumbing check).

Each rank holds some points ``y_i`` in ``ndim`` dimensions; the partial sumstats are the
per-dimension sums of squared residuals ``s_j = sum_i (y_ij - theta_j)^2`` and the loss is
their sum divided by the global point count, minimised at the global mean of the points.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from ..parallel.comm import get_world_comm
from .onepoint import OnePointModel

__all__ = ["SumOfSquaresModel", "make_toy_data"]


def make_toy_data(ndim: int = 10, npoints: int = 1000, seed: int = 0, comm=None) -> dict:
    comm = get_world_comm() if comm is None else comm
    rng = np.random.default_rng(seed)
    y = rng.normal(loc=np.linspace(-1, 1, ndim), scale=0.5, size=(npoints, ndim))
    return {"y": torch.as_tensor(np.array_split(y, comm.size)[comm.rank], dtype=torch.float32),
            "n_total": npoints, "mean": y.mean(0)}


@dataclass(eq=False)
class SumOfSquaresModel(OnePointModel):
    aux_data: dict = None

    def calc_partial_sumstats_from_params(self, params, randkey=None):
        y = self.aux_data["y"].to(params.device, params.dtype)
        return ((y - params) ** 2).sum(0)

    def calc_loss_from_sumstats(self, sumstats, sumstats_aux=None, randkey=None):
        return sumstats.sum() / self.aux_data["n_total"]
