"""The population SMF model written in plain PyTorch ops (no custom kernels).

This is what a user of the reference writes: a ``OnePointModel`` whose hooks are ordinary
differentiable array code (the reference's are ``jax.numpy``, tests/smf_example/
smf_grad_descent.py:32-82; here ``torch``).  It computes the same summed statistics as
:class:`~multigrad_amd.models.population.PopulationSMFModel` -- one ``(a, log10 sigma)``
pair per population, log-MSE loss -- through autograd, so it exercises the *generic*
device paths: the eager distributed chain rule (``OnePointModel._vjp``) and the
graph-captured generic engine (:mod:`multigrad_amd.engine.generic`).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from ..ops.smf import logmse_loss
from .onepoint import OnePointModel

__all__ = ["TorchPopulationSMFModel", "StochasticTorchPopulationSMFModel", "torch_population_data"]


def torch_population_data(data: dict) -> dict:
    """Plain-tensor aux data (halo masses, population ids, bins) from
    :func:`~multigrad_amd.models.population.make_population_data` output, with the
    target SMF filled in (``PopulationSMFModel.set_target_from_truth`` first)."""
    sh = data["shard"]
    bins = data["bins"]
    dev = sh.x.device
    return dict(x=sh.x.float(), pop=sh.pop.long(),
                edges=torch.tensor(bins.edges, dtype=torch.float32, device=dev),
                scale=torch.tensor(bins.scale, dtype=torch.float32, device=dev),
                target=data["target_sumstats"].float().to(dev), eps=float(data["loss_eps"]),
                npop=int(data["npop"]))


@dataclass(eq=False)
class TorchPopulationSMFModel(OnePointModel):
    """``aux_data`` from :func:`torch_population_data`; parameters interleaved
    ``(a_c, log10 sigma_c)``."""

    aux_data: dict = None

    def calc_partial_sumstats_from_params(self, params, randkey=None):
        return self._sumstats(params, self.aux_data["x"])

    def _sumstats(self, params, x):
        d = self.aux_data
        th = params.reshape(-1, 2)
        a = th[:, 0][d["pop"]]
        sigma = torch.pow(10.0, th[:, 1])[d["pop"]]
        z = (d["edges"][None, :] - (x + a)[:, None]) / sigma[:, None]
        cdf = torch.special.ndtr(z)
        return (cdf[:, 1:] - cdf[:, :-1]).sum(0) * d["scale"]

    def calc_loss_from_sumstats(self, sumstats, sumstats_aux=None, randkey=None):
        d = self.aux_data
        return logmse_loss(sumstats, d["target"].to(sumstats.dtype), d["eps"])


@dataclass(eq=False)
class StochasticTorchPopulationSMFModel(TorchPopulationSMFModel):
    """The same model with per-evaluation Monte-Carlo scatter: every halo's log mass is
    perturbed by ``scatter * N(0, 1)`` drawn from ``randkey.generator(device)`` -- a
    stochastic forward model, fitted with a fresh key per Adam step (reference
    multigrad/adam.py:59-62) or a constant one (``const_randkey``)."""

    scatter: float = 0.02

    def calc_partial_sumstats_from_params(self, params, randkey=None):
        x = self.aux_data["x"]
        if randkey is not None:
            x = x + self.scatter * torch.randn(x.shape, generator=randkey.generator(x.device),
                                               device=x.device, dtype=x.dtype)
        return self._sumstats(params, x)
