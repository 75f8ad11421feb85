"""Utility functions: simple gradient descent, Latin hypercube sampling, scatter.

Public API of the reference's ``multigrad.util`` (``multigrad/util.py:37-134``):
``simple_grad_descent``, ``GradDescentResult``, ``latin_hypercube_sampler``,
``scatter_nd``.
"""
from __future__ import annotations

from typing import Any, NamedTuple, Union

import numpy as np
import torch
from scipy.stats import qmc

from ..parallel.subcomm import scatter_nd
from .hooks import StepHooks, driver_guard
from .progress import trange
from .tensors import as_param_tensor

__all__ = ["simple_grad_descent", "GradDescentResult", "latin_hypercube_sampler",
           "scatter_nd", "value_and_grad"]


class GradDescentResult(NamedTuple):
    loss: torch.Tensor
    params: torch.Tensor
    aux: Union[torch.Tensor, list]


def latin_hypercube_sampler(xmin, xmax, n_dim, num_evaluations, seed=None,
                            optimization=None) -> np.ndarray:
    """``num_evaluations`` Latin-hypercube draws in the box ``[xmin, xmax]^n_dim``."""
    xmin = np.zeros(n_dim) + xmin
    xmax = np.zeros(n_dim) + xmax
    sampler = qmc.LatinHypercube(n_dim, seed=seed, optimization=optimization)
    unit = sampler.random(num_evaluations)
    return qmc.scale(unit, xmin, xmax)


def value_and_grad(loss_func, has_aux: bool = False, **call_kwargs):
    """Autograd equivalent of ``jax.value_and_grad``: ``f(p) -> ((loss[, aux]), grad)``."""

    def f(params):
        p = as_param_tensor(params).detach().requires_grad_(True)
        with torch.enable_grad():
            out = loss_func(p, **call_kwargs)
            loss = out[0] if has_aux else out
            (g,) = torch.autograd.grad(loss, p, allow_unused=True)
        if g is None:
            g = torch.zeros_like(p)
        if has_aux:
            return (loss.detach(), out[1]), g
        return loss.detach(), g

    return f


def simple_grad_descent(loss_func, guess, nsteps, learning_rate, loss_and_grad_func=None,
                        grad_loss_func=None, has_aux=False, *, comm=None, callback=None,
                        **kwargs) -> GradDescentResult:
    """Fixed-learning-rate gradient descent (reference ``multigrad/util.py:80-134``).

    SPMD: every rank runs the same loop with identical all-reduced gradients, so no
    broadcast is needed.  The recorded ``params[i]`` are the parameters at which
    ``loss[i]`` was evaluated (the final update is not recorded), exactly as in the
    reference.  Losses and parameters stay on the parameters' device until the end.
    ``comm`` (the communicator the gradient is reduced over) and ``callback(step, loss,
    None)`` feed the per-step driver hooks (:mod:`multigrad_amd.utils.hooks`).
    """
    if loss_and_grad_func is None:
        if grad_loss_func is None:
            loss_and_grad_func = value_and_grad(loss_func, has_aux=has_aux, **kwargs)
        else:
            def loss_and_grad_func(params):
                return loss_func(params), grad_loss_func(params)

    params = as_param_tensor(guess)
    losses, plist, auxes = [], [], []
    hooks = StepHooks(comm, callback)  # MULTIGRAD_CHECK_EVERY / MULTIGRAD_METRICS
    with driver_guard(comm):
        for step in trange(nsteps, desc="Simple Gradient Descent Progress"):
            (loss, grad), aux = loss_and_grad_func(params), None
            if has_aux:
                (loss, aux), grad = loss, grad
            losses.append(torch.as_tensor(loss).detach())
            plist.append(params)
            auxes.append(aux)
            params = params - learning_rate * torch.as_tensor(grad, device=params.device,
                                                              dtype=params.dtype)
            if hooks.active:
                hooks(step, loss, None, lambda: params)
    loss_t = torch.stack(losses) if losses else torch.zeros(0)
    params_t = torch.stack(plist) if plist else torch.zeros((0,) + tuple(params.shape))
    aux_out: Any = auxes
    if has_aux:
        try:
            aux_out = torch.stack([torch.as_tensor(a) for a in auxes])
        except (TypeError, RuntimeError, ValueError):
            pass
    return GradDescentResult(loss=loss_t, params=params_t, aux=aux_out)
