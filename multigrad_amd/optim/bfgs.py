"""L-BFGS-B driver (host scipy path) -- reference ``multigrad/bfgs.py:32-113``.

The root rank runs ``scipy.optimize.minimize(method="L-BFGS-B", jac=True)``; every other
rank services its function evaluations so that it can join the collectives inside
``loss_and_grad_fn``.  Instead of the reference's two pickled broadcasts per evaluation
(``"compute"`` then ``params``) the command and the parameters travel in
ONE float64 tensor broadcast ``[cmd, x_0 .. x_{n-1}]``; the final ``OptimizeResult`` is
broadcast once (M13) so every rank returns an identical result.

For large parameter counts use :func:`multigrad_amd.optim.lbfgs.run_lbfgs_device`
(SPMD on the GPU with batched RCCL-all-reduced dot products).
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np
import scipy.optimize
import torch

from ..utils.hooks import StepHooks, driver_guard
from ..utils.progress import progress_enabled
from ..utils.random import init_randkey
from ..utils.tensors import as_param_tensor

__all__ = ["run_bfgs", "RootAborted"]

_CMD_COMPUTE, _CMD_EXIT, _CMD_ABORT = 1.0, 0.0, -1.0


class RootAborted(RuntimeError):
    """Raised on the worker ranks of a root-driven fit whose root rank failed."""


def _bfgs_pbar(maxsteps):
    if progress_enabled():
        from tqdm import auto as tqdm
        return tqdm.trange(maxsteps, desc="BFGS Gradient Descent Progress", leave=True)
    return None


def _scalar_loss(loss):
    if isinstance(loss, (tuple, list)):
        loss = loss[0]
    return float(torch.as_tensor(loss).detach().cpu().double())


def run_bfgs(loss_and_grad_fn: Callable, params, maxsteps: int = 100, param_bounds=None,
             randkey=None, comm=None, *, dtype=None, device=None, options: Optional[dict] = None):
    """Minimise with L-BFGS-B.

    Parameters
    ----------
    loss_and_grad_fn : ``(params[, randkey=key]) -> (loss, grad)``
    params : initial guess
    maxsteps : maximum number of L-BFGS iterations (scipy ``maxiter``)
    param_bounds : ``(ndim, 2)`` bounds passed straight to scipy (``None`` = unbounded)
    randkey : held constant for every evaluation (a deterministic objective)
    comm : communicator whose ranks all take part (default: serial)

    Returns
    -------
    scipy.optimize.OptimizeResult, identical on every rank.
    """
    kwargs = {}
    if randkey is not None:
        kwargs["randkey"] = init_randkey(randkey)
    x0_t = as_param_tensor(params, device=device)
    shape, pdtype, pdev = x0_t.shape, dtype or x0_t.dtype, x0_t.device
    x0 = x0_t.detach().cpu().double().numpy().reshape(-1)
    n = x0.size
    multi = comm is not None and comm.size > 1
    cmd = torch.empty(n + 1, dtype=torch.float64)

    def evaluate(x: np.ndarray):
        xt = torch.as_tensor(x, dtype=pdtype, device=pdev).reshape(shape)
        loss, grad = loss_and_grad_fn(xt, **kwargs)
        g = torch.as_tensor(grad).detach().reshape(-1).cpu().double().numpy()
        return _scalar_loss(loss), g

    if not multi or comm.rank == 0:
        with driver_guard(comm if multi else None):
            return _root(fun_eval=evaluate, x0=x0, maxsteps=maxsteps, param_bounds=param_bounds,
                         options=options, comm=comm if multi else None, cmd=cmd)
    # workers: service the root's evaluations (reference multigrad/bfgs.py:96-106).  A
    # failure here, or inside the objective's collectives on any rank, tears the process
    # group down (driver_guard) so no rank waits for the process-group timeout.
    with driver_guard(comm):
        while True:
            comm.broadcast(cmd, root=0)
            c = cmd[0].item()
            if c == _CMD_EXIT:
                break
            if c == _CMD_ABORT:
                raise RootAborted(f"root rank of {comm.name!r} aborted the fit: "
                                  f"{comm.bcast(None, root=0)}")
            evaluate(cmd[1:].numpy().copy())
        return scipy.optimize.OptimizeResult(comm.bcast(None, root=0))


def _root(fun_eval, x0, maxsteps, param_bounds, options, comm, cmd):
    """The root's scipy L-BFGS-B run.  An exception raised between evaluations (scipy, a
    callback, a hook) is sent to the workers as an abort command, so they leave their
    command loop with the root's error; one raised inside an evaluation propagates to
    ``driver_guard``, whose process-group teardown ends the workers' pending collective."""
    pbar = _bfgs_pbar(maxsteps)
    in_eval = [False]

    def fun(x):
        if comm is not None:
            cmd[0] = _CMD_COMPUTE
            cmd[1:] = torch.from_numpy(np.asarray(x, dtype=np.float64))
            comm.broadcast(cmd, root=0)
        in_eval[0] = True
        out = fun_eval(x)
        in_eval[0] = False
        return out

    hooks = StepHooks(None)  # metrics only: the workers are inside the command loop
    nit = [0]

    def callback(*a, **_k):
        if pbar is not None:
            pbar.update()
        if hooks.active:
            res = _k.get("intermediate_result")
            hooks(nit[0], None if res is None else float(res.fun), None)
        nit[0] += 1

    from ..utils.tensors import blas_single_thread
    try:
        with blas_single_thread():  # keep the cores for the model evaluations
            result = scipy.optimize.minimize(fun, x0=x0, method="L-BFGS-B", jac=True,
                                             options=dict(maxiter=maxsteps, **(options or {})),
                                             callback=callback, bounds=param_bounds)
    except BaseException as exc:
        if comm is not None and not in_eval[0]:
            cmd[0] = _CMD_ABORT
            comm.broadcast(cmd, root=0)
            comm.bcast(f"{type(exc).__name__}: {exc}", root=0)
        raise
    finally:
        if pbar is not None:
            pbar.close()
    if comm is not None:
        cmd[0] = _CMD_EXIT
        comm.broadcast(cmd, root=0)
        comm.bcast(dict(result), root=0)
    return result
