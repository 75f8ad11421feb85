"""One-point models: differentiable summary statistics summed over data shards.

Reference: ``multigrad/multigrad.py:186-607`` (``OnePointModel``, ``OnePointGroup``).

The distributed chain rule (reference ``_vjp``, ``:508-538``)::

    S(theta) = sum_r s_r(theta)                   # partial sumstats, all-reduced
    L(theta) = l(S(theta))                        # loss on the total, every rank
    dL/dtheta = sum_r J_{s_r}(theta)^T dl/dS      # local VJP with the global cotangent,
                                                  # then all-reduced

is evaluated here with PyTorch-ROCm autograd on the rank's GPU.  Both reductions are
device collectives (RCCL over xGMI, stream ordered; gloo on CPU) -- there is no
host round trip per step as in the reference's numpy-staged MPI calls.  Models whose
sumstats are produced by hand-written HIP kernels plug in through custom autograd
functions (see :mod:`multigrad_amd.models.smf`) or the fused-engine protocol
(:mod:`multigrad_amd.engine`).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Any, Tuple, Union

import numpy as np
import torch

from ..optim import adam as _adam
from ..optim import bfgs as _bfgs
from ..parallel.comm import get_world_comm
from ..utils import util
from ..utils.random import init_randkey
from ..utils.tensors import as_param_tensor, detach_tree, infer_device

__all__ = ["OnePointModel", "OnePointGroup"]


def _rk(randkey):
    return {} if randkey is None else {"randkey": randkey}


class _OptimizerFrontEnds:
    """``run_simple_grad_descent`` / ``run_adam`` / ``run_bfgs`` shared by models and groups
    (reference ``multigrad/multigrad.py:226-352``, ``:583-599``)."""

    def _opt_comm(self):
        raise NotImplementedError

    def param_device(self) -> torch.device:
        raise NotImplementedError

    def _engine_members(self):
        return tuple(self.models) if isinstance(self, OnePointGroup) else (self,)

    def _generic_engine_ok(self, x0, loss_aux_ok: bool = True) -> bool:
        """Whether this model's (or group's) optimizer steps can go through the captured
        generic engine (engine/generic.py): torch OnePointModels on a GPU, an fp32 guess
        (the engine's Adam state is fp32; an fp64 fit keeps the eager loop), no fused-engine
        protocol (a single model that has one uses the fused engine), not disabled."""
        members = self._engine_members()
        single_fused = (not isinstance(self, OnePointGroup)
                        and getattr(self, "fused_engine", None) is not None)
        return (x0.is_cuda and x0.dtype == torch.float32 and not single_fused
                and all(isinstance(m, OnePointModel) for m in members)
                and (loss_aux_ok or not any(m.loss_func_has_aux for m in members))
                and os.environ.get("MULTIGRAD_GENERIC_ENGINE", "1") != "0")

    def _step_engine(self, x0, comm=None):
        """The model's cached fused step engine (``fused_step_engine``: the shared-parameter
        SMF models, engine/smf2.py) for an fp32 device guess, or None."""
        fn = getattr(self, "fused_step_engine", None)
        if fn is None or not (x0.is_cuda and x0.dtype == torch.float32) or \
                os.environ.get("MULTIGRAD_GENERIC_ENGINE", "1") == "0":
            return None
        return fn(comm=self._opt_comm() if comm is None else comm)

    def run_simple_grad_descent(self, guess, nsteps: int = 100, learning_rate: float = 0.01):
        """Fixed-learning-rate gradient descent.

        Returns ``GradDescentResult(loss, params, aux)`` where ``params[i]`` is the point at
        which ``loss[i]`` was evaluated.
        """
        has_aux = bool(getattr(self, "loss_func_has_aux", False))
        x0 = as_param_tensor(guess, device=self.param_device())
        eng = self._step_engine(x0)
        if eng is not None and not has_aux:
            # fused device step (engine/smf2.py): one pass + one exchange per step
            return eng.run_simple_grad_descent(x0, nsteps=nsteps, learning_rate=learning_rate)
        if self._generic_engine_ok(x0, loss_aux_ok=False):
            # one captured step replayed per iteration (engine/generic.py)
            from ..engine.generic import GraphAdamEngine
            return GraphAdamEngine(self, comm=self._opt_comm()).run_simple_grad_descent(
                x0, nsteps=nsteps, learning_rate=learning_rate)
        return util.simple_grad_descent(
            None, guess=as_param_tensor(guess, device=self.param_device()), nsteps=nsteps,
            learning_rate=learning_rate,
            loss_and_grad_func=self.calc_loss_and_grad_from_params, has_aux=has_aux,
            comm=self._opt_comm())

    def run_adam(self, guess, nsteps: int = 100, param_bounds=None, learning_rate: float = 0.01,
                 randkey=None, const_randkey: bool = False, comm=None, **kw):
        """Adam from ``guess``; returns the parameter trajectory ``(nsteps+1, ndim)``.

        ``randkey`` (int or :class:`~multigrad_amd.utils.random.PRNGKey`) gives a fresh key
        per step, or the same key every step with ``const_randkey=True``.  Extra keywords
        (``history``, ``checkpoint_path``, ``checkpoint_every``, ``resume_from``,
        ``legacy_bounds_jacobian``, ``b1``, ``b2``, ``eps``, ``callback``) go to
        :func:`multigrad_amd.optim.adam.run_adam`.  Every rank returns the trajectory.
        """
        comm = self._opt_comm() if comm is None else comm
        guess = as_param_tensor(guess, device=self.param_device())
        if const_randkey:
            assert randkey is not None, "Must pass randkey if const_randkey"
            const_key = init_randkey(randkey) if not hasattr(randkey, "split") else randkey
            randkey = None

            def loss_and_grad_fn(x, _, **k):
                return self.calc_loss_and_grad_from_params(x, randkey=const_key, **k)
        else:
            def loss_and_grad_fn(x, _, **k):
                return self.calc_loss_and_grad_from_params(x, **k)
        fused = getattr(self, "fused_engine", None)
        use_engine = kw.pop("use_engine", True)
        keyed = randkey is not None or const_randkey
        step_kw = ("history", "legacy_bounds_jacobian", "b1", "b2", "eps", "callback")
        if use_engine and all(k in step_kw for k in kw) and (
                not keyed or getattr(self, "engine_randkey_invariant", False)):
            eng = self._step_engine(guess, comm)
            if eng is not None:
                return eng.run_adam(guess, nsteps=nsteps, param_bounds=param_bounds,
                                    learning_rate=learning_rate, **kw)
        if fused is not None and use_engine and (
                not keyed or getattr(self, "engine_randkey_invariant", False)):
            # a fused-protocol model whose hooks ignore randkey gives the same trajectory
            # with or without keys (engine_randkey_invariant)
            eng = fused()
            if eng is not None:
                try:
                    return eng.run_adam(guess, nsteps=nsteps, param_bounds=param_bounds,
                                        learning_rate=learning_rate, **kw)
                finally:
                    if not getattr(eng, "cached", False):  # a model's cached engine stays up
                        eng.close()
        # any other model or group on a GPU: one captured step replayed per iteration
        # (engine/generic.py), per-step or constant keys included
        graph_kw = {k: kw[k] for k in kw if k in ("history", "legacy_bounds_jacobian", "b1",
                                                   "b2", "eps", "callback")}
        if use_engine and len(graph_kw) == len(kw) and self._generic_engine_ok(guess):
            from ..engine.generic import GraphAdamEngine
            return GraphAdamEngine(self, comm=comm).run_adam(
                guess, nsteps=nsteps, param_bounds=param_bounds, learning_rate=learning_rate,
                randkey=const_key if const_randkey else randkey, const_randkey=const_randkey,
                **graph_kw)
        return _adam.run_adam(loss_and_grad_fn, params=guess, data=None, nsteps=nsteps,
                              param_bounds=param_bounds, learning_rate=learning_rate,
                              randkey=randkey, comm=comm, **kw)

    def run_bfgs(self, guess, maxsteps: int = 100, param_bounds=None, randkey=None,
                 comm=None, method: str = "auto", **kw):
        """L-BFGS(-B); returns a ``scipy.optimize.OptimizeResult`` on every rank.

        ``method="scipy"``: scipy's L-BFGS-B on the root rank, other ranks serve its
        evaluations (the reference's protocol).
        ``method="device"``: SPMD device L-BFGS with all-reduced dot products; with
        ``param_bounds`` it is L-BFGS-B (generalized Cauchy point, subspace minimisation,
        projected line search: :mod:`multigrad_amd.optim.lbfgsb`), so bounded fits keep
        scipy's semantics (``bounds_mode="transform"`` uses the Adam reparameterisation
        instead).  Models with the fused-engine protocol run it over the engine's (ZeRO-
        or owner-) sharded vectors.  ``"auto"`` picks ``device`` above 1e5 parameters.
        """
        comm = self._opt_comm() if comm is None else comm
        x0 = as_param_tensor(guess, device=self.param_device())
        if method == "auto":
            method = "device" if x0.numel() > 100_000 else "scipy"
        if method == "scipy":
            fn = self.calc_loss_and_grad_from_params
            eng = None
            step_eng = self._step_engine(x0, comm) if (
                getattr(self, "engine_randkey_invariant", False) or randkey is None) else None
            if step_eng is not None:
                # each scipy evaluation is one fused device evaluation (engine/smf2.py)
                fn = step_eng.evaluator()
            elif self._generic_engine_ok(x0):
                # each scipy evaluation replays one captured evaluation (engine/generic.py)
                from ..engine.generic import GraphAdamEngine
                eng = GraphAdamEngine(self, comm=comm)
                fn = eng.evaluator(x0, randkey=None if randkey is None else init_randkey(randkey)
                                   if not hasattr(randkey, "split") else randkey)
            try:
                return _bfgs.run_bfgs(fn, x0, maxsteps=maxsteps,
                                      param_bounds=param_bounds, randkey=randkey, comm=comm,
                                      device=self.param_device(), **kw)
            finally:
                if eng is not None:
                    eng.close()
        from ..optim import lbfgs as _lbfgs
        from ..optim import lbfgsb as _lbfgsb
        hist = kw.pop("history", 10)
        mode = kw.pop("bounds_mode", "project")
        if mode not in ("project", "transform"):
            raise ValueError("bounds_mode must be 'project' or 'transform'")
        fused = getattr(self, "fused_engine", None)
        if fused is not None and randkey is None and (param_bounds is None or mode == "project"):
            eng = fused(comm=comm, **{k: kw.pop(k) for k in ("zero", "chunks") if k in kw})
            if eng is not None:
                try:
                    obj = eng.lbfgs_objective(x0)
                    if param_bounds is None:
                        return _lbfgs.lbfgs_minimize(obj, maxiter=maxsteps, m=hist, **kw)
                    lo, hi = obj.local_box(param_bounds)
                    return _lbfgsb.lbfgsb_minimize(obj, lo, hi, maxiter=maxsteps, m=hist, **kw)
                finally:
                    if not getattr(eng, "cached", False):
                        eng.close()
        if param_bounds is not None and mode == "project":
            return _lbfgsb.run_lbfgsb_device(self.calc_loss_and_grad_from_params, x0,
                                             maxsteps=maxsteps, param_bounds=param_bounds,
                                             randkey=randkey, comm=comm, history=hist, **kw)
        return _lbfgs.run_lbfgs_device(self.calc_loss_and_grad_from_params, x0, maxsteps=maxsteps,
                                       param_bounds=param_bounds, randkey=randkey, comm=comm,
                                       history=hist, **kw)


@dataclass
class OnePointModel(_OptimizerFrontEnds):
    """Differentiable one-point model whose summary statistics add across ranks.

    Subclasses implement two torch-differentiable hooks:

    * ``calc_partial_sumstats_from_params(params[, randkey])`` -> this rank's partial
      sumstats (or ``(sumstats, aux)`` if ``sumstats_func_has_aux``);
    * ``calc_loss_from_sumstats(sumstats[, sumstats_aux][, randkey])`` -> loss (or
      ``(loss, aux)`` if ``loss_func_has_aux``).

    ``randkey`` is forwarded only when not ``None``.  (The reference docstring swaps the
    two ``*_has_aux`` descriptions; the behaviour above follows its code.)

    Parameters
    ----------
    aux_data : any auxiliary data for the hooks (typically this rank's data shard)
    comm : communicator (default: world)
    loss_func_has_aux, sumstats_func_has_aux : aux flags as above
    device : device of the parameters (default: inferred from ``aux_data`` tensors)
    dtype : parameter dtype for non-tensor guesses (default float32)
    """

    aux_data: Any = None
    comm: Any = None
    loss_func_has_aux: bool = False
    sumstats_func_has_aux: bool = False
    device: Any = None
    dtype: Any = None

    # ------------------------------------------------------------------ user hooks
    def calc_partial_sumstats_from_params(self, params, randkey=None):
        """Custom method to map parameters to (partial) summary statistics."""
        raise NotImplementedError(
            "Subclass must implement `calc_partial_sumstats_func_from_params`")

    def calc_loss_from_sumstats(self, sumstats, sumstats_aux=None, randkey=None):
        """Custom method to map summary statistics to loss."""
        raise NotImplementedError("Subclass must implement `calc_loss_func_from_sumstats`")

    # ------------------------------------------------------------------ plumbing
    def __post_init__(self):
        if self.comm is None:
            self.comm = get_world_comm()

    def _opt_comm(self):
        return self.comm

    def param_device(self) -> torch.device:
        if self.device is not None:
            return torch.device(self.device)
        return infer_device(self.aux_data)

    def _params(self, params) -> torch.Tensor:
        return as_param_tensor(params, device=self.param_device(), dtype=self.dtype)

    def _allreduce(self, x: torch.Tensor) -> torch.Tensor:
        x = x.detach().contiguous()
        if self.comm is not None and self.comm.size > 1:
            x = x.clone()
            self.comm.all_reduce(x)
        return x

    def run_lhs_param_scan(self, xmins, xmaxs, n_dim, num_evaluations, seed=None,
                           randkey=None):
        """Sumstats and loss over a Latin-hypercube sample of parameters.

        The sample is drawn on rank 0 and broadcast, so every rank evaluates the same
        points even with ``seed=None`` (reference Q8); with ``sumstats_func_has_aux`` the
        aux is passed to the loss properly (Q9).

        Returns ``(params[num_eval, n_dim], sumstats[num_eval, ...], losses[num_eval])``.
        """
        params = None
        if self.comm is None or self.comm.rank == 0:
            params = util.latin_hypercube_sampler(xmins, xmaxs, n_dim, num_evaluations, seed=seed)
        if self.comm is not None and self.comm.size > 1:
            params = self.comm.bcast(params, root=0)
        rk = _rk(randkey)
        # all partial sumstats first, then ONE all-reduce of the stacked [num_eval, ...]
        # tensor instead of one small collective per evaluation (reference
        # multigrad/multigrad.py:354-388 reduces inside the loop)
        partials, auxes = [], []
        with torch.no_grad():
            for x in params:
                r = self.calc_partial_sumstats_from_params(self._params(x), **rk)
                a = None
                if self.sumstats_func_has_aux:
                    r, a = r
                partials.append(torch.as_tensor(r))
                auxes.append(a)
        if not partials:
            return params, np.array([]), np.array([])
        totals = self._allreduce(torch.stack(partials))
        sumstats, losses = [], []
        for s, a in zip(totals, auxes):
            args = (s, a) if self.sumstats_func_has_aux else (s,)
            loss = self.calc_loss_from_sumstats(*args, **rk)
            if self.loss_func_has_aux:
                loss = loss[0]
            sumstats.append(np.asarray(s.cpu()))
            losses.append(float(loss))
        return params, np.array(sumstats), np.array(losses)

    # ------------------------------------------------------------------ sumstats
    def calc_sumstats_from_params(self, params, total: bool = True, randkey=None):
        """Summary statistics at ``params``, summed over ``comm`` when ``total``."""
        with torch.no_grad():
            result = self.calc_partial_sumstats_from_params(self._params(params), **_rk(randkey))
            aux = None
            if self.sumstats_func_has_aux:
                result, aux = result
            if total:
                result = self._allreduce(torch.as_tensor(result))
        return (result, aux) if self.sumstats_func_has_aux else result

    def calc_dloss_dsumstats(self, sumstats, sumstats_aux=None, randkey=None):
        """Gradient of the loss w.r.t. the (total) sumstats (``(grad, aux)`` with loss aux)."""
        s = torch.as_tensor(sumstats).detach().clone().requires_grad_(True)
        args = (s, sumstats_aux) if self.sumstats_func_has_aux else (s,)
        with torch.enable_grad():
            out = self.calc_loss_from_sumstats(*args, **_rk(randkey))
            loss = out[0] if self.loss_func_has_aux else out
            (g,) = torch.autograd.grad(loss, s, allow_unused=True)
        if g is None:
            g = torch.zeros_like(s)
        return (g, detach_tree(out[1])) if self.loss_func_has_aux else g

    def calc_loss_from_params(self, params, randkey=None):
        """Loss at ``params`` (sumstats summed over all ranks first)."""
        rk = _rk(randkey)
        with torch.no_grad():
            s = self.calc_sumstats_from_params(params, **rk)
            args = s if self.sumstats_func_has_aux else (s,)
            return detach_tree(self.calc_loss_from_sumstats(*args, **rk))

    def calc_dloss_dparams(self, params, randkey=None):
        """Gradient of the loss w.r.t. ``params`` (distributed chain rule)."""
        return self._vjp(params, randkey=randkey, include_loss=False)

    def calc_loss_and_grad_from_params(self, params, randkey=None):
        """``(loss, grad)`` -- cheaper than computing them separately."""
        return self._vjp(params, randkey=randkey, include_loss=True)

    def _vjp(self, params, randkey=None, include_loss=True):
        rk = _rk(randkey)
        p = self._params(params).detach().requires_grad_(True)
        with torch.enable_grad():
            out = self.calc_partial_sumstats_from_params(p, **rk)
            if self.sumstats_func_has_aux:
                partial, saux = out
            else:
                partial, saux = out, None
            partial = torch.as_tensor(partial)
            # (1) all-reduce the partial sumstats
            total = self._allreduce(partial).requires_grad_(True)
            args = (total, saux) if self.sumstats_func_has_aux else (total,)
            # (2) loss and its cotangent on the total sumstats (redundant on every rank)
            loss_out = self.calc_loss_from_sumstats(*args, **rk)
            loss = loss_out[0] if self.loss_func_has_aux else loss_out
            (cot,) = torch.autograd.grad(loss, total, allow_unused=True)
            if cot is None:
                cot = torch.zeros_like(total)
            # (3) local pullback with the global cotangent
            if partial.requires_grad:
                (g,) = torch.autograd.grad(partial, p, cot, allow_unused=True)
            else:
                g = None
        if g is None:
            g = torch.zeros_like(p)
        # (4) all-reduce the parameter gradient
        grad = self._allreduce(g)
        if include_loss:
            return detach_tree(loss_out), grad
        return grad

    # ------------------------------------------------------------------ identity
    def __hash__(self):
        name = getattr(self.comm, "name", None)
        return hash((name, type(self).calc_loss_from_sumstats))

    def __eq__(self, other):
        # identity equality (the reference compares against OnePointGroup)
        return self is other


@dataclass
class OnePointGroup(_OptimizerFrontEnds):
    """Sum of several models' losses, each model on its own sub-communicator.

    Only each sub-communicator's rank 0 contributes its model's ``(loss, grad)``; the
    contributions are summed with ONE all-reduce of a packed ``[loss, grad...]`` vector
    over ``main_comm`` (reference: two pickled allgathers, ``multigrad/multigrad.py:578-580``).
    Ranks may hold different numbers of models.
    """

    models: Union[Tuple[OnePointModel, ...], OnePointModel] = ()
    main_comm: Any = None

    def __post_init__(self):
        if self.main_comm is None:
            self.main_comm = get_world_comm()
        if isinstance(self.models, OnePointModel):
            self.models = (self.models,)
        self.models = tuple(self.models)
        assert len(self.models) and isinstance(self.models[0], OnePointModel)

    def _opt_comm(self):
        return self.main_comm

    @property
    def comm(self):
        return self.main_comm

    def param_device(self) -> torch.device:
        return self.models[0].param_device()

    def calc_loss_and_grad_from_params(self, params, randkey=None):
        rk = _rk(randkey)
        packed, gshape = None, None
        for model in self.models:
            loss, grad = model.calc_loss_and_grad_from_params(params, **rk)
            if isinstance(loss, (tuple, list)):
                loss = loss[0]
            gshape = grad.shape
            vec = torch.cat([torch.as_tensor(loss).reshape(1).to(grad), grad.reshape(-1)])
            if model.comm is not None and model.comm.rank:
                vec = torch.zeros_like(vec)
            packed = vec if packed is None else packed + vec
        if self.main_comm is not None and self.main_comm.size > 1:
            packed = packed.contiguous()
            self.main_comm.all_reduce(packed)
        return packed[0], packed[1:].reshape(gshape)

    def calc_loss_from_params(self, params, randkey=None):
        return self.calc_loss_and_grad_from_params(params, randkey=randkey)[0]

    def calc_dloss_dparams(self, params, randkey=None):
        return self.calc_loss_and_grad_from_params(params, randkey=randkey)[1]

    def __hash__(self):
        return hash((getattr(self.main_comm, "name", None), self.models[0]))

    def __eq__(self, other):
        return self is other
