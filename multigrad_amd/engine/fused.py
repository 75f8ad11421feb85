"""Fused, device-resident Adam engine (HIP kernels + stream-ordered collectives).

The generic path (``OnePointModel.run_adam``) runs the distributed chain rule through
autograd with Python in the loop.  Models that expose the *engine protocol* run instead
as a fixed sequence of device operations per step, with no host synchronisation:

    partial sumstats  (fwd kernel + deterministic slab reduce)     -> S
    all-reduce(S)     (RCCL, latency bound, K floats)
    loss + edge weights from S (1 tiny kernel)                     -> loss, h
    local VJP         (segmented per-population kernel)            -> g
    all-reduce(g)     (RCCL, bandwidth bound, P floats) -- or reduce-scatter + all-gather
                      with the optimizer sharded across ranks (ZeRO-1 style)
    fused Adam        (1 HBM pass: moments, bias correction, transform, trajectory row)

On a single GPU the whole step is captured once into a HIP graph and replayed
(``torch.cuda.CUDAGraph``); the device step counter inside the Adam kernel makes the
replay self-advancing.  This replaces the reference's per-step host round trips
(4 host crossings per Adam step, 2 of them pickled broadcasts).

Engine protocol (see :class:`~multigrad_amd.models.population.PopulationSMFModel`):
``engine_sizes() -> (P, nS, nH, fwd_blocks)``, ``engine_partial_into(theta, S, slab)``,
``engine_loss_into(S, loss, h)``, ``engine_vjp_into(theta, h, grad)``.
"""
from __future__ import annotations

import os
import time
from typing import Optional

import torch

from ..optim.adam import History
from ..optim.transforms import Bounds
from ..ops import adam as adam_ops

__all__ = ["FusedAdamEngine"]


def _env_flag(name: str, default: Optional[bool]) -> Optional[bool]:
    v = os.environ.get(name)
    if v is None:
        return default
    return v.lower() not in ("0", "false", "off", "no")


class FusedAdamEngine:
    """Device-resident Adam for a model implementing the engine protocol.

    Parameters
    ----------
    model : the model (its ``comm`` is used for the collectives)
    graph : capture the step into a HIP graph (default: on for a single rank; env
        ``MULTIGRAD_GRAPH`` overrides)
    """

    def __init__(self, model, comm=None, graph: Optional[bool] = None):
        self.model = model
        self.comm = model.comm if comm is None else comm
        self.size = 1 if self.comm is None else self.comm.size
        g = _env_flag("MULTIGRAD_GRAPH", graph)
        self.use_graph = (self.size == 1) if g is None else bool(g)
        self.graph = None
        self.ready = False

    # ------------------------------------------------------------------ setup
    def setup(self, guess, nsteps: int, param_bounds=None, learning_rate: float = 0.01,
              b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8, history="full",
              legacy_bounds_jacobian: bool = False):
        P, nS, nH, nblk = self.model.engine_sizes()
        dev = self.model.param_device()
        p0 = torch.as_tensor(guess).detach().reshape(-1).to(device=dev, dtype=torch.float32)
        assert p0.numel() == P, f"guess has {p0.numel()} params, model expects {P}"
        self.P = P
        self.lr, self.b1, self.b2, self.eps = float(learning_rate), float(b1), float(b2), float(eps)
        self.bounds = Bounds.from_spec(param_bounds, P, device=dev)
        self.legacy = bool(legacy_bounds_jacobian)
        if self.bounds is not None:
            self.u = self.bounds.forward(p0).contiguous()
            self.theta = self.bounds.inverse(self.u).contiguous()
        else:
            self.u = p0.clone()
            self.theta = self.u
        self.m = torch.zeros_like(self.u)
        self.v = torch.zeros_like(self.u)
        self.grad = torch.zeros_like(self.u)
        self.S = torch.zeros(nS, dtype=torch.float32, device=dev)
        self.slab = torch.zeros(max(nblk, 1) * nS, dtype=torch.float32, device=dev)
        self.h = torch.zeros(nH, dtype=torch.float32, device=dev)
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self.step_dev = torch.zeros(2, dtype=torch.int32, device=dev)
        self.step_host = 0
        self.nsteps = int(nsteps)
        self.history = History(history, nsteps, self.theta.detach().clone())
        self.graph = None
        self.ready = True
        return self

    # ------------------------------------------------------------------ one step
    def _enqueue_step(self):
        md = self.model
        md.engine_partial_into(self.theta, self.S, slab=self.slab)
        if self.size > 1:
            self.comm.all_reduce(self.S)
        md.engine_loss_into(self.S, self.loss, self.h)
        md.engine_vjp_into(self.theta, self.h, self.grad)
        if self.size > 1:
            self.comm.all_reduce(self.grad)
        traj_base, stride = None, 0
        if self.history.mode == "full":
            traj_base, stride = self.history.buf.reshape(-1), self.P
        adam_ops.fused_adam_(self.u, self.m, self.v, self.grad,
                             self.theta if self.bounds is not None else None, self.step_dev,
                             self.lr, self.b1, self.b2, self.eps, self.bounds, self.legacy,
                             traj_base=traj_base, traj_stride=stride)

    def _capture(self):
        # warm the allocator/stream state on a side stream, then capture one step
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        torch.cuda.current_stream().wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._enqueue_step()

    def step(self):
        """Enqueue one optimizer step (asynchronous)."""
        assert self.ready, "call setup() first"
        if self.step_host >= self.nsteps and self.history.mode == "full":
            raise RuntimeError("more steps than the trajectory buffer was sized for")
        if self.use_graph:
            if self.graph is None:
                self._capture()
            self.graph.replay()
        else:
            self._enqueue_step()
        self.step_host += 1
        if self.history.mode != "full":
            self.history.record(self.step_host - 1, self.theta)

    def params(self) -> torch.Tensor:
        return self.theta

    def last_loss(self) -> float:
        return float(self.loss.item())

    # ------------------------------------------------------------------ driver
    def run_adam(self, guess, nsteps: int = 100, param_bounds=None, learning_rate: float = 0.01,
                 b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8, history="full",
                 legacy_bounds_jacobian: bool = False, callback=None, **unused):
        """Adam with the reference's return contract: trajectory ``(nsteps+1, P)``."""
        self.setup(guess, nsteps, param_bounds, learning_rate, b1, b2, eps, history,
                   legacy_bounds_jacobian)
        for i in range(int(nsteps)):
            self.step()
            if callback is not None:
                callback(i, self.loss, self)
        return self.history.result()
