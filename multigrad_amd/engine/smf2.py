"""Fused optimizer steps of the shared-parameter SMF models (the reference's own workload).

Reference: the 2-parameter SMF fits, tests/smf_example/smf_grad_descent.py:32-82 (the
``MySMFModel`` of :mod:`multigrad_amd.models.smf`) and docs/source/notebooks/
smf_gradient_descent.py:19-91 (``DocsSMFModel``), driven by ``run_simple_grad_descent``
(multigrad/util.py:80-134, the path timed by tests/smf_example/benchmark.py:10-46) or
``run_adam`` (multigrad/adam.py:52-68).

A step is the kernels of ``csrc/smf.hip`` "shared-parameter fused step": ONE pass over the
halos yields, per edge, the bin masses and the two VJP residual sums, and because both
parameters are shared by every halo the gradient is linear in those sums -- so the sumstat
all-reduce and the gradient all-reduce of the reference (multigrad/multigrad.py:522,531-532)
become ONE 32-float one-shot exchange, and the loss, cotangent, gradient and update run in
the same workgroup.  Two schedules:

* ``loop`` (shards of at most ``MULTIGRAD_SMF2_LOOP_MAX`` halos on every rank, default
  65536): one persistent workgroup runs up to ``MULTIGRAD_SMF2_LOOP_STEPS`` whole steps per
  launch -- a step is a few microseconds, so the launch cost is paid once per block.
* ``grid``: a grid forward plus a one-workgroup step kernel per step, replayed from HIP
  graphs of ``graph_steps`` steps (single rank or with the peer-memory exchange; RCCL/gloo
  reductions are not captured, the step then splits around them).

The engine is cached on its model (:meth:`Smf2Engine.for_model`): a second ``run_*`` call
with the same shapes re-uses its buffers, its graphs and its schedule (``stats`` counts
captures), the analogue of JAX's jit cache the reference relies on
(tests/smf_example/benchmark.py:41-46).
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from ._stream import EngineStream, make_engine_stream, on_engine_stream

__all__ = ["Smf2Engine", "smf2_eligible"]


def _ext():
    from ..ops._ext import ext
    return ext()


def smf2_eligible(model) -> bool:
    """Whether ``model`` (an SMF model of :mod:`multigrad_amd.models.smf`) can run on the
    fused step: on a GPU, absolute tails, at most 16 (padded) bins, fp32 shard."""
    if os.environ.get("MULTIGRAD_SMF2", "1").lower() in ("0", "off", "false", "no"):
        return False
    if getattr(model, "dtype", None) not in (None, torch.float32):
        return False   # an fp64 model keeps the PyTorch path
    try:
        dev = model.param_device()
        if dev.type != "cuda":
            return False
        shard, bins = model._setup()
        if bins.rel_tail or shard.pop is not None:
            return False
        return int(_ext().smf_padded_bins(bins.nb)) <= int(_ext().smf2_max_bins())
    except Exception:  # noqa: BLE001  (no extension: the generic path)
        return False


class Smf2Engine:
    """Device-resident fused GD / Adam / evaluation for a shared-parameter SMF model."""

    def __init__(self, model, comm=None):
        self.model = model
        self.comm = model.comm if comm is None else comm
        self.size = 1 if self.comm is None else self.comm.size
        self.rank = 0 if self.comm is None else self.comm.rank
        shard, bins = model._setup()
        self.shard, self.bins = shard, bins
        self.x = shard.x
        self.n = int(shard.n)
        self.device = shard.device
        self.log_sigma = bool(model._log_sigma)
        self.loss_eps = float(model._loss_eps)
        self.target = model._target
        self.edges, self.scale = list(bins.edges), list(bins.scale)
        self.R = 3 * int(_ext().smf_padded_bins(bins.nb)) + 2
        self._es = None
        self.stats = {"captures": 0, "setups": 0, "launches": 0}
        self._graphs = {}
        self._cap = -1
        self.oneshot = None
        nmax = self.n
        if self.size > 1:
            t = torch.tensor([self.n], dtype=torch.int64)
            self.comm.all_reduce(t, op="max")
            nmax = int(t.item())
            from ..parallel.xgmi import get_oneshot
            self.oneshot = get_oneshot(self.comm)  # collective
        self.nmax = nmax
        lm = int(os.environ.get("MULTIGRAD_SMF2_LOOP_MAX", str(1 << 16)))
        sched = os.environ.get("MULTIGRAD_SMF2_SCHEDULE", "auto").lower()
        # the persistent loop carries its exchange inside the launch: it needs the peer
        # exchange on several ranks
        loop_ok = self.size == 1 or self.oneshot is not None
        self.schedule = ("loop" if (sched == "loop" or (sched == "auto" and nmax <= lm))
                         and loop_ok else "grid")
        self.loop_steps = max(1, int(os.environ.get("MULTIGRAD_SMF2_LOOP_STEPS", "1000")))
        self.graph_steps = max(1, int(os.environ.get("MULTIGRAD_SMF2_GRAPH_STEPS", "16")))
        self.use_graph = (os.environ.get("MULTIGRAD_GRAPH", "1") != "0"
                          and (self.size == 1 or self.oneshot is not None))
        blocks = int(_ext().smf2_fwd_max_blocks(bins.nb, self.log_sigma))
        # at least MULTIGRAD_SMF2_HALOS_PER_THREAD halos per thread: fewer slab rows for the
        # one-workgroup step kernel to sum when the shard is small
        hpt = max(1, int(os.environ.get("MULTIGRAD_SMF2_HALOS_PER_THREAD", "16")))
        self.nblocks = max(1, min(blocks, -(-max(self.n, 1) // (256 * hpt)), 65535))
        f32 = dict(dtype=torch.float32, device=self.device)
        self.slab = torch.zeros(self.nblocks * self.R, **f32)
        self.theta = torch.zeros(2, **f32)
        self.u = torch.zeros(2, **f32)
        self.m = torch.zeros(2, **f32)
        self.v = torch.zeros(2, **f32)
        self.step_dev = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.grad = torch.zeros(2, **f32)
        self.S = torch.zeros(max(16, bins.nb), **f32)
        self.loss = torch.zeros(1, **f32)
        self.vals = torch.zeros(64, **f32)
        self.loss_hist = torch.zeros(1, **f32)
        self.param_hist = torch.zeros(2, **f32)
        self.nsteps = 0
        self.scalars = None
        self.step_host = 0
        self._warm()

    @on_engine_stream(always=True)
    def _warm(self) -> None:
        """One evaluation at a dummy point: loads the code objects before anything is
        captured (the first ``run_*`` call is the "compile" step, as jit's first call)."""
        self.setup(torch.tensor([0.0, 1.0]), 0, "eval")
        if self.schedule == "loop":
            peers, rank, seq, err = self._peer_args()
            _ext().smf2_loop(self.x, self.edges, self.scale, self.log_sigma, self._state(),
                             self.scalars, peers, rank, seq, err, 1)
        else:
            self._launch_grid_step()

    # ------------------------------------------------------------------ cache
    @classmethod
    def for_model(cls, model, comm=None) -> Optional["Smf2Engine"]:
        """The model's cached engine (created on first use, collective on several ranks);
        rebuilt when the model's data, device or communicator changed; None when the
        model is not eligible (:func:`smf2_eligible`)."""
        comm = model.comm if comm is None else comm
        if not smf2_eligible(model):
            return None
        shard, _ = model._setup()
        key = (id(shard), id(comm), str(shard.device))
        eng = model.__dict__.get("_smf2_engine")
        if eng is not None and eng._key == key:
            return eng
        eng = cls(model, comm)
        eng._key = key
        model.__dict__["_smf2_engine"] = eng
        return eng

    # ------------------------------------------------------------------ stream
    def _engine_stream(self):
        self._es = make_engine_stream(self._es, self.device)
        return self._es

    def _stream_wanted(self) -> bool:
        return True

    # ------------------------------------------------------------------ state
    def _ensure_capacity(self, nsteps: int) -> None:
        if nsteps > self._cap:
            cap = max(nsteps, 2 * max(self._cap, 0), 4096)
            f32 = dict(dtype=torch.float32, device=self.device)
            self.loss_hist = torch.zeros(cap, **f32)
            self.param_hist = torch.zeros(2 * (cap + 1), **f32)
            self._cap = cap
            self._graphs.clear()  # captured with the old buffers

    def _state(self):
        return [self.target, self.theta, self.u, self.m, self.v, self.step_dev, self.loss_hist,
                self.param_hist, self.grad, self.S, self.loss, self.vals]

    @on_engine_stream(always=True)
    def setup(self, guess, nsteps: int, opt: str = "gd", learning_rate: float = 0.01,
              b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8, param_bounds=None,
              legacy_bounds_jacobian: bool = False):
        """Start a run of ``nsteps`` steps from ``guess`` (``opt``: gd | adam | eval)."""
        from ..optim.transforms import Bounds
        nsteps = int(nsteps)
        self._ensure_capacity(max(nsteps, 1))
        p0 = torch.as_tensor(guess, dtype=torch.float32).reshape(-1).to(self.device)
        if p0.numel() != 2:
            raise ValueError(f"the shared-parameter SMF models take 2 parameters, got {p0.numel()}")
        lo, hi = [-math.inf, -math.inf], [math.inf, math.inf]
        bounded = False
        if param_bounds is not None and opt == "adam":
            bnd = Bounds.from_spec(param_bounds, 2, device=self.device)
            if bnd is not None:
                bounded = True
                lo = [float(v) for v in bnd.lo.cpu()]
                hi = [float(v) for v in bnd.hi.cpu()]
                u0 = bnd.forward(p0)
                p0 = bnd.inverse(u0)        # the recorded start is T^-1(T(guess))
                self.u.copy_(u0)
        if not bounded:
            self.u.copy_(p0)
        self.theta.copy_(p0)
        self.m.zero_()
        self.v.zero_()
        self.step_dev.zero_()
        self.param_hist[:2].copy_(p0)
        self.nsteps = nsteps
        code = {"gd": 0, "adam": 1, "eval": 2}[opt]
        timeout = self.oneshot.timeout_s if self.oneshot is not None else 5.0
        self.scalars = [self.loss_eps, float(learning_rate), float(b1), float(b2), float(eps),
                        float(code), float(bool(legacy_bounds_jacobian)), float(bounded),
                        float(self._cap), lo[0], lo[1], hi[0], hi[1], float(timeout)]
        self.step_host = 0
        self.stats["setups"] += 1
        if self.schedule == "grid" and self.use_graph and code != 2 and self.graph_steps > 1:
            # captured once per schedule (even by a 1-step warm-up call: the "compile" step
            # of the reference's benchmark), then cached
            self._graph(self.graph_steps)
        return self

    # ------------------------------------------------------------------ launches
    def _peer_args(self):
        if self.size > 1 and self.oneshot is not None:
            return self.oneshot.peers, self.oneshot.rank, self.oneshot.seq, self.oneshot.err
        return [], 0, None, None

    def _launch_grid_step(self):
        E = _ext()
        E.smf2_forward(self.x, self.theta, self.edges, self.scale, self.log_sigma, self.slab,
                       self.nblocks)
        peers, rank, seq, err = self._peer_args()
        if self.size > 1 and self.oneshot is None:
            # no peer exchange: local sums -> RCCL / gloo all-reduce -> the rest of the step
            E.smf2_step(self.slab, self.nblocks, self.edges, self.scale, self.log_sigma,
                        self._state(), self.scalars, [], 0, None, None, 1)
            self.comm.all_reduce(self.vals[:self.R])
            E.smf2_step(self.slab, self.nblocks, self.edges, self.scale, self.log_sigma,
                        self._state(), self.scalars, [], 0, None, None, 2)
        else:
            E.smf2_step(self.slab, self.nblocks, self.edges, self.scale, self.log_sigma,
                        self._state(), self.scalars, peers, rank, seq, err, 0)
        self.stats["launches"] += 2

    def _graph_key(self, k: int):
        return (k, tuple(self.scalars))

    def _graph(self, k: int):
        """The graph of k grid steps for the current scalars (captured on first use; a
        capture runs nothing, the kernels read all state from device memory)."""
        key = self._graph_key(k)
        g = self._graphs.get(key)
        if g is None and not torch.cuda.is_current_stream_capturing():
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=torch.cuda.current_stream()):
                for _ in range(k):
                    self._launch_grid_step()
            # one graph per scalar set (learning rate, optimizer, bounds): a sweep over
            # learning rates must not grow the cache without bound
            while len(self._graphs) >= 8:
                self._graphs.pop(next(iter(self._graphs)))
            self._graphs[key] = g
            self.stats["captures"] += 1
        return g

    def _replay(self, k: int) -> bool:
        g = self._graph(k)
        if g is None:
            return False
        g.replay()
        return True

    @on_engine_stream(always=True)
    def steps(self, n: int) -> None:
        """Run ``n`` optimizer steps (no host synchronisation)."""
        n = int(n)
        if n <= 0:
            return
        if self.step_host + n > self.nsteps and self.scalars[5] != 2:
            raise RuntimeError(f"{self.step_host + n} steps requested, setup() was for "
                               f"{self.nsteps}")
        E = _ext()
        if self.schedule == "loop":
            peers, rank, seq, err = self._peer_args()
            done = 0
            while done < n:
                k = min(self.loop_steps, n - done)
                E.smf2_loop(self.x, self.edges, self.scale, self.log_sigma, self._state(),
                            self.scalars, peers, rank, seq, err, k)
                self.stats["launches"] += 1
                done += k
        else:
            done = 0
            G = self.graph_steps
            while n - done >= G and self.use_graph and G > 1:
                if not self._replay(G):
                    break
                done += G
            while done < n:
                self._launch_grid_step()
                done += 1
        self.step_host += n

    def check(self, where: str = "") -> None:
        if self.oneshot is not None:
            self.oneshot.check(where or "SMF fused step", comm=self.comm)

    # ------------------------------------------------------------------ drivers
    @on_engine_stream(always=True)
    def run_simple_grad_descent(self, guess, nsteps: int = 100, learning_rate: float = 0.01,
                                callback=None):
        """Reference multigrad/util.py:80-134: ``GradDescentResult(loss[i], params[i], aux)``
        with ``params[i]`` the point ``loss[i]`` was evaluated at."""
        from ..utils.hooks import StepHooks, driver_guard
        from ..utils.util import GradDescentResult
        self.setup(guess, nsteps, "gd", learning_rate)
        hooks = StepHooks(self.comm, callback)
        with driver_guard(self.comm):
            self._drive(nsteps, hooks)
        self.check("simple_grad_descent")
        n = int(nsteps)
        return GradDescentResult(loss=self.loss_hist[:n].clone(),
                                 params=self.param_hist[:2 * n].reshape(n, 2).clone(),
                                 aux=[None] * n)

    @on_engine_stream(always=True)
    def run_adam(self, guess, nsteps: int = 100, param_bounds=None, learning_rate: float = 0.01,
                 b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8, history="full",
                 legacy_bounds_jacobian: bool = False, callback=None, **unused):
        """Reference multigrad/adam.py:52-68: trajectory ``(nsteps+1, 2)`` (``history``:
        full, last, or a stride)."""
        if unused:
            raise TypeError(f"unsupported run_adam options for the SMF fused step: {sorted(unused)}")
        from ..utils.hooks import StepHooks, driver_guard
        self.setup(guess, nsteps, "adam", learning_rate, b1, b2, eps, param_bounds,
                   legacy_bounds_jacobian)
        hooks = StepHooks(self.comm, callback)
        with driver_guard(self.comm):
            self._drive(nsteps, hooks)
        self.check("run_adam")
        n = int(nsteps)
        traj = self.param_hist[:2 * (n + 1)].reshape(n + 1, 2)
        if history == "last":
            return traj[-1:].clone()
        if history not in (None, "full"):
            stride = int(history)
            idx = list(range(0, n + 1, stride))
            if idx[-1] != n:
                idx.append(n)
            return traj[idx].clone()
        return traj.clone()

    def _drive(self, nsteps: int, hooks) -> None:
        if not hooks.active:
            self.steps(nsteps)
            return
        for i in range(int(nsteps)):
            self.steps(1)
            hooks(i, self.loss, self, lambda: self.theta.clone())

    # L-BFGS / scipy evaluations: loss and gradient at a point, no update
    def evaluator(self):
        """``fn(params) -> (loss, grad)`` device tensors: one fused evaluation (forward,
        exchange, loss, residual VJP) per call, no update -- the evaluation function of the
        scipy L-BFGS-B driver (reference multigrad/bfgs.py:72-77)."""
        def fn(params, randkey=None):
            with EngineStream(self):
                if self.scalars is None or self.scalars[5] != 2:
                    self.setup(params, 0, "eval")
                self.theta.copy_(torch.as_tensor(params, dtype=torch.float32).reshape(-1)
                                 .to(self.device))
                if self.schedule == "loop":
                    peers, rank, seq, err = self._peer_args()
                    _ext().smf2_loop(self.x, self.edges, self.scale, self.log_sigma,
                                     self._state(), self.scalars, peers, rank, seq, err, 1)
                else:
                    self._launch_grid_step()
                loss, grad = self.loss[0].clone(), self.grad.clone()
            return loss, grad
        return fn

    # engine API of the model front-ends
    def params(self) -> torch.Tensor:
        return self.theta.clone()

    def close(self) -> None:
        """Kept for the engine interface: the cached engine stays alive with its model."""
        return None
