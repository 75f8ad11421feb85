"""Graph-captured Adam engine for ANY torch ``OnePointModel`` or ``OnePointGroup``.

The reference's distributed chain rule works for every user model
(multigrad/multigrad.py:508-538) and its Adam loop is ``jax.example_libraries`` Adam
driven from Python (multigrad/adam.py:52-68).  The eager equivalent here
(``OnePointModel._vjp`` + :func:`multigrad_amd.optim.adam.run_adam`) launches every torch
op of the user's hooks from Python each step.  This engine instead records ONE optimizer
step of a user model -- its autograd forward, the sumstat all-reduce, the loss cotangent,
the VJP, the dense-gradient sum and the fused Adam update with the trajectory write --
into a HIP graph, and replays it:

    partial = calc_partial_sumstats_from_params(p[, randkey])   # user hook, autograd
    S = sum_ranks(partial)       one-shot xGMI kernel (<= 64 fp32) | RCCL
    cot = d loss(S[, aux][, randkey]) / dS                      # user hook, autograd
    g = VJP(partial, p, cot)
    world 1:  fused Adam (bounded or not) + trajectory row  (csrc/adam.hip)
    world W:  two-shot kernel: reduce-scatter g -> Adam on the owned 1/W -> all-gather p
              (csrc/xgmi.hip), or RCCL all-reduce + fused Adam

What the reference API allows, the engine runs (reference multigrad/multigrad.py):

* ``sumstats_func_has_aux`` (``:518-523``): the aux stays on its rank and goes to the loss
  hook as its second argument, exactly as in the eager chain rule.
* per-step ``randkey`` / ``const_randkey`` (``multigrad/adam.py:59-62``,
  ``multigrad.py:289-300``): the keys follow the eager driver's sequence (one split per
  step, the same on every rank).  Eager steps hand the hooks the step's key.  A captured
  step hands them a capture key whose ``generator(device)`` returns a CUDA generator
  registered with the graph; before each replay the engine seeds those generators with
  the step's key, so a replay draws exactly what a fresh ``key.generator(device)`` would
  (same Philox seed, offset 0).  Any other use of the key inside a hook (its integer
  value, a split, a host generator) cannot be replayed and sends the run down the eager
  path, decided collectively.
* ``OnePointGroup`` (``:547-607``): each member's chain rule runs on its own
  sub-communicator (one-shot sumstat sum per sub-communicator); every rank adds its local
  VJPs, and the main communicator sums ``[grad]`` once -- the two-shot Adam exchange -- and
  the group loss (each sub-communicator's rank 0 contributes its member's loss) with one
  1-float one-shot exchange.  The reference all-reduces each member's gradient on its
  sub-communicator and then all-gathers ``[loss, grad]`` over the main communicator; the
  sum is the same, with one dense exchange instead of two.

A step is replayable only if every collective in it is a peer-memory kernel with its
sequence number on the device (one rank, or one-shot + two-shot) with fp32 sumstats of at
most 64 values, and the user hooks make no host synchronisation; the step counter lives on
the device so replays self-advance.  Anything else runs the same step eagerly (the reason
is kept in ``fallback_reason``).  By default the engine times a few eager steps against a
few replays and keeps the faster mode (``tuning``).

On several ranks the two-shot exchange owns the parameters in peer memory (uncached); the
hooks read a cached copy refreshed once per step (``p``), so a gather-heavy torch model
does not read its parameters through uncached memory.

The gradient exchange is one bucket after the VJP: the reference API gives a model ONE
parameter array (multigrad/multigrad.py:482), so autograd delivers the whole gradient at
once and there is nothing to overlap inside the VJP.
"""
from __future__ import annotations

import math
import os
import weakref
from typing import Optional

import torch

from ._stream import EngineStream, make_engine_stream, on_engine_stream
from ..ops.adam import adam_step_
from ..optim.adam import History
from ..optim.transforms import Bounds
from ..utils.random import PRNGKey, init_randkey
from ..utils.tensors import as_param_tensor


def _give_back_ar(ts, pins) -> None:
    """Finalizer of an engine's hold on a two-shot all-reduce context: the hold and the
    pins of the engine's captured graphs (``pins``: a one-element list, updated by the
    engine as it captures)."""
    from ..parallel.xgmi import release_twoshot_allreduce, unpin_twoshot_allreduce
    unpin_twoshot_allreduce(ts, pins[0])
    pins[0] = 0
    release_twoshot_allreduce(ts)


__all__ = ["GraphAdamEngine", "KeyNotCapturable"]


class KeyNotCapturable(RuntimeError):
    """A hook used its randkey in a way a graph replay cannot reproduce."""


class KeyAttributeNotCapturable(KeyNotCapturable, AttributeError):
    """An attribute of the capture-time randkey other than ``generator``: also an
    AttributeError, so ``hasattr(randkey, name)`` is False and ``getattr(randkey, name,
    default)`` returns the default inside a captured step (a hook that only probes the key
    stays capturable); using the attribute sends the run to the eager path."""


class _CaptureKey:
    """The ``randkey`` the hooks see while a step is captured: only
    ``generator(<cuda device>)`` is allowed (graph-registered, seeded before each replay)."""

    dtype = "prng_key"

    def __init__(self, eng: "GraphAdamEngine"):
        object.__setattr__(self, "_eng", eng)

    def generator(self, device="cpu") -> torch.Generator:
        return self._eng._next_generator(device)

    def __getattr__(self, name):
        if name.startswith("__") and name.endswith("__"):
            raise AttributeError(name)  # protocol probes (copy, pickle, ...)
        raise KeyAttributeNotCapturable(
            f"randkey.{name} inside a captured step: only randkey.generator(<cuda device>) "
            f"can be replayed with a fresh key per step")


class _no_gc:
    """Collect garbage now and keep the cyclic collector off during a graph capture: a
    CUDAGraph freed by the collector while another graph is being captured aborts the
    process (hipGraphExecDestroy is not permitted on a capturing stream)."""

    def __enter__(self):
        import gc
        gc.collect()
        self._was = gc.isenabled()
        gc.disable()

    def __exit__(self, *exc):
        import gc
        if self._was:
            gc.enable()
        return False


def _leaf_view(p: torch.Tensor, shape) -> torch.Tensor:
    return p.detach().view(shape).requires_grad_(True)


def _step_replay_default() -> bool:
    """``MULTIGRAD_STEP_REPLAY``: whether direct ``step()`` calls may replay graphs."""
    return os.environ.get("MULTIGRAD_STEP_REPLAY", "0").strip().lower() in ("1", "on", "true", "yes")


class GraphAdamEngine:
    """Adam over a generic :class:`~multigrad_amd.models.onepoint.OnePointModel` (or a
    :class:`~multigrad_amd.models.onepoint.OnePointGroup` of them).

    ``graph``: None (default) = capture when the step is capturable; False = eager;
    True = capture or raise.  ``MULTIGRAD_GRAPH`` overrides None."""

    def __init__(self, model, comm=None, graph: Optional[bool] = None):
        from ..models.onepoint import OnePointGroup
        self.model = model
        self.group = isinstance(model, OnePointGroup)
        self.members = tuple(model.models) if self.group else (model,)
        default = model.main_comm if self.group else model.comm
        self.comm = default if comm is None else comm
        self.size = 1 if self.comm is None else self.comm.size
        self.rank = 0 if self.comm is None else self.comm.rank
        env = os.environ.get("MULTIGRAD_GRAPH")
        if graph is None and env is not None:
            graph = env.lower() not in ("0", "false", "off", "no")
        self.graph_req = graph
        self.graph = None
        self._kgraph = None
        self.graph_steps = max(1, int(os.environ.get("MULTIGRAD_GRAPH_STEPS", "16")))
        # direct step() calls replay graphs only when the caller promises to launch nothing
        # on the legacy default stream between them (engine/_stream.py); the engine's own
        # drivers (steps(), run_adam, run_simple_grad_descent) always may
        self.step_replay = _step_replay_default()
        self.use_graph = False
        self.fallback_reason = None
        self.oneshot = None          # main-communicator one-shot (group loss)
        self.m_oneshot = [None] * len(self.members)  # per-member sumstat one-shot
        self.twoshot = None
        self.ar = None
        self.mode = "adam"   # "sgd": fixed-rate gradient descent; "eval": scipy objective
        self._gens = []
        self._gen_i = 0
        self._cap_key = _CaptureKey(self)
        self.key_mode = None     # None | "step" | "const"
        self.ready = False
        self._es = None          # the engine's own stream (stream())
        self._dev_step_stale = False  # eager steps ran since the device step was last set

    # ------------------------------------------------------------------ stream
    def _engine_stream(self):
        dev = getattr(self, "device", None)
        self._es = make_engine_stream(self._es, dev if dev is not None
                                      else self.members[0].param_device())
        return self._es

    def _stream_wanted(self) -> bool:
        """Launch on the engine stream while a graph may be replayed: graph mode, or any
        captured graph still held (eager steps between replays belong there too)."""
        return bool(getattr(self, "use_graph", False) or getattr(self, "graph", None) is not None
                    or getattr(self, "_kgraph", None) is not None)

    def stream(self):
        """Context manager: the current stream becomes the engine's own (non-default) HIP
        stream, ordered after the caller's stream on entry and before it on exit.

        Every public method of the engine runs its GPU work -- eager steps, captures, graph
        replays, and the user hooks and callbacks it calls -- inside this context.  On this
        ROCm runtime a graph replay that follows a host synchronisation and any launch on
        the legacy default stream since the graph's previous replay computes wrong results
        (garbage in the graph's intermediates), while the same schedules with nothing
        launched on the default stream match eager launches bit for bit
        (tools/dbg/torch_replay_bisect.py, torch only; docs/design.md "Graph replays and the
        default stream").  User code that calls :meth:`step` directly and launches its own
        GPU work between the calls should do that work inside ``with engine.stream():``."""
        return EngineStream(self, always=False)

    # ------------------------------------------------------------------ keys
    def _next_generator(self, device) -> torch.Generator:
        dev = torch.device(device)
        if dev.type != "cuda":
            raise KeyNotCapturable(
                f"randkey.generator({device!r}) inside a captured step: a host generator's "
                f"draws would be frozen into the graph; use the model's CUDA device")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        if self._gen_i == len(self._gens):
            self._gens.append(torch.Generator(device=dev))
        g = self._gens[self._gen_i]
        if g.device != dev:
            raise KeyNotCapturable(f"randkey.generator({device!r}) on another device than "
                                   f"the engine's {self.device}")
        self._gen_i += 1
        return g

    def _step_key(self) -> Optional[PRNGKey]:
        """This step's key (host; the eager driver's sequence, multigrad/adam.py:59-62)."""
        if self.key_mode is None:
            return None
        if self.key_mode == "const":
            return self.key
        self.key, k = self.key.split(2)
        return k

    def _seed_generators(self, key: Optional[PRNGKey]) -> None:
        if key is not None:
            for g in self._gens:
                g.manual_seed(key.seed)

    # ------------------------------------------------------------------ setup
    @on_engine_stream(always=True)
    def setup(self, guess, nsteps: int, param_bounds=None, learning_rate: float = 0.01,
              b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8, history="full",
              legacy_bounds_jacobian: bool = False, randkey=None, const_randkey: bool = False):
        self.close()
        md0 = self.members[0]
        p0 = as_param_tensor(guess, device=md0.param_device()).detach()
        self.shape = tuple(p0.shape)
        p0 = p0.reshape(-1).to(torch.float32)
        dev = p0.device
        self.device = dev
        self.P = P = p0.numel()
        W = self.size
        self.lr, self.b1, self.b2, self.eps = float(learning_rate), float(b1), float(b2), float(eps)
        self.legacy = bool(legacy_bounds_jacobian)
        if const_randkey:
            assert randkey is not None, "Must pass randkey if const_randkey"
            self.key_mode, self.key = "const", (randkey if hasattr(randkey, "split")
                                                else init_randkey(randkey))
        elif randkey is not None:
            self.key_mode, self.key = "step", init_randkey(randkey)
        else:
            self.key_mode, self.key = None, None
        bounds = Bounds.from_spec(param_bounds, P, device=dev)
        cuda = dev.type == "cuda"
        sgd = self.mode in ("sgd", "eval")   # modes that need the summed gradient itself
        self.ar = None
        self.twoshot = None
        self.oneshot = None
        self.m_oneshot = [None] * len(self.members)
        if cuda:
            from ..parallel.xgmi import (acquire_twoshot, get_oneshot, get_twoshot_allreduce,
                                         twoshot_enabled)
            if W > 1:
                q = 4 * W
                P_pad = -(-P // q) * q
                if sgd:  # the summed gradient itself is needed: a capturable all-reduce
                    self.ar = get_twoshot_allreduce(self.comm, P, hold=True)
                    # the hold and the pins of this engine's graphs go back to the
                    # communicator's cache at close() -- or when the engine is dropped
                    # without it (the finalizer holds no reference to the engine)
                    self._ar_pins = [0]
                    self._ar_fin = weakref.finalize(self, _give_back_ar, self.ar, self._ar_pins)
                else:
                    self.twoshot = acquire_twoshot(self.comm, P_pad) if twoshot_enabled() else None
                if self.group:
                    self.oneshot = get_oneshot(self.comm)  # the group loss
            # collective per sub-communicator (every member rank runs setup)
            self.m_oneshot = [get_oneshot(md.comm) if md.comm is not None and md.comm.size > 1
                              else None for md in self.members]
        self.P_pad = P_pad if self.twoshot is not None else P
        # which dense-gradient exchange the run uses (kept after close())
        self.grad_exchange = ("none" if W == 1 else "two-shot" if self.twoshot is not None
                              else "two-shot all-reduce" if self.ar is not None else "rccl/gloo")
        f32 = dict(dtype=torch.float32, device=dev)
        # the hooks read p (cached memory); with the two-shot exchange the parameters live
        # in its uncached peer-memory region and p is refreshed from it after each step
        self.p = torch.zeros(self.P_pad, **f32)
        if self.twoshot is not None:
            self.theta = self.twoshot.theta
            self.theta.zero_()
            self.gbuf = self.twoshot.grad
            self.gbuf.zero_()
        else:
            self.theta = self.p
            self.gbuf = None
        start = bounds.inverse(bounds.forward(p0)) if bounds is not None else p0
        self.theta[:P].copy_(start)
        if self.theta is not self.p:
            self.p[:P].copy_(start)
        if bounds is not None and self.P_pad > P:
            pad = self.P_pad - P
            bounds = Bounds(torch.cat([bounds.lo, torch.full((pad,), -math.inf, **f32)]),
                            torch.cat([bounds.hi, torch.full((pad,), math.inf, **f32)]),
                            torch.cat([bounds.kind, torch.zeros(pad, dtype=torch.int8, device=dev)]))
        self.bounds = bounds
        if self.twoshot is not None:
            lo_, n_ = self.twoshot.slice()
            self.own = (lo_, lo_ + n_)
            self.m = torch.zeros(n_, **f32)
            self.v = torch.zeros(n_, **f32)
            self.bounds_loc = None if bounds is None else Bounds(
                bounds.lo[lo_:lo_ + n_].contiguous(), bounds.hi[lo_:lo_ + n_].contiguous(),
                bounds.kind[lo_:lo_ + n_].contiguous())
            self.u = None if bounds is None else self.bounds_loc.forward(self.theta[lo_:lo_ + n_]).contiguous()
        else:
            self.own = (0, self.P_pad)
            self.m = torch.zeros(self.P_pad, **f32)
            self.v = torch.zeros(self.P_pad, **f32)
            self.bounds_loc = bounds
            self.u = bounds.forward(self.p).contiguous() if bounds is not None else self.p
        self.step_dev = torch.zeros(2, dtype=torch.int32, device=dev)
        self._dev_step_stale = False
        self.loss = torch.zeros(1, **f32)
        self.nsteps = int(nsteps)
        self.step_host = 0
        self.history_mode = history
        if self.twoshot is not None and history == "full":
            a, b = self.own
            self.traj_loc = torch.zeros((self.nsteps + 1, b - a), **f32)
            self.traj_loc[0] = self.theta[a:b]
            self.history = History("last", nsteps, self.p[:P].clone())
        else:
            self.traj_loc = None
            self.history = History(history, nsteps, self.p[:P].clone())
        if self.mode == "sgd":  # losses and the parameters they were evaluated at
            self.loss_hist = torch.zeros(self.nsteps, **f32)
            self.param_hist = torch.zeros((self.nsteps, P), **f32)
        if self.mode == "eval":  # loss and summed gradient, packed for one host copy
            self.lg = torch.zeros(1 + P, **f32)
        self.graph = None
        self._kgraph = None
        self.graph_steps = max(1, int(os.environ.get("MULTIGRAD_GRAPH_STEPS", "16")))
        self.tuning = None
        self._times = {}
        self.fallback_reason = None
        exch = self.ar if sgd else self.twoshot
        capturable = cuda and (W == 1 or exch is not None) and \
            (not self.group or W == 1 or self.oneshot is not None) and \
            all(o is not None or md.comm is None or md.comm.size == 1
                for o, md in zip(self.m_oneshot, self.members))
        if self.graph_req is True and not capturable:
            raise RuntimeError("this step is not capturable (RCCL collectives in it)")
        self.use_graph = capturable and self.graph_req is not False
        if self.use_graph and not self._probe_capture(capture=W > 1):
            # a rank's hooks cannot be captured, or a sumstat vector does not fit the
            # one-shot kernel: every rank runs eagerly (a per-rank fallback would leave the
            # ranks' collective sequences out of step)
            if self.graph_req is True:
                raise RuntimeError(f"the step is not capturable: {self.fallback_reason}")
            self.use_graph = False
        if not capturable and self.graph_req is None:
            self.fallback_reason = "RCCL / gloo collectives in the step" if W > 1 else \
                "CPU tensors"
        if W > 1 and cuda:
            # the ranks meet here before the first peer-memory exchange (its wait for a
            # peer is bounded by MULTIGRAD_ONESHOT_TIMEOUT)
            torch.cuda.synchronize()
            self.comm.barrier()
        self.ready = True
        return self

    @on_engine_stream
    def close(self) -> None:
        """Give the two-shot context back to the communicator's pool (collective: every
        rank closes its engine the same way); setup() calls it before re-connecting.  Graphs
        that recorded exchanges on the all-reduce context are dropped with it (their pins go
        back with the hold)."""
        if self.ar is not None and getattr(self, "_ar_pins", [0])[0]:
            self.graph = None
            self._kgraph = None
        if self.twoshot is not None:
            from ..parallel.xgmi import release_twoshot
            release_twoshot(self.comm, self.twoshot)
        fin = getattr(self, "_ar_fin", None)
        if fin is not None:
            fin()  # release the hold and this engine's pins (once)
            self._ar_fin = None
        self.twoshot = None
        self.ar = None
        self.ready = False

    # ------------------------------------------------------------------ the step
    def _member(self, i: int, key, exchange: bool):
        """Member i's chain rule up to its local VJP: ``(loss, g_local)``; with
        ``exchange`` the partial sumstats are summed over the member's communicator."""
        md, P = self.members[i], self.P
        rk = {} if key is None else {"randkey": key}
        with torch.enable_grad():
            leaf = _leaf_view(self.p[:P], self.shape)
            out = md.calc_partial_sumstats_from_params(leaf, **rk)
            if md.sumstats_func_has_aux:
                partial, saux = out
            else:
                partial, saux = out, None
            partial = torch.as_tensor(partial)
            self._S_meta[i] = (partial.dtype, partial.numel())
            total = partial.detach().clone()
            if exchange:
                total = self._sumstats_allreduce(i, total)
            total = total.to(partial.dtype).requires_grad_(True)
            args = (total, saux) if md.sumstats_func_has_aux else (total,)
            lout = md.calc_loss_from_sumstats(*args, **rk)
            loss = lout[0] if md.loss_func_has_aux else lout
            (cot,) = torch.autograd.grad(loss, total, allow_unused=True)
            if cot is None:
                cot = torch.zeros_like(total)
            g = None
            if partial.requires_grad:
                (g,) = torch.autograd.grad(partial, leaf, cot, allow_unused=True)
        return loss.detach(), g

    def _hooks_only(self, key):
        """The user's part of a step (forward, loss, cotangent, VJP) without collectives."""
        self._S_meta = [None] * len(self.members)
        self._gen_i = 0
        for i in range(len(self.members)):
            self._member(i, key, exchange=False)

    def _probe_capture(self, capture: bool) -> bool:
        """Collective on several ranks: can every rank capture its user hooks?  The
        collective-free part of a step runs once eagerly on a side stream (lazy
        initialisation; it also records the sumstat shapes and counts the randkey
        generators) and, with ``capture``, into a throw-away graph; every sumstat vector
        summed over more than one rank must fit the one-shot kernel (fp32, <= 64 values:
        an RCCL call must never be recorded into a graph).  The verdicts are all-gathered
        so all ranks take the same path."""
        from ..parallel.xgmi import MAX_FLOATS
        ok, reason = True, None
        key = self._cap_key if self.key_mode is not None else None
        try:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                self._hooks_only(key)
            torch.cuda.current_stream().wait_stream(s)
            for i, md in enumerate(self.members):
                if md.comm is not None and md.comm.size > 1:
                    dt, n = self._S_meta[i]
                    if dt != torch.float32 or n > MAX_FLOATS:
                        raise RuntimeError(
                            f"sumstats of {n} x {dt} do not fit the capturable one-shot "
                            f"all-reduce (fp32, <= {MAX_FLOATS} values)")
            if capture:
                g = torch.cuda.CUDAGraph()
                for gen in self._gens:
                    g.register_generator_state(gen)
                with _no_gc():
                    with torch.cuda.graph(g):
                        self._hooks_only(key)
                del g
        except Exception as exc:  # noqa: BLE001  (host sync / dynamic shapes in user code)
            torch.cuda.synchronize()
            ok, reason = False, f"capture failed: {type(exc).__name__}: {exc}"
        if self.size > 1:
            verdicts = self.comm.allgather((ok, reason))
        else:
            verdicts = [(ok, reason)]
        bad = [(r, why) for r, (good, why) in enumerate(verdicts) if not good]
        if bad:
            self.fallback_reason = f"rank {bad[0][0]}: {bad[0][1]}" if self.size > 1 else bad[0][1]
        return not bad

    def _sumstats_allreduce(self, i: int, S: torch.Tensor) -> torch.Tensor:
        mc = self.members[i].comm
        if mc is None or mc.size == 1:
            return S
        S = S.contiguous()
        o = self.m_oneshot[i]
        if o is not None and S.dtype == torch.float32 and S.numel() <= 64:
            o(S)
            return S
        mc.all_reduce(S)
        return S

    def _group_loss(self, losses) -> torch.Tensor:
        """Sum of the members' losses over the group: sub-communicator rank 0 contributes."""
        tot = torch.zeros(1, dtype=torch.float32, device=self.device)
        for md, l in zip(self.members, losses):
            if md.comm is None or md.comm.rank == 0:
                tot = tot + l.reshape(1).to(torch.float32)
        if self.size > 1:
            tot = tot.contiguous()
            if self.oneshot is not None:
                self.oneshot(tot)
            else:
                self.comm.all_reduce(tot)
        return tot

    def _body(self, host_step: Optional[int], key):
        P = self.P
        self._S_meta = [None] * len(self.members)
        self._gen_i = 0
        g, losses = None, []
        for i in range(len(self.members)):
            loss, gi = self._member(i, key, exchange=True)
            losses.append(loss)
            if gi is not None:
                g = gi if g is None else g + gi
        if self.group:
            self.loss.copy_(self._group_loss(losses))
        else:
            self.loss.copy_(losses[0].reshape(1).to(torch.float32))
        g = torch.zeros(self.shape, device=self.device) if g is None else g
        g = g.reshape(-1).to(torch.float32)
        if self.mode == "eval":
            if self.size > 1:
                g = g.contiguous()
                if self.ar is not None:
                    self.ar.all_reduce_(g)
                else:
                    self.comm.all_reduce(g)
            self.lg[:1].copy_(self.loss)
            self.lg[1:].copy_(g)
            return
        if self.mode == "sgd":
            # record (loss, parameters at evaluation) at the device step, then p -= lr g;
            # the step counter advances on the device, so eager steps and replays agree
            idx = self.step_dev[:1].long()
            self.loss_hist.index_copy_(0, idx, self.loss)
            self.param_hist.index_copy_(0, idx, self.p[:P].view(1, P))
            if self.size > 1:
                g = g.contiguous()
                if self.ar is not None:
                    self.ar.all_reduce_(g)
                else:
                    self.comm.all_reduce(g)
            self.p[:P].add_(g, alpha=-self.lr)
            self.step_dev[:1].add_(1)
            return
        hb = self.history.buf.reshape(-1) if self.history.mode == "full" else None
        if self.twoshot is not None:
            self.gbuf[:P].copy_(g)
            a, b = self.own
            bnd = self.bounds_loc
            mode = 1 if bnd is None else (3 if self.legacy else 2)
            traj = None if self.traj_loc is None else self.traj_loc.reshape(-1)
            self.twoshot.step(a, b - a, mode, m=self.m, v=self.v, u=self.u, bounds=bnd,
                              traj=traj, traj_stride=0 if traj is None else b - a,
                              step=self.step_dev, host_step=host_step, lr=self.lr, b1=self.b1,
                              b2=self.b2, eps=self.eps)
            self.p[:P].copy_(self.theta[:P])  # the cached copy the next step's hooks read
            return
        if self.size > 1:
            g = g.contiguous()
            self.comm.all_reduce(g)
        bnd = self.bounds
        adam_step_(self.u, self.m, self.v, g, self.p if bnd is not None else None,
                   self.step_dev, self.lr, self.b1, self.b2, self.eps, bnd, self.legacy,
                   traj_base=hb, traj_stride=P if hb is not None else 0, host_step=host_step)

    def _capture(self):
        """Warm up on a side stream (allocator, autograd and kernel loading), restore the
        state the warm-up moved, then capture one step.  Collectives in the warm-up run on
        every rank alike, so their device sequence numbers stay in lockstep."""
        saved = [t.clone() for t in (self.p, self.m, self.v, self.step_dev)]
        th_saved = self.theta.clone() if self.theta is not self.p else None
        u_saved = self.u.clone() if self.u is not None and self.u is not self.p else None
        traj_saved = None if self.traj_loc is None else self.traj_loc[1].clone()
        hist_saved = None if self.history.mode != "full" else self.history.buf[1].clone()
        key = self._cap_key if self.key_mode is not None else None
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self._body(None, key)  # one warm-up step (it writes trajectory row 1, restored below)
        torch.cuda.current_stream().wait_stream(s)
        for t, v in zip((self.p, self.m, self.v, self.step_dev), saved):
            t.copy_(v)
        if th_saved is not None:
            self.theta.copy_(th_saved)
        if u_saved is not None:
            self.u.copy_(u_saved)
        if traj_saved is not None:
            self.traj_loc[1].copy_(traj_saved)
        if hist_saved is not None:
            self.history.buf[1].copy_(hist_saved)
        graph = torch.cuda.CUDAGraph()
        for gen in self._gens:
            graph.register_generator_state(gen)
        pins = self._ar_pin_count()
        with _no_gc():
            with torch.cuda.graph(graph):
                self._body(None, key)
        self._ar_note_pins(pins)
        return graph

    def _ar_pin_count(self) -> int:
        return self.ar.pins if self.ar is not None else 0

    def _ar_note_pins(self, before: int) -> None:
        """Account the exchanges a capture recorded on the all-reduce context (pins held
        until close())."""
        if self.ar is not None:
            self._ar_pins[0] += self.ar.pins - before

    def _replay(self, key) -> None:
        """Replay the captured step (on the engine stream, like every launch of the engine:
        see :meth:`stream`).  After eager steps, the device step counter is set from the
        host first (eager steps keep the count on the host)."""
        self._sync_dev_step()
        self._seed_generators(key)
        self.graph.replay()

    def _sync_dev_step(self) -> None:
        if self._dev_step_stale:
            self.step_dev[0] = self.step_host
            self._dev_step_stale = False

    def _tuning_phase(self) -> bool:
        return (self.graph_req is None and self.tuning is None and
                self.nsteps > 3 * self._TUNE + self._TUNE_WARM)

    def _block_ok(self) -> bool:
        """Whether the next steps may replay a graph of ``graph_steps`` unrolled steps:
        graph mode after its tuning, a step with no per-step key (the generators are seeded
        once per replay), and no per-step host bookkeeping beyond the last parameters."""
        return (self.use_graph and self.graph is not None and self.graph_steps > 1 and
                self.key_mode is None and self.mode in ("adam", "sgd") and
                not self._tuning_phase() and
                (self.history.mode in ("full", "last") or self.traj_loc is not None))

    def _capture_block(self, k: int):
        """Capture ``k`` steps into one graph (after the one-step capture, which warmed up
        the allocator and the kernels); each step reads and advances the device step."""
        g = torch.cuda.CUDAGraph()
        pins = self._ar_pin_count()
        with _no_gc():
            with torch.cuda.graph(g):
                for _ in range(int(k)):
                    self._body(None, None)
        self._ar_note_pins(pins)
        return g

    @on_engine_stream
    def steps(self, n: int):
        """``n`` optimizer steps: :meth:`step` one by one, or -- once graph mode is settled
        for an unkeyed step -- replays of a graph of ``graph_steps`` unrolled steps (the
        whole-loop capture of the reference's lax.scan, multigrad/mpi4jax/multigrad.py:
        57-58, in blocks), with the remainder as one-step replays."""
        n, K = int(n), self.graph_steps
        while n > 0:
            if n >= K and self._block_ok():
                if self.step_host + K > self.nsteps:
                    raise RuntimeError("more steps than the trajectory buffer was sized for")
                if self._kgraph is None or self._kgraph[0] != K:
                    self._kgraph = (K, self._capture_block(K))
                self._sync_dev_step()
                self._kgraph[1].replay()
                self.step_host += K
                n -= K
                if self.history.mode != "full" and self.traj_loc is None:
                    self.history.record(self.step_host - 1, self.p[:self.P])
            else:
                self._step()
                n -= 1

    def _drive(self, nsteps: int, hooks, *hook_args, **hook_kw):
        """Run ``nsteps`` steps; with per-step hooks one at a time, else as one
        :meth:`steps` call (graph blocks)."""
        if not hooks.active:
            self.steps(nsteps)
            return
        for i in range(int(nsteps)):
            self._step()
            hooks(i, self.loss, *hook_args, **hook_kw)

    _TUNE = 6       # steps per timed window of the auto policy
    _TUNE_WARM = 3  # eager steps before the first window (lazy init, first launches, clocks)

    def _tuned_step(self, key):
        """Auto policy (``graph=None``): after ``_TUNE_WARM`` eager steps, a window of
        ``_TUNE`` eager steps, then the capture and one untimed replay, then a window of
        ``_TUNE`` replays; each window is timed as a whole (no synchronisation inside it,
        so eager launches overlap the GPU as in steady state).  Replay is kept only if it
        beats eager by 3% -- a collective decision -- and then simply continues.  Measured
        on one MI355X (profiles/graph_modes/): replay wins when the step is launch bound
        and loses slightly when it is GPU bound."""
        import time
        k, T, W = self.step_host, self._TUNE, self._TUNE_WARM
        # phase: -1 warm-up, 0 eager window, 1 first (untimed) replay, 2 replay window
        ph = -1 if k < W else 0 if k < W + T else 1 if k == W + T else 2
        if ph >= 1 and self.graph is None:
            self.step_dev[0] = k   # eager steps keep the count on the host
            self._dev_step_stale = False
            try:
                self.graph = self._capture()
            except Exception as exc:  # noqa: BLE001
                if self.size > 1:
                    raise
                torch.cuda.synchronize()
                self.use_graph = False
                self.fallback_reason = f"capture failed: {type(exc).__name__}: {exc}"
                self._body(k, key)
                self._dev_step_stale = True
                return
        if k in (W, W + T + 1):
            torch.cuda.synchronize()
            self._t0 = time.perf_counter()
        if ph >= 1:
            self._replay(key)
        else:
            self._body(k, key)
            self._dev_step_stale = True
        if k in (W + T - 1, W + 2 * T):
            torch.cuda.synchronize()
            self._times[ph] = time.perf_counter() - self._t0
        if k == W + 2 * T:
            te, tg = self._times[0] / T, self._times[2] / T
            keep = 1 if tg < 0.97 * te else 0
            if self.size > 1:
                keep = int(all(self.comm.allgather(keep)))
            self.tuning = {"eager_s": te, "graph_s": tg, "graph": bool(keep)}
            if not keep:
                self.use_graph = False
                self.graph = None
                self.fallback_reason = f"eager measured faster ({te * 1e3:.3f} vs {tg * 1e3:.3f} ms/step)"

    @on_engine_stream
    def step(self):
        """One optimizer step.  A direct call launches the step eagerly even in graph mode,
        unless ``step_replay`` is set (``MULTIGRAD_STEP_REPLAY=1``): between direct calls
        the caller may launch kernels on the legacy default stream and synchronise, after
        which a graph replay computes garbage on this HIP runtime (docs/design.md "Graph
        replays and the default stream"); a caller that keeps its own GPU work inside
        :meth:`stream` may opt in.  The engine's drivers (:meth:`steps`, ``run_adam``,
        ``run_simple_grad_descent``) own every launch and replay."""
        self._step(replay=self.step_replay)

    def _step(self, replay: bool = True):
        assert self.ready, "call setup() first"
        if self.step_host >= self.nsteps and (self.history.mode == "full" or self.traj_loc is not None
                                              or self.mode == "sgd"):
            raise RuntimeError("more steps than the trajectory buffer was sized for")
        key = self._step_key()
        if not replay and self.use_graph:
            self._body(self.step_host, key)
            self._dev_step_stale = True
            self.step_host += 1
            if self.history.mode != "full" and self.traj_loc is None:
                self.history.record(self.step_host - 1, self.p[:self.P])
            return
        if self.use_graph and self.graph_req is None and self.tuning is None and \
                self.nsteps > 3 * self._TUNE + self._TUNE_WARM:
            self._tuned_step(key)
            self.step_host += 1
            if self.history.mode != "full" and self.traj_loc is None:
                self.history.record(self.step_host - 1, self.p[:self.P])
            return
        if self.use_graph and self.graph is None:
            try:
                self.graph = self._capture()
            except Exception as exc:  # noqa: BLE001  (host sync / dynamic shapes in user code)
                if self.graph_req is True or self.size > 1:
                    raise
                torch.cuda.synchronize()
                self.use_graph = False
                self.fallback_reason = f"capture failed: {type(exc).__name__}: {exc}"
        if self.use_graph:
            self._replay(key)
        else:
            self._body(self.step_host, key)
            self._dev_step_stale = True
        self.step_host += 1
        if self.history.mode != "full" and self.traj_loc is None:
            self.history.record(self.step_host - 1, self.p[:self.P])

    # ------------------------------------------------------------------ results
    def check(self, where: str = "", collective: bool = False) -> None:
        comm = self.comm if collective else None
        for ctx in (self.twoshot, self.ar, self.oneshot):
            if ctx is not None:
                ctx.check(where or f"generic engine step {self.step_host}", comm=comm)
        for md, ctx in zip(self.members, self.m_oneshot):
            if ctx is not None:
                ctx.check(where or f"generic engine step {self.step_host}",
                          comm=md.comm if collective else None)

    @on_engine_stream
    def last_loss(self) -> float:
        v = float(self.loss.item())
        self.check("last_loss")
        return v

    @on_engine_stream
    def params(self) -> torch.Tensor:
        self.check("params", collective=True)
        return self.p[:self.P].reshape(self.shape).clone()

    @on_engine_stream
    def trajectory(self) -> torch.Tensor:
        self.check("trajectory", collective=True)
        if self.traj_loc is not None:
            rows = self.step_host + 1
            loc = self.traj_loc[:rows].contiguous()
            gathered = torch.empty((self.size,) + tuple(loc.shape), dtype=loc.dtype,
                                   device=self.device)
            self.comm.all_gather_into_tensor(gathered.reshape(-1), loc.reshape(-1))
            full = gathered.permute(1, 0, 2).reshape(rows, -1)[:, :self.P]
            return full.reshape((rows,) + self.shape)
        t = self.history.result()[:, :self.P] if self.history.mode == "full" else self.history.result()
        return t.reshape((t.shape[0],) + self.shape)

    @on_engine_stream(always=True)
    def evaluator(self, x0, randkey=None):
        """``f(x) -> (loss, grad)`` replaying one captured evaluation of the distributed
        chain rule (autograd forward, sumstat all-reduce, cotangent, VJP, gradient sum):
        the objective of the root-driven scipy L-BFGS-B (optim/bfgs.py), which calls it
        once per function evaluation with a constant ``randkey`` (multigrad/bfgs.py:63-66).
        Falls back to eager launches when the step cannot be captured; collective on
        several ranks (every rank evaluates every point)."""
        self.mode = "eval"
        self.setup(x0, nsteps=1, history="last", randkey=randkey,
                   const_randkey=randkey is not None)
        P, shape = self.P, self.shape
        if self.use_graph and self.graph_req is not False:
            try:
                self.graph = self._capture()
            except Exception as exc:  # noqa: BLE001  (host sync in user code, ...)
                if self.graph_req is True or self.size > 1:
                    raise
                torch.cuda.synchronize()
                self.use_graph = False
                self.fallback_reason = f"capture failed: {type(exc).__name__}: {exc}"

        def f(x, **kw):
            kw.pop("randkey", None)  # the engine holds the (constant) key
            if kw:
                raise TypeError(f"the captured evaluator takes no keywords: {sorted(kw)}")
            with self.stream():
                self.p[:P].copy_(torch.as_tensor(x).reshape(-1))
                key = self._step_key()
                if self.use_graph:
                    self._replay(key)
                else:
                    self._body(None, key)
                out = self.lg.cpu()  # loss and gradient in ONE device->host copy
            return out[0], out[1:].reshape(shape)

        return f

    @on_engine_stream(always=True)
    def run_simple_grad_descent(self, guess, nsteps: int = 100, learning_rate: float = 0.01,
                                callback=None):
        """Fixed-rate gradient descent with the reference's result contract
        (``GradDescentResult``: ``loss[i]`` and the ``params[i]`` it was evaluated at,
        multigrad/util.py:100-134), one captured step replayed per iteration."""
        from ..utils.hooks import StepHooks, driver_guard
        from ..utils.util import GradDescentResult
        self.mode = "sgd"
        self.setup(guess, nsteps, learning_rate=learning_rate, history="last")
        hooks = StepHooks(self.comm, callback)
        with driver_guard(self.comm):
            self._drive(nsteps, hooks, None, self.params)
        self.check("simple_grad_descent", collective=True)
        n = self.step_host
        res = GradDescentResult(loss=self.loss_hist[:n].clone(),
                                params=self.param_hist[:n].reshape((n,) + self.shape).clone(),
                                aux=[None] * n)
        self.close()
        return res

    @on_engine_stream(always=True)
    def run_adam(self, guess, nsteps: int = 100, param_bounds=None, learning_rate: float = 0.01,
                 b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8, history="full",
                 legacy_bounds_jacobian: bool = False, callback=None, randkey=None,
                 const_randkey: bool = False, **unused):
        """Adam with the reference's contract: trajectory ``(nsteps+1, *shape)``."""
        if unused:
            raise TypeError(f"unsupported run_adam options for the graph engine: {sorted(unused)}")
        from ..utils.hooks import StepHooks, driver_guard
        self.mode = "adam"
        self.setup(guess, nsteps, param_bounds, learning_rate, b1, b2, eps, history,
                   legacy_bounds_jacobian, randkey=randkey, const_randkey=const_randkey)
        hooks = StepHooks(self.comm, callback)
        with driver_guard(self.comm):
            W = self.size

            def comm_bytes():  # sumstat exchange + dense-gradient exchange, bytes sent
                nS = sum(m[1] for m in getattr(self, "_S_meta", []) if m is not None)
                return 0 if W == 1 else int(4 * (W - 1) * (nS + 2 * (self.P // W)))

            self._drive(nsteps, hooks, self, self.params, comm_bytes=comm_bytes)
            traj = self.trajectory()
        self.close()
        return traj
