"""Fused, device-resident Adam engine (HIP kernels + stream-ordered RCCL collectives).

The generic path (``OnePointModel.run_adam``) runs the distributed chain rule through
autograd with Python in the loop.  Models that expose the *engine protocol* run instead
as a fixed sequence of device operations per step, with no host synchronisation:

    forward per chunk      (HIP kernel -> per-workgroup slab rows)
    slab reduce            (fixed-order sum)                               -> S
    all-reduce(S)          (RCCL, latency bound, K floats)
    loss + edge weights    (1 tiny kernel)                                 -> loss, h
    VJP per chunk          (segmented per-population kernel)               -> g_c
    ZeRO-1 (world > 1, default):
        reduce-scatter(g_c)  issued right after VJP_c on RCCL's stream, so it overlaps
                             VJP_{c+1} on the compute stream
        fused Adam on the owned 1/W slice of chunk c (as soon as RS_c lands)
        all-gather(theta_c)  overlapping Adam_{c+1} and, across the step boundary, the
                             next step's forward of chunk c-1...
    replicated (world == 1, or zero=False):
        all-reduce(g) + fused Adam over every parameter

RS + AG move exactly the bytes of one all-reduce, but the optimizer work and the Adam
state drop to 1/W per GPU and every collective hides behind compute of a neighbouring
chunk.  Parameters stay bitwise identical across ranks (each slice has one owner).

Owner mode (world > 1, model data placed by parameter ownership): when the model
reports unit bounds ``engine_owner_units() -> [W+1]`` and every rank's data touches only
units inside its own range (``engine_support_units()``, verified collectively at setup),
the chunks ARE the ranks' ranges.  Rank r's gradient on its range is then complete
locally and zero elsewhere, so the step is

    forward(own chunk) -> all-reduce(S) -> loss -> VJP(own chunk) -> Adam(own chunk)

with the K-float sumstat all-reduce as the only collective: the dense P-float
gradient reduction of data parallelism (reference multigrad/multigrad.py:531-532)
is provably all zeros outside the owner's range and is not sent.  Parameters, moments and
trajectory are sharded by owner and assembled on request.

On a single GPU the whole step is captured once into a HIP graph and replayed; the
device step counter inside the Adam kernel makes the replay self-advancing.  This
replaces the reference's per-step host round trips (4 host crossings per
Adam step, 2 of them pickled broadcasts).

Engine protocol (implemented by :class:`~multigrad_amd.models.population.PopulationSMFModel`):
``engine_units() -> (J, params_per_unit)``, ``engine_set_chunks(unit_bounds)``,
``engine_nS()``, ``engine_fwd_rows(chunk)``, ``engine_forward_chunk(theta, slab, chunk)
-> rows``, ``engine_reduce(slab, rows, S)``, ``engine_loss_into(S, loss, h)``,
``engine_vjp_into(theta, h, grad, chunk)``, optionally ``engine_param_perm()`` (the
unit order the model wants the engine vectors in) and ``engine_layout_hint(guess)`` (the
starting parameters, before ``engine_set_chunks``, for a data layout that depends on
them).  Every method works on CPU tensors too (PyTorch reference math), which is how the
multi-rank orchestration is tested on gloo.
"""
from __future__ import annotations

import math
import os
import time
from typing import List, Optional

import torch

import contextlib

from ._stream import EngineStream, make_engine_stream, on_engine_stream
from ..optim.adam import History
from ..optim.transforms import Bounds, KIND_NONE
from ..ops.adam import adam_step_
from ..utils.profiling import PhaseTimer
from ..utils.trace import trace

__all__ = ["FusedAdamEngine", "plan_chunks"]


def _env_flag(name: str, default: Optional[bool]) -> Optional[bool]:
    v = os.environ.get(name)
    if v is None:
        return default
    return v.lower() not in ("0", "false", "off", "no")


def _side_stream_mode() -> str:
    """``MULTIGRAD_TWOSHOT_SIDE_STREAM``: 1/on, 0/off, unset/auto (measured at setup)."""
    v = os.environ.get("MULTIGRAD_TWOSHOT_SIDE_STREAM", "auto").strip().lower()
    if v in ("1", "on", "true", "yes"):
        return "on"
    if v in ("0", "off", "false", "no"):
        return "off"
    return "auto"


def _autotune_mode() -> str:
    """``MULTIGRAD_AUTOTUNE``: ``auto`` (default) -- the setup autotune and the settle steps
    get at most ``MULTIGRAD_TUNE_BUDGET`` (0.1) of the requested run's estimated time, and a
    run too short for the minimum windows keeps the default schedule (the first candidate);
    ``on`` -- always the full autotune (bench.py); ``off`` -- never."""
    v = os.environ.get("MULTIGRAD_AUTOTUNE", "auto").strip().lower()
    if v in ("0", "off", "false", "no"):
        return "off"
    if v in ("1", "on", "true", "yes", "full"):
        return "on"
    return "auto"


def _best_ms(tuning) -> float:
    """Fastest measured candidate of an autotune record (dropped candidates have no time)."""
    ms = [c["ms"] for c in tuning["candidates"] if c.get("ms") is not None]
    return min(ms) if ms else math.inf


def plan_chunks(J: int, upp: int, world: int, nchunks: int):
    """Unit-aligned chunk boundaries whose parameter counts are multiples of 4*world
    (float4 lanes on every reduce-scatter slice); the last chunk is padded.

    Returns (unit_bounds, param_bounds, P_pad, chunk_lengths)."""
    q = 4 * world
    a = q // math.gcd(q, upp)  # units per alignment block
    C = max(1, min(int(nchunks), J))
    ub = sorted({min(J, int(round(c * J / C / a)) * a) for c in range(C)} | {0, J})
    ub = [u for u in ub if u <= J]
    # drop empty chunks (duplicates already removed); keep J as the final bound
    pb = [u * upp for u in ub]
    last = pb[-1] - pb[-2]
    P_pad = pb[-2] + (-(-last // q) * q if last else 0)
    lengths = [pb[i + 1] - pb[i] for i in range(len(pb) - 2)] + [P_pad - pb[-2]]
    return ub, pb, P_pad, lengths


class FusedAdamEngine:
    """Device-resident Adam for a model implementing the engine protocol.

    Parameters
    ----------
    model : the model (its ``comm`` is used for the collectives)
    graph : capture the step into a HIP graph (default: on for a single GPU rank;
        ``MULTIGRAD_GRAPH`` overrides)
    zero : shard the optimizer across ranks (reduce-scatter / all-gather); default on
        for more than one rank (``MULTIGRAD_ZERO``)
    chunks : number of parameter chunks for collective/compute overlap (default 1 on a
        single rank, 4 otherwise; ``MULTIGRAD_CHUNKS``)
    owner : owner mode (see the module docstring): default whenever the model's data
        placement allows it on more than one rank (``MULTIGRAD_OWNER``)

    With ZeRO the parameter all-gathers run on a second communicator (its own RCCL
    stream), so the all-gather of chunk c overlaps the reduce-scatter of chunk c+1
    instead of queueing behind it; the trajectory is stored sharded (each rank records
    the slices it owns, written by the Adam kernel) and assembled by one all-gather when
    it is requested -- the analogue of the reference's end-of-run trajectory broadcast.
    """

    @property
    def graph(self):
        """The captured one-step graph (None: capture on first use).  Dropping it also
        drops the graph of a block of steps."""
        return self._graph

    @graph.setter
    def graph(self, g):
        self._graph = g
        if g is None:
            self._kgraph = None

    def __init__(self, model, comm=None, graph: Optional[bool] = None,
                 zero: Optional[bool] = None, chunks: Optional[int] = None,
                 owner: Optional[bool] = None, repartition: Optional[bool] = None):
        self.model = model
        self.comm = model.comm if comm is None else comm
        self.size = 1 if self.comm is None else self.comm.size
        self.rank = 0 if self.comm is None else self.comm.rank
        z = _env_flag("MULTIGRAD_ZERO", zero)
        self.zero = (self.size > 1) if z is None else bool(z) and self.size > 1
        # owner mode: None = whenever the model's placement allows it on >1 rank; True =
        # also on a single rank (exercises the owner schedule); False = never
        o = _env_flag("MULTIGRAD_OWNER", owner)
        self.allow_owner = True if o is None else bool(o)
        self.force_owner = bool(o)
        self.owner = False
        # re-partition a data-parallel (hashed) shard by parameter owner at setup: one
        # all-to-all-v of the data (model.engine_repartition), after which owner mode needs
        # only the sumstat all-reduce per step.  None = on for several ranks unless owner
        # mode or ZeRO was asked for explicitly; MULTIGRAD_REPARTITION overrides
        r = _env_flag("MULTIGRAD_REPARTITION", repartition)
        if r is None:
            r = self.size > 1 and self.allow_owner and z is None
        self.repartition = bool(r) and self.size > 1 and self.allow_owner
        self.repartitioned = None  # the model's re-partition record, once done
        # kept across setup() calls of this engine (a model's cached engine serves every
        # run_* call, models/population.py fused_engine): device buffers of the same shape,
        # the autotune verdicts and -- when every buffer and scalar a graph captured is
        # unchanged -- the captured graphs (the analogue of JAX's jit cache)
        self._bufs = {}
        self._tune_cache = {}
        self._gkey = None
        self.stats = {"setups": 0, "captures": 0, "trial_steps": 0, "layouts": 0}
        self.closed = False
        self.fuse_vjp_adam = bool(_env_flag("MULTIGRAD_FUSED_VJP_ADAM", True))
        # slab reduction (+ one-shot cross-rank sum) + loss in one launch
        self.fuse_epilogue = bool(_env_flag("MULTIGRAD_FUSED_EPILOGUE", True))
        self.oneshot = None
        # two-shot xGMI reduce-scatter -> Adam -> all-gather of the dense gradient (ZeRO
        # mode on GPUs; parallel/xgmi.py): None = RCCL collectives
        self.twoshot = None
        self._ts_keep = None  # the acquired two-shot context (kept across setups)
        nc = chunks if chunks is not None else int(os.environ.get("MULTIGRAD_CHUNKS", "0")) or None
        self._chunks_explicit = nc is not None
        self.nchunks_req = nc if nc is not None else (1 if self.size == 1 else 4)
        self.comm_ag = None  # second communicator (own RCCL stream) for parameter all-gathers
        g = _env_flag("MULTIGRAD_GRAPH", graph)
        self._graph_auto = g is None
        self.use_graph = (self.size == 1) if g is None else bool(g)
        # whole-loop capture (the analogue of the reference's lax.scan over the optimizer
        # loop, multigrad/mpi4jax/multigrad.py:57-58): graph mode replays graphs of
        # graph_steps unrolled steps, so the ~10 us host launch and the ~10 us device gap
        # between consecutive graph launches are paid once per block, not per step
        # (profiles/graph_modes/); MULTIGRAD_GRAPH_STEPS, 1 = one step per graph
        self.graph_steps = max(1, int(os.environ.get("MULTIGRAD_GRAPH_STEPS", "16")))
        # direct step() calls replay graphs only on request (engine/generic.py step())
        from .generic import _step_replay_default
        self.step_replay = _step_replay_default()
        self._kgraph = None
        self.graph = None
        self._capturing = False
        self._es = None  # the engine's own stream (stream(), engine/_stream.py)
        # eager launches of a pipelined step that read/advance the device step counter like
        # graph replays do (benchmarks/graph_modes.py "eager-dev": separates the cost of the
        # device counter from the cost of graph dispatch); MULTIGRAD_DEVICE_STEP=1
        self.device_step = _env_flag("MULTIGRAD_DEVICE_STEP", False)
        self.pending = False
        self.pipeline = False
        self.ready = False
        # per-phase HIP-event timing of eager steps (MULTIGRAD_PROFILE=1 or bench.py
        # --profile-phases); never active inside a graph capture
        self.timer = PhaseTimer()

    def _buf(self, name: str, shape, dtype=torch.float32) -> torch.Tensor:
        """A zeroed device buffer, the one of the previous setup when the shape matches."""
        shape = tuple(int(v) for v in (shape if isinstance(shape, (tuple, list)) else (shape,)))
        t = self._bufs.get(name)
        if t is None or tuple(t.shape) != shape or t.dtype != dtype or t.device != self.device:
            t = torch.zeros(shape, dtype=dtype, device=self.device)
            self._bufs[name] = t
        else:
            t.zero_()
        return t

    # ------------------------------------------------------------------ stream
    def _engine_stream(self):
        dev = getattr(self, "device", None)
        self._es = make_engine_stream(self._es, dev if dev is not None
                                      else self.model.param_device())
        return self._es

    def _stream_wanted(self) -> bool:
        """Launch on the engine stream while a graph may be replayed: graph mode, or any
        captured graph still held (eager steps between replays belong there too)."""
        return bool(getattr(self, "use_graph", False) or getattr(self, "graph", None) is not None
                    or getattr(self, "_kgraph", None) is not None)

    def stream(self):
        """Context manager: the engine's own HIP stream becomes current (ordered after the
        caller's stream on entry, before it on exit).  Every public method runs its launches
        there, never on the legacy default stream (engine/_stream.py: graph replays after
        default-stream launches and a host synchronisation compute garbage on this runtime)."""
        return EngineStream(self, always=False)

    # ------------------------------------------------------------------ setup
    @on_engine_stream(always=True)
    def setup(self, guess, nsteps: int, param_bounds=None, learning_rate: float = 0.01,
              b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8, history="full",
              legacy_bounds_jacobian: bool = False):
        """Allocate the device state for ``nsteps`` steps from ``guess`` (collective).

        Hashed placement on several GPUs with the two-shot exchange and no explicit chunk
        count: the two-chunk layout (whose exchange may overlap the VJP on a side stream) is
        timed against one chunk (one cross-rank rendezvous per step instead of two) and,
        when the overlapped two-chunk schedule won, against four overlapped chunks
        (``MULTIGRAD_MAX_CHUNKS``, default 4); the fastest is kept -- all by the same
        setup-time measurement as the rest of the schedule (:meth:`_autotune`)."""
        kw = dict(param_bounds=param_bounds, learning_rate=learning_rate, b1=b1, b2=b2,
                  eps=eps, history=history, legacy_bounds_jacobian=legacy_bounds_jacobian)
        self._chunks_override = None
        self._maybe_repartition()
        ck = ("chunks", self.size, bool(param_bounds is None), history == "full")
        if ck in self._tune_cache and not self._chunks_explicit:
            # the chunk count this engine measured before (hashed two-shot schedule)
            self._chunks_override = self._tune_cache[ck]
        self._setup(guess, nsteps, **kw)
        tun = self.tuning
        if not (tun and self.twoshot is not None and not self.owner and self.C == 2
                and not self._chunks_explicit and "ts_side" in tun["chosen"]
                and not tun.get("budget_skipped") and not tun.get("cached")):
            return self
        t2 = _best_ms(tun)
        skip = getattr(self, "_skip_autotune", False)
        self._chunks_override = 1
        self._skip_autotune = True
        try:
            self._setup(guess, nsteps, **kw)
        finally:
            self._skip_autotune = skip
        cands = [{"ts_side": False, "rccl_exchange": False}]
        if os.environ.get("MULTIGRAD_HASHED_EXCHANGE", "auto").strip().lower() != "twoshot":
            cands.append({"ts_side": False, "rccl_exchange": True})
        self._autotune(cands, min_window_s=1e-3 * float(
            os.environ.get("MULTIGRAD_AUTOTUNE_WINDOW_MS", "30")))
        t1 = _best_ms(self.tuning)
        tun1 = self.tuning
        chunk_times = {"1": t1, "2": t2}
        tuned = {1: tun1, 2: tun}
        current = 1
        nmax = int(os.environ.get("MULTIGRAD_MAX_CHUNKS", "4"))
        if nmax >= 4 and t2 < t1:
            # the overlapped schedule won with two chunks: four give the exchange of each
            # chunk a shorter wait behind its VJP and the next forward a shorter wait behind
            # its exchange (one more cross-rank rendezvous per extra chunk)
            self._chunks_override = 4
            self._skip_autotune = True
            try:
                self._setup(guess, nsteps, **kw)
            finally:
                self._skip_autotune = skip
            if self.C == 4 and self.comm_stream is not None:
                self._autotune([{"ts_side": True, "rccl_exchange": False}],
                               min_window_s=1e-3 * float(
                                   os.environ.get("MULTIGRAD_AUTOTUNE_WINDOW_MS", "30")))
                chunk_times["4"] = _best_ms(self.tuning)
                tuned[4] = self.tuning
                current = 4
        best = min(tuned, key=lambda c: chunk_times[str(c)])
        if best != current:
            self._chunks_override = best
            self._skip_autotune = True
            try:
                self._setup(guess, nsteps, **kw)
            finally:
                self._skip_autotune = skip
            for k, v in tuned[best]["chosen"].items():
                setattr(self, k, v)
            self.graph = None
        self.tuning = dict(tuned[best], chunks=dict(chunk_times, chosen=best))
        self._tune_cache[ck] = best
        dropped = [dict(d, chunks=n) for n, t in tuned.items() for d in t.get("dropped", [])]
        if dropped:  # candidates dropped in any of the chunk-count tunings, with the reason
            self.tuning["dropped"] = dropped
        return self

    def _setup(self, guess, nsteps: int, param_bounds=None, learning_rate: float = 0.01,
               b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8, history="full",
               legacy_bounds_jacobian: bool = False):
        md = self.model
        dev = md.param_device()
        self.device = dev
        if dev.type != "cuda":
            self.use_graph = False
        J, upp = md.engine_units()
        P = J * upp
        self.upp = upp
        owner_ub = self._owner_units(md, J)
        self.owner = owner_ub is not None
        if self.owner:
            ub = owner_ub
            pb = [u * upp for u in ub]
            P_pad = P
            lengths = [pb[i + 1] - pb[i] for i in range(len(pb) - 1)]
        else:
            W = self.size if self.zero else 1
            self.twoshot = None
            if self.zero and dev.type == "cuda":
                # two-shot: 2 chunks by default when the overlapped schedule may be chosen
                # (side stream auto), else 1 -- each chunk is one more cross-rank rendezvous
                side_mode = _side_stream_mode()
                nch = self._chunks_override or (
                    self.nchunks_req if self._chunks_explicit else (2 if side_mode == "auto" else 1))
                ub, pb, P_pad, lengths = plan_chunks(J, upp, W, nch)
                self.twoshot = self._connect_twoshot(P_pad)  # collective
            if self.twoshot is None:
                ub, pb, P_pad, lengths = plan_chunks(J, upp, W, self.nchunks_req)
        hint = getattr(md, "engine_layout_hint", None)
        changed = True
        if hint is not None:  # e.g. lanes grouped by forward path at the starting point
            changed = bool(hint(guess))
        cur = getattr(md, "engine_chunks_current", None)
        if changed or cur is None or not cur(ub):
            # (a model that reports its current chunks keeps its layout when neither the
            # chunks nor the layout classes changed: no rebuild on a repeated run)
            trace(f"engine: layout ({'owner' if self.owner else 'dense'}, {len(ub) - 1} chunks)")
            md.engine_set_chunks(ub)
            self.stats["layouts"] += 1
        self._ub = list(ub)
        if self.size > 1 and dev.type == "cuda" and self.fuse_epilogue:
            from ..parallel.xgmi import get_oneshot
            trace("engine: one-shot connect")
            self.oneshot = get_oneshot(self.comm)  # collective (all ranks run setup)
            trace(f"engine: one-shot {'up' if self.oneshot is not None else 'unavailable'}")
        # Internal order: models may keep the engine vectors in their own unit order
        # (e.g. the lanes layout's slot order, for coalesced parameter/gradient access).
        # It must keep every chunk's units inside the chunk, and be the same on all ranks;
        # user-facing values (guess, bounds, params, trajectory) are permuted at the edge.
        self.pidx, self.inv_pidx = self._param_order(md, P, upp, dev)
        self.P, self.P_pad, self.pb, self.lengths = P, P_pad, pb, lengths
        self.C = len(lengths)
        self.lr, self.b1, self.b2, self.eps = float(learning_rate), float(b1), float(b2), float(eps)
        self.legacy = bool(legacy_bounds_jacobian)
        p0 = torch.as_tensor(guess).detach().reshape(-1).to(device=dev, dtype=torch.float32)
        assert p0.numel() == P, f"guess has {p0.numel()} params, model expects {P}"
        f32 = dict(dtype=torch.float32, device=dev)
        bounds = Bounds.from_spec(param_bounds, P, device=dev)
        if self.pidx is not None:
            p0 = p0[self.pidx]
            if bounds is not None:
                bounds = Bounds(bounds.lo[self.pidx].contiguous(), bounds.hi[self.pidx].contiguous(),
                                bounds.kind[self.pidx].contiguous())
        if bounds is not None and P_pad > P:
            pad = P_pad - P
            bounds = Bounds(torch.cat([bounds.lo, torch.full((pad,), -math.inf, **f32)]),
                            torch.cat([bounds.hi, torch.full((pad,), math.inf, **f32)]),
                            torch.cat([bounds.kind, torch.full((pad,), KIND_NONE, dtype=torch.int8,
                                                               device=dev)]))
        old_b = getattr(self, "bounds", None)
        if bounds is not None and old_b is not None and bounds.lo.shape == old_b.lo.shape and \
                torch.equal(bounds.lo, old_b.lo) and torch.equal(bounds.hi, old_b.hi):
            bounds = old_b  # the same box: the same tensors (graphs captured on them stay valid)
        self.bounds = bounds
        if self.twoshot is not None:
            # parameters and gradient live in the exported peer-memory regions
            theta = self.twoshot.theta
            theta.zero_()
            self.grad = self.twoshot.grad
            self.grad.zero_()
        else:
            theta = self._buf("theta", P_pad)
        theta[:P] = p0
        if bounds is not None:  # the recorded start is T^-1(T(guess)), as the reference
            theta.copy_(bounds.inverse(bounds.forward(theta)))
        self.theta = theta
        if self.twoshot is None:
            self.grad = self._buf("grad", P_pad)
        nS = md.engine_nS()
        self.nS = nS
        self.rows = [md.engine_fwd_rows(c) for c in range(self.C)]
        self.S = self._buf("S", nS)
        self.slab = self._buf("slab", max(1, sum(self.rows)) * nS)
        self.h = self._buf("h", nS + 1)
        self.loss = self._buf("loss", 1)
        self.step_dev = self._buf("step_dev", (self.C, 2), torch.int32)
        if self.owner:
            a, b = pb[self.rank], pb[self.rank + 1]
            self.own_range = (a, b)
            n = b - a
            self.m = self._buf("m", n)
            self.v = self._buf("v", n)
            if bounds is not None:
                self.bounds_loc = Bounds(bounds.lo[a:b].contiguous(), bounds.hi[a:b].contiguous(),
                                         bounds.kind[a:b].contiguous())
                self.u_loc = self.bounds_loc.forward(theta[a:b]).contiguous()
            else:
                self.bounds_loc = None
                self.u_loc = None
        elif self.zero:
            self.loc_len = [L // W for L in lengths]
            self.loc_off = [sum(self.loc_len[:c]) for c in range(self.C)]
            nloc = sum(self.loc_len)
            self.own = [(pb[c] + self.rank * self.loc_len[c], pb[c] + (self.rank + 1) * self.loc_len[c])
                        for c in range(self.C)]
            self.m = self._buf("m", nloc)
            self.v = self._buf("v", nloc)
            self.g_loc = self._buf("g_loc", nloc)
            if bounds is not None:
                idx = torch.cat([torch.arange(a, b, device=dev) for a, b in self.own])
                self.bounds_loc = Bounds(bounds.lo[idx].contiguous(), bounds.hi[idx].contiguous(),
                                         bounds.kind[idx].contiguous())
                self.u_loc = self.bounds_loc.forward(theta[idx]).contiguous()
            else:
                self.bounds_loc = None
                self.u_loc = None
        else:
            if bounds is not None:
                self.u = self._buf("u", P_pad)
                self.u.copy_(bounds.forward(theta))
            else:
                self.u = theta
            self.m = self._buf("m", P_pad)
            self.v = self._buf("v", P_pad)
        self.step_host = 0
        self.nsteps = int(nsteps)
        sharded = self.zero or self.owner
        hmode = history if not (sharded and history == "full") else "last"
        self.history = History(hmode, nsteps, theta[:P].detach().clone(),
                               buf=self._bufs.get("history") if hmode == "full" else None)
        if hmode == "full":
            self._bufs["history"] = self.history.buf
        self.traj_loc = None
        self.history_mode = history
        if self.owner:
            if history == "full":
                a, b = self.own_range
                self.traj_loc = self._buf("traj_loc", (self.nsteps + 1, b - a))
                self.traj_loc[0] = theta[a:b]
        elif self.zero:
            if history == "full":
                self.traj_loc = self._buf("traj_loc", (self.nsteps + 1, sum(self.loc_len)))
                for c in range(self.C):
                    a, b = self.own[c]
                    o, n = self.loc_off[c], self.loc_len[c]
                    self.traj_loc[0, o:o + n] = theta[a:b]
            if self.comm_ag is None and self.size > 1 and self.twoshot is None and \
                    _env_flag("MULTIGRAD_AG_COMM", True):
                self.comm_ag = self.comm.split(0)
        self._ag: List = [None] * self.C
        self.comm_stream = None
        self.ts_side = False
        # hashed placement with the two-shot context up: RCCL reduce-scatter / all-gather
        # stays available as an autotune candidate (on the same buffers and shard layout)
        self.rccl_exchange = False
        xmode = os.environ.get("MULTIGRAD_HASHED_EXCHANGE", "auto").strip().lower()
        if self.twoshot is not None and xmode == "rccl":
            self.rccl_exchange = True
        side_mode = _side_stream_mode()
        if self.twoshot is not None and self.C > 1 and side_mode != "off":
            # overlapped schedule: the two-shot exchange of chunk c runs on a side stream as
            # soon as the VJP of chunk c is done (overlapping the VJP of chunk c+1), and the
            # next step's forward of chunk c waits only for that chunk's exchange; its grid
            # is capped so the compute kernels keep most CUs.  "auto" (default) times both
            # schedules on this machine at setup (_autotune) and keeps the faster: with
            # two ranks sharing one GPU the side stream only adds event waits, across xGMI
            # it hides part of the exchange behind compute.
            self.comm_stream = torch.cuda.Stream(device=dev)
            self.ts_blocks = int(os.environ.get("MULTIGRAD_TWOSHOT_BLOCKS", "256"))
            self.ev_vjp = [torch.cuda.Event() for _ in range(self.C)]
            self.ev_ts = [torch.cuda.Event() for _ in range(self.C)]
            self.ts_side = side_mode == "on"
        self._ts_pending = [False] * self.C
        # fused exchange ("ts_fused"): the two-shot exchange of chunk c-1 runs in the first
        # workgroups of chunk c's VJP launch and the last chunk's in the next step's first
        # forward launch (csrc/twoshot.h) -- overlap with compute on ONE stream, no events.
        # >= 2 chunks on a model whose kernels carry it (bounded fits: modes 2 / 3).
        # MULTIGRAD_TWOSHOT_FUSED: auto (an autotune candidate), on (always, no tuning), off
        self._x_pending = None  # packed exchange of the last chunk, for the next launch
        fmode = os.environ.get("MULTIGRAD_TWOSHOT_FUSED", "auto").strip().lower()
        self.ts_fused_ok = bool(
            fmode not in ("0", "off", "false", "no") and self.twoshot is not None
            and self.C > 1
            and getattr(md, "engine_fused_exchange_ok", lambda: False)())
        self.ts_fused = self.ts_fused_ok and fmode in ("1", "on", "true", "yes")
        if self.ts_fused:
            self.ts_side = False
        if self.ts_fused_ok and not hasattr(self, "ts_blocks"):
            self.ts_blocks = int(os.environ.get("MULTIGRAD_TWOSHOT_BLOCKS", "256"))
        self.pending = False
        ok = getattr(md, "engine_pipeline_ok", None)
        pchunk = self.rank if self.owner else None
        self.pipeline = bool(
            _env_flag("MULTIGRAD_PIPELINE", True) and self.fuse_vjp_adam
            and (self.owner or (not self.zero and self.C == 1 and self.size == 1))
            and ok is not None and hasattr(md, "engine_forward_update_chunk")
            and (ok(pchunk) if bounds is None else ok(pchunk, bounded=True)))
        # a step can be captured when every collective in it is a peer-memory kernel with
        # its sequence number in device memory (one-shot sumstats, two-shot gradient) --
        # RCCL/gloo calls are not captured
        # (the fused exchange carries a step's last exchange into the next step: eager only)
        self.capturable = dev.type == "cuda" and not self.ts_fused and (
            self.size == 1 or (self.oneshot is not None and self.fuse_epilogue and
                               (self.owner or (self.twoshot is not None and not self.ts_side))))
        if self._graph_auto:
            # a pipelined step is two launches (forward+update, epilogue); replaying them
            # from a graph measured 1-5% slower than eager launches (tools/archive/graph_ab_full.sh).
            # Multi-rank steps are capturable (MULTIGRAD_GRAPH=1, tested bitwise against
            # eager) but replays measured 7x slower than the 4 eager launches of the hashed
            # step with two ranks on one GPU (profiles/twoshot_2rank.md): eager by default.
            self.use_graph = self.capturable and not self.pipeline and self.size == 1
        elif self.use_graph and not self.capturable:
            self.use_graph = False  # e.g. RCCL collectives in the step: eager launches
        gk = self._graph_key()
        if gk != self._gkey:  # a buffer or scalar the captured graphs baked in changed
            self.graph = None
            self._gkey = gk
        self.tuning = None
        self._tuning = False
        self._relayout_init()
        self.ready = True
        if self.size > 1 and dev.type == "cuda":
            # line the ranks up before the first peer-memory exchange: a kernel waits for
            # its peers at most MULTIGRAD_ONESHOT_TIMEOUT, and the setup above (data layout,
            # sorts, first code-object loads) takes different times on different ranks
            torch.cuda.synchronize()
            self.comm.barrier()
        cands = []
        if self.comm_stream is not None and side_mode == "auto" and not self.use_graph and \
                xmode != "rccl" and not self.ts_fused:
            # hashed: where the exchange runs -- two-shot on the compute stream, on the side
            # stream, or RCCL's reduce-scatter / all-gather (measured, not assumed;
            # MULTIGRAD_HASHED_EXCHANGE=twoshot|rccl pins it)
            cands = [{"ts_side": False, "rccl_exchange": False, "ts_fused": False},
                     {"ts_side": True, "rccl_exchange": False, "ts_fused": False}]
            if self.ts_fused_ok:
                cands.append({"ts_side": False, "rccl_exchange": False, "ts_fused": True})
            if xmode != "twoshot":
                cands.append({"ts_side": False, "rccl_exchange": True, "ts_fused": False})
        elif self._graph_auto and self.capturable and (self.size == 1 or self.owner):
            # eager launches vs one-step replays vs replays of blocks of steps
            cands = [{"use_graph": False}, {"use_graph": True, "graph_steps": 1}]
            if self.graph_steps > 1 and (self.history.mode == "full" or self.traj_loc is not None):
                cands.append({"use_graph": True, "graph_steps": self.graph_steps})
        self.stats["setups"] += 1
        if cands and dev.type == "cuda" and _autotune_mode() != "off" and \
                not getattr(self, "_skip_autotune", False):
            self._autotune(cands, min_window_s=1e-3 * float(
                os.environ.get("MULTIGRAD_AUTOTUNE_WINDOW_MS", "30")))
        return self

    def _graph_key(self):
        """Everything a captured step bakes in: the identity of every buffer it reads or
        writes and the launch scalars.  Equal keys across setups keep the graphs."""
        ids = [id(getattr(self, n, None)) for n in (
            "theta", "grad", "S", "slab", "h", "loss", "step_dev", "m", "v", "u", "g_loc",
            "traj_loc", "u_loc", "oneshot", "twoshot")]
        for b in (getattr(self, "bounds", None), getattr(self, "bounds_loc", None)):
            ids += [None] if b is None else [id(b.lo), id(b.hi), id(b.kind)]
        hist = getattr(self, "history", None)
        ids.append(id(getattr(hist, "buf", None)) if hist is not None else None)
        epoch = getattr(self.model, "engine_layout_epoch", None)
        return (tuple(ids), self.lr, self.b1, self.b2, self.eps, self.legacy, self.pipeline,
                self.owner, self.zero, self.C, None if epoch is None else epoch())

    def _tune_key(self, cands):
        return (tuple(tuple(sorted(c.items())) for c in cands), self.P, self.size, self.owner,
                self.zero, self.pipeline, self.C, self.history.mode == "full",
                self.traj_loc is not None, self.bounds is None)

    @staticmethod
    def _param_order(md, P: int, upp: int, dev):
        """``(pidx, inv_pidx)``: internal -> user and user -> internal parameter index of
        the model's unit order (``engine_param_perm``), or ``(None, None)``."""
        perm = getattr(md, "engine_param_perm", lambda: None)()
        if perm is None:
            return None, None
        perm = torch.as_tensor(perm, device=dev).to(torch.int64)
        ar = torch.arange(upp, device=dev, dtype=torch.int64)
        pidx = (perm[:, None] * upp + ar).reshape(-1)      # internal -> user index
        inv = torch.empty_like(pidx)
        inv[pidx] = torch.arange(P, device=dev)            # user -> internal index
        return pidx, inv

    # ------------------------------------------------------------------ re-layout
    # A fit can move populations across the Euler-Maclaurin limit (the reference's own SMF
    # fit takes sigma from 0.5 to 0.2 dex on 0.1-dex bins, tests/smf_example/
    # smf_grad_descent.py:103,113): the lane classes laid out at setup then no longer
    # match, narrow populations sit scattered in wide groups and most groups take the
    # per-edge path (1% scattered narrow populations: ~47% of the groups).  Every
    # MULTIGRAD_RELAYOUT_EVERY (16) steps the engine measures on the device, without a host sync,
    # the share of groups the forward at the current parameters sends down the per-edge
    # path (model.engine_relayout_probe), reads it back a few steps later, and when it
    # differs from the share the classes were laid out for by more than
    # MULTIGRAD_RELAYOUT_MARGIN it re-classifies at the step boundary: the lanes are rebuilt
    # on the GPU (ops/_schedule.py:build_lanes_torch, ms) and theta / m / v / u / bounds are
    # permuted into the new internal order.  Trajectory rows keep the order they were
    # written in; each row range is mapped back to the user order with its own permutation.
    def _relayout_init(self) -> None:
        md = self.model
        every = int(os.environ.get("MULTIGRAD_RELAYOUT_EVERY", "16") or 0)
        self.relayout_every = every
        self.relayout_margin = float(os.environ.get("MULTIGRAD_RELAYOUT_MARGIN", "0.02"))
        self._relayout_on = bool(
            every > 0 and _env_flag("MULTIGRAD_RELAYOUT", True) and self.device.type == "cuda"
            and (self.size == 1 or self.owner) and self.pidx is not None
            and hasattr(md, "engine_relayout_probe") and hasattr(md, "engine_layout_share"))
        self._probe_step = None
        self._probe_last = 0
        self._probe_host = None
        self._probe_ev = None
        self._share_ref = self._probe_now() if self._relayout_on else None
        self.relayouts: List[dict] = []
        # trajectory row ranges and the user -> internal map they were written with
        self._segs = [(0, self.inv_pidx)]

    def _probe_now(self) -> Optional[float]:
        """The probe's per-edge share at the current parameters (host sync)."""
        v = self.model.engine_relayout_probe(self.theta, self.rank if self.owner else None)
        return None if v is None else float(v)

    def _maybe_relayout(self) -> None:
        """Step-boundary hook: launch the device probe every ``relayout_every`` steps and act
        on its value ``_PROBE_DELAY`` steps later (deterministic step: owner ranks vote)."""
        if not getattr(self, "_relayout_on", False) or self._tuning or self._capturing:
            return
        k = self.step_host
        if self._probe_step is None:
            if k - self._probe_last < self.relayout_every:
                return
            v = self.model.engine_relayout_probe(self.theta, self.rank if self.owner else None)
            if v is None:
                self._relayout_on = False
                return
            if self._probe_host is None:
                self._probe_host = torch.zeros(1, dtype=torch.float32, pin_memory=True)
                self._probe_ev = torch.cuda.Event()
            self._probe_host.copy_(v.reshape(1), non_blocking=True)
            self._probe_ev.record()
            self._probe_step = k
            return
        if k - self._probe_step < self._PROBE_DELAY:
            return
        self._probe_ev.synchronize()  # recorded _PROBE_DELAY steps ago: normally long done
        f_cur = float(self._probe_host[0])
        self._probe_step, self._probe_last = None, k
        # the probe's share right after the last (re)layout is the reference: a drift by
        # more than the margin either way means populations crossed the limit since
        f_ref = self._share_ref if self._share_ref is not None else 0.0
        go = abs(f_cur - f_ref) > self.relayout_margin
        if self.owner and self.size > 1:
            flag = torch.tensor([1 if go else 0], dtype=torch.int64)
            self.comm.all_reduce(flag, op="max")
            go = bool(flag[0])
        if go and not self.relayout(reason=dict(step=k, share_probe=round(f_cur, 4),
                                                share_ref=round(f_ref, 4))):
            self._share_ref = f_cur  # classes unchanged: nothing to gain, stop re-trying

    _PROBE_DELAY = 4

    @on_engine_stream
    def relayout(self, reason: Optional[dict] = None) -> bool:
        """Re-classify the lane groups at the current parameters and rebuild the layout
        (collective in owner mode).  Returns whether the classes changed."""
        md = self.model
        if self.pidx is None or not hasattr(md, "engine_layout_hint"):
            return False
        t0 = time.perf_counter()
        self.drain()
        P, dev = self.P, self.device
        if self.owner:
            a, b = self.own_range
            full = self._assemble(self.theta[a:b])
        else:
            full = self.theta[:P]
        band = float(os.environ.get("MULTIGRAD_RELAYOUT_BAND", "0.02"))
        if not md.engine_layout_hint(self.to_user(full), band=band):
            return False
        old_inv = self.inv_pidx
        md.engine_set_chunks(self._ub)
        pidx, inv = self._param_order(md, P, self.upp, dev)
        g = old_inv[pidx]  # new internal position i holds old internal position g[i]
        if self.owner:
            a, b = self.own_range
            loc = g[a:b] - a
            self.theta[a:b] = self.theta[g[a:b]]
            for name in ("m", "v", "u_loc"):
                t = getattr(self, name, None)
                if t is not None:
                    t.copy_(t[loc])
            if self.bounds_loc is not None:
                bl = self.bounds_loc
                self.bounds_loc = Bounds(bl.lo[loc].contiguous(), bl.hi[loc].contiguous(),
                                         bl.kind[loc].contiguous())
        else:
            self.theta[:P] = self.theta[:P][g]
            for name in ("m", "v"):
                t = getattr(self, name)
                t[:P] = t[:P][g]
            if self.bounds is not None:
                self.u[:P] = self.u[:P][g]
        if self.bounds is not None:
            bd = self.bounds
            pad = torch.arange(P, bd.lo.numel(), device=dev)
            gi = torch.cat([g, pad])
            self.bounds = Bounds(bd.lo[gi].contiguous(), bd.hi[gi].contiguous(),
                                 bd.kind[gi].contiguous())
        if self.history.mode != "full":
            self.history.rows = [r[g] for r in self.history.rows]
        self.pidx, self.inv_pidx = pidx, inv
        self._segs.append((self.step_host + 1, inv))
        rows = [md.engine_fwd_rows(c) for c in range(self.C)]
        if sum(rows) * self.nS > self.slab.numel():
            self.slab = torch.zeros(sum(rows) * self.nS, dtype=torch.float32, device=dev)
        self.rows = rows
        self.graph = None  # captured with the old layout's buffers
        torch.cuda.synchronize()
        self._share_ref = self._probe_now()
        rec = dict(reason or {}, step=self.step_host, seconds=round(time.perf_counter() - t0, 4),
                   share_new=round(self._share_ref, 4) if self._share_ref is not None else None,
                   share_layout=round(md.engine_layout_share(self.rank if self.owner else None), 4))
        self.relayouts.append(rec)
        return True

    def _traj_to_user(self, t: torch.Tensor) -> torch.Tensor:
        """Trajectory rows (internal order of the layout they were written in) -> user order."""
        segs = getattr(self, "_segs", None)
        if self.pidx is None or not segs or len(segs) == 1:
            return self.to_user(t)
        out = torch.empty_like(t)
        n = t.shape[0]
        for i, (r0, inv) in enumerate(segs):
            r1 = segs[i + 1][0] if i + 1 < len(segs) else n
            r0, r1 = min(r0, n), min(r1, n)
            if r1 > r0:
                out[r0:r1] = t[r0:r1][..., inv]
        return out

    # ------------------------------------------------------------------ setup-time tuning
    def _tl(self):
        """The sharded trajectory buffer, or None while the autotune steps run."""
        return None if self._tuning else self.traj_loc

    def _hb(self):
        """The replicated trajectory buffer (flat), or None (not recorded / autotune)."""
        if self._tuning or self.history.mode != "full":
            return None
        return self.history.buf.reshape(-1)

    def _autotune(self, cands, warm: int = 2, min_window_s: float = 0.008, **kw):
        key = self._tune_key(cands)
        hit = self._tune_cache.get(key)
        if hit is not None and hit.get("budget_skipped"):
            # a short run kept the default schedule before: again, unless this run's budget
            # (from the probe step time measured then) now affords the windows
            est = hit["step_ms_probe"] * 1e-3
            budget = float(os.environ.get("MULTIGRAD_TUNE_BUDGET", "0.1")) * est * max(1, self.nsteps)
            rounds_b = max(1, int(os.environ.get("MULTIGRAD_AUTOTUNE_ROUNDS", "2")))
            extra = warm + (self.graph_steps if any(c.get("use_graph") for c in cands) else 0)
            if _autotune_mode() == "on" or \
                    int(budget / max(est, 1e-9) / (len(cands) * rounds_b)) - extra >= 8:
                hit = None
        if hit is not None:
            # this engine timed these candidates before (a repeated run_* call): no trial
            # steps, the verdict is applied as it is
            changed = False
            for k, v in hit["chosen"].items():
                if getattr(self, k, None) != v:
                    setattr(self, k, v)
                    # use_graph / graph_steps choose whether (and which) graphs replay; the
                    # graphs themselves stay valid (their buffers are in the graph key)
                    changed = changed or k not in ("use_graph", "graph_steps")
            if changed:
                self.graph = None
            self.tuning = dict(hit, cached=True)
            trace(f"engine: autotune verdict cached {hit['chosen']}")
            return
        trace(f"engine: autotune {cands}")
        try:
            self._autotune_impl(cands, warm, min_window_s, **kw)
        finally:
            trace(f"engine: autotune done {getattr(self, 'tuning', None)}")
        if self.tuning is not None:
            self._tune_cache[key] = {k: v for k, v in self.tuning.items() if k != "cached"}

    def _autotune_impl(self, cands, warm: int = 2, min_window_s: float = 0.008,
                  max_reps: int = 400):
        """Collective: time each candidate schedule (a dict of engine attributes) over a
        window of at least ``min_window_s`` of work after ``warm`` steps, with syncs only
        at the window edges; keep the candidate whose slowest rank was fastest, then
        restore the optimizer state.  No trajectory rows are written while tuning, so the
        recorded trajectory is that of the real steps alone.

        Besides picking the schedule measured fastest on this machine (eager launches vs
        graph replay; the hashed exchange on the compute or a side stream), the window
        length brings the GPU to its working clock before the first real step: after a
        cold start the same step ran 0.88 ms and ~0.64 ms only after ~15 ms of work
        (profiles/step_timeline.md)."""
        state = [self.theta, self.m, self.v, self.step_dev]
        for name in ("u", "u_loc"):
            t = getattr(self, name, None)
            if t is not None and all(t is not x for x in state):
                state.append(t)
        saved = [t.clone() for t in state]
        multi = self.size > 1

        def restore():
            self._drain_all()
            torch.cuda.synchronize()
            for t, v in zip(state, saved):
                t.copy_(v)
            self.pending = False
            self.step_host = 0

        def apply(c):
            for k, v in c.items():
                setattr(self, k, v)
            self.graph = None

        def window(n):
            self._drain_all()
            torch.cuda.synchronize()
            if multi:
                self.comm.barrier()
            t0 = time.perf_counter()
            self._run_steps(n)
            self._drain_all()
            torch.cuda.synchronize()
            dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
            if multi:
                self.comm.all_reduce(dt, op="max")
            return float(dt) / n

        from ..parallel.xgmi import CollectiveTimeout

        def verdict(c):
            """Collective: None if every rank's peer-memory exchanges of candidate ``c``
            completed, else the reason (and the protocols are reset on every rank, so the
            next candidate starts clean)."""
            ctxs = [x for x in (self.twoshot, self.oneshot) if x is not None]
            if not multi or not ctxs:
                return None
            flags = torch.zeros(self.size, dtype=torch.int64)
            flags[self.rank] = int(any(int(x.err.item()) for x in ctxs))
            self.comm.all_reduce(flags)
            bad = [r for r in range(self.size) if int(flags[r])]
            if not bad:
                return None
            for x in ctxs:
                x.reset(self.comm)
            return f"peer-memory exchange timed out on rank(s) {bad}"

        cands = [dict(c) for c in cands]
        dropped = []
        self._fault_seen = set()
        self._tuning = True
        try:
            apply(cands[0])
            for _ in range(warm):
                self._raw_step()
            est = window(2)
            reps = int(min(max_reps, max(8, math.ceil(min_window_s / max(est, 1e-6)))))
            restore()
            why = verdict(cands[0])
            if why is not None:  # the probe of the first candidate already failed
                dropped.append(dict(cands[0], reason=why))
            self.stats["trial_steps"] += warm + 2
            rounds_b = max(1, int(os.environ.get("MULTIGRAD_AUTOTUNE_ROUNDS", "2")))
            budget_s = None
            if _autotune_mode() == "auto":
                # at most MULTIGRAD_TUNE_BUDGET of the requested run (est: the slowest rank's
                # step, identical on every rank, so every rank takes the same branch)
                budget_s = float(os.environ.get("MULTIGRAD_TUNE_BUDGET", "0.1")) * est * \
                    max(1, self.nsteps)
                extra = warm + (self.graph_steps if any(c.get("use_graph") for c in cands) else 0)
                fit = int(budget_s / max(est, 1e-9) / (len(cands) * rounds_b)) - extra
                if fit < 8 and why is None:
                    apply(cands[0])
                    self.tuning = {"chosen": cands[0], "budget_skipped": True,
                                   "budget_ms": round(1e3 * budget_s, 3),
                                   "step_ms_probe": round(1e3 * est, 4)}
                    self._settle(est, restore, budget_s=budget_s)
                    if multi:
                        torch.cuda.synchronize()
                        self.comm.barrier()
                    return
                reps = max(8, min(reps, fit))
            times = [math.inf] * len(cands)
            # MULTIGRAD_AUTOTUNE_ROUNDS (2) rounds, the order reversed every other round, the
            # best window of each candidate kept: a single pass in a fixed order let the
            # clock ramp of the first windows decide (the headline's eager candidate timed
            # 0.470 ms against 0.455 for 16-step replays in the first window, while
            # alternating runs measured eager 0.438 vs 0.447, profiles/graph_modes)
            rounds = max(1, int(os.environ.get("MULTIGRAD_AUTOTUNE_ROUNDS", "2")))
            for r in range(rounds):
                order = list(range(len(cands)))
                if r % 2:
                    order.reverse()
                for i in order:
                    c = cands[i]
                    if any(d.items() >= c.items() for d in dropped):
                        times[i] = math.inf
                        continue
                    apply(c)
                    self._fault_c = c
                    for _ in range(warm):
                        self._raw_step()
                    if self._block_ok():
                        self._run_steps(self.graph_steps)  # capture (and first replay) untimed
                    t = window(reps)
                    self.stats["trial_steps"] += warm + reps
                    self._fault_c = None
                    restore()
                    why = verdict(c)
                    if why is not None:
                        dropped.append(dict(c, reason=why))
                        times[i] = math.inf
                        continue
                    times[i] = min(times[i], t)
            if all(math.isinf(t) for t in times) and self.twoshot is not None:
                # no peer-memory schedule survived: the RCCL exchange on the same buffers
                fb = {k: False for k in cands[0]}
                fb["rccl_exchange"] = True
                if fb in cands:
                    times[cands.index(fb)] = math.inf
                apply(fb)
                for _ in range(warm):
                    self._raw_step()
                t = window(reps)
                restore()
                why = verdict(fb)
                if why is not None:
                    raise CollectiveTimeout(f"setup autotune: every exchange schedule failed ({why})")
                if fb not in cands:
                    cands.append(fb)
                    times.append(t)
                else:
                    times[cands.index(fb)] = t
            self.check("setup autotune", collective=multi)
        finally:
            self._tuning = False
            self._fault_c = None
        if all(math.isinf(t) for t in times):
            raise CollectiveTimeout(f"setup autotune: every candidate failed: {dropped}")
        best = min(range(len(cands)), key=lambda i: times[i])
        apply(cands[best])
        self.tuning = {"candidates": [dict(c, ms=round(1e3 * t, 4) if math.isfinite(t) else None)
                                      for c, t in zip(cands, times)],
                       "chosen": cands[best], "steps_per_window": reps, "rounds": rounds}
        if dropped:
            self.tuning["dropped"] = dropped
        if self.use_graph:
            # capture the real (trajectory-writing) step now rather than inside the first
            # timed step
            pend = self.pending
            self.pending = self.pipeline
            self._capture()
            if self._block_ok():
                self._capture(self.graph_steps)
            self.pending = pend
        used = rounds * len(cands) * (reps + warm) * est
        self._settle(est, restore, budget_s=None if budget_s is None else max(0.0, budget_s - used))
        if multi:
            torch.cuda.synchronize()
            self.comm.barrier()

    def _settle(self, step_s: float, restore, budget_s: Optional[float] = None) -> None:
        """End the setup with ``MULTIGRAD_SETTLE_MS`` (60) of eager steps (no trajectory
        rows; the optimizer state is restored afterwards), so the first real steps do not
        start from an idle GPU.  Measured on one MI355X (profiles/narrow_sweep/README.md):
        after the ~0.1 s of host work that follows the autotune windows, the forward kernel
        ran 410 us for a few steps, then 500-585 us and only back at ~445 us after ~50 steps
        -- the power controller's transient after an idle gap; a 20-step timing from there
        measured ~1850 steps/s against ~2250 in steady state."""
        ms = float(os.environ.get("MULTIGRAD_SETTLE_MS", "60"))
        if budget_s is not None:  # MULTIGRAD_AUTOTUNE=auto: what is left of the tuning budget
            ms = min(ms, 1e3 * budget_s)
        if ms <= 0 or self.device.type != "cuda" or (budget_s is not None and ms < 1e3 * step_s):
            return
        n = int(min(2000, max(1, math.ceil(1e-3 * ms / max(step_s, 1e-5)))))
        self.stats["trial_steps"] += n
        use_graph = self.use_graph
        self._tuning = True
        self.use_graph = False  # eager launches: the captured graphs write trajectory rows
        try:
            for _ in range(n):
                self._raw_step()
            restore()
        finally:
            self._tuning = False
            self.use_graph = use_graph


    def _drain_all(self):
        self._flush_exchange()
        for c in range(self.C):
            self._drain(c)

    # ------------------------------------------------------------------ helpers
    def _connect_twoshot(self, numel: int):
        """The two-shot context for ``numel`` floats (kept across setups of the same
        size), connecting it now if needed -- collective; None: use RCCL."""
        from ..parallel.xgmi import acquire_twoshot, release_twoshot, twoshot_enabled
        if not twoshot_enabled() or self.size > 8:
            return None
        ts = self._ts_keep
        if ts is not None:
            torch.cuda.synchronize()  # no exchange of a previous run still in flight
        if ts is not None and ts.numel == numel:
            return ts
        if ts is not None:
            release_twoshot(self.comm, ts)
            self._ts_keep = None
        self._ts_keep = acquire_twoshot(self.comm, numel)
        return self._ts_keep

    @on_engine_stream
    def close(self) -> None:
        """Give the engine's peer-memory exchange context back to the communicator's pool
        (collective: every rank closes its engine).  The engine cannot step afterwards."""
        from ..parallel.xgmi import release_twoshot
        if getattr(self, "_ts_keep", None) is not None:
            release_twoshot(self.comm, self._ts_keep)
        self._ts_keep = None
        self.twoshot = None
        self.ready = False
        self.closed = True
        self.graph = None
        self._gkey = None

    def _ts_pack(self, c: int) -> bytes:
        """Chunk c's two-shot exchange (reduce-scatter -> Adam -> all-gather; bounded fits:
        Adam on u, modes 2 / 3) as packed launch arguments for a compute launch that carries
        it (fused exchange)."""
        a, b = self.own[c]
        o, n = self.loc_off[c], self.loc_len[c]
        tl = self._tl()
        traj = None if tl is None else tl.reshape(-1)[o:]
        bnd = self._bslice(c)
        mode = 1 if bnd is None else (3 if self.legacy else 2)
        return self.twoshot.pack(a, b - a, mode, m=self.m[o:o + n], v=self.v[o:o + n], traj=traj,
                                 traj_stride=0 if traj is None else self.traj_loc.shape[1],
                                 step=self.step_dev[c], host_step=self._hstep(), lr=self.lr,
                                 b1=self.b1, b2=self.b2, eps=self.eps, max_blocks=self.ts_blocks,
                                 u=None if self.u_loc is None else self.u_loc[o:o + n],
                                 bounds=bnd)

    def _flush_exchange(self):
        """Launch the pending exchange of the last chunk on its own (fused exchange)."""
        if self._x_pending is not None:
            from ..ops._ext import ext
            xs, self._x_pending = self._x_pending, None
            if not self._inject_fault():
                ext().xgmi_twoshot_launch_packed(xs)

    def _twoshot_update(self, c: int):
        """Chunk c: dense-gradient reduce-scatter + Adam on the owned slice + all-gather,
        one launch on the side stream after the chunk's VJP."""
        side = self.ts_side
        if self._inject_fault():
            return  # test hook: this rank skips one exchange, so its peers time out
        if side:
            self.ev_vjp[c].record(torch.cuda.current_stream())
            self.comm_stream.wait_event(self.ev_vjp[c])
        a, b = self.own[c]
        o, n = self.loc_off[c], self.loc_len[c]
        bnd = self._bslice(c)
        mode = 1 if bnd is None else (3 if self.legacy else 2)
        tl = self._tl()
        traj = None if tl is None else tl.reshape(-1)[o:]
        with torch.cuda.stream(self.comm_stream) if side else contextlib.nullcontext():
            self.twoshot.step(a, b - a, mode, m=self.m[o:o + n], v=self.v[o:o + n],
                              u=None if self.u_loc is None else self.u_loc[o:o + n],
                              bounds=bnd, traj=traj,
                              traj_stride=0 if traj is None else self.traj_loc.shape[1],
                              step=self.step_dev[c], host_step=self._hstep(), lr=self.lr,
                              b1=self.b1, b2=self.b2, eps=self.eps,
                              max_blocks=self.ts_blocks if side else 0)
        if side:
            self.ev_ts[c].record(self.comm_stream)
            self._ts_pending[c] = True

    def _inject_fault(self) -> bool:
        """Test hook ``MULTIGRAD_AUTOTUNE_FAULT=<attr>=<0|1>:<rank>``: while the setup
        autotune times a candidate with that attribute value, the given rank skips one
        two-shot exchange (once per matching candidate and tuning), so its peers' exchange times
        out (bounded wait) -- the way an exchange that fails on a real xGMI node shows up."""
        spec = os.environ.get("MULTIGRAD_AUTOTUNE_FAULT")
        c = getattr(self, "_fault_c", None)
        if not spec or c is None:
            return False
        cond, _, rank = spec.partition(":")
        key, _, val = cond.partition("=")
        if key not in c or bool(c[key]) != (val.strip() == "1") or int(rank or 0) != self.rank:
            return False
        seen = self.__dict__.setdefault("_fault_seen", set())
        ck = tuple(sorted(c.items()))
        if ck in seen:
            return False  # once per matching candidate
        seen.add(ck)
        return True

    def _maybe_repartition(self) -> None:
        """Collective: move the model's data to the parameter owners once (see
        ``repartition`` in ``__init__``); a model without ``engine_repartition``, or whose
        data already follow the owners, is left as it is."""
        if not self.repartition or self.repartitioned is not None:
            return
        fn = getattr(self.model, "engine_repartition", None)
        if fn is None:
            return
        trace("engine: re-partition by owner")
        info = fn()
        self.repartitioned = dict(info) if info else {}
        trace(f"engine: re-partition done {self.repartitioned}")

    def _owner_units(self, md, J):
        """Owner-mode unit bounds if the model's data placement allows it on every rank."""
        if not self.allow_owner or (self.size == 1 and not self.force_owner):
            return None
        fn = getattr(md, "engine_owner_units", None)
        ub = fn() if fn is not None else None
        if ub is None and self.size == 1 and self.force_owner:
            ub = [0, J]
        ok = ub is not None and len(ub) == self.size + 1 and ub[0] == 0 and ub[-1] == J \
            and all(x <= y for x, y in zip(ub, ub[1:]))
        if ok:
            lo, hi = md.engine_support_units()
            ok = hi <= lo or (ub[self.rank] <= lo and hi <= ub[self.rank + 1])
        flag = torch.tensor([1 if ok else 0], dtype=torch.int64)
        self.comm.all_reduce(flag, op="min")
        return [int(u) for u in ub] if int(flag[0]) == 1 else None

    def _assemble(self, own: torch.Tensor) -> torch.Tensor:
        """Owner mode: the full (model-order) vector(s) from every rank's owned slices;
        ``own`` is ``[..., n_own]`` (identical leading shape on all ranks)."""
        lead = tuple(own.shape[:-1])
        L = max(self.lengths)
        buf = torch.zeros(lead + (L,), dtype=own.dtype, device=self.device)
        buf[..., :own.shape[-1]] = own
        gathered = torch.empty((self.size,) + lead + (L,), dtype=own.dtype, device=self.device)
        self.comm.all_gather_into_tensor(gathered.reshape(-1), buf.reshape(-1))
        out = torch.empty(lead + (self.P,), dtype=own.dtype, device=self.device)
        for r in range(self.size):
            a, b = self.pb[r], self.pb[r + 1]
            out[..., a:b] = gathered[r][..., :b - a]
        return out

    def _ph(self, name: str):
        if self._capturing or not self.timer.enabled:
            return contextlib.nullcontext()
        return self.timer.phase(name)

    def _bslice(self, c):
        if self.bounds_loc is None:
            return None
        o, n = self.loc_off[c], self.loc_len[c]
        b = self.bounds_loc
        return Bounds(b.lo[o:o + n], b.hi[o:o + n], b.kind[o:o + n])

    def _drain(self, c):
        """Wait for chunk c's parameter all-gather (stream-ordered)."""
        if self._ts_pending[c]:
            torch.cuda.current_stream().wait_event(self.ev_ts[c])
            self._ts_pending[c] = False
        w = self._ag[c]
        if w is None:
            return
        w.wait()
        self._ag[c] = None

    @on_engine_stream
    def drain(self):
        """Join pending parameter all-gathers and exchanges and apply a pending (pipelined)
        update."""
        self._flush_exchange()
        for c in range(self.C):
            self._drain(c)
        if self.pending:
            self.pending = False
            idx = self.step_host - 1
            ok = True
            if self.bounds is not None:
                self._drain_bounded(idx)
            elif self.owner:
                a, b = self.own_range
                tl = self._tl()
                tb = None if tl is None else tl.reshape(-1)
                ok = self._fused_vjp_adam(self.rank, a, tb, b - a, host_step=self._hstep(idx))
            else:
                hb = self._hb()
                ok = self._fused_vjp_adam(None, 0, hb, self.P if hb is not None else 0,
                                          host_step=self._hstep(idx))
            assert ok, "pipelined engine lost its fused VJP + Adam path"

    def _drain_bounded(self, idx: int) -> None:
        """The pending update of step ``idx`` of a bounded pipelined fit: residual VJP and
        the bounded Adam kernel (csrc/adam.hip; the end of a run or a checkpoint)."""
        md = self.model
        hs = self._hstep(idx)
        if self.owner:
            a, b = self.own_range
            md.engine_vjp_into(self.theta, self.h, self.grad, chunk=self.rank)
            tl = self._tl()
            tb = None if tl is None else tl.reshape(-1)
            adam_step_(self.u_loc, self.m, self.v, self.grad[a:b], self.theta[a:b],
                       self.step_dev[0], self.lr, self.b1, self.b2, self.eps, self.bounds_loc,
                       self.legacy, traj_base=tb, traj_stride=(b - a) if tb is not None else 0,
                       host_step=hs)
            return
        md.engine_vjp_into(self.theta, self.h, self.grad, chunk=None)
        hb = self._hb()
        P, bnd = self.P, self.bounds
        adam_step_(self.u[:P], self.m[:P], self.v[:P], self.grad[:P], self.theta[:P],
                   self.step_dev[0], self.lr, self.b1, self.b2, self.eps,
                   Bounds(bnd.lo[:P], bnd.hi[:P], bnd.kind[:P]), self.legacy, traj_base=hb,
                   traj_stride=P if hb is not None else 0, host_step=hs)

    # ------------------------------------------------------------------ one step
    def _update_args(self, step_idx: int) -> dict:
        """Arguments of the pending (pipelined) VJP + Adam of step ``step_idx``."""
        if self.owner:
            a, b = self.own_range
            tl = self._tl()
            traj = None if tl is None else tl.reshape(-1)
            stride = b - a
        else:
            a = 0
            traj = self._hb()
            stride = self.P
        args = dict(h=self.h, m=self.m, v=self.v, unit_offset=a // self.upp,
                    step=self.step_dev[0], host_step=self._hstep(step_idx), lr=self.lr,
                    b1=self.b1, b2=self.b2, eps=self.eps, traj=traj,
                    traj_stride=stride if traj is not None else 0)
        if self.bounds is not None:  # bounded: Adam on u (indexed like m, v), p = T^-1(u)
            bnd = self.bounds_loc if self.owner else self.bounds
            args.update(u=self.u_loc if self.owner else self.u, lo=bnd.lo, hi=bnd.hi,
                        legacy=self.legacy)
        return args

    def _forward_loss(self, update: bool = False):
        md = self.model
        row = 0
        fused = getattr(md, "engine_reduce_loss_into", None)
        fused_ok = (fused is not None and self.fuse_epilogue
                    and (self.size == 1 or self.oneshot is not None) and self.slab.is_cuda)
        advance = None
        # the last chunk's forward host call also issues the epilogue launch (one host call
        # per step fewer; ops/smf.py:smf_forward_into, csrc/smf.hip:smf_forward_lanes)
        fold = fused_ok and _env_flag("MULTIGRAD_FOLD_EPILOGUE", True) and \
            getattr(md, "engine_forward_epilogue_ok", lambda: False)()
        chunks = [self.rank] if self.owner else list(range(self.C))
        folded = False
        with self._ph("forward"):
            for i, c in enumerate(chunks):
                self._drain(c)
                epi = None
                if fold and i == len(chunks) - 1:
                    epi = dict(slab=self.slab, row0=row, S=self.S, loss=self.loss, h=self.h,
                               oneshot=self.oneshot if self.size > 1 else None, advance=None)
                if update:  # the previous step's VJP + Adam, fused into this forward
                    args = self._update_args(self.step_host - 1)
                    if fused_ok and args["host_step"] is None:
                        # device step counter: advanced by the epilogue launch, not a kernel
                        args["defer_advance"] = True
                        advance = args["step"]
                    if epi is not None:
                        epi["advance"] = advance
                    kw = {} if epi is None else {"epilogue": epi}
                    n = md.engine_forward_update_chunk(self.theta, self.slab[row * self.nS:], c,
                                                       args, **kw)
                else:
                    kw = {} if epi is None else {"epilogue": epi}
                    if i == 0 and self._x_pending is not None:
                        # the previous step's exchange of the last chunk, in this launch's
                        # first workgroups (this chunk's parameters are already complete)
                        kw["exchange"] = self._x_pending
                        self._x_pending = None
                        if self._inject_fault():
                            del kw["exchange"]
                    n = md.engine_forward_chunk(self.theta, self.slab[row * self.nS:], c, **kw)
                folded = epi is not None
                row += n
        if folded:
            return
        if fused_ok:
            with self._ph("sumstat_epilogue"):
                if fused(self.slab, row, self.S, self.loss, self.h, self.oneshot,
                         advance=advance):
                    return
        assert advance is None, "the step counter advance was deferred to the epilogue"
        with self._ph("forward"):
            md.engine_reduce(self.slab, row, self.S)
        if self.size > 1:
            with self._ph("sumstat_allreduce"):
                self.comm.all_reduce(self.S)
        with self._ph("loss"):
            md.engine_loss_into(self.S, self.loss, self.h)

    def _enqueue_step(self):
        md = self.model
        if self.pipeline:
            # step k = [VJP + Adam of step k-1 fused into the forward of step k] + epilogue;
            # the update of step k stays pending until the next step or drain()
            self._forward_loss(update=self.pending)
            self.pending = True
            return
        self._forward_loss()
        hb = self._hb()
        tl = self._tl()
        if self.owner and self._fused_vjp_adam(self.rank, self.own_range[0],
                                               None if tl is None else tl.reshape(-1),
                                               self.own_range[1] - self.own_range[0]):
            pass
        elif self.owner:
            c = self.rank
            with self._ph("vjp"):
                md.engine_vjp_into(self.theta, self.h, self.grad, chunk=c)
            a, b = self.own_range
            u = self.u_loc if self.u_loc is not None else self.theta[a:b]
            p = self.theta[a:b] if self.u_loc is not None else None
            tb = None if tl is None else tl.reshape(-1)
            with self._ph("adam"):
                adam_step_(u, self.m, self.v, self.grad[a:b], p, self.step_dev[0], self.lr,
                           self.b1, self.b2, self.eps, self.bounds_loc, self.legacy,
                           traj_base=tb, traj_stride=(b - a) if tb is not None else 0,
                           host_step=self._hstep())
        elif self.zero and self.twoshot is not None and not self.rccl_exchange and self.ts_fused:
            # VJP_0, [VJP_1 + X_0], ..., [VJP_{C-1} + X_{C-2}]; X_{C-1} rides on the next
            # step's first forward launch (or drain())
            for c in range(self.C):
                xs = self._ts_pack(c - 1) if c > 0 else None
                with self._ph("vjp"):
                    md.engine_vjp_into(self.theta, self.h, self.grad, chunk=c, exchange=xs)
            self._x_pending = self._ts_pack(self.C - 1)
        elif self.zero and self.twoshot is not None and not self.rccl_exchange:
            for c in range(self.C):
                with self._ph("vjp"):
                    md.engine_vjp_into(self.theta, self.h, self.grad, chunk=c)
                self._twoshot_update(c)
        elif self.zero:
            rs = []
            for c in range(self.C):
                with self._ph("vjp"):
                    md.engine_vjp_into(self.theta, self.h, self.grad, chunk=c)
                a, L = self.pb[c], self.lengths[c]
                o, n = self.loc_off[c], self.loc_len[c]
                rs.append(self.comm.reduce_scatter_tensor(self.g_loc[o:o + n], self.grad[a:a + L],
                                                          async_op=True))
            for c in range(self.C):
                with self._ph("grad_reduce_scatter_wait"):
                    rs[c].wait()
                a, b = self.own[c]
                o, n = self.loc_off[c], self.loc_len[c]
                u = self.u_loc[o:o + n] if self.u_loc is not None else self.theta[a:b]
                p = self.theta[a:b] if self.u_loc is not None else None
                tb = None if tl is None else tl.reshape(-1)[o:]
                with self._ph("adam"):
                    adam_step_(u, self.m[o:o + n], self.v[o:o + n], self.g_loc[o:o + n], p,
                               self.step_dev[c], self.lr, self.b1, self.b2, self.eps,
                               self._bslice(c), self.legacy, traj_base=tb,
                               traj_stride=self.traj_loc.shape[1] if tb is not None else 0,
                               host_step=self._hstep())
                pa, L = self.pb[c], self.lengths[c]
                agc = self.comm_ag if self.comm_ag is not None else self.comm
                self._ag[c] = agc.all_gather_into_tensor(self.theta[pa:pa + L], self.theta[a:b],
                                                         async_op=True)
        elif self.C == 1 and self._fused_vjp_adam(None, 0, hb, self.P if hb is not None else 0):
            pass
        else:
            with self._ph("vjp"):
                for c in range(self.C):
                    md.engine_vjp_into(self.theta, self.h, self.grad,
                                       chunk=c if self.C > 1 else None)
            if self.size > 1:
                with self._ph("grad_allreduce"):
                    self.comm.all_reduce(self.grad)
            with self._ph("adam"):
                self._replicated_adam(hb)

    def _replicated_adam(self, hb):
        stride = self.P if hb is not None else 0
        bnd = self.bounds
        if hb is not None and self.P_pad != self.P:
            # trajectory rows are P long: update the real parameters and the padding
            # separately so the kernel writes exactly one row
            P = self.P
            adam_step_(self.u[:P], self.m[:P], self.v[:P], self.grad[:P],
                       self.theta[:P] if bnd is not None else None, self.step_dev[0],
                       self.lr, self.b1, self.b2, self.eps,
                       None if bnd is None else Bounds(bnd.lo[:P], bnd.hi[:P], bnd.kind[:P]),
                       self.legacy, traj_base=hb, traj_stride=stride, host_step=self._hstep())
        else:
            adam_step_(self.u, self.m, self.v, self.grad,
                       self.theta if bnd is not None else None, self.step_dev[0],
                       self.lr, self.b1, self.b2, self.eps, bnd, self.legacy,
                       traj_base=hb, traj_stride=stride, host_step=self._hstep())

    def _fused_vjp_adam(self, chunk, p0: int, traj, traj_stride: int, host_step="auto") -> bool:
        """Fused VJP + Adam when the gradient is complete locally (owner mode, or one
        replicated chunk), the parameters are unbounded and the model offers it."""
        fn = getattr(self.model, "engine_vjp_adam_into", None)
        if fn is None or not self.fuse_vjp_adam or self.bounds is not None:
            return False
        with self._ph("vjp_adam"):
            hs = self._hstep() if host_step == "auto" else host_step
            return bool(fn(self.theta, self.h, self.m, self.v, p0 // self.upp, self.step_dev[0],
                           hs, self.lr, self.b1, self.b2, self.eps, traj_base=traj,
                           traj_stride=traj_stride, chunk=chunk))

    def _hstep(self, idx: Optional[int] = None):
        """The 0-based step for eager launches; None inside a graph capture and for every
        launch of a graph-mode engine (the Adam kernels then keep the step in device
        memory, so graph replays and eager launches -- e.g. direct step() calls, which
        launch eagerly -- agree)."""
        if self._capturing or self.use_graph or (self.device_step and self.pipeline):
            return None
        return self.step_host if idx is None else idx

    def _capture(self, k: int = 1):
        """Capture ``k`` consecutive steps into one graph (k = 1: ``self.graph``; k > 1:
        the block graph).  Every step inside reads and advances the device step counter,
        so a block replays exactly like k one-step replays."""
        prep = getattr(self.model, "engine_prepare", None)
        if prep is not None:
            prep([self.rank] if self.owner else list(range(self.C)))
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        torch.cuda.current_stream().wait_stream(s)
        from .generic import _no_gc
        g = torch.cuda.CUDAGraph()
        pend = self.pending
        self._capturing = True
        try:
            with _no_gc():  # no CUDAGraph may be freed by the collector during a capture
                with torch.cuda.graph(g):
                    for _ in range(int(k)):
                        self._enqueue_step()  # pipelined: sets pending for the next one
        finally:
            self._capturing = False
            self.pending = pend
        self.stats["captures"] += 1
        if k == 1:
            self.graph = g
        else:
            self._kgraph = (int(k), g)

    def _block_ok(self) -> bool:
        """Whether steps may run as replays of a multi-step graph: graph mode, and no
        per-step host work (the trajectory rows are written on the device)."""
        return (self.use_graph and self.graph_steps > 1 and
                (self.history.mode == "full" or self.traj_loc is not None))

    def _run_steps(self, n: int):
        """``n`` steps without the host-side history bookkeeping: blocks of
        ``graph_steps`` steps replayed from one graph where allowed, the rest one by one."""
        n = int(n)
        K = self.graph_steps
        while n > 0:
            if n >= K and self._block_ok() and (self.pending or not self.pipeline):
                if self._kgraph is None or self._kgraph[0] != K:
                    self._capture(K)
                self._kgraph[1].replay()
                if self.pipeline:
                    self.pending = True
                self.step_host += K
                n -= K
            else:
                self._raw_step()
                n -= 1
            self._maybe_relayout()

    @on_engine_stream
    def steps(self, n: int):
        """Enqueue ``n`` optimizer steps (asynchronous on GPU): :meth:`step` ``n`` times,
        with blocks of ``graph_steps`` steps replayed from one graph in graph mode."""
        assert self.ready, "call setup() first"
        n = int(n)
        if n <= 0:
            return
        if not self._block_ok():
            for _ in range(n):
                self._step(replay=True)
            return
        if self.step_host + n > self.nsteps and self.history.mode == "full":
            raise RuntimeError("more steps than the trajectory buffer was sized for")
        self._run_steps(n)

    def _raw_step(self, replay: bool = True):
        if replay and self.use_graph and (self.pending or not self.pipeline):
            if self.graph is None:
                self._capture()
            self.graph.replay()
            if self.pipeline:
                self.pending = True
        else:
            self._enqueue_step()
        self.step_host += 1

    @on_engine_stream
    def step(self):
        """Enqueue one optimizer step (asynchronous on GPU).  A direct call launches eagerly
        even in graph mode unless ``step_replay`` is set (``MULTIGRAD_STEP_REPLAY=1``), as
        :meth:`GraphAdamEngine.step <multigrad_amd.engine.generic.GraphAdamEngine.step>`;
        :meth:`steps` and ``run_adam`` replay."""
        self._step(replay=self.step_replay)

    def _step(self, replay: bool = True):
        assert self.ready, "call setup() first"
        if self.step_host >= self.nsteps and self.history.mode == "full":
            raise RuntimeError("more steps than the trajectory buffer was sized for")
        self._raw_step(replay)
        self._record_history()
        self._maybe_relayout()

    def _record_history(self) -> None:
        """Host-side trajectory bookkeeping after a step (history "last" / stride)."""
        if self.history.mode != "full" and self.traj_loc is None:
            if self.pipeline:
                st = self.history.stride
                if not (self.step_host == self.history.nsteps or
                        (st and self.step_host % st == 0)):
                    return
            self.drain()
            if self.owner:
                st = self.history.stride
                if self.step_host == self.history.nsteps or (st and self.step_host % st == 0):
                    a, b = self.own_range
                    self.history.record(self.step_host - 1, self._assemble(self.theta[a:b]))
            else:
                self.history.record(self.step_host - 1, self.theta[:self.P])

    def to_user(self, t: torch.Tensor) -> torch.Tensor:
        """Engine (internal) parameter order -> the model's parameter order (last dim)."""
        if self.pidx is None:
            return t
        return t[..., self.inv_pidx]

    @on_engine_stream
    def trajectory(self) -> torch.Tensor:
        """The recorded parameter trajectory (assembled across ranks under ZeRO)."""
        self.drain()
        self.check("trajectory", collective=True)
        if self.traj_loc is None:
            if self.history.mode == "full":
                out = self._traj_to_user(self.history.result())
                if out.untyped_storage().data_ptr() == self.history.buf.untyped_storage().data_ptr():
                    out = out.clone()  # the buffer is the engine's: a later run rewrites it
                return out
            return self.to_user(self.history.result())
        if self.owner:
            rows = self.step_host + 1
            return self._traj_to_user(self._assemble(self.traj_loc[:rows].contiguous()))
        W = self.size
        nloc = self.traj_loc.shape[1]
        rows = self.step_host + 1
        gathered = torch.empty((W, rows, nloc), dtype=self.traj_loc.dtype, device=self.device)
        self.comm.all_gather_into_tensor(gathered.reshape(-1),
                                         self.traj_loc[:rows].contiguous().reshape(-1))
        out = torch.empty((rows, self.P_pad), dtype=self.traj_loc.dtype, device=self.device)
        for c in range(self.C):
            o, n = self.loc_off[c], self.loc_len[c]
            for r in range(W):
                a = self.pb[c] + r * n
                out[:, a:a + n] = gathered[r, :, o:o + n]
        return self.to_user(out[:, :self.P])

    @on_engine_stream
    def params(self) -> torch.Tensor:
        self.drain()
        self.check("params", collective=True)
        if self.owner:
            a, b = self.own_range
            return self.to_user(self._assemble(self.theta[a:b]))
        # a copy: theta may be the peer-memory region a later engine reuses
        return self.to_user(self.theta[:self.P]).clone()

    @on_engine_stream
    def last_loss(self) -> float:
        loss = float(self.loss.item())
        self.check("last_loss")
        return loss

    @on_engine_stream
    def check(self, where: str = "", collective: bool = False) -> None:
        """Raise :class:`~multigrad_amd.parallel.xgmi.CollectiveTimeout` if a peer-memory
        exchange of this engine (one-shot sumstats, two-shot gradient) timed out -- its
        results are NaN-poisoned; a host sync.

        ``collective=True`` all-reduces the verdict so every rank raises together (used
        where the caller goes on to a collective: ``params``, ``trajectory``,
        checkpoints, the periodic check of :meth:`run_adam`); ``last_loss`` and
        ``state_dict`` check locally."""
        where = where or f"engine step {self.step_host}"
        comm = self.comm if collective else None
        for ctx in (self.twoshot, self.oneshot):
            if ctx is not None:
                ctx.check(where, comm=comm)

    def grad_collective_name(self) -> str:
        """Human-readable name of the per-step gradient collective (bench records)."""
        if self.size == 1:
            return "none (1 rank)"
        if self.owner:
            return "none: owner-local gradients, sumstat all-reduce only"
        if self.zero and self.twoshot is not None and self.rccl_exchange:
            return ("RCCL reduce-scatter + all-gather (ZeRO-1), measured faster than the "
                    "two-shot kernel at setup")
        if self.zero and self.twoshot is not None:
            if self.ts_fused:
                sched = (f", {self.C} chunks, each exchange in the first workgroups of the "
                         f"next compute launch (fused exchange, one stream, no events)")
            elif self.ts_side:
                sched = f", {self.C} chunks on a side stream overlapping compute"
            else:
                sched = f", {self.C} chunk(s) on the compute stream"
            return ("xGMI two-shot kernel: reduce-scatter + Adam + all-gather in one launch per "
                    "chunk (self-tested)" + sched)
        if self.zero:
            return "RCCL reduce-scatter + all-gather (ZeRO-1)"
        return "RCCL all-reduce"

    def comm_bytes_per_step(self) -> int:
        """Bytes this rank sends through collectives in one step: the sumstat exchange,
        plus the dense-gradient exchange of the hashed placement (reduce-scatter and
        parameter all-gather, or an all-reduce: 2 (W-1)/W of the vector either way)."""
        W = self.size
        if W == 1:
            return 0
        nbytes = 4 * self.nS * (W - 1)  # one-shot push (RCCL moves about as much)
        if not self.owner:
            nbytes += int(2 * (W - 1) * (self.P_pad // W) * 4)
        return nbytes

    def sumstat_collective_name(self) -> str:
        if self.size == 1:
            return "none (1 rank)"
        return "xGMI one-shot kernel (self-tested)" if self.oneshot is not None else "RCCL"

    # ------------------------------------------------------------------ L-BFGS objective
    def lbfgs_objective(self, guess):
        """Objective over this rank's optimizer-owned parameters for
        :func:`multigrad_amd.optim.lbfgs.lbfgs_minimize` (sharded under ZeRO)."""
        self._skip_autotune = True  # the objective never runs optimizer steps
        try:
            self.setup(guess, nsteps=1, history="last")
        finally:
            self._skip_autotune = False
        return _EngineObjective(self)

    # ------------------------------------------------------------------ checkpoints
    @property
    def sharded(self) -> bool:
        return self.size > 1 and (self.zero or self.owner)

    def _local_theta(self) -> torch.Tensor:
        if self.owner:
            a, b = self.own_range
            return self.theta[a:b]
        if self.zero:
            return torch.cat([self.theta[a:b] for a, b in self.own])
        return self.theta

    @on_engine_stream
    def state_dict(self) -> dict:
        """This rank's optimizer state after ``step_host`` steps: owned slices under ZeRO
        and owner mode (one file per rank), everything otherwise."""
        self.drain()
        self.check("state_dict")  # never checkpoint NaN-poisoned state
        mode = "owner" if self.owner else "zero" if self.zero else "replicated"
        u = self.u_loc if self.sharded else (self.u if self.bounds is not None else None)
        st = {"mode": mode, "size": self.size, "rank": self.rank, "P": self.P,
              "pb": list(self.pb), "step": self.step_host, "lr": self.lr,
              "theta": self._local_theta().detach().cpu().clone(),
              "m": self.m.detach().cpu().clone(), "v": self.v.detach().cpu().clone(),
              "u": None if u is None else u.detach().cpu().clone()}
        rows = self.step_host + 1
        if self.traj_loc is not None:
            st["traj"] = self._traj_rows_to_current(self.traj_loc[:rows]).detach().cpu().clone()
        elif self.history.mode == "full":
            st["traj"] = self._traj_rows_to_current(self.history.buf[:rows]).detach().cpu().clone()
        else:
            st["history_rows"] = [r.detach().cpu().clone() for r in self.history.rows]
        if self.pidx is not None:
            # the user parameter index of every local element: a checkpoint written after a
            # re-layout loads into an engine laid out differently (e.g. at the guess)
            st["units_order"] = self._local_order().cpu().clone()
            if self.history.mode != "full" and self.traj_loc is None:
                st["units_order_full"] = self.pidx.cpu().clone()
        return st

    def _local_order(self) -> torch.Tensor:
        """User parameter index of each element of this rank's optimizer vectors."""
        if self.owner:
            a, b = self.own_range
            return self.pidx[a:b]
        return self.pidx

    def _traj_rows_to_current(self, t: torch.Tensor) -> torch.Tensor:
        """Trajectory rows (each in the layout it was written in) -> the current internal
        order (columns: this rank's local elements)."""
        segs = getattr(self, "_segs", None)
        if self.pidx is None or not segs or len(segs) == 1:
            return t
        base = self.own_range[0] if self.owner else 0
        cur = self._local_order()
        out = t.clone()
        n = t.shape[0]
        for i, (r0, inv) in enumerate(segs[:-1]):
            r1 = min(segs[i + 1][0], n)
            if r1 > min(r0, n):
                out[r0:r1, :cur.numel()] = t[r0:r1][:, inv[cur] - base]
        return out

    @on_engine_stream
    def load_state_dict(self, st: dict) -> int:
        """Restore a :meth:`state_dict` into a :meth:`setup` engine of the same shape;
        returns the step to continue from."""
        # finish this engine's in-flight work first: a pending fused exchange (the last chunk's
        # reduce-scatter -> Adam -> all-gather, carried by the next launch) or a pending
        # pipelined update would otherwise run on top of the loaded state
        self.drain()
        mode = "owner" if self.owner else "zero" if self.zero else "replicated"
        if st["mode"] != mode or st["size"] != self.size or st["P"] != self.P or \
                list(st["pb"]) != list(self.pb):
            raise ValueError(f"checkpoint ({st['mode']}, {st['size']} ranks) does not match "
                             f"this engine ({mode}, {self.size} ranks)")
        dev = self.device
        step = int(st["step"])
        from ..utils.checkpoint import check_loaded_step
        check_loaded_step(step, self.comm if self.size > 1 else None)
        self.m.copy_(st["m"].to(dev))
        self.v.copy_(st["v"].to(dev))
        th = st["theta"].to(dev)
        if self.owner:
            a, b = self.own_range
            self.theta[a:b].copy_(th)
        elif self.zero:
            for c in range(self.C):
                a, b = self.own[c]
                o, n = self.loc_off[c], self.loc_len[c]
                self.theta[a:b].copy_(th[o:o + n])
                pa, L = self.pb[c], self.lengths[c]
                agc = self.comm_ag if self.comm_ag is not None else self.comm
                self._ag[c] = agc.all_gather_into_tensor(self.theta[pa:pa + L], self.theta[a:b],
                                                         async_op=True)
            self.drain()
        else:
            self.theta.copy_(th)
        if st.get("u") is not None:
            (self.u_loc if self.sharded else self.u).copy_(st["u"].to(dev))
        elif not self.sharded and self.bounds is None:
            self.u = self.theta
        if "traj" in st:
            tr = st["traj"].to(dev)
            dst = self.traj_loc if self.traj_loc is not None else self.history.buf
            dst[:tr.shape[0]].copy_(tr)
        elif "history_rows" in st:
            self.history.rows = [r.to(dev) for r in st["history_rows"]]
        if st.get("units_order") is not None and self.pidx is not None:
            full = st.get("units_order_full")
            self._reorder_loaded(st["units_order"].to(dev), None if full is None else full.to(dev))
        self._segs = [(0, self.inv_pidx)]
        self.step_host = step
        self.step_dev[:, 0] = step
        self.step_dev[:, 1] = 0
        return step

    def _reorder_loaded(self, saved: torch.Tensor, saved_full: Optional[torch.Tensor]) -> None:
        """Permute freshly loaded vectors from the checkpoint's internal order (``saved``:
        user index per local element; ``saved_full``: per element of the full vector) into
        this engine's."""
        def positions(order):
            pos = torch.empty(self.P, dtype=torch.int64, device=order.device)
            pos[order] = torch.arange(order.numel(), device=order.device)
            return pos

        cur = self._local_order()
        if not torch.equal(saved, cur) and self.zero and not self.owner:
            # ZeRO slices are cut from the internal order: a different lanes layout gives
            # every rank different parameters in its slices
            raise ValueError(
                "this ZeRO checkpoint was written with a different lanes layout (parameter "
                "order) than this engine's -- e.g. resumed from another starting point whose "
                "narrow populations group the lanes differently; resume with the run's own "
                "guess, with zero=False, or with MULTIGRAD_LANE_CLASSES=0 on both runs")
        if not torch.equal(saved, cur):
            idx = positions(saved)[cur]  # position of each current local element when saved
            n = cur.numel()
            if self.owner:
                a, b = self.own_range
                self.theta[a:b] = self.theta[a:b][idx]
                vecs = [self.m, self.v] + ([self.u_loc] if self.u_loc is not None else [])
            else:
                self.theta[:n] = self.theta[:n][idx]
                vecs = [self.m, self.v] + ([self.u] if self.bounds is not None else [])
            for t in vecs:
                t[:n] = t[:n][idx]
            traj = self.traj_loc if self.traj_loc is not None else (
                self.history.buf if self.history.mode == "full" else None)
            if traj is not None:
                traj[:, :n] = traj[:, :n][:, idx]
        if saved_full is not None and self.history.mode != "full" and self.traj_loc is None \
                and not torch.equal(saved_full, self.pidx):
            idx = positions(saved_full)[self.pidx]
            self.history.rows = [r[idx] for r in self.history.rows]

    @on_engine_stream
    def save_checkpoint(self, path: str) -> None:
        from ..utils import checkpoint as ckpt
        self.drain()
        self.check("checkpoint", collective=True)
        ckpt.save_optimizer_state(path, self.state_dict(), comm=self.comm if self.size > 1 else None,
                                  sharded=self.sharded)

    @on_engine_stream
    def load_checkpoint(self, path: str) -> int:
        from ..utils import checkpoint as ckpt
        return self.load_state_dict(ckpt.load_optimizer_state(
            path, rank=self.rank, sharded=self.sharded,
            comm=self.comm if self.size > 1 and self.sharded else None))

    # ------------------------------------------------------------------ driver
    @on_engine_stream(always=True)
    def run_adam(self, guess, nsteps: int = 100, param_bounds=None, learning_rate: float = 0.01,
                 b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8, history="full",
                 legacy_bounds_jacobian: bool = False, callback=None,
                 checkpoint_path: Optional[str] = None, checkpoint_every: int = 0,
                 resume_from: Optional[str] = None, **unused):
        """Adam with the reference's return contract: trajectory ``(nsteps+1, P)``.

        ``checkpoint_path``/``checkpoint_every`` write a resumable state every k steps
        (owner-/ZeRO-sharded runs write one file per rank, ``<path>.rank<r>``);
        ``resume_from`` continues such a run (same number of ranks and placement)."""
        if unused:
            raise TypeError(f"unsupported run_adam options for the fused engine: {sorted(unused)}")
        self.setup(guess, nsteps, param_bounds, learning_rate, b1, b2, eps, history,
                   legacy_bounds_jacobian)
        start = self.load_checkpoint(resume_from) if resume_from is not None else 0
        from ..utils.hooks import StepHooks, driver_guard
        hooks = StepHooks(self.comm, callback)  # MULTIGRAD_CHECK_EVERY / MULTIGRAD_METRICS
        err_every = int(os.environ.get("MULTIGRAD_ERR_CHECK_EVERY", "100") or 0)
        err_every = err_every if (self.oneshot is not None or self.twoshot is not None) else 0
        ck_every = checkpoint_every if checkpoint_path else 0
        with driver_guard(self.comm):
            comm_bytes = self.comm_bytes_per_step()
            i, end = start, int(nsteps)
            while i < end:
                # steps up to the next host event run as one call (graph blocks)
                n = 1 if hooks.active else min(
                    [end - i] + [e - i % e for e in (err_every, ck_every) if e])
                self.steps(n)
                i += n
                if hooks.active:
                    hooks(i - 1, self.loss, self, self.params, comm_bytes=comm_bytes)
                if err_every and i % err_every == 0:
                    self.check(collective=True)
                if ck_every and i % ck_every == 0:
                    self.save_checkpoint(checkpoint_path)
            return self.trajectory()


class _EngineObjective:
    """Loss and gradient over the engine's owned parameter slices.

    ZeRO (world > 1): x is the concatenation of this rank's slices of every chunk; an
    evaluation all-gathers the chunks, runs forward + loss + per-chunk VJP, and
    reduce-scatters the gradient back to the owned slices -- L-BFGS vectors and history
    are sharded 1/W and its dot products are all-reduced by the optimizer.  With the
    two-shot peer-memory context up, the all-gather is its mode 5 (each rank pushes its
    slices into every rank's parameter region) and the reduce-scatter its mode 4 (rank-order
    sum of the owned slices of every rank's gradient region): the evaluation makes no RCCL
    or host collective.  Otherwise RCCL reduce-scatter / all-gather on the same layout.
    Owner placement: x is the owned parameter range, whose gradient is complete locally
    (only the sumstats cross ranks, inside the forward's epilogue).
    Replicated: x is the full (padded) parameter vector and the gradient is all-reduced.
    """

    def __init__(self, eng: FusedAdamEngine):
        self.e = eng
        self.comm = eng.comm
        self.sharded = eng.zero or eng.owner
        self.device = eng.device
        self.ts = eng.twoshot if (eng.zero and not eng.owner) else None
        if eng.owner:
            self.n_local = eng.own_range[1] - eng.own_range[0]
        else:
            self.n_local = sum(eng.loc_len) if eng.zero else eng.P_pad

    def local_box(self, param_bounds):
        """``(lo, hi)`` of this objective's vector (user-order spec -> internal order,
        padding unbounded, then this rank's owned slices) for the device L-BFGS-B."""
        from ..optim.lbfgsb import bounds_arrays
        e = self.e
        lo_u, hi_u = bounds_arrays(param_bounds, e.P)
        out = []
        for arr, fill in ((lo_u, -math.inf), (hi_u, math.inf)):
            v = torch.full((e.P_pad,), fill, dtype=torch.float32, device=self.device)
            if arr is not None:
                t = torch.as_tensor(arr, dtype=torch.float32, device=self.device)
                v[:e.P] = t[e.pidx] if e.pidx is not None else t
            if e.owner:
                a, b = e.own_range
                v = v[a:b]
            elif e.zero:
                v = torch.cat([v[a:b] for a, b in e.own])
            out.append(v.contiguous())
        return out[0], out[1]

    def x0(self) -> torch.Tensor:
        e = self.e
        if e.owner:
            a, b = e.own_range
            return e.theta[a:b].clone()
        if not e.zero:
            return e.theta.clone()
        return torch.cat([e.theta[a:b] for a, b in e.own]).contiguous()

    def _load(self, x: torch.Tensor):
        e = self.e
        if e.owner:
            a, b = e.own_range
            e.theta[a:b].copy_(x)
            return
        if not e.zero:
            e.theta.copy_(x)
            return
        for c in range(e.C):
            a, b = e.own[c]
            o, n = e.loc_off[c], e.loc_len[c]
            if self.ts is not None:
                # this rank's slice into every rank's parameter region (its own included);
                # the launch returns when every rank's slice of the chunk has landed here
                self.ts.all_gather_(x[o:o + n], a, n)
                continue
            e.theta[a:b].copy_(x[o:o + n])
            pa, L = e.pb[c], e.lengths[c]
            agc = e.comm_ag if e.comm_ag is not None else e.comm
            e._ag[c] = agc.all_gather_into_tensor(e.theta[pa:pa + L], e.theta[a:b], async_op=True)

    def __call__(self, x: torch.Tensor):
        loss, g = self.device_call(x)
        f = float(loss.double().item())
        self.e.check("L-BFGS evaluation")
        return f, g

    def check(self, where: str = "L-BFGS") -> None:
        """Collective: raise :class:`~multigrad_amd.parallel.xgmi.CollectiveTimeout` on every
        rank if any peer-memory exchange of the engine's evaluations timed out (the two-shot
        reduce-scatter / all-gather of the ZeRO evaluations, the one-shot sumstats) -- their
        results were NaN-poisoned.  :meth:`device_call` does not sync, so the optimizers call
        this at the end of a run, next to their reducer's check."""
        self.e.check(where, collective=True)

    def device_call(self, x: torch.Tensor):
        """``(loss, grad)`` with the loss left on the device (1-element tensor), so the
        optimizer can fetch it together with its own reductions in one copy."""
        e, md = self.e, self.e.model
        self._nev = getattr(self, "_nev", 0) + 1
        if self._fault_now():
            # test hook: this rank skips the gradient exchange of one evaluation, so its
            # peers' bounded waits time out (the engine's error word, NaN-poisoned slices)
            return e.loss, e.g_loc if (e.zero and not e.owner) else e.grad
        self._load(x)
        e._forward_loss()
        if e.owner:
            md.engine_vjp_into(e.theta, e.h, e.grad, chunk=e.rank)
            a, b = e.own_range
            g = e.grad[a:b]
        elif e.zero and self.ts is not None:
            for c in range(e.C):
                md.engine_vjp_into(e.theta, e.h, e.grad, chunk=c)
                a, b = e.own[c]
                o, n = e.loc_off[c], e.loc_len[c]
                self.ts.reduce_scatter_(e.g_loc[o:o + n], a, n)
            g = e.g_loc
        elif e.zero:
            works = []
            for c in range(e.C):
                md.engine_vjp_into(e.theta, e.h, e.grad, chunk=c)
                a, L = e.pb[c], e.lengths[c]
                o, n = e.loc_off[c], e.loc_len[c]
                works.append(e.comm.reduce_scatter_tensor(e.g_loc[o:o + n], e.grad[a:a + L],
                                                          async_op=True))
            for w in works:
                w.wait()
            g = e.g_loc
        else:
            for c in range(e.C):
                md.engine_vjp_into(e.theta, e.h, e.grad, chunk=c if e.C > 1 else None)
            if e.size > 1:
                e.comm.all_reduce(e.grad)
            g = e.grad
        return e.loss, g

    def _fault_now(self) -> bool:
        """``MULTIGRAD_LBFGS_FAULT=<rank>:<evaluation>`` (tests): that rank skips the whole
        evaluation number ``evaluation`` (1-based) -- every exchange in it."""
        spec = os.environ.get("MULTIGRAD_LBFGS_FAULT")
        if not spec or self.e.size == 1:
            return False
        r, _, k = spec.partition(":")
        return int(r) == self.e.rank and int(k or 1) == self._nev

    def full(self, x: torch.Tensor) -> torch.Tensor:
        """The full parameter vector (model order) for the optimizer's vector x."""
        self._load(x)
        self.e.drain()
        if self.e.owner:
            return self.e.params().clone()
        return self.e.to_user(self.e.theta[:self.e.P]).clone()
