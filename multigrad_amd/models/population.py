"""Population SMF model: the 1e6-1e8 parameter "SMF-style summed-loss model".

BASELINE.json's headline configuration is a 1e7-parameter summed-loss model; the
reference only ships a 2-parameter SMF fit (tests/smf_example/smf_grad_descent.py).  Its
structure is kept: each halo belongs to one of J populations and every
population has its own ``(a_c, log10 sigma_c)`` pair, so P = 2J and

    S_k = scale_k sum_i [Phi((e_{k+1} - x_i - a_{c_i}) / sigma_{c_i}) - Phi((e_k - ...) / ...)]

with the reference's log-MSE loss (docs variant, ``+1e-10`` in the logs).  With halos
spread over every rank the gradient is dense, so each optimizer step needs a full
P-float gradient reduction -- the all-reduce-bandwidth workload of BASELINE configs 2-5.

Synthetic data are generated from a counter-based hash of the *global* halo index, so
every rank builds exactly its ``array_split`` shard of the same global data set (strong
scaling: the total data is independent of the number of GPUs), on its own GPU.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from ..ops.smf import (PopulationShard, SmfBins, logmse_loss, prepare_forward, smf_edge_weights_into,
                       smf_forward_into, smf_forward_slab, smf_slab_reduce, smf_sumstats,
                       smf_vjp_adam_into, smf_vjp_into)
from ..parallel.comm import get_world_comm
from .onepoint import OnePointModel

__all__ = ["PopulationSMFModel", "make_population_data", "hash_uniform", "owner_bounds",
           "owner_bounds_from_counts", "repartition_by_owner"]

_M1 = -7046029254386353131   # 0x9E3779B97F4A7C15 as int64
_M2 = -4658895280553007687   # 0xBF58476D1CE4E5B9
_M3 = -7723592293110705685   # 0x94D049BB133111EB


def _mix(i: torch.Tensor, seed: int) -> torch.Tensor:
    z = i * _M1 + (seed * 0x632BE59B + 0x1234567)
    z = (z ^ (z >> 30)) * _M2
    z = (z ^ (z >> 27)) * _M3
    return z ^ (z >> 31)


def hash_uniform(i: torch.Tensor, seed: int) -> torch.Tensor:
    """Deterministic U(0,1) (float64) from int64 indices (same bits on CPU and GPU)."""
    z = _mix(i, seed) & ((1 << 52) - 1)
    return (z.to(torch.float64) + 0.5) / float(1 << 52)


def _rank_range(n: int, rank: int, size: int):
    base, rem = divmod(n, size)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


_GEN_CHUNK = 1 << 24


def _global_pop(idx: torch.Tensor, seed: int, npop: int) -> torch.Tensor:
    return (_mix(idx, seed) & 0x7FFFFFFF) % npop


def owner_bounds(num_halos: int, npop: int, seed: int, size: int, device) -> list:
    """Population bounds ``Q[0..size]`` (even, so every owned parameter slice starts on a
    16-byte boundary) that split the global catalog into ``size`` contiguous population
    ranges of nearly equal halo counts -- ``np.array_split`` of the catalog sorted by
    population, moved to the nearest population boundary so that no population straddles
    two ranks.  Every rank derives the same bounds from the global counts (one pass over
    the counter-based hash, no communication)."""
    counts = torch.zeros(npop, dtype=torch.int64, device=device)
    for a in range(0, int(num_halos), _GEN_CHUNK):
        idx = torch.arange(a, min(int(num_halos), a + _GEN_CHUNK), dtype=torch.int64, device=device)
        counts += torch.bincount(_global_pop(idx, seed, npop), minlength=npop)
    return owner_bounds_from_counts(counts, size)


def owner_bounds_from_counts(counts: torch.Tensor, size: int) -> list:
    """:func:`owner_bounds` from the global per-population halo counts ``[J]`` (any device):
    ``size`` contiguous, even-aligned population ranges of nearly equal halo counts."""
    npop = int(counts.numel())
    cum = torch.cumsum(counts.to(torch.int64), 0).cpu().numpy()
    total = int(cum[-1]) if npop else 0
    bounds = [0]
    for r in range(1, size):
        target = r * total / size
        q = int(np.searchsorted(cum, target, side="left")) + 1   # first pop after the split
        q = min(max(q - (q & 1), bounds[-1]), npop)
        bounds.append(q)
    bounds.append(npop)
    return bounds


def repartition_by_owner(data: dict, comm=None, layout: str = "lanes",
                         lane_order: str = "global") -> dict:
    """Re-partition a data-parallel population shard by parameter owner, in place.

    ``data`` is any rank's shard of the population model (:func:`make_population_data`
    with ``placement="hashed"``, or a user's ``np.array_split`` of a catalog -- reference
    tests/smf_example/smf_grad_descent.py:28).  Collective over ``comm``:

    1. the per-population halo counts are summed across ranks (one all-reduce of ``J``
       int64) and cut into ``W`` contiguous population ranges of nearly equal halo counts
       (:func:`owner_bounds_from_counts`, the rule of the ``"owner"`` placement);
    2. the shard is already sorted by population, so the halos bound for rank ``d`` are one
       contiguous run: ONE all-to-all-v of ``(log mass, population)`` rows
       (:meth:`Comm.all_to_all_v`: xGMI peer pulls, RCCL or gloo) moves every halo to the
       rank that owns its population;
    3. the received rows (source ranks in order, each sorted by population and, within a
       population, in the source's order) are rebuilt into a shard in ``layout``.

    A halo's order inside its population is its order in the concatenation of the source
    shards, so an ``array_split`` of a catalog gives exactly the shard the ``"owner"``
    placement generates.  Afterwards every rank's gradient is complete on its own
    populations and zero elsewhere: the fused engine's owner mode drops the P-float gradient
    all-reduce (reference multigrad/multigrad.py:531-532) and keeps only the sumstat
    all-reduce.  Returns ``data`` (``shard``, ``placement="owner"``, ``owner_units`` and
    ``repartition`` -- timing and row counts -- replaced)."""
    import time
    comm = get_world_comm() if comm is None else comm
    t0 = time.perf_counter()
    sh: PopulationShard = data["shard"]
    if sh.pop is None:
        raise ValueError("repartition_by_owner needs a population shard (pop ids)")
    dev = sh.device
    npop = sh.npop
    gcounts = sh.counts.to(dev, torch.int64)
    if comm.size > 1:
        comm.all_reduce(gcounts)
    bounds = owner_bounds_from_counts(gcounts, comm.size)
    off = sh.offsets                                   # local cumsum of counts (host)
    send_counts = [int(off[bounds[d + 1]] - off[bounds[d]]) for d in range(comm.size)]
    rows = torch.stack([sh.x.reshape(-1).view(torch.int32), sh.pop.reshape(-1).to(torch.int32)], 1)
    n_before = int(rows.shape[0])
    from ..utils.trace import trace
    trace(f"repartition: owner bounds done, all-to-all-v of {n_before} rows")
    recv, recv_counts = comm.all_to_all_v(rows, send_counts)
    trace("repartition: all-to-all-v done, building the owner shard")
    del rows
    t_x = time.perf_counter() - t0
    x = recv[:, 0].contiguous().view(torch.float32)
    pop = recv[:, 1].contiguous()
    del recv
    chunks = 1
    new = PopulationShard(x, pop, npop, device=dev, chunks=chunks, layout=layout, comm=comm,
                          lane_order=lane_order)
    del x, pop
    data["shard"] = new
    data["placement"] = "owner"
    data["owner_units"] = bounds
    data["repartition"] = {"halos_before": n_before, "halos_after": int(new.n),
                           "sent_to": send_counts, "received_from": list(recv_counts),
                           "exchange_s": round(t_x, 4),
                           "total_s": round(time.perf_counter() - t0, 4)}
    return data


def make_population_data(num_params: int = 10_000_000, num_halos: int = 1 << 27, seed: int = 0,
                         comm=None, device=None, nbins: int = 10, chunks: int = 1,
                         truth_offset=(0.1, 0.1), tail: str = "absolute",
                         layout: str = "auto", placement: str = "hashed",
                         lane_order: Optional[str] = None, narrow_frac: float = 0.0,
                         narrow_log_sigma: float = -1.1,
                         narrow_guess_log_sigma: Optional[float] = None) -> dict:
    """This rank's shard of the synthetic population-SMF data set.

    The global catalog (halo i: population ``hash(i) mod J``, log mass from a second hash)
    is the same for every placement and every number of ranks; ``placement`` only decides
    which rank holds which halo:

    ``"hashed"``: rank r holds the r-th contiguous block of halo indices (the reference's
        ``np.array_split`` of an unsorted catalog).  Every rank touches every population,
        so the gradient is dense on every rank and must be summed across ranks.
    ``"owner"``: the catalog is split by population (:func:`owner_bounds`), as
        ``np.array_split`` of a catalog sorted by population / host halo would (the
        reference's diffdesi tree utilities sort by host, reference
        multigrad/diffdesi_experimental/util.py:20-35).  Each rank's gradient is then
        non-zero only on its own populations and the engine skips the gradient collective
        (``data["owner_units"]``, see :class:`~multigrad_amd.engine.fused.FusedAdamEngine`).

    ``layout`` (device layout of the shard, :class:`~multigrad_amd.ops.smf.PopulationShard`)
    and ``lane_order``: ``"auto"`` picks the lanes layout (one lane per population, slots
    in the global order, per-population VJP residuals) for a single rank and the owner
    placement, where a rank holds every halo of its populations (~27 per population at
    the headline size); and ``"tiles"`` (halo-parallel forward, segmented recomputing VJP)
    for hashed shards on several ranks, where a rank holds only ~27/W halos per population:
    there the residuals cost more HBM traffic than recomputing the few halos, and lanes
    spend most of their time on per-group overhead.  Measured per-rank proxies at 1/8 of
    the halos (profiles/hashed_proxy.md): tiles 94 + 63 us (forward + VJP), lanes with
    the local slot order and the recomputing VJP (``lane_order="local"``) 120 + 136 us,
    lanes global order with residuals 140 + 146 us.

    ``narrow_frac``: the fraction of populations (chosen by a hash of the population id, so
    scattered over the catalog) whose true log10 sigma is ``narrow_log_sigma`` (default
    -1.1: sigma = 0.079 dex, a bin width of 1.26 sigma at the truth and 1.0 sigma at the
    default guess), outside the Euler-Maclaurin forward's range of 0.5 sigma; these
    populations take the per-edge path (profiles/narrow_sweep/).  ``narrow_guess_log_sigma``:
    the starting log10 sigma of those populations (default: truth + offset, as the others);
    a wide start (e.g. -0.6, inside the Euler-Maclaurin range) makes a fit move them across
    the limit while it runs (the engine's re-layout, engine/fused.py).

    Returns a dict with the sorted device shard (``shard``), bins, volume, true
    parameters ``truth`` (interleaved, device) and a starting ``guess``; the target SMF is
    filled in by :meth:`PopulationSMFModel.set_target_from_truth`.
    """
    comm = get_world_comm() if comm is None else comm
    assert num_params % 2 == 0, "parameters come in (a, log_sigma) pairs"
    if placement not in ("hashed", "owner"):
        raise ValueError("placement must be 'hashed' or 'owner'")
    if layout == "auto":
        layout = "tiles" if placement == "hashed" and comm.size > 1 else "lanes"
    if lane_order is None:
        lane_order = "global"
    npop = num_params // 2
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
            else torch.device("cpu")
    owner_units = None
    if placement == "owner":
        owner_units = owner_bounds(num_halos, npop, seed, comm.size, device)
        lo, hi = owner_units[comm.rank], owner_units[comm.rank + 1]
        parts = []
        for a in range(0, int(num_halos), _GEN_CHUNK):
            idx = torch.arange(a, min(int(num_halos), a + _GEN_CHUNK), dtype=torch.int64,
                               device=device)
            pp = _global_pop(idx, seed, npop)
            parts.append(idx[(pp >= lo) & (pp < hi)])
            del idx, pp
        idx = torch.cat(parts) if parts else torch.zeros(0, dtype=torch.int64, device=device)
        del parts
    else:
        start, end = _rank_range(int(num_halos), comm.rank, comm.size)
        idx = torch.arange(start, end, dtype=torch.int64, device=device)
    pop = _global_pop(idx, seed, npop)
    q = 0.9 * hash_uniform(idx, seed + 1)
    logm = (10.0 - torch.log10(1.0 - q)).to(torch.float32)          # log10(1e10/(1-q))
    del idx, q
    shard = PopulationShard(logm, pop.to(torch.int32), npop, device=device, chunks=chunks,
                            layout=layout, comm=comm, lane_order=lane_order)
    del logm, pop
    cidx = torch.arange(npop, dtype=torch.int64, device=device)
    truth = torch.empty(2 * npop, dtype=torch.float32, device=device)
    truth[0::2] = (-2.0 + 0.2 * (hash_uniform(cidx, seed + 2) - 0.5)).to(torch.float32)
    truth[1::2] = (-0.5 + 0.2 * (hash_uniform(cidx, seed + 3) - 0.5)).to(torch.float32)
    narrow = None
    if narrow_frac > 0:
        narrow = hash_uniform(cidx, seed + 4) < float(narrow_frac)
        truth[1::2] = torch.where(narrow, torch.full_like(truth[1::2], float(narrow_log_sigma)),
                                  truth[1::2])
    guess = truth.clone()
    guess[0::2] += truth_offset[0]
    guess[1::2] += truth_offset[1]
    if narrow is not None and narrow_guess_log_sigma is not None:
        guess[1::2] = torch.where(narrow, torch.full_like(guess[1::2], float(narrow_guess_log_sigma)),
                                  guess[1::2])
    edges = np.linspace(8.5, 9.5, nbins + 1)
    # volume normalises the SMF to O(1e-2) per bin like the reference's tests
    volume = 10.0 * num_halos
    return dict(shard=shard, bins=SmfBins.make(edges, volume, tail), volume=volume, truth=truth,
                guess=guess, npop=npop, num_halos=int(num_halos), target_sumstats=None,
                loss_eps=1e-10, placement=placement, owner_units=owner_units)


@dataclass(eq=False)
class PopulationSMFModel(OnePointModel):
    """SMF-style summed-loss model with one ``(a, log10 sigma)`` pair per population.

    ``aux_data`` comes from :func:`make_population_data`.  The hooks are differentiable
    (custom autograd function over the HIP kernels), so every generic multigrad path
    works; :meth:`fused_engine` additionally exposes the device protocol used by the
    graph-captured fused Adam engine.
    """

    aux_data: dict = None

    # the hooks ignore randkey (a deterministic model), so a keyed run_adam gives the
    # keyless trajectory and may use the fused engine
    engine_randkey_invariant = True

    @property
    def shard(self) -> PopulationShard:
        return self.aux_data["shard"]

    @property
    def bins(self) -> SmfBins:
        return self.aux_data["bins"]

    @property
    def nparams(self) -> int:
        return 2 * self.aux_data["npop"]

    def param_device(self) -> torch.device:
        return self.shard.device

    def calc_partial_sumstats_from_params(self, params, randkey=None):
        return smf_sumstats(torch.as_tensor(params).reshape(-1), self.shard, self.bins, True)

    def calc_loss_from_sumstats(self, sumstats, sumstats_aux=None, randkey=None):
        t = self.aux_data["target_sumstats"]
        return logmse_loss(sumstats, t.to(sumstats.device, sumstats.dtype), self.aux_data["loss_eps"])

    def set_target_from_truth(self):
        """Target SMF = total sumstats at the true parameters (all ranks)."""
        self.aux_data["target_sumstats"] = torch.ones(self.bins.nb, device=self.param_device())
        S = self.calc_sumstats_from_params(self.aux_data["truth"])
        self.aux_data["target_sumstats"] = S.to(torch.float32)
        return S

    # ------------------------------------------------------------ fused-engine protocol
    # (see multigrad_amd.engine.fused): parameters are grouped in "units" of 2 (one
    # population); the engine chooses unit-aligned chunk boundaries.
    def fused_engine(self, cache: bool = True, **kw):
        """The model's fused Adam engine.  Cached per model and keyword set (``cache``): a
        repeated ``run_adam`` / ``run_bfgs`` re-uses its buffers, layout, autotune verdict
        and -- with unchanged buffers and scalars -- its captured graphs (engine/fused.py
        ``stats``), the analogue of the jit cache the reference's benchmark warms once
        (tests/smf_example/benchmark.py:41-46).  Replacing ``aux_data`` entries (a new
        shard) or closing the engine drops it."""
        from ..engine.fused import FusedAdamEngine
        if not cache:
            return FusedAdamEngine(self, **kw)
        comm = kw.get("comm", None)
        sid = id(self.aux_data.get("shard"))
        key = (tuple(sorted((k, repr(v)) for k, v in kw.items())), sid,
               id(self.comm if comm is None else comm))
        store = self.__dict__.setdefault("_engine_cache", {})
        # engines of a replaced shard are dropped (each holds its shard, its layout and
        # O(params) device buffers; a cached engine keeps its shard alive, so a shard id in
        # the key cannot be reused by new data while the entry exists)
        for k in [k for k in store if k[1] != sid]:
            del store[k]
        eng = store.get(key)
        if eng is None or getattr(eng, "closed", False):
            eng = FusedAdamEngine(self, **kw)
            eng.cached = True
            eng._cache_shard = self.aux_data.get("shard")  # pins the id in the key
            store[key] = eng
        return eng

    def engine_chunks_current(self, unit_bounds) -> bool:
        """Whether the shard is already cut at ``unit_bounds`` (the engine then keeps the
        layout instead of rebuilding it, when the lane classes did not change either)."""
        return list(getattr(self.shard, "chunk_pops", [])) == [int(u) for u in unit_bounds]

    def engine_layout_epoch(self):
        """Changes whenever the device layout is rebuilt (part of the engine's graph key)."""
        sh = self.shard
        return (id(sh), getattr(sh, "layout_version", 0))

    def engine_units(self):
        """(number of parameter units, parameters per unit)."""
        return self.aux_data["npop"], 2

    def engine_set_chunks(self, unit_bounds):
        self.shard.set_chunks(unit_bounds)

    def lane_fallback_groups(self, params) -> tuple:
        """``(groups on the per-edge path, groups)`` of the lanes forward at ``params``
        (user order): a group leaves the Euler-Maclaurin path when any of its lanes has a bin
        width above 0.5 sigma.  (0, 0) for other layouts."""
        sh = self.shard
        d = self.bins.delta
        if sh.layout != "lanes" or sh.device.type != "cuda" or d <= 0:
            return 0, 0
        s = torch.as_tensor(params, device=sh.device).reshape(-1)[1::2].float()
        narrow = (s < math.log10(2.0 * d)).to(torch.int32)
        sp = sh.slot_pop.long()
        per_slot = torch.where(sp >= 0, narrow[sp.clamp(min=0)], torch.zeros_like(narrow[:1]))
        g = per_slot.reshape(-1, 64).amax(1)
        return int(g.sum()), int(g.numel())

    def engine_layout_hint(self, guess, band: float = 0.0) -> bool:
        """Group the lanes by forward path at ``guess`` (user-order parameters; called by the
        fused engine before :meth:`engine_set_chunks`, at setup and when it re-lays the lanes
        out during a fit): populations whose bin width exceeds the Euler-Maclaurin range
        (h = delta / sigma > 0.5, csrc/smf.hip kEmHMax) get lane groups of their own, so a
        few narrow populations do not send whole groups to the per-edge path.  Returns
        whether the classes changed.  ``MULTIGRAD_LANE_CLASSES=0`` turns it off."""
        sh = self.shard
        if not self._lane_classes_apply():
            return False
        d = self.bins.delta
        g = torch.as_tensor(guess).reshape(-1)
        s = g[1::2].detach()
        s = s.to(torch.float64) if s.is_cuda else s.to("cpu", torch.float64)
        # h = delta / 10^s > 0.5  <=>  s < log10(2 delta); ``band`` (re-layouts during a fit)
        # also groups the populations within band dex above the limit with the narrow ones,
        # so a fit that moves them across it a little later needs no second re-layout
        return sh.set_lane_classes((s < math.log10(2.0 * d) + band).to(torch.int64))

    def _lane_classes_apply(self) -> bool:
        sh = self.shard
        return (sh.layout == "lanes" and os.environ.get("MULTIGRAD_LANE_CLASSES", "1") != "0"
                and self.bins.delta > 0 and not self.bins.rel_tail)

    def engine_relayout_probe(self, theta, chunk=None):
        """Device scalar (no host sync): the share of the lane groups of ``chunk`` that the
        forward at ``theta`` (engine internal order) sends down the per-edge path -- groups
        with any lane outside the Euler-Maclaurin range.  The engine compares it with
        :meth:`engine_layout_share` (the share the current lane classes were laid out for)
        and re-lays the lanes out when a fit has moved populations across the limit.  None
        when classes do not apply."""
        sh = self.shard
        if not self._lane_classes_apply() or sh.device.type != "cuda":
            return None
        g0, g1 = sh.group_range(chunk)
        if g1 <= g0:
            return torch.zeros((), device=theta.device)
        sp = sh.slot_pidx[64 * g0:64 * g1].long()
        s = theta.reshape(-1)[1:2 * self.aux_data["npop"]:2]
        narrow = (sp >= 0) & (s[sp.clamp(min=0)] < math.log10(2.0 * self.bins.delta))
        return narrow.view(-1, 64).any(1).float().mean()

    def engine_layout_share(self, chunk=None) -> float:
        """The per-edge group share the current lane classes imply (host)."""
        return self.shard.per_edge_share(chunk)

    def engine_repartition(self) -> Optional[dict]:
        """Fused-engine hook (collective): a data-parallel shard on several ranks is moved
        to the parameter owners (:func:`repartition_by_owner`: one all-to-all-v), so the
        engine runs in owner mode.  Returns the re-partition record, or None when there is
        nothing to do (one rank, data already placed by owner)."""
        d = self.aux_data
        if self.comm is None or self.comm.size == 1 or d.get("placement") == "owner" \
                or self.shard.pop is None:
            return None
        old = id(d.get("shard"))
        repartition_by_owner(d, self.comm)
        # the engines cached for the data-parallel shard now run on the owner shard: re-key
        # them, so the next run_* call finds the same engine (fused_engine drops entries of
        # any other shard)
        store = self.__dict__.get("_engine_cache", {})
        for k in [k for k in store if k[1] == old]:
            eng = store.pop(k)
            eng._cache_shard = d["shard"]
            store[(k[0], id(d["shard"]), k[2])] = eng
        return d["repartition"]

    def engine_owner_units(self):
        """Population (unit) bounds ``[W+1]`` of the owner placement, or None."""
        return self.aux_data.get("owner_units")

    def engine_support_units(self):
        """``(lo, hi)``: the populations this rank's data touches lie in ``[lo, hi)``
        (``(0, 0)`` for an empty shard)."""
        nz = torch.nonzero(self.shard.counts > 0).reshape(-1)
        if nz.numel() == 0:
            return 0, 0
        return int(nz[0]), int(nz[-1]) + 1

    def engine_param_perm(self):
        """Internal unit order of the engine vectors (lanes layout with the global slot
        order: populations in slot order, so parameter reads and gradient writes are
        coalesced), or None (population order)."""
        return self.shard.perm if self._engine_order() == "internal" else None

    def _engine_order(self) -> str:
        sh = self.shard
        return "internal" if sh.layout == "lanes" and sh.lane_order == "global" else "user"

    def engine_nS(self) -> int:
        return self.bins.nbp

    def engine_fwd_rows(self, chunk=None) -> int:
        if self.shard.device.type != "cuda":
            return 1
        h0, h1 = self.shard.halo_range(chunk)
        return self.shard.fwd_rows(max(h1 - h0, 1), self.bins.nb, True, self.bins.rel_tail,
                                   chunk, resid=True)

    def engine_forward_chunk(self, theta, slab, chunk=None, epilogue=None, exchange=None) -> int:
        # the engine always runs the VJP of a chunk after this forward at the same theta,
        # so the forward stores the VJP residuals (lanes layout) -- unless the VJP
        # recomputes (local slot order: few halos per population)
        return smf_forward_slab(theta, self.shard, self.bins, True, slab, chunk,
                                resid=not self.shard.vjp_recompute, order=self._engine_order(),
                                epilogue=self._epilogue_spec(epilogue), exchange=exchange)

    def engine_fused_exchange_ok(self) -> bool:
        """The forward / VJP launches can carry a packed two-shot exchange in their first
        workgroups (``exchange=``): the tiles layout of the hashed placement."""
        return self.shard.device.type == "cuda" and self.shard.layout == "tiles"

    def engine_forward_epilogue_ok(self) -> bool:
        """The sumstat epilogue can ride on the last forward launch sequence of a step
        (lanes layout on a GPU): ``engine_forward_*chunk(..., epilogue=...)``."""
        return self.shard.device.type == "cuda" and self.shard.layout == "lanes" and \
            not self.shard.vjp_recompute

    def _epilogue_spec(self, e):
        if e is None:
            return None
        return dict(e, target=self.aux_data["target_sumstats"],
                    eps=float(self.aux_data["loss_eps"]))

    def engine_prepare(self, chunks):
        """Host-side schedule construction for the given chunks (called by the engine
        before it captures a step into a HIP graph)."""
        for c in chunks:
            prepare_forward(self.shard, self.bins, True, c)

    def engine_pipeline_ok(self, chunk=None, bounded: bool = False) -> bool:
        """Whether :meth:`engine_forward_chunk` can also apply the previous step's VJP and
        Adam update (lanes layout on the GPU, internal order, no split populations);
        ``bounded``: the bounded form (box-constrained Adam in u-space), which needs the
        Euler-Maclaurin / per-edge residual forward (uniform bins, absolute tails)."""
        sh = self.shard
        if sh.device.type != "cuda" or self._engine_order() != "internal":
            return False
        if bounded and (self.bins.rel_tail or self.bins.delta <= 0):
            return False
        k0, k1 = (0, sh.giant.shape[0]) if chunk is None else \
            (sh.chunk_giant[chunk], sh.chunk_giant[chunk + 1])
        return k1 == k0

    def engine_forward_update_chunk(self, theta, slab, chunk, update: dict, epilogue=None) -> int:
        """Forward of ``chunk`` that first applies the pending VJP + Adam of the previous
        step per population (``update``: h, m, v, unit_offset, step, host_step, lr, b1, b2,
        eps, traj, traj_stride) -- one pass instead of a VJP kernel plus a forward."""
        return smf_forward_slab(theta, self.shard, self.bins, True, slab, chunk, resid=True,
                                order=self._engine_order(), update=update,
                                epilogue=self._epilogue_spec(epilogue))

    def engine_reduce(self, slab, nrows, S):
        return smf_slab_reduce(slab, nrows, self.bins, S)

    def engine_loss_into(self, S_total, loss_out, h_out):
        t = self.aux_data["target_sumstats"]
        eps = float(self.aux_data["loss_eps"])
        if S_total.device.type != "cuda":
            s = S_total[:self.bins.nb].detach().double().clone().requires_grad_(True)
            with torch.enable_grad():
                loss = logmse_loss(s, t.double(), eps)
                (g,) = torch.autograd.grad(loss, s)
            loss_out[0] = loss.detach().to(loss_out.dtype)
            smf_edge_weights_into(g.float(), self.bins, h_out)
            return
        from ..ops._ext import ext
        if getattr(self, "_empty", None) is None or self._empty.device != S_total.device:
            self._empty = torch.empty(0, device=S_total.device)
        ext().smf_logmse(S_total, t, eps, list(self.bins.edges), list(self.bins.scale),
                         loss_out, self._empty, h_out)

    def engine_reduce_loss_into(self, slab, nrows, S, loss_out, h_out, oneshot=None,
                                advance=None) -> bool:
        """Fused epilogue: slab reduction, (with ``oneshot``: the cross-rank sum through
        the one-shot peer exchange) and loss + edge weights in one launch.  False where it
        does not apply (CPU), the engine then runs reduce / all-reduce / loss separately.
        ``advance``: an int32 device counter the launch increments (the pipelined engine's
        step counter)."""
        if slab.device.type != "cuda":
            return False
        from ..ops._ext import ext
        t = self.aux_data["target_sumstats"]
        if oneshot is None:
            ext().smf_epilogue(slab, int(nrows), list(self.bins.edges), list(self.bins.scale), t,
                               float(self.aux_data["loss_eps"]), S, loss_out, h_out, [], 0,
                               None, None, 5.0, advance)
        else:
            ext().smf_epilogue(slab, int(nrows), list(self.bins.edges), list(self.bins.scale), t,
                               float(self.aux_data["loss_eps"]), S, loss_out, h_out,
                               oneshot.peers, oneshot.rank, oneshot.seq, oneshot.err,
                               oneshot.timeout_s, advance)
        return True

    def engine_vjp_into(self, theta, h, grad, chunk=None, exchange=None):
        return smf_vjp_into(theta, self.shard, self.bins, True, h, grad, chunk=chunk,
                            residuals_ready=True, order=self._engine_order(),
                            recompute=self.shard.vjp_recompute, exchange=exchange)

    def engine_vjp_adam_into(self, theta, h, m, v, unit_offset, step, host_step, lr, b1, b2,
                             eps, traj_base=None, traj_stride=0, chunk=None) -> bool:
        """Optional fused VJP + (unbounded) Adam; False where it does not apply."""
        if self._engine_order() != "internal":
            return False
        return smf_vjp_adam_into(theta, self.shard, self.bins, True, h, m, v, unit_offset,
                                 step, host_step, lr, b1, b2, eps, traj_base, traj_stride, chunk)

    # simple (unchunked) protocol helpers
    def engine_partial_into(self, theta, out, slab=None, chunk=None):
        return smf_forward_into(theta, self.shard, self.bins, True, out, slab=slab, chunk=chunk,
                                order=self._engine_order())
