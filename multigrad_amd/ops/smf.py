"""SMF summed-statistic ops: HIP forward/VJP kernels + fp32/fp64 PyTorch references.

Device tensors run ``csrc/smf.hip`` (one pass over the halos for all bins, deterministic
reductions, segmented per-population VJP).  CPU tensors use the PyTorch formulation
below, which is also the numerics oracle for the kernel tests.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from ._ext import ext
from ..utils.trace import trace

__all__ = ["SmfBins", "PopulationShard", "smf_sumstats", "smf_sumstats_reference",
           "logmse_loss", "normal_cdf", "TILE_HALOS", "TILE_POPS"]

TILE_HALOS = 2048
TILE_POPS = 2048
FWD_BLOCKS_MAX = 2048  # 8 workgroups per CU on 256 CUs, grid-stride beyond
LANE_WINDOW = 4096     # lanes layout: populations sorted by size within windows of this many
LANE_LMAX = 4096       # lanes layout: populations with more halos are split into parts
LPT_OVERHEAD = float(os.environ.get("MULTIGRAD_LPT_OVERHEAD", "3"))  # per-group cost, halo rows


@dataclass(frozen=True)
class SmfBins:
    """Bin edges and per-bin scale ``1/(volume*width)`` of a stellar-mass function.

    ``tail`` selects the accuracy contract of the HIP forward's normal-CDF evaluation:
    ``"absolute"`` (default): every edge CDF to 1.1e-7 absolute -- the accuracy of the
    float32 ``erf`` the reference evaluates (tests/smf_example/smf_grad_descent.py:32-48);
    ``"relative"``: every CDF tail to ~1.2e-6 *relative*, so bins fed only by the far
    Gaussian tails of halos keep ~6 significant digits (the reference's float32 erf
    difference loses them all); ~12% slower forward.
    """

    edges: tuple
    scale: tuple
    tail: str = "absolute"

    @staticmethod
    def make(edges, volume: float, tail: str = "absolute") -> "SmfBins":
        if tail not in ("relative", "absolute"):
            raise ValueError("tail must be 'relative' or 'absolute'")
        e = np.asarray(torch.as_tensor(edges).detach().cpu().double().numpy() if
                       isinstance(edges, torch.Tensor) else edges, dtype=np.float64)
        w = np.diff(e)
        return SmfBins(tuple(float(v) for v in e), tuple(float(1.0 / (volume * d)) for d in w),
                       tail)

    @property
    def rel_tail(self) -> bool:
        return self.tail == "relative"

    @property
    def delta(self) -> float:
        """Edge spacing when the edges are uniformly spaced (the Euler-Maclaurin forward's
        condition, csrc/smf.hip make_bins), else 0."""
        e = np.asarray(self.edges, dtype=np.float64)
        d = (e[-1] - e[0]) / max(len(e) - 1, 1)
        ok = d > 0 and np.all(np.abs(e - (e[0] + d * np.arange(len(e)))) <=
                              1e-6 * np.maximum(1.0, np.abs(e)))
        return float(d) if ok else 0.0

    @property
    def nb(self) -> int:
        return len(self.scale)

    @property
    def nbp(self) -> int:
        for s in (1, 2, 4, 8, 10, 16, 32):
            if self.nb <= s:
                return s
        raise ValueError("at most 32 bins supported by the HIP kernels")


def normal_cdf(z: torch.Tensor) -> torch.Tensor:
    return torch.special.ndtr(z)


def smf_sumstats_reference(theta: torch.Tensor, x: torch.Tensor, pop: Optional[torch.Tensor],
                           bins: SmfBins, log_sigma: bool) -> torch.Tensor:
    """Differentiable PyTorch SMF (any dtype/device): S_k = scale_k sum_i dPhi_ik."""
    th = theta.reshape(-1, 2)
    a = th[:, 0]
    s = th[:, 1]
    if pop is None:
        a_i, s_i = a[0], s[0]
    else:
        idx = pop.long()
        a_i, s_i = a[idx], s[idx]
    sigma = torch.pow(torch.as_tensor(10.0, dtype=theta.dtype, device=theta.device), s_i) \
        if log_sigma else s_i
    mu = x.to(theta.dtype) + a_i
    edges = torch.as_tensor(bins.edges, dtype=theta.dtype, device=theta.device)
    scale = torch.as_tensor(bins.scale, dtype=theta.dtype, device=theta.device)
    if sigma.dim() == 0:
        z = (edges[None, :] - mu[:, None]) / sigma
    else:
        z = (edges[None, :] - mu[:, None]) / sigma[:, None]
    cdf = normal_cdf(z)
    mass = (cdf[:, 1:] - cdf[:, :-1]).sum(0)
    return mass * scale


def logmse_loss(sumstats: torch.Tensor, target: torch.Tensor, eps: float = 0.0) -> torch.Tensor:
    """Reduced chi^2 with unit errors in log10 space (reference smf_grad_descent.py:78-82)."""
    return torch.mean((torch.log10(sumstats + eps) - torch.log10(target + eps)) ** 2)


class PopulationShard:
    """This rank's data shard sorted by population, with the device tile schedule.

    Parameters
    ----------
    x : (N,) float tensor of log halo masses (any order)
    pop : (N,) int tensor of population ids in ``[0, npop)``, or None for a single
        shared-parameter population (the reference's 2-parameter models)
    npop : number of populations (parameters = 2 * npop)
    device : device for the kernels
    chunks : number of contiguous population chunks (tiles never straddle a chunk, so
        per-chunk VJPs can overlap per-chunk gradient collectives)
    layout : device layout of a population shard on the GPU.
        ``"lanes"`` (default with populations): one wavefront lane per population slot,
        halos interleaved per 64-slot group (runtime.cpp:build_lanes); the forward keeps
        per-population residuals and the VJP is a memory-bound pass over them.
        ``"tiles"``: halos sorted by population, segmented-scan VJP over a tile schedule
        that recomputes every halo (no residual memory).  Shared-parameter shards
        (``pop=None``) always use the plain halo array.
    lane_order : lanes layout, how populations are grouped into 64-slot groups (sorted by
        size within windows): ``"global"`` (default) by the cross-rank counts, so every
        rank of a data-parallel job derives the same slot order and the engine can keep
        its vectors in that internal order; ``"local"`` by this rank's own counts, so the
        lanes of a group have nearly equal local lengths even when the rank holds only a
        few halos of each population (hashed shards) -- vectors then stay in population
        order and the VJP recomputes the halos instead of keeping residuals.
    """

    def __init__(self, x, pop=None, npop: int = 1, device=None, chunks: int = 1,
                 tile_halos: int = TILE_HALOS, tile_pops: int = TILE_POPS,
                 layout: str = "lanes", lane_window: int = LANE_WINDOW,
                 lane_lmax: int = LANE_LMAX, comm=None, lane_order: str = "global"):
        x = torch.as_tensor(x)
        device = torch.device(device) if device is not None else x.device
        self.device = device
        if layout not in ("lanes", "tiles"):
            raise ValueError("layout must be 'lanes' or 'tiles'")
        # lanes on the CPU builds the schedule and the internal parameter order only (the
        # math runs through the PyTorch reference), which is how the engine's internal
        # ordering is exercised by the multi-rank CPU tests
        self.layout = layout if pop is not None else "tiles"
        self._comm = comm
        if lane_order not in ("global", "local"):
            raise ValueError("lane_order must be 'global' or 'local'")
        self.lane_order = lane_order
        self._lane_window, self._lane_lmax = int(lane_window), int(lane_lmax)
        self.resid = None          # lanes: [ngroups, 2 (nbp+1), 64] residuals of the last forward
        self.resid_epoch = 0       # bumped by every residual-writing forward
        self.npop = int(npop)
        self.n = int(x.numel())
        if pop is None:
            assert self.npop == 1
            xs = x.reshape(-1).to(device=device, dtype=torch.float32).contiguous()
            counts = torch.tensor([self.n], dtype=torch.int64)
            self.pop = None
        else:
            pop = torch.as_tensor(pop).reshape(-1)
            trace(f"shard: sort {pop.numel()} halos into {self.npop} populations")
            if pop.device.type == "cuda":
                # device radix sort + histogram; only the J counts come back to the host
                spop, order, counts = stable_population_sort(pop.to(torch.int32), self.npop)
                counts = counts.cpu().to(torch.int64)
                xs = x.reshape(-1).to(pop.device)[order].to(device=device, dtype=torch.float32)
                self.pop = spop.to(device).contiguous()
                del order
            else:
                pop_cpu = pop.to("cpu", torch.int32).contiguous()
                order, counts = _sort_by_population(pop_cpu, self.npop)
                xs = x.reshape(-1)[order.to(x.device)].to(device=device, dtype=torch.float32)
                self.pop = pop_cpu[order].to(device).contiguous()
            xs = xs.contiguous()
        self.x = xs
        self.counts = counts
        # the lanes population order must be identical on every rank of a data-parallel
        # job: it is decided by the cross-rank sums of the counts
        self.order_counts = None
        self.lane_class = None  # optional per-population class that groups lanes first
        if self.layout == "lanes" and lane_order == "global" and comm is not None and comm.size > 1:
            trace("shard: all-reduce of the population counts (global lane order)")
            oc = counts.clone().to(torch.int64)
            comm.all_reduce(oc)
            self.order_counts = oc
        trace("shard: counts ready")
        self.offsets = torch.zeros(self.npop + 1, dtype=torch.int64)
        self.offsets[1:] = torch.cumsum(counts, 0)
        self._tile_halos, self._tile_pops = tile_halos, tile_pops
        bounds = np.linspace(0, self.npop, max(1, min(int(chunks), self.npop)) + 1).round()
        self.set_chunks([int(b) for b in bounds])

    def set_chunks(self, pop_bounds) -> None:
        """(Re)cut the shard into contiguous population chunks ``[b_c, b_{c+1})`` and
        rebuild the tile schedule so that no tile straddles a chunk boundary."""
        pb = [int(b) for b in pop_bounds]
        assert pb[0] == 0 and pb[-1] == self.npop and all(a <= b for a, b in zip(pb, pb[1:]))
        # bumped by every (re)build: engines key their captured graphs on it
        self.layout_version = getattr(self, "layout_version", 0) + 1
        self.nchunks = len(pb) - 1
        self.chunk_pops = pb
        self.chunk_halos = [int(self.offsets[b]) for b in pb]
        if self.layout == "lanes":
            self._build_lanes(pb)
            return
        if self.device.type != "cuda":
            self.tiles = torch.zeros((0, 4), dtype=torch.int64)
            self.giant = torch.zeros((0, 3), dtype=torch.int32)
            self.chunk_tiles = [0] * (self.nchunks + 1)
            self.chunk_giant = [0] * (self.nchunks + 1)
            self.nslots = 0
            self.partials = torch.zeros(2, dtype=torch.float32)
            return
        tiles, giant, ct, cg, nslots = _build_tiles(self.counts, pb[1:-1], self._tile_halos,
                                                    self._tile_pops)
        self.tiles = tiles.to(self.device)
        self.giant = giant.to(self.device)
        self.chunk_tiles = [int(v) for v in ct]
        self.chunk_giant = [int(v) for v in cg]
        self.nslots = int(nslots)
        self.partials = torch.zeros(max(self.nslots, 1) * 2, dtype=torch.float32,
                                    device=self.device)

    def set_lane_classes(self, cls: Optional[torch.Tensor]) -> bool:
        """Per-population class (int, [npop], CPU or on the shard's device) that orders the
        slots of a lanes window before the halo count: populations of one class share 64-lane
        groups.  The Euler-Maclaurin forward takes a group's fast path only when every lane's
        bin width is inside its range, so the narrow populations of a fit (bin width > 0.5
        sigma) are kept out of the other groups -- at 1% narrow populations in random
        places, 47% of the groups would otherwise hold one.  Takes effect at the next
        :meth:`set_chunks`; the class must be the same on every rank.  Returns whether it
        changed.  Kept on the shard's device when given there (the engine's re-layout
        computes it on the GPU: no host round trip of 5e6-entry vectors)."""
        if cls is not None:
            cls = torch.as_tensor(cls).reshape(-1).to(torch.int64)
            if cls.device != self.device and cls.device.type != "cpu":
                cls = cls.to(self.device)
            assert cls.numel() == self.npop
            if not bool((cls != 0).any()):
                cls = None
        old = self.lane_class
        self.lane_class = cls
        if old is None or cls is None:
            return not (old is None and cls is None)
        return not torch.equal(old.to(cls.device), cls)

    def per_edge_share(self, chunk: Optional[int] = None) -> float:
        """Share of the lane groups (of ``chunk``, default all) that hold a population of
        lane class != 0 (the narrow populations of :meth:`set_lane_classes`): the groups the
        residual forward evaluates by per-edge tails.  Cached per layout."""
        if self.layout != "lanes" or self.lane_class is None or self.ngroups == 0:
            return 0.0
        cache = self.__dict__.setdefault("_pe_share", None)
        if cache is None:
            cls = self.lane_class
            sp = self.slot_pop.to(cls.device, torch.int64)
            c = torch.where(sp >= 0, cls[sp.clamp(min=0)], torch.zeros_like(sp))
            per_group = (c.reshape(-1, 64).amax(1) > 0).double()
            # cumulative counts: any chunk's share from one host copy
            cum = torch.zeros(per_group.numel() + 1, dtype=torch.float64, device=per_group.device)
            cum[1:] = torch.cumsum(per_group, 0)
            cache = self._pe_share = cum.cpu()
        g0, g1 = self.group_range(chunk)
        return float((cache[g1] - cache[g0]) / (g1 - g0)) if g1 > g0 else 0.0

    def _order_key(self):
        key = self.order_counts
        if self.lane_class is None:
            return key
        cls = self.lane_class
        if cls.device.type != "cpu":
            if getattr(self, "_key_base_dev", None) is None or self._key_base_dev.device != cls.device:
                base = self.counts if key is None else key
                self._key_base_dev = base.to(device=cls.device, dtype=torch.int64)
            return self._key_base_dev + (cls << 40)
        base = self.counts.to(torch.int64) if key is None else key
        return base + (cls << 40)

    def _build_lanes(self, pb) -> None:
        from ._schedule import build_lanes_py, build_lanes_torch
        key = self._order_key()
        out = None
        if self.device.type == "cuda" and os.environ.get("MULTIGRAD_LANES_BUILDER", "device") != "host":
            # the same schedule from sorts and scatters on the GPU (~ms; the host builder takes
            # ~1 s at 5e6 populations): what makes a re-layout during a fit affordable
            if getattr(self, "_counts_dev", None) is None:
                self._counts_dev = self.counts.to(self.device, torch.int64)
            out = build_lanes_torch(self._counts_dev, pb[1:-1], self._lane_window,
                                    self._lane_lmax, key, device=self.device)
        if out is None:
            try:
                out = ext().build_lanes(self.counts.to(torch.int64), list(pb[1:-1]),
                                        self._lane_window, self._lane_lmax, key)
            except ImportError:
                out = build_lanes_py(self.counts, pb[1:-1], self._lane_window, self._lane_lmax, key)
        (slot_pop, slot_src, slot_len, slot_part, group_base, group_len, chunk_groups, giant,
         chunk_giant, fwd_order, slot_pidx, perm) = out
        trace(f"shard: lanes schedule built ({int(group_len.numel())} groups)")
        dev = self.device
        self.nslots = int(slot_pop.numel())
        self.ngroups = int(group_len.numel())
        self.chunk_groups = [int(v) for v in chunk_groups]
        self.chunk_giant = [int(v) for v in chunk_giant]
        self.slot_pop = slot_pop.to(dev)
        self.slot_part = slot_part.to(dev)
        self.group_base = group_base.to(dev)
        self.group_len = group_len.to(dev)
        self.fwd_order = fwd_order.to(dev)
        self._group_len_cpu, self._fwd_order_cpu = group_len.cpu(), fwd_order.cpu()
        self._wave_cache = {}
        self.giant = giant.to(dev).contiguous()
        # internal parameter order (see build_lanes): perm[i] = population of unit i
        self.slot_pidx = slot_pidx.to(dev)
        self.perm = perm.to(torch.int64).to(dev)
        self.inv_perm = torch.empty_like(self.perm)
        self.inv_perm[self.perm] = torch.arange(self.npop, device=dev)
        gi = giant.clone()
        if gi.numel():
            gi[:, 0] = self.inv_perm.cpu()[gi[:, 0].long()].to(torch.int32)
        self.giant_int = gi.to(dev).contiguous()
        nparts = int(giant[:, 2].max()) if giant.numel() else 0
        self.partials = torch.zeros(max(nparts, 1) * 2, dtype=torch.float32, device=dev)
        if dev.type == "cuda":
            # tail padding: the forward's prefetch loads run up to 2*unroll+1 rows past a
            # group's end unconditionally (values masked), so the last group stays in bounds
            self.xi = torch.full((int(group_base[-1]) + 64 * 16,), -1e30, dtype=torch.float32,
                                 device=dev)
            ext().smf_lanes_pack(self.x, slot_src.to(dev), slot_len.to(dev), self.group_base,
                                 self.group_len, self.xi)
        else:
            self.xi = None
        self.resid = None
        self.resid_epoch += 1
        self._pe_share = None
        trace("shard: lanes packed")

    def fwd_schedule(self, chunk: Optional[int], nblocks: int):
        """Work distribution of the lanes forward over ``chunk`` with ``nblocks``
        workgroups: ``(wave_order, wave_start, queues)``, at most one part set.

        ``MULTIGRAD_LPT``: ``static`` -- per-wave LPT lists built on the host
        (runtime.cpp:lpt_waves); ``dynamic`` -- 256 device work queues drawn by atomic
        tickets (waves that the oldest-first issue arbitration favours take more groups);
        ``0`` -- grid-stride over the longest-first order; ``auto`` (default) -- static.
        The static lists run with issue-priority feedback (``MG_FWD_PRIO`` in smf.hip: a
        wave's priority falls as its list drains), which removes most of the
        oldest-wave-first tail.  Until round 5 ``auto`` took the dynamic queues when every
        wave got >= 8 groups (the headline); round 6 measured static faster at every size
        of the pipelined step, same box, 3 alternating pairs (profiles/r6_owner_tail/):
        headline 0.4335-0.4341 vs 0.4352-0.4354 ms, 1/4 owner proxy 0.1137-0.1139 vs
        0.1181-0.1185, 1/8 0.0628-0.0630 vs 0.0713-0.0718.  Static lists also make the
        forward's bin sums run-to-run reproducible: a wave accumulates its groups in list
        order, while the dynamic draws change which wave sums which group (one of the
        three dynamic 1/4 runs ended at a different last-digit loss).
        """
        mode = os.environ.get("MULTIGRAD_LPT", "auto")
        if mode == "0":
            return None, None, None
        g0, g1 = self.group_range(chunk)
        nwaves = int(nblocks) * (256 // 64)
        if mode == "dynamic":
            if getattr(self, "_queues", None) is None:
                if self.device.type == "cuda" and torch.cuda.is_current_stream_capturing():
                    return None, None, None
                self._queues = torch.zeros(int(os.environ.get("MULTIGRAD_FWD_QUEUES", "256")),
                                           dtype=torch.int32, device=self.device)
            return None, None, self._queues
        key = (chunk, int(nblocks))
        if key not in self._wave_cache:
            if self.device.type == "cuda" and torch.cuda.is_current_stream_capturing():
                return None, None, None  # no host->device copies inside a graph capture
            order, start = ext().lpt_waves(self._group_len_cpu, self._fwd_order_cpu, g0, g1,
                                           nwaves, LPT_OVERHEAD)
            self._wave_cache[key] = (order.to(self.device), start.to(self.device))
        return self._wave_cache[key] + (None,)

    def resid_buffer(self, nbp: int) -> torch.Tensor:
        """Residual storage of the lanes forward, group-major [ngroups, 2 (nbp+1), 64]."""
        shape = (self.ngroups, 2 * (nbp + 1), 64)
        if self.resid is None or tuple(self.resid.shape) != shape:
            self.resid = torch.empty(shape, dtype=torch.float32, device=self.device)
        return self.resid

    def fwd_rows(self, nhalos: int, nbins: int = 10, log_sigma: bool = True,
                 rel_tail: bool = False, chunk: Optional[int] = None, resid: bool = True) -> int:
        """Slab rows a forward over ``chunk`` writes: one per workgroup of the forward grid
        (:meth:`fwd_blocks`).  ``resid`` is accepted for the engine interface; the residual
        forwards have no extra rows since the deferral list's fix-up launch was removed."""
        return self.fwd_blocks(nhalos, nbins, log_sigma, rel_tail, chunk)

    @property
    def vjp_recompute(self) -> bool:
        """Lanes layout with local slot order: the VJP re-evaluates the halos (no
        residuals) -- the cheaper choice at few halos per population."""
        return self.layout == "lanes" and self.lane_order == "local"

    def slot_index(self, order: str) -> torch.Tensor:
        """Slot -> parameter unit index for ``order`` in {"user", "internal"}."""
        return self.slot_pidx if order == "internal" else self.slot_pop

    def to_user_units(self, t: torch.Tensor) -> torch.Tensor:
        """(J, k) rows in internal order -> user (population) order."""
        return t[self.inv_perm]

    def group_range(self, chunk: Optional[int] = None):
        if chunk is None:
            return 0, self.ngroups
        return self.chunk_groups[chunk], self.chunk_groups[chunk + 1]

    def halo_range(self, chunk: Optional[int] = None):
        if chunk is None:
            return 0, self.n
        return self.chunk_halos[chunk], self.chunk_halos[chunk + 1]

    def fwd_blocks(self, nhalos: int, nbins: int = 10, log_sigma: bool = True,
                   rel_tail: bool = False, chunk: Optional[int] = None) -> int:
        """Forward grid: enough 256-thread workgroups for the halos (tiles layout) or for
        the 64-slot groups (lanes layout, one per wavefront), capped at one fully
        resident wave of workgroups."""
        if self.device.type != "cuda":
            return 1
        if self.layout == "lanes":
            g0, g1 = self.group_range(chunk)
            key = ("lanes", nbins, bool(log_sigma), bool(rel_tail))
            if key not in _GRID_CACHE:
                _GRID_CACHE[key] = int(ext().smf_fwd_lanes_max_blocks(
                    nbins, bool(log_sigma), bool(rel_tail), True))
            cap = min(_GRID_CACHE[key], int(os.environ.get("MULTIGRAD_FWD_MAX_BLOCKS", "1000000")))
            return int(max(1, min(cap, math.ceil(max(g1 - g0, 1) / 4))))
        cap = FWD_BLOCKS_MAX
        if self.device.type == "cuda":
            key = (nbins, bool(log_sigma), self.pop is not None, bool(rel_tail))
            if key not in _GRID_CACHE:
                _GRID_CACHE[key] = int(ext().smf_fwd_max_blocks(nbins, bool(log_sigma),
                                                                self.pop is not None,
                                                                bool(rel_tail)))
            cap = _GRID_CACHE[key]
        return int(max(1, min(cap, math.ceil(nhalos / 256))))


_GRID_CACHE: dict = {}
# Share of per-edge lane groups (narrow populations, PopulationShard.per_edge_share) from
# which the residual lanes forward runs the per-edge kernel for every group (LMODE 4)
# instead of the Euler-Maclaurin kernel with its out-of-line per-edge call: measured on one
# MI355X (profiles/narrow_sweep/, rocprof kernel averages) the EM kernel takes about
# 446 + 410 f us at a per-edge share f and the per-edge kernel 617-627 us, so they cross
# near f = 0.42.
PER_EDGE_SHARE = float(os.environ.get("MULTIGRAD_PER_EDGE_SHARE", "0.45"))


def _sort_by_population(pop_cpu: torch.Tensor, npop: int):
    try:
        return ext().sort_by_population(pop_cpu, npop)
    except ImportError:
        order = torch.argsort(pop_cpu.long(), stable=True)
        counts = torch.bincount(pop_cpu.long(), minlength=npop)
        return order, counts


_SORT_CHUNK = 1 << 30  # torch.sort refuses more than INT_MAX elements


def stable_population_sort(pop: torch.Tensor, npop: int, chunk: Optional[int] = None):
    """``(sorted_pop, order, counts)`` of a stable sort of the int32 population ids, on
    the ids' device.  Up to ``chunk`` elements this is one radix sort.  Longer shards (a
    288 GB GPU holds several 1e9 halos) are sorted in chunks and placed by a stable
    counting sort across them: a halo of population p that is the r-th of p in chunk c
    goes to ``start[p] + (p's count in chunks < c) + r`` -- the same order one global
    stable sort would give."""
    chunk = _SORT_CHUNK if chunk is None else int(chunk)
    n = pop.numel()
    if n <= chunk:
        spop, order = torch.sort(pop, stable=True)
        return spop, order, torch.bincount(spop, minlength=npop)
    dev = pop.device
    counts = torch.zeros(npop, dtype=torch.int64, device=dev)
    for c0 in range(0, n, chunk):
        counts += torch.bincount(pop[c0:c0 + chunk], minlength=npop)
    placed = torch.cumsum(counts, 0) - counts      # start of p, then + p's halos so far
    order = torch.empty(n, dtype=torch.int64, device=dev)
    for c0 in range(0, n, chunk):
        sp, o = torch.sort(pop[c0:c0 + chunk], stable=True)
        cc = torch.bincount(sp, minlength=npop)
        first = torch.cumsum(cc, 0) - cc              # first position of p in this chunk
        sp64 = sp.long()
        pos = placed[sp64] + (torch.arange(sp.numel(), device=dev) - first[sp64])
        order[pos] = o + c0
        placed += cc
        del sp, o, cc, first, sp64, pos
    spop = torch.repeat_interleave(torch.arange(npop, dtype=torch.int32, device=dev), counts,
                                   output_size=n)
    return spop, order, counts


def _build_tiles(counts, breaks, tile_halos, tile_pops):
    try:
        return ext().build_tiles(counts.to(torch.int64), list(breaks), tile_halos, tile_pops)
    except ImportError:
        from ._schedule import build_tiles_py
        return build_tiles_py(counts, breaks, tile_halos, tile_pops)


# ---------------------------------------------------------------------------- device ops
def _user_theta(theta: torch.Tensor, shard: PopulationShard, order: str) -> torch.Tensor:
    """Parameters in population (user) order, from ``order`` (CPU reference paths)."""
    if order != "internal":
        return theta
    t = theta.reshape(-1)[:2 * shard.npop].reshape(-1, 2)
    return shard.to_user_units(t).reshape(-1)


def smf_forward_slab(theta: torch.Tensor, shard: PopulationShard, bins: SmfBins, log_sigma: bool,
                     slab: torch.Tensor, chunk: Optional[int] = None, resid: bool = False,
                     order: str = "user", update: Optional[dict] = None,
                     epilogue: Optional[dict] = None, exchange: Optional[bytes] = None) -> int:
    """Forward of the shard (or one population chunk) into per-workgroup slab rows;
    returns the number of rows written.  CPU: one row from the PyTorch reference.
    ``resid`` (lanes layout): also store the VJP residuals of these populations.
    ``order="internal"`` (lanes layout): ``theta`` is in the shard's internal parameter
    order (``shard.perm``), the order the fused engine keeps its vectors in; chunks are
    the same population ranges in either order.  ``exchange``: a packed two-shot exchange
    of another parameter chunk that the tiles forward runs in its first workgroups (fused
    exchange); other paths launch it on its own first."""
    if order == "internal" and shard.layout != "lanes":
        raise ValueError("internal parameter order needs the lanes layout")
    if exchange and (theta.device.type != "cuda" or shard.layout == "lanes"):
        _launch_exchange(exchange)
        exchange = None
    h0, h1 = shard.halo_range(chunk)
    if theta.device.type != "cuda":
        with torch.no_grad():
            xs = shard.x[h0:h1]
            ps = None if shard.pop is None else shard.pop[h0:h1]
            th = _user_theta(theta, shard, order)
            row = smf_sumstats_reference(th.reshape(-1).float(), xs, ps, bins, log_sigma)
            sc = torch.as_tensor(bins.scale, dtype=row.dtype)
        slab[:bins.nbp].zero_()
        slab[:bins.nb] = (row / sc).to(slab.dtype)  # unscaled bin sums (scale at reduce)
        return 1
    nblk = shard.fwd_blocks(max(h1 - h0, 1), bins.nb, log_sigma, bins.rel_tail, chunk)
    if shard.layout == "lanes":
        g0, g1 = shard.group_range(chunk)
        rbuf = shard.resid_buffer(bins.nbp) if resid else None
        w_order, w_start, queues = shard.fwd_schedule(chunk, nblk)
        upd, usc = None, []
        if update is not None:  # pipelined residual VJP + Adam of the previous step
            u = update
            traj = u.get("traj")
            upd = [u["h"], u["m"], u["v"], u["step"],
                   traj if traj is not None else torch.empty(0, device=theta.device)]
            usc = [float(u["unit_offset"]), float(-1 if u.get("host_step") is None else u["host_step"]),
                   float(u["lr"]), float(u["b1"]), float(u["b2"]), float(u["eps"]),
                   float(u.get("traj_stride", 0)), float(bool(u.get("defer_advance", False)))]
            if u.get("u") is not None:  # bounded: Adam on u, p = T^-1(u) (csrc/adam.h)
                upd += [u["u"], u["lo"], u["hi"]]
                usc.append(float(bool(u.get("legacy", False))))
        et, es, ep = [], [], []
        if epilogue is not None:  # the sumstat epilogue launched by the same host call
            e = epilogue
            none = torch.empty(0, dtype=torch.int32, device=theta.device)
            os_ = e.get("oneshot")
            adv = e.get("advance")
            et = [e["slab"], e["target"], e["S"], e["loss"], e["h"],
                  none if os_ is None else os_.seq, none if os_ is None else os_.err,
                  none if adv is None else adv]
            es = [float(e["row0"]), float(e["eps"]), float(0 if os_ is None else os_.rank),
                  float(5.0 if os_ is None else os_.timeout_s)]
            ep = [] if os_ is None else list(os_.peers)
        rows = ext().smf_forward_lanes(shard.xi, shard.slot_index(order), shard.group_base,
                                       shard.group_len, shard.fwd_order, theta, list(bins.edges),
                                       list(bins.scale), bool(log_sigma), g0, g1, slab, nblk,
                                       bins.rel_tail, rbuf, w_order, w_start, queues, upd, usc,
                                       et, es, ep,
                                       bool(resid and shard.per_edge_share(chunk) >= PER_EDGE_SHARE))
        if resid:
            shard.resid_epoch += 1
        return int(rows)
    assert epilogue is None, "the folded epilogue is a lanes-layout launch"
    ext().smf_forward(shard.x, shard.pop, theta, list(bins.edges), list(bins.scale),
                      bool(log_sigma), h0, h1, slab, nblk, bins.rel_tail, exchange or b"")
    return nblk


def prepare_forward(shard: "PopulationShard", bins: SmfBins, log_sigma: bool = True,
                    chunk: Optional[int] = None) -> None:
    """Build (outside any graph capture) the host-side schedules the forward over
    ``chunk`` will use, e.g. the lanes layout's per-wave LPT lists."""
    if shard.device.type != "cuda" or shard.layout != "lanes":
        return
    h0, h1 = shard.halo_range(chunk)
    nblk = shard.fwd_blocks(max(h1 - h0, 1), bins.nb, log_sigma, bins.rel_tail, chunk)
    shard.fwd_schedule(chunk, nblk)


def smf_vjp_adam_into(theta: torch.Tensor, shard: "PopulationShard", bins: SmfBins,
                      log_sigma: bool, h: torch.Tensor, m: torch.Tensor, v: torch.Tensor,
                      unit_offset: int, step: torch.Tensor, host_step: Optional[int], lr: float,
                      b1: float, b2: float, eps: float, traj_base: Optional[torch.Tensor] = None,
                      traj_stride: int = 0, chunk: Optional[int] = None) -> bool:
    """Fused residual VJP + unbounded Adam (lanes layout, internal order, residuals of a
    forward at this ``theta``): theta, m, v and the trajectory row of the chunk's units are
    updated in place and no gradient is materialised.  ``m``/``v`` (and trajectory rows)
    cover units ``[unit_offset, unit_offset + m.numel() // 2)``.  Returns False (nothing
    done) where the fused path does not apply: CPU tensors, other layouts, or split
    populations in the chunk (their gradient needs the cross-part finalize)."""
    if theta.device.type != "cuda" or shard.layout != "lanes" or shard.resid is None:
        return False
    k0, k1 = (0, shard.giant.shape[0]) if chunk is None else \
        (shard.chunk_giant[chunk], shard.chunk_giant[chunk + 1])
    if k1 > k0:
        return False
    g0, g1 = shard.group_range(chunk)
    ext().smf_vjp_adam_lanes(shard.slot_index("internal"), shard.slot_part, theta, h,
                             shard.resid_buffer(bins.nbp), 64 * g0, 64 * g1, list(bins.scale),
                             bool(log_sigma), m, v, int(unit_offset), step,
                             -1 if host_step is None else int(host_step), float(lr), float(b1),
                             float(b2), float(eps), traj_base, int(traj_stride))
    return True


def smf_slab_reduce(slab: torch.Tensor, nrows: int, bins: SmfBins, out: torch.Tensor) -> torch.Tensor:
    """Fixed-order sum of ``nrows`` slab rows per bin, times the bin scale -> ``out``."""
    if slab.device.type != "cuda":
        rows = slab[:nrows * bins.nbp].reshape(nrows, bins.nbp).double().sum(0)
        sc = torch.zeros(bins.nbp, dtype=torch.float64)
        sc[:bins.nb] = torch.as_tensor(bins.scale, dtype=torch.float64)
        out[:bins.nbp] = (rows * sc).to(out.dtype)
        return out
    ext().smf_slab_reduce(slab, nrows, list(bins.edges), list(bins.scale), out)
    return out


def smf_forward_into(theta: torch.Tensor, shard: PopulationShard, bins: SmfBins, log_sigma: bool,
                     out: torch.Tensor, slab: Optional[torch.Tensor] = None,
                     chunk: Optional[int] = None, resid: bool = False,
                     order: str = "user") -> torch.Tensor:
    """Partial sumstats of the shard (or one population chunk) into ``out[:nbp]``."""
    if slab is None:
        h0, h1 = shard.halo_range(chunk)
        nblk = shard.fwd_rows(max(h1 - h0, 1), bins.nb, log_sigma, bins.rel_tail, chunk, resid)
        slab = torch.empty(nblk * bins.nbp, dtype=torch.float32, device=theta.device)
    nrows = smf_forward_slab(theta, shard, bins, log_sigma, slab, chunk, resid, order)
    return smf_slab_reduce(slab, nrows, bins, out)


def _launch_exchange(exchange: Optional[bytes]) -> None:
    """A packed two-shot exchange (parallel.xgmi.TwoShot.pack) launched on its own, for
    the paths whose kernels do not carry one (enqueued before them: same stream order)."""
    if exchange:
        ext().xgmi_twoshot_launch_packed(exchange)


def smf_vjp_into(theta: torch.Tensor, shard: PopulationShard, bins: SmfBins, log_sigma: bool,
                 h: torch.Tensor, grad: torch.Tensor, chunk: Optional[int] = None,
                 residuals_ready: bool = False, order: str = "user",
                 recompute: bool = False, exchange: Optional[bytes] = None) -> torch.Tensor:
    """Per-population VJP with edge weights ``h`` into ``grad`` (the chunk's parameters
    only).  CPU: autograd of the PyTorch reference restricted to the chunk's halos.

    Lanes layout: the VJP reads the residuals of a forward at the same ``theta``.  Pass
    ``residuals_ready=True`` only when the caller has just run
    ``smf_forward_*(..., resid=True)`` at this ``theta`` for this chunk (the fused engine
    does); otherwise the residual forward is recomputed here first.  ``order`` as in
    :func:`smf_forward_slab` (``grad`` is written in the same order as ``theta``).
    ``recompute`` (lanes layout): re-evaluate the halos instead of reading residuals
    (``smf_vjp_lanes_rc_kernel``).  ``exchange``: a packed two-shot exchange of another
    parameter chunk (fused exchange) that the tiles VJP runs in its first workgroups; other
    paths launch it on its own first."""
    if order == "internal" and shard.layout != "lanes":
        raise ValueError("internal parameter order needs the lanes layout")
    if exchange and (theta.device.type != "cuda" or shard.layout == "lanes"):
        _launch_exchange(exchange)
        exchange = None
    if theta.device.type != "cuda":
        h0, h1 = shard.halo_range(chunk)
        p0, p1 = (0, shard.npop) if chunk is None else (shard.chunk_pops[chunk], shard.chunk_pops[chunk + 1])
        th = _user_theta(theta.detach(), shard, order)
        th = th.reshape(-1)[:2 * shard.npop].double().clone().requires_grad_(True)
        xs = shard.x[h0:h1].double()
        ps = None if shard.pop is None else shard.pop[h0:h1]
        hw = h[:bins.nb + 1].double() * math.sqrt(2 * math.pi)
        with torch.enable_grad():
            t2 = th.reshape(-1, 2)
            a = t2[:, 0][ps.long()] if ps is not None else t2[0, 0]
            sg = t2[:, 1][ps.long()] if ps is not None else t2[0, 1]
            sigma = torch.pow(torch.tensor(10.0, dtype=th.dtype), sg) if log_sigma else sg
            e = torch.as_tensor(bins.edges, dtype=th.dtype)
            z = (e[None, :] - (xs + a)[:, None]) / (sigma[:, None] if torch.is_tensor(sigma) and sigma.dim() else sigma)
            f = (normal_cdf(z) * hw[None, :]).sum()
            (g,) = torch.autograd.grad(f, th, allow_unused=True)
        if g is None:
            g = torch.zeros_like(th)
        if order == "internal":  # internal units [p0, p1) are populations perm[p0:p1]
            g = g.reshape(-1, 2)[shard.perm].reshape(-1)
        grad.reshape(-1)[2 * p0:2 * p1] = g[2 * p0:2 * p1].to(grad.dtype)
        return grad
    E = ext()
    if shard.layout == "lanes" and recompute:
        g0, g1 = shard.group_range(chunk)
        k0, k1 = (0, shard.giant.shape[0]) if chunk is None else \
            (shard.chunk_giant[chunk], shard.chunk_giant[chunk + 1])
        giant = shard.giant_int if order == "internal" else shard.giant
        E.smf_vjp_lanes_rc(shard.xi, shard.slot_index(order), shard.slot_part, shard.group_base,
                           shard.group_len, theta, h, list(bins.edges), list(bins.scale),
                           bool(log_sigma), g0, g1, grad, shard.partials, giant[k0:k1])
        return grad
    if shard.layout == "lanes":
        if not residuals_ready or shard.resid is None:
            nblk = shard.fwd_rows(1, bins.nb, log_sigma, bins.rel_tail, chunk, resid=True)
            slab = torch.empty(nblk * bins.nbp, dtype=torch.float32, device=theta.device)
            smf_forward_slab(theta, shard, bins, log_sigma, slab, chunk, resid=True, order=order)
        g0, g1 = shard.group_range(chunk)
        k0, k1 = (0, shard.giant.shape[0]) if chunk is None else \
            (shard.chunk_giant[chunk], shard.chunk_giant[chunk + 1])
        giant = shard.giant_int if order == "internal" else shard.giant
        E.smf_vjp_lanes(shard.slot_index(order), shard.slot_part, theta, h,
                        shard.resid_buffer(bins.nbp), 64 * g0, 64 * g1, list(bins.scale),
                        bool(log_sigma), grad, shard.partials, giant[k0:k1])
        return grad
    if chunk is None:
        t0, t1 = 0, shard.tiles.shape[0]
        g0, g1 = 0, shard.giant.shape[0]
    else:
        t0, t1 = shard.chunk_tiles[chunk], shard.chunk_tiles[chunk + 1]
        g0, g1 = shard.chunk_giant[chunk], shard.chunk_giant[chunk + 1]
    E.smf_vjp(shard.x, shard.pop, theta, shard.tiles, t0, t1, h, list(bins.edges),
              list(bins.scale), bool(log_sigma), grad, shard.partials, shard.giant[g0:g1],
              exchange or b"")
    return grad


def smf_edge_weights_into(g: torch.Tensor, bins: SmfBins, h: torch.Tensor) -> torch.Tensor:
    """h_e = (g_{e-1} scale_{e-1} - g_e scale_e) / sqrt(2 pi) for e in [0, nb]."""
    if g.device.type != "cuda":
        sc = torch.as_tensor(bins.scale, dtype=torch.float64)
        gg = g[:bins.nb].double() * sc
        hh = torch.zeros(bins.nbp + 1, dtype=torch.float64)
        hh[1:bins.nb + 1] += gg
        hh[:bins.nb] -= gg
        h[:bins.nbp + 1] = (hh / math.sqrt(2 * math.pi)).to(h.dtype)
        return h
    ext().smf_edge_weights(g, list(bins.edges), list(bins.scale), h)
    return h


class _SmfSumstats(torch.autograd.Function):
    @staticmethod
    def forward(ctx, theta, shard, bins, log_sigma):
        out = torch.empty(bins.nbp, dtype=torch.float32, device=theta.device)
        resid = theta.requires_grad and shard.layout == "lanes"
        smf_forward_into(theta.detach().contiguous(), shard, bins, log_sigma, out, resid=resid)
        ctx.shard, ctx.bins, ctx.log_sigma = shard, bins, log_sigma
        ctx.epoch = shard.resid_epoch if resid else None
        ctx.save_for_backward(theta)
        return out[:bins.nb].clone()

    @staticmethod
    def backward(ctx, gS):
        (theta,) = ctx.saved_tensors
        bins = ctx.bins
        g = gS.detach().to(torch.float32).contiguous()
        h = torch.empty(bins.nbp + 1, dtype=torch.float32, device=theta.device)
        smf_edge_weights_into(g, bins, h)
        grad = torch.empty_like(theta, dtype=torch.float32)
        # residuals are still those of this forward unless another forward ran since
        ready = ctx.epoch is not None and ctx.epoch == ctx.shard.resid_epoch
        smf_vjp_into(theta.detach().contiguous(), ctx.shard, bins, ctx.log_sigma, h, grad,
                     residuals_ready=ready)
        return grad.to(theta.dtype), None, None, None


def smf_sumstats(theta: torch.Tensor, shard: PopulationShard, bins: SmfBins,
                 log_sigma: bool = True) -> torch.Tensor:
    """Partial SMF of this rank's shard; differentiable w.r.t. interleaved ``theta``.

    ``theta`` holds ``(a_c, s_c)`` per population (``2 * npop`` values).  On a GPU this
    runs the HIP kernels (float32); on CPU the PyTorch reference.
    """
    if theta.device.type == "cuda":
        th = theta.reshape(-1)
        if th.dtype != torch.float32:
            th = th.to(torch.float32)
        return _SmfSumstats.apply(th, shard, bins, bool(log_sigma)).to(theta.dtype)
    return smf_sumstats_reference(theta.reshape(-1), shard.x.to(theta.device),
                                  None if shard.pop is None else shard.pop.to(theta.device),
                                  bins, log_sigma)
