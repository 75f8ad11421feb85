"""One-shot xGMI all-reduce for tiny device vectors (``csrc/xgmi.hip``).

Every rank exports an uncached 2.3 KB region with ``hipIpcGetMemHandle``; the handles
are exchanged once over the communicator's object channel (gloo) and mapped with
``hipIpcOpenMemHandle``.  A call is one single-wavefront kernel: push the K values into
every peer's inbox, signal, poll the local flags, sum the W inboxes in rank order.

It replaces RCCL for tiny device all-reduces (K <= 64 fp32, SUM: the engine's per-step
sumstats) on up to 8 ranks.  The context is built on the first eligible call and checked
by a self-test on the actual hardware; only if every rank passes it is it used --
otherwise (or with ``MULTIGRAD_ALLREDUCE=rccl``, or without IPC, e.g. ranks on several
nodes, or without the native extension) RCCL is.

``MULTIGRAD_ALLREDUCE``:
  ``auto`` (default) -- the fused engine's per-step sumstat exchange uses it;
      ``Comm.all_reduce`` of user code stays on RCCL.
  ``oneshot`` -- additionally every eligible ``Comm.all_reduce`` (checked after each call).
  ``rccl`` -- never.

Failure is loud: a peer that does not signal within ``MULTIGRAD_ONESHOT_TIMEOUT`` seconds
sets the device error word and poisons the result with NaN (``csrc/xgmi.h``); the engine
reads the word at its host sync points (``FusedAdamEngine.check``) and raises
:class:`CollectiveTimeout` naming the rank and sequence number.  :meth:`reset`
(collective) re-zeroes the protocol state so a caller can continue after handling it.

Reference counterpart: the per-evaluation ``MPI.Allreduce`` of the sumstats,
multigrad/multigrad.py:522.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

__all__ = ["OneShotAllReduce", "CollectiveTimeout", "oneshot_enabled", "oneshot_mode",
           "connect", "get_oneshot", "maybe_oneshot", "MAX_FLOATS", "MAX_RANKS", "TwoShot",
           "WideOneShot", "get_wide_oneshot", "MAX_WIDE",
           "connect_twoshot", "twoshot_enabled", "get_twoshot_allreduce", "acquire_twoshot",
           "release_twoshot", "release_twoshot_allreduce", "status", "STRESS_REPS",
           "peer_all_gather"]

MAX_FLOATS = 64
MAX_WIDE = 1024    # fp64 values per wide one-shot call (csrc/xgmi.h kXwMax)
MAX_RANKS = 8
STRESS_REPS = 32   # back-to-back device-only exchanges in each connect-time self-test


def _corrupt_rank() -> int:
    """Test hook: the rank that corrupts one self-test exchange (-1: none)."""
    try:
        return int(os.environ.get("MULTIGRAD_XGMI_SELFTEST_CORRUPT", "-1"))
    except ValueError:
        return -1


def _record(comm, kind: str, **info) -> None:
    """Per-communicator verdict log of the peer-memory contexts (``status(comm)``)."""
    try:
        log = comm.__dict__.setdefault("_xgmi_status", {})
    except AttributeError:
        return
    log.setdefault(kind, []).append(info)


def status(comm) -> dict:
    """What the connect-time checks of ``comm``'s peer-memory collectives decided:
    ``{"one-shot": [...], "two-shot": [...]}``, one entry per connect attempt with
    ``ok``, the number of stress exchanges that passed and the fallback reason (RCCL)
    otherwise.  bench.py records it in its JSON line."""
    return dict(getattr(comm, "_xgmi_status", {}) or {})


class CollectiveTimeout(RuntimeError):
    """A peer-memory collective timed out waiting for a peer: its result is invalid."""


def oneshot_mode() -> str:
    m = os.environ.get("MULTIGRAD_ALLREDUCE", "auto").lower()
    return m if m in ("auto", "oneshot", "rccl") else "auto"


def oneshot_enabled() -> bool:
    """Whether the engine's sumstat exchange may use the one-shot kernel."""
    return oneshot_mode() in ("auto", "oneshot")


def _timeout_s() -> float:
    return float(os.environ.get("MULTIGRAD_ONESHOT_TIMEOUT", "5"))


class OneShotAllReduce:
    """One rank's side of the one-shot all-reduce; build it with :func:`connect`."""

    kind = "one-shot"

    def __init__(self, rank: int, size: int, base: int, peers, timeout_s: float = 5.0):
        self.rank, self.size = int(rank), int(size)
        self.base = base
        self.peers = list(peers)
        self.timeout_s = float(timeout_s)
        dev = torch.device("cuda", torch.cuda.current_device())
        self.seq = torch.zeros(1, dtype=torch.int32, device=dev)
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)

    @staticmethod
    def supports(t: torch.Tensor, op) -> bool:
        return (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()
                and 1 <= t.numel() <= MAX_FLOATS
                and (op is None or str(op).lower() in ("sum", "reduceop.sum")
                     or getattr(op, "name", "") == "SUM"))

    def __call__(self, t: torch.Tensor) -> torch.Tensor:
        from ..ops._ext import ext
        ext().xgmi_allreduce(t, self.peers, self.rank, self.seq, self.err, self.timeout_s)
        return t

    def ok(self) -> bool:
        """False if any call timed out waiting for a peer (host sync)."""
        return int(self.err.item()) == 0

    def check(self, where: str = "", comm=None) -> None:
        """Raise :class:`CollectiveTimeout` if any exchange so far timed out (host sync).

        With ``comm`` the verdict is all-reduced first (collective: every rank raises
        together, so no rank is left waiting in a later collective)."""
        e, s = (int(x) for x in torch.cat([self.err, self.seq]).tolist())
        bad = [self.rank] if e else []
        if comm is not None and comm.size > 1:
            flags = torch.zeros(comm.size, dtype=torch.int64)
            flags[comm.rank] = 1 if e else 0
            comm.all_reduce(flags)
            bad = [r for r in range(comm.size) if int(flags[r])]
        if bad:
            raise CollectiveTimeout(
                f"rank {self.rank}/{self.size}: {self.kind} xGMI exchange timed out after "
                f"{self.timeout_s:g} s waiting for a peer on rank(s) {bad} (sequence {s}"
                f"{', ' + where if where else ''}); its sums are NaN-poisoned.  A rank "
                f"skipped a collective or fell behind by more than MULTIGRAD_ONESHOT_TIMEOUT; "
                f"call reset() on every rank (collective) before reusing the communicator")

    @staticmethod
    def region_bytes() -> int:
        return 0  # the extension's default: the one-shot region

    def reset(self, comm) -> None:
        """Collective: return the protocol to its initial state on every rank (after a
        timeout was handled).  Every rank's kernels are drained first."""
        from ..ops._ext import ext
        torch.cuda.synchronize()
        comm.barrier()
        ext().xgmi_zero(self.base, self.region_bytes())
        self.seq.zero_()
        self.err.zero_()
        torch.cuda.synchronize()
        comm.barrier()

    def self_test(self, reps: int = STRESS_REPS) -> bool:
        """Stress self-test on the real peers: ``reps`` back-to-back exchanges with no host
        synchronisation in between, each with step-unique rank-dependent values whose sums
        are exact in fp32 (so a read of the previous exchange's slot, a lost flag or a
        reordered store shows up as a wrong sum), every result copied aside on the device
        and verified once at the end.  True when every sum is right and no wait timed
        out.  ``MULTIGRAD_XGMI_SELFTEST_CORRUPT=<rank>`` (test hook) makes that rank
        perturb its contribution to one exchange, so every rank must fail."""
        dev = self.seq.device
        corrupt = _corrupt_rank() == self.rank
        res = torch.zeros((reps, MAX_FLOATS), dtype=torch.float32, device=dev)
        bufs = [torch.empty(1 + (7 * i) % MAX_FLOATS, dtype=torch.float32, device=dev)
                for i in range(reps)]
        for i, t in enumerate(bufs):
            n = t.numel()
            torch.arange(n, out=t)
            t.add_((self.rank + 1) * (i + 1))
            if corrupt and i == reps // 2:
                t.add_(0.5)
            self(t)
            res[i, :n].copy_(t)
        got = res.cpu()
        for i, t in enumerate(bufs):
            n = t.numel()
            want = (torch.arange(n, dtype=torch.float32) * self.size
                    + (i + 1) * self.size * (self.size + 1) / 2)
            if not torch.equal(got[i, :n], want):
                return False
        return self.ok()

    def close(self) -> None:
        from ..ops._ext import ext
        E = ext()
        for r, p in enumerate(self.peers):
            if r != self.rank and p:
                E.xgmi_close(p)
        if self.base:
            E.xgmi_free(self.base)
        self.peers, self.base = [], 0


def connect(comm, timeout_s: float = 5.0, test: bool = True,
            cls=None) -> Optional[OneShotAllReduce]:
    """Collective: export, exchange and map the regions of every rank of ``comm``, then
    self-test.  Each phase ends with an all-gather of the per-rank verdicts, so all ranks
    take the same branch; returns None (use RCCL) if any rank failed any phase -- a
    missing native extension included.  ``cls``: :class:`OneShotAllReduce` (default) or
    :class:`WideOneShot`."""
    cls = OneShotAllReduce if cls is None else cls
    E = None
    base, handle = 0, None
    try:
        from ..ops._ext import ext
        E = ext()
        base = E.xgmi_alloc(cls.region_bytes())
        handle = bytes(E.xgmi_handle(base))
    except Exception as exc:  # noqa: BLE001  (no extension / no IPC on this rank)
        _debug(exc)
    handles = comm.allgather(handle)
    peers, ok = [], all(h is not None for h in handles)
    if ok:
        try:
            peers = [base if r == comm.rank else E.xgmi_open(handles[r]) for r in range(comm.size)]
        except Exception as exc:  # noqa: BLE001  (no IPC between these ranks)
            ok = False
            _debug(exc)
    if not all(comm.allgather(ok)):
        if E is not None:
            for r, p in enumerate(peers):
                if r != comm.rank and p:
                    E.xgmi_close(p)
            if base:
                E.xgmi_free(base)
        _record(comm, cls.kind, ok=False, stress_exchanges=0,
                fallback="RCCL: peer-memory export/map unavailable on some rank")
        return None
    ar = cls(comm.rank, comm.size, base, peers, timeout_s)
    comm.barrier()  # every region is zeroed and mapped before any rank writes into it
    ok = ar.self_test() if test else True
    verdicts = comm.allgather(bool(ok))
    if not all(verdicts):
        torch.cuda.synchronize()
        ar.close()
        _record(comm, cls.kind, ok=False, stress_exchanges=0,
                fallback=f"RCCL: stress self-test failed on rank(s) "
                         f"{[r for r, v in enumerate(verdicts) if not v]}")
        return None
    _record(comm, cls.kind, ok=True, stress_exchanges=STRESS_REPS if test else 0, fallback=None)
    return ar


def device_share(comm) -> int:
    """How many ranks of ``comm`` (this one included) run on this rank's GPU (collective on
    first use, cached): 1 on a normal one-process-per-GPU node, W when W processes share one
    GPU (the single-GPU rehearsals of multi-rank runs)."""
    n = getattr(comm, "_device_share", None)
    if n is None:
        import socket
        ident = None
        try:
            from ..ops._ext import ext
            ident = (socket.gethostname(), str(ext().device_pci_bus_id()))
        except Exception as exc:  # noqa: BLE001
            _debug(exc)
        ids = comm.allgather(ident)
        n = max(1, sum(1 for i in ids if i is not None and i == ident))
        try:
            comm._device_share = n
        except AttributeError:
            pass
    return int(n)


# Workgroups of one two-shot exchange launch with the GPU to itself (the grid-stride loop
# covers any size).  Exchange workgroups wait for their peers' flags; when several ranks
# share one GPU, every rank's grid is cut to 1/share of this so all of them can be resident
# together and no waiting grid can keep a peer's signalling workgroup off the GPU (an
# exchange grid that fills the GPU made the 4- and 8-process one-GPU rehearsals time out).
TWOSHOT_GRID = 1024


def _debug(exc) -> None:
    if os.environ.get("MULTIGRAD_DEBUG"):
        print(f"[multigrad] one-shot all-reduce unavailable: {exc}", flush=True)


def maybe_oneshot(comm, t: torch.Tensor, op) -> Optional[torch.Tensor]:
    """``Comm.all_reduce`` hook: run ``t`` through the communicator's one-shot all-reduce
    when ``MULTIGRAD_ALLREDUCE=oneshot`` (opt-in for user code) and applicable; None
    otherwise (the caller uses RCCL).  Each call is checked (host sync) so a timed-out
    exchange raises here instead of returning a wrong sum."""
    if oneshot_mode() != "oneshot" or comm.size > MAX_RANKS or not OneShotAllReduce.supports(t, op):
        return None
    ar = getattr(comm, "_oneshot", None)
    if ar is None:
        ar = comm._oneshot = connect(comm, _timeout_s()) or False
    if ar is False:
        return None
    ar(t)
    ar.check("Comm.all_reduce")
    return t


def get_oneshot(comm) -> Optional[OneShotAllReduce]:
    """The communicator's one-shot context for the fused engine, connecting it now if
    needed (collective: call on every rank); None when disabled or unavailable (use
    RCCL)."""
    if comm is None or comm.size == 1 or not oneshot_enabled() or comm.size > MAX_RANKS:
        return None
    if not torch.cuda.is_available():
        return None
    ar = getattr(comm, "_oneshot", None)
    if ar is None:
        ar = comm._oneshot = connect(comm, _timeout_s()) or False
    return ar or None


class WideOneShot(OneShotAllReduce):
    """fp64 one-shot all-reduce of up to :data:`MAX_WIDE` values per call, a summed part
    followed by a max-reduced part, both in rank order (every rank gets the same bits):
    the optimizers' per-iteration reductions (device L-BFGS / L-BFGS-B inner products,
    line-search directional derivatives, max|g|), stream ordered, no host round trip.
    Build it with :func:`get_wide_oneshot` (collective, self-tested)."""

    kind = "wide one-shot"

    @staticmethod
    def region_bytes() -> int:
        from ..ops._ext import ext
        return int(ext().xgmi_wide_region_bytes())

    @staticmethod
    def supports(t: torch.Tensor, op=None) -> bool:
        return (t.is_cuda and t.dtype == torch.float64 and t.is_contiguous()
                and 1 <= t.numel() <= MAX_WIDE)

    def __call__(self, t: torch.Tensor, nsum: Optional[int] = None, nmax: int = 0) -> torch.Tensor:
        """In place: ``t[:nsum]`` summed, ``t[nsum:nsum + nmax]`` max-reduced across the
        ranks (``nsum`` defaults to the rest of ``t``)."""
        from ..ops._ext import ext
        nsum = t.numel() - nmax if nsum is None else int(nsum)
        ext().xgmi_allreduce_wide(t, int(nsum), int(nmax), self.peers, self.rank, self.seq,
                                  self.err, self.timeout_s)
        return t

    def self_test(self, reps: int = STRESS_REPS) -> bool:
        """``reps`` back-to-back exchanges without host synchronisation, each with
        rank- and call-dependent values whose sums and maxima are exact in fp64 (about 47
        significant bits: integers up to ~2^23 with 2^-24 fractions), sizes up to
        the full width; verified once at the end (the test hook
        ``MULTIGRAD_XGMI_SELFTEST_CORRUPT`` perturbs one rank's contribution)."""
        dev = self.seq.device
        corrupt = _corrupt_rank() == self.rank
        W = self.size
        sizes = [1 + (131 * i) % MAX_WIDE for i in range(reps)]
        sizes[-1] = MAX_WIDE
        bufs, outs = [], []
        for i, n in enumerate(sizes):
            nmax = min(n // 3, 16)
            t = torch.arange(n, dtype=torch.float64, device=dev) * 2.0 ** -24
            t += (self.rank + 1) * (i + 1) * 1024.0
            if corrupt and i == reps // 2:
                t[0] += 0.5
            self(t, n - nmax, nmax)
            bufs.append((n, nmax))
            outs.append(t)
        got = [o.cpu() for o in outs]
        for i, ((n, nmax), g) in enumerate(zip(bufs, got)):
            base = torch.arange(n, dtype=torch.float64) * 2.0 ** -24
            want = base * W + (i + 1) * 1024.0 * W * (W + 1) / 2
            want[n - nmax:] = base[n - nmax:] + W * (i + 1) * 1024.0
            if not torch.equal(g, want):
                return False
        return self.ok()


def get_wide_oneshot(comm) -> Optional[WideOneShot]:
    """The communicator's wide one-shot context, connecting it now if needed (collective:
    call on every rank); None when disabled (``MULTIGRAD_ALLREDUCE=rccl``), on CPU, on more
    than :data:`MAX_RANKS` ranks or when peer memory is unavailable (the caller uses RCCL
    or gloo)."""
    if comm is None or comm.size == 1 or not oneshot_enabled() or comm.size > MAX_RANKS:
        return None
    if not torch.cuda.is_available():
        return None
    ar = getattr(comm, "_wide_oneshot", None)
    if ar is None:
        ar = comm._wide_oneshot = connect(comm, _timeout_s(), cls=WideOneShot) or False
    return ar or None


# ============================================================================ two-shot
def twoshot_enabled() -> bool:
    """Whether the ZeRO engine may sum its dense gradient with the two-shot kernel
    (``MULTIGRAD_ALLREDUCE`` auto/oneshot and ``MULTIGRAD_TWOSHOT`` not 0)."""
    if os.environ.get("MULTIGRAD_TWOSHOT", "1").lower() in ("0", "off", "false", "no"):
        return False
    return oneshot_mode() in ("auto", "oneshot")


class TwoShot:
    """Two-shot reduce-scatter -> Adam -> all-gather over peer memory (``csrc/xgmi.hip``).

    Owns three uncached, IPC-exported regions per rank: the gradient buffer ``grad`` the
    VJP writes, the parameter buffer ``theta`` the forward reads (both ``numel`` floats,
    exposed as tensors aliasing the regions) and a flag region.  One :meth:`step` per
    optimizer step pulls rank r's 1/W slice of every peer's gradient, sums it in rank order,
    applies Adam to the slice and pushes the new parameters into every peer's ``theta``;
    the launch returns (on the device) only when every slice has landed everywhere.
    Build it with :func:`connect_twoshot` (collective, self-tested).
    """

    kind = "two-shot"

    def __init__(self, comm, numel: int, regions, peers, timeout_s: float, share: int = 1):
        from ..ops._ext import ext
        E = ext()
        self.rank, self.size = comm.rank, comm.size
        # grid cap of every launch (TWOSHOT_GRID / ranks sharing this GPU)
        self.block_cap = max(16, TWOSHOT_GRID // max(1, int(share)))
        self.numel = int(numel)
        self.regions = regions            # (grad, theta, flags) base addresses, this rank
        self.gpeers, self.tpeers, self.fpeers = peers
        self.timeout_s = float(timeout_s)
        dev = torch.device("cuda", torch.cuda.current_device())
        self.grad = E.xgmi_tensor(regions[0], self.numel)
        self.theta = E.xgmi_tensor(regions[1], self.numel)
        self.seq = torch.zeros(1, dtype=torch.int32, device=dev)
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        self._step0 = torch.zeros(2, dtype=torch.int32, device=dev)
        # users of a cached all-reduce context (get_twoshot_allreduce): engines that hold it
        # between calls, and graphs captured around it (pinned: a replay may come any time);
        # the cache evicts only contexts that nobody holds
        self.holders = 0
        # exchanges recorded into graphs that may still be replayed; the capturer gives them
        # back with unpin() when it drops its graphs (generic engine close(), ingraph's loop)
        self.pins = 0

    def _blocks(self, max_blocks: int) -> int:
        mb = int(max_blocks)
        return self.block_cap if mb <= 0 else min(mb, self.block_cap)

    def slice(self, rank: Optional[int] = None):
        """Owned float range ``(lo, n)`` of ``rank`` (default: this rank)."""
        r = self.rank if rank is None else rank
        n = self.numel // self.size
        return r * n, n

    def step(self, lo: int, n: int, mode: int, m=None, v=None, u=None, bounds=None, traj=None,
             traj_stride: int = 0, step: Optional[torch.Tensor] = None,
             host_step: Optional[int] = None, lr: float = 0.0, b1: float = 0.9, b2: float = 0.999,
             eps: float = 1e-8, max_blocks: int = 0) -> None:
        """Enqueue one exchange on the current stream.  ``mode`` 0: theta = sum of the
        gradients (self-test); 1: unbounded Adam; 2/3: bounded (3: legacy Jacobian);
        4: reduce-scatter into ``u``; 5: all-gather of ``u`` (:meth:`reduce_scatter_`,
        :meth:`all_gather_`).  ``max_blocks`` caps the grid (0: the default 1024)."""
        from ..ops._ext import ext
        if not self.regions:
            raise RuntimeError("two-shot context used after close() (its peer memory is "
                               "unmapped)")
        lo_b = hi_b = kind = None
        if bounds is not None:
            lo_b, hi_b, kind = bounds.lo, bounds.hi, bounds.kind
        ext().xgmi_twoshot(self.gpeers, self.tpeers, self.fpeers, self.rank, int(lo), int(n),
                           self.numel, int(mode), u, m, v, lo_b, hi_b, kind, traj,
                           self._step0 if step is None else step, self.seq, self.err,
                           [float(-1 if host_step is None else host_step), float(lr), float(b1),
                            float(b2), float(eps), self.timeout_s, float(traj_stride),
                            float(self._blocks(max_blocks))])

    def pack(self, lo: int, n: int, mode: int, m=None, v=None, traj=None, traj_stride: int = 0,
             step: Optional[torch.Tensor] = None, host_step: Optional[int] = None,
             lr: float = 0.0, b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8,
             max_blocks: int = 0, u=None, bounds=None) -> bytes:
        """The launch arguments of one Adam exchange (``mode`` 1: unbounded; 2 / 3: bounded
        with ``u`` and ``bounds`` of the owned slice), packed for a compute launch that runs
        it in its first workgroups (fused exchange, csrc/twoshot.h; ops.smf ``exchange=``).
        Nothing is enqueued here."""
        from ..ops._ext import ext
        if not self.regions:
            raise RuntimeError("two-shot context used after close() (its peer memory is "
                               "unmapped)")
        lo_b = hi_b = kind = None
        if bounds is not None:
            lo_b, hi_b, kind = bounds.lo, bounds.hi, bounds.kind
        return ext().xgmi_twoshot_pack(
            self.gpeers, self.tpeers, self.fpeers, self.rank, int(lo), int(n), self.numel,
            int(mode), u, m, v, lo_b, hi_b, kind, traj,
            self._step0 if step is None else step, self.seq, self.err,
            [float(-1 if host_step is None else host_step), float(lr), float(b1), float(b2),
             float(eps), self.timeout_s, float(traj_stride), float(self._blocks(max_blocks))])

    def check(self, where: str = "", comm=None) -> None:
        OneShotAllReduce.check(self, where, comm)  # same err/seq protocol words

    def reduce_scatter_(self, out: torch.Tensor, lo: int, n: int, max_blocks: int = 0) -> None:
        """Mode 4: ``out[:n]`` = rank-order sum over the ranks of ``grad[lo:lo+n]`` (this
        rank's owned slice of every peer's gradient region); nothing is pushed."""
        self.step(lo, n, 4, u=out, max_blocks=max_blocks)

    def all_gather_(self, src: torch.Tensor, lo: int, n: int, max_blocks: int = 0) -> None:
        """Mode 5: ``theta[lo:lo+n]`` = ``src[:n]`` on every rank (this rank's slice pushed
        into every peer's parameter region); nothing is pulled."""
        self.step(lo, n, 5, u=src, max_blocks=max_blocks)

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum of a contiguous fp32 tensor of at most ``numel`` elements over the
        ranks, stream ordered and graph capturable (mode-0 exchange: every rank sums the
        peers' slices in rank order, so all ranks get bitwise identical results).

        Reusing the regions across calls is safe without host syncs: an exchange returns
        only when every peer has pulled this rank's ``grad`` and pushed into its ``theta``,
        and a peer's next exchange waits for this rank's next launch, which follows this
        rank's copy-out in stream order."""
        k = t.numel()
        if k > self.numel or t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("two-shot all_reduce_: contiguous fp32 tensor of at most "
                             f"{self.numel} elements expected, got {t.dtype} x {k}")
        flat = t.view(-1)
        if torch.cuda.is_current_stream_capturing():
            self.pins += 1  # a replay of this graph may come at any time: never evict
        self.grad[:k].copy_(flat)
        lo, n = self.slice()
        self.step(lo, n, 0)
        flat.copy_(self.theta[:k])
        return t

    def ok(self) -> bool:
        return int(self.err.item()) == 0

    def self_test(self, reps: int = STRESS_REPS) -> bool:
        """Stress self-test: ``reps`` back-to-back mode-0 exchanges over the whole region
        with no host synchronisation in between.  Exchange i sums gradients
        ``(idx mod 97) + (rank + 1)(i + 1)`` -- exact in fp32 and different in every
        exchange, so a slice pulled from a peer before it was rewritten (the previous
        exchange's value), a parameter slice that did not land, or a flag raised too early
        all give a wrong sum.  A strided sample of ``theta`` covering every rank's slice is
        copied aside on the device after each exchange and verified once at the end.
        ``MULTIGRAD_XGMI_SELFTEST_CORRUPT=<rank>`` (test hook): that rank corrupts its
        gradient slice in one exchange, so every rank must fail."""
        dev = self.grad.device
        corrupt = _corrupt_rank() == self.rank
        stride = max(1, self.numel // 4096)
        sample = torch.arange(0, self.numel, stride, device=dev)
        idx = torch.arange(self.numel, device=dev, dtype=torch.float32)
        base = torch.remainder(idx, 97.0)
        res = torch.empty((reps, sample.numel()), dtype=torch.float32, device=dev)
        lo, n = self.slice()
        for i in range(reps):
            torch.add(base, float((self.rank + 1) * (i + 1)), out=self.grad)
            if corrupt and i == reps // 2:
                self.grad[::7].add_(0.5)
            self.step(lo, n, 0)
            res[i].copy_(self.theta[sample])
        got = res.cpu()
        b = base[sample].cpu()
        ok = True
        for i in range(reps):
            want = b * self.size + (i + 1) * self.size * (self.size + 1) / 2
            if not torch.equal(got[i], want):
                ok = False
                break
        self.grad.zero_()
        self.theta.zero_()
        torch.cuda.synchronize()
        return ok and self.ok()

    def reset(self, comm) -> None:
        from ..ops._ext import ext
        torch.cuda.synchronize()
        comm.barrier()
        ext().xgmi_zero(self.regions[2], ext().xgmi_twoshot_flag_bytes())
        self.seq.zero_()
        self.err.zero_()
        torch.cuda.synchronize()
        comm.barrier()

    def close(self) -> None:
        from ..ops._ext import ext
        if not self.regions:
            return
        torch.cuda.synchronize()
        E = ext()
        for peers in (self.gpeers, self.tpeers, self.fpeers):
            for r, p in enumerate(peers):
                if r != self.rank and p:
                    E.xgmi_close(p)
        for b in self.regions:
            E.xgmi_free(b)
        self.regions = ()
        self.grad = self.theta = None


_MAX_AR_CONTEXTS = 4


def get_twoshot_allreduce(comm, numel: int, hold: bool = False) -> Optional[TwoShot]:
    """A cached two-shot context able to sum ``numel`` fp32 values over ``comm`` (for
    capturable user-level all-reduces, :func:`multigrad_amd.ingraph.reduce_sum`);
    collective on first use for a given size class.  None when disabled or unavailable
    (the caller uses RCCL).

    The smallest cached context that is large enough is reused.  Connecting is
    collective and synchronises the host, so it is refused while a graph is being
    captured (connect before capturing: call once eagerly with the same size).  At most
    ``_MAX_AR_CONTEXTS`` working contexts that nobody uses are kept; connecting a larger one
    closes the smallest of those (every rank makes the same calls in the same order, so the
    caches agree).  A context is in use while a caller holds it (``hold=True``, given back
    with :func:`release_twoshot_allreduce`) or while a graph that captured an exchange on it
    may still be replayed (``pins``, given back with :func:`unpin_twoshot_allreduce` by the
    capturer when it drops the graph); a closed context raises on use instead of touching
    unmapped peer memory."""
    if (comm is None or comm.size < 2 or comm.size > MAX_RANKS or not twoshot_enabled()
            or not torch.cuda.is_available()):
        return None
    quantum = 4 * comm.size
    want = max(quantum, -(-int(numel) // quantum) * quantum)
    cache = getattr(comm, "_twoshot_ar", None)
    if cache is None:
        cache = comm._twoshot_ar = {}
    fits = sorted(have for have, ts in cache.items() if ts and have >= want)
    if fits:
        ts = cache[fits[0]]
        ts.holders += int(hold)
        return ts
    if any(not ts and have <= want for have, ts in cache.items()):
        return None  # a failed connect at this size or below: the peers are unusable
    if torch.cuda.is_current_stream_capturing():
        raise RuntimeError(
            f"two-shot all-reduce of {numel} floats: no connected context is large enough "
            f"and connecting is collective (host synchronisation), which a graph capture "
            f"cannot contain; run one eager call of this size on every rank first")
    ts = connect_twoshot(comm, want, _timeout_s()) or False
    cache[want] = ts
    if ts:
        ts.holders += int(hold)
    idle = sorted(have for have, t in cache.items() if t and not t.holders and not t.pins)
    while len(idle) > _MAX_AR_CONTEXTS:
        torch.cuda.synchronize()
        comm.barrier()
        cache.pop(idle[0]).close()
        idle.pop(0)
    return ts or None


def peer_all_gather(comm, out: torch.Tensor, inp: torch.Tensor) -> bool:
    """``out`` (``[W * inp.numel()]`` elements, any dtype) = every rank's ``inp`` in rank
    order, through a cached two-shot context (mode 5: each rank pushes its piece into every
    peer's region; the bits are moved, never added, so fp64 and integer data pass
    unchanged).  Collective.  False (nothing done) where peer memory is unavailable; the
    caller then uses ``comm.all_gather_into_tensor``."""
    if comm is None or comm.size < 2 or not inp.is_cuda:
        return False
    nb = inp.numel() * inp.element_size()
    if nb % 4 or not inp.is_contiguous() or not out.is_contiguous():
        return False
    n = -(-(nb // 4) // 4) * 4  # floats per rank, float4 aligned
    ts = get_twoshot_allreduce(comm, n * comm.size, hold=True)
    if ts is None:
        return False
    try:
        src = inp.reshape(-1).view(torch.float32)
        if src.numel() != n or src.data_ptr() % 16:
            pad = torch.zeros(n, dtype=torch.float32, device=inp.device)
            pad[:src.numel()] = src
            src = pad
        ts.all_gather_(src, comm.rank * n, n)
        k = nb // 4
        rows = ts.theta[:n * comm.size].view(comm.size, n)[:, :k]
        out.reshape(-1).view(torch.float32).view(comm.size, k).copy_(rows)
    finally:
        release_twoshot_allreduce(ts)
    return True


def release_twoshot_allreduce(ts: Optional[TwoShot]) -> None:
    """Give back a context taken with ``get_twoshot_allreduce(..., hold=True)``."""
    if ts:
        ts.holders = max(0, ts.holders - 1)


def unpin_twoshot_allreduce(ts: Optional[TwoShot], n: int) -> None:
    """Give back ``n`` pins (exchanges captured into graphs the caller has dropped)."""
    if ts:
        ts.pins = max(0, ts.pins - int(n))


def acquire_twoshot(comm, numel: int) -> Optional[TwoShot]:
    """Collective: a two-shot context of exactly ``numel`` floats for an engine, taken
    from ``comm``'s pool of released contexts when every rank has one (no new peer
    memory, no new IPC mappings), connected (and stress-tested) otherwise.  Give it back
    with :func:`release_twoshot` when the engine is done."""
    pool = comm.__dict__.setdefault("_twoshot_pool", {})
    free = pool.get(int(numel), [])
    if all(comm.allgather(bool(free))):
        ts = free.pop()
        torch.cuda.synchronize()
        ts.theta.zero_()
        ts.grad.zero_()
        return ts
    return connect_twoshot(comm, numel)


def release_twoshot(comm, ts: Optional[TwoShot], keep: int = 2) -> None:
    """Return an engine's two-shot context to ``comm``'s pool (``keep`` per size; the
    rest are closed).  Every rank releases in the same order, so the pools stay paired."""
    if ts is None or not ts.regions:
        return
    torch.cuda.synchronize()
    pool = comm.__dict__.setdefault("_twoshot_pool", {})
    free = pool.setdefault(ts.numel, [])
    free.append(ts)
    while len(free) > keep:
        comm.barrier()
        free.pop(0).close()


def connect_twoshot(comm, numel: int, timeout_s: Optional[float] = None,
                    test: bool = True) -> Optional[TwoShot]:
    """Collective: allocate, export, exchange and map the three regions of every rank,
    then self-test; None (use RCCL) if any rank failed any phase.  ``numel`` must be a
    multiple of ``4 * comm.size`` (float4 slices)."""
    numel = int(numel)
    if comm is None or comm.size < 2 or comm.size > MAX_RANKS or numel % (4 * comm.size):
        return None
    timeout_s = _timeout_s() if timeout_s is None else float(timeout_s)
    E, regions, handles = None, [], None
    try:
        from ..ops._ext import ext
        E = ext()
        sizes = (4 * numel, 4 * numel, E.xgmi_twoshot_flag_bytes())
        for nb in sizes:
            regions.append(E.xgmi_alloc(nb))
        handles = [bytes(E.xgmi_handle(b)) for b in regions]
    except Exception as exc:  # noqa: BLE001
        _debug(exc)
        handles = None
    allh = comm.allgather(handles)
    ok = all(h is not None for h in allh)
    peers = ([], [], [])
    if ok:
        try:
            for k in range(3):
                peers[k].extend(regions[k] if r == comm.rank else E.xgmi_open(allh[r][k])
                                for r in range(comm.size))
        except Exception as exc:  # noqa: BLE001
            ok = False
            _debug(exc)
    if not all(comm.allgather(ok)):
        if E is not None:
            for k in range(3):
                for r, p in enumerate(peers[k]):
                    if r != comm.rank and p:
                        E.xgmi_close(p)
            for b in regions:
                E.xgmi_free(b)
        _record(comm, "two-shot", ok=False, numel=numel, stress_exchanges=0,
                fallback="RCCL: peer-memory export/map unavailable on some rank")
        return None
    ts = TwoShot(comm, numel, tuple(regions), peers, timeout_s, share=device_share(comm))
    comm.barrier()
    ok = ts.self_test() if test else True
    verdicts = comm.allgather(bool(ok))
    if not all(verdicts):
        ts.close()
        _record(comm, "two-shot", ok=False, numel=numel, stress_exchanges=0,
                fallback=f"RCCL: stress self-test failed on rank(s) "
                         f"{[r for r, v in enumerate(verdicts) if not v]}")
        return None
    _record(comm, "two-shot", ok=True, numel=numel, grid=ts.block_cap,
            stress_exchanges=STRESS_REPS if test else 0, fallback=None)
    return ts
