"""Device L-BFGS-B: box-constrained L-BFGS on (optionally sharded) device vectors.

The reference hands its bounds to scipy's L-BFGS-B (``multigrad/bfgs.py:83-86``).  At
1e6-1e8 parameters that optimizer has to live on the GPUs, so this is L-BFGS-B itself
(Byrd, Lu, Nocedal & Zhu 1995, with the projected subspace step of Morales & Nocedal
2011, as in scipy's L-BFGS-B 3.0) in an SPMD form:

* **Generalized Cauchy point.**  The first local minimiser of the quadratic model
  ``m(x) = f + g'(x-x_k) + (x-x_k)'B(x-x_k)/2`` (compact form ``B = theta I - W M W'``,
  ``W = [Y, theta S]``) along the projected gradient path ``P(x - t g)``.  The path
  has one breakpoint per coordinate; each rank sends the ``K`` smallest of its own (with
  the gradient entry and the ``2m`` row of ``W``), so every rank holds the ``K`` globally
  smallest, sorted, and runs the same sequential segment scan on the host -- identical
  decisions everywhere without broadcasts.  The Cauchy point is then ``P(x - t* g)``, one
  elementwise pass on the device.  (If the minimiser lies beyond the ``K``-th breakpoint,
  ``K`` grows and the scan repeats.)
* **Subspace minimisation** over the free variables by the direct primal method.  The
  ``2m x 2m`` Gram matrix of ``W`` over the free rows is the full Gram matrix (kept from
  the history inner products) minus the rows of the active set, which are gathered; the
  step is projected onto the box and falls back to the feasible truncation if the
  projected step is not a descent direction.
* **Line search** along ``d = xbar - x`` (strong Wolfe, cubic interpolation, step <= 1 so
  the iterate stays feasible), on loss values and directional derivatives that are
  all-reduced, i.e. bitwise identical on every rank.
* **Host traffic.**  Two device->host copies per iteration besides the function
  evaluations: (A) the new pair's inner products with the history together with every
  Cauchy-point input, (B) the subspace inner products; the first evaluation of the line
  search also carries the directional derivative at the start point.

Termination as scipy: ``max|P(x-g)-x| <= pgtol`` or ``(f_k-f_{k+1})/max(|f_k|,|f_{k+1}|,1)
<= factr * eps`` or ``maxiter``.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import scipy.linalg
import scipy.optimize
import torch

from ..ops.lbfgs import MultiDot, lincomb_
from ._reduce import DeviceReducer
from .lbfgs import _zoom

__all__ = ["lbfgsb_minimize", "run_lbfgsb_device", "BoxObjective"]

_EPS = np.finfo(np.float64).eps
_B_CAP_MULTI = 1 << 16  # breakpoints per rank and Cauchy-point batch on several ranks


class BoxObjective:
    """Replicated objective ``loss_and_grad_fn(x) -> (loss, grad)`` in the parameters
    themselves (no transform), for :func:`lbfgsb_minimize`."""

    def __init__(self, loss_and_grad_fn, x0: torch.Tensor, comm=None, **fn_kwargs):
        self.fn, self.kw, self.comm = loss_and_grad_fn, fn_kwargs, comm
        self.sharded = False
        x0 = x0.detach().reshape(-1).to(torch.float32)
        self.device, self.shape = x0.device, x0.shape
        self._x0 = x0.clone()
        self.n_local = x0.numel()

    def x0(self):
        return self._x0.clone()

    def full(self, x):
        return x

    def __call__(self, x):
        loss, grad = self.fn(x, **self.kw)
        if isinstance(loss, (tuple, list)):
            loss = loss[0]
        g = torch.as_tensor(grad).detach().reshape(-1).to(device=x.device, dtype=torch.float32)
        return float(torch.as_tensor(loss).detach().double()), g.contiguous()


def _box(lo, hi, n, device):
    lo = torch.full((n,), -math.inf, device=device) if lo is None else \
        torch.as_tensor(lo, dtype=torch.float32, device=device).reshape(-1).clone()
    hi = torch.full((n,), math.inf, device=device) if hi is None else \
        torch.as_tensor(hi, dtype=torch.float32, device=device).reshape(-1).clone()
    return lo.contiguous(), hi.contiguous()


class _History:
    """m accepted (s, y) pairs in a ring of m+1 device slots (a new pair is measured in the
    spare slot before it is accepted), with their inner products."""

    def __init__(self, m: int, n: int, device):
        self.m = int(m)
        self.R = self.m + 1
        self.HS = torch.zeros((2 * self.R, n), dtype=torch.float32, device=device)  # s_q, y_q
        self.SY = np.zeros((self.R, self.R))  # s_i . y_j
        self.SS = np.zeros((self.R, self.R))
        self.YY = np.zeros((self.R, self.R))
        self.order: list = []   # accepted slots, oldest first
        self.theta = 1.0

    def spare(self) -> int:
        return min(set(range(self.R)) - set(self.order))

    def s(self, q):
        return self.HS[q]

    def y(self, q):
        return self.HS[self.R + q]

    def accept(self, q: int, dots: np.ndarray) -> bool:
        """dots[r] = (HS_r . s_q, HS_r . y_q) for every row r; decide and record."""
        sy, yy = dots[q, 1], dots[self.R + q, 1]
        if not (sy > _EPS * yy and yy > 0):
            return False
        for o in self.order + [q]:
            self.SY[o, q] = dots[o, 1]
            self.SY[q, o] = dots[self.R + o, 0]
            self.SS[o, q] = self.SS[q, o] = dots[o, 0]
            self.YY[o, q] = self.YY[q, o] = dots[self.R + o, 1]
        self.order.append(q)
        if len(self.order) > self.m:
            self.order.pop(0)
        self.theta = yy / sy
        return True

    def compact(self):
        """``(idx, M, WWt)`` for the accepted pairs: ``M`` (2k x 2k) and the full Gram
        matrix ``W W'`` of ``W = [Y, theta S]`` (rows in ``idx`` order)."""
        idx = np.asarray(self.order, dtype=np.int64)
        k = idx.size
        if k == 0:
            return idx, np.zeros((0, 0)), np.zeros((0, 0))
        th = self.theta
        sy = self.SY[np.ix_(idx, idx)]
        D = np.diag(np.diag(sy))
        Lm = np.tril(sy, -1)
        ss = self.SS[np.ix_(idx, idx)]
        K = np.block([[-D, Lm.T], [Lm, th * ss]])
        M = np.linalg.inv(K)
        yy = self.YY[np.ix_(idx, idx)]
        ys = sy.T  # y_i . s_j
        WWt = np.block([[yy, th * ys], [th * ys.T, th * th * ss]])
        return idx, M, WWt

    def rows(self, idx):
        """Row indices of ``W = [Y_idx, S_idx]`` in HS and the theta factor per row."""
        rows = np.concatenate([self.R + idx, idx]).astype(np.int64)
        fac = np.concatenate([np.ones(idx.size), np.full(idx.size, self.theta)])
        return rows, fac


def _lbfgsb_minimize_impl(obj, lo=None, hi=None, maxiter: int = 100, m: int = 10,
                    factr: float = 1e7, pgtol: float = 1e-5, maxls: int = 20,
                    c1: float = 1e-4, c2: float = 0.9, K: Optional[int] = None,
                    callback=None, gtol: Optional[float] = None,
                    ftol: Optional[float] = None) -> scipy.optimize.OptimizeResult:
    """Minimise ``obj`` subject to ``lo <= x <= hi`` (local slices of the optimizer's
    vector, +-inf allowed).  ``obj`` as for :func:`multigrad_amd.optim.lbfgs.lbfgs_minimize`
    (``x0()``, ``__call__(x) -> (f, g)``, optional ``device_call``, ``full(x)``, ``comm``,
    ``sharded``).  ``gtol`` / ``ftol`` are accepted as aliases of ``pgtol`` /
    ``factr * eps`` (the unbounded driver's names)."""
    if gtol is not None:
        pgtol = gtol
    if ftol is not None:
        factr = ftol / _EPS
    comm, sharded = obj.comm, obj.sharded
    n = obj.n_local
    dev = obj.device
    lo, hi = _box(lo, hi, n, dev)
    lo64, hi64 = lo.double(), hi.double()
    x = torch.minimum(torch.maximum(obj.x0().contiguous(), lo), hi)
    f, g = obj(x)
    g = g.clone()
    nfev = 1
    H = _History(m, n, dev)
    R = H.R
    dot = MultiDot(2 * R, n, dev)
    dev_call = getattr(obj, "device_call", None) if dev.type == "cuda" else None
    ftol = factr * _EPS
    pending = None  # slot of a measured, not yet accepted pair
    status, message, nit = 1, "STOP: TOTAL NO. of ITERATIONS REACHED LIMIT", 0
    xt = torch.empty_like(x)

    red = DeviceReducer(comm, sharded, dev)  # collective (may connect peer memory)
    # the first Cauchy-point batch all-gathers (1 + B0) x (2 + 2m) fp64 records per rank:
    # connect that context now; the geometric growth to larger batches (rare: the Cauchy
    # point usually lies among the first few thousand breakpoints) connects its larger
    # context on demand, collectively (every rank reaches the same batch together) -- about
    # 1.2 MB per rank at m = 10 instead of 11.5 MB reserved for a 2^16 batch up front
    b0 = int(K) if K is not None else min(1 << 14, _B_CAP_MULTI)
    red.reserve_gather((1 + b0) * (2 + 2 * m) * 8)

    from ..utils.hooks import StepHooks
    hooks = StepHooks(comm, what="L-BFGS-B iterate")  # MULTIGRAD_CHECK_EVERY / _METRICS
    host0 = getattr(comm, "host_collectives", 0) if comm is not None else 0

    def run_callback(xv):
        nonlocal host0
        h0 = getattr(comm, "host_collectives", 0) if comm is not None else 0
        callback(obj.full(xv))
        if comm is not None:  # the callback's own collectives are not the loop's
            host0 += getattr(comm, "host_collectives", 0) - h0

    for k in range(maxiter + 1):
        # ------------------------------------------------ copy A: pair dots + GCP inputs
        t = torch.where(g < 0, (x - hi) / g, torch.where(g > 0, (x - lo) / g,
                                                          torch.full_like(g, math.inf)))
        t = torch.where(torch.isnan(t), torch.full_like(t, math.inf), t)
        free_path = t > 0
        d = torch.where(free_path, -g, torch.zeros_like(g))
        xd = x.double()
        pg = (torch.minimum(torch.maximum(xd - g.double(), lo64), hi64) - xd).abs()
        vecs = [d] if pending is None else [H.s(pending), H.y(pending), d]
        dots_dev = dot(H.HS, 2 * R, vecs)
        tc = torch.where(free_path & torch.isfinite(t), t, torch.full_like(t, math.inf))
        pg_l = pg.max().double() if n else torch.zeros((), dtype=torch.float64, device=dev)
        # one reduction and one copy: [d.d, HS.vecs (summed), max|pg| (max), #finite (local)]
        packA = red.reduce(sums=[(d.double() * d.double()).sum(), dots_dev],
                           maxes=[pg_l], local=[torch.isfinite(tc).sum()])
        dd = packA[0]
        dots_np = packA[1:1 + 2 * R * len(vecs)].reshape(2 * R, len(vecs))
        pgmax = float(packA[-2])
        nfin_l = packA[-1]
        if pending is not None:
            H.accept(pending, dots_np[:, :2])
            pending = None
        Wd = dots_np[:, -1]  # HS rows . d
        if k > 0 and callback is not None:
            run_callback(x)
        if pgmax <= pgtol:
            status, message = 0, "CONVERGENCE: NORM_OF_PROJECTED_GRADIENT_<=_PGTOL"
            break
        if k == maxiter:
            break
        # ------------------------------------------------ generalized Cauchy point
        idx, M, WWt = H.compact()
        rows, fac = H.rows(idx)
        th = H.theta
        tstar, cvec = _cauchy_point(dd, Wd[rows] * fac, M, th, tc, int(nfin_l), g, H.HS,
                                    rows, fac, red, K)
        xcp = torch.minimum(torch.maximum(x - tstar * g, lo), hi)
        free = (xcp > lo) & (xcp < hi)
        # ------------------------------------------------ copy B: subspace inner products
        kk2 = idx.size
        if kk2:
            Mc = M @ cvec
            coef = np.zeros(2 * R)
            coef[rows] = Mc * fac
            wmc = torch.empty_like(x)
            lincomb_(H.HS, 2 * R, torch.from_numpy(coef.astype(np.float32)).to(dev), 0.0, None, wmc)
            r = g + th * (xcp - x) - wmc
        else:
            r = g + th * (xcp - x)
        rF = torch.where(free, r, torch.zeros_like(r))
        WtZr = dot(H.HS, 2 * R, [rF])[:, 0]
        if kk2:
            act = torch.nonzero(~free).reshape(-1)  # a host sync: only where it is used
            rows_d = torch.as_tensor(rows, device=dev)
            GA = _gram(H.HS[rows_d[:, None], act[None, :]].double())
        else:
            GA = torch.zeros((0, 0), dtype=torch.float64, device=dev)
        redB = red.reduce(sums=[WtZr, GA])
        WtZr_np = redB[:2 * R]
        GA_np = redB[2 * R:].reshape(kk2 * 2, kk2 * 2) if kk2 else np.zeros((0, 0))
        if kk2:
            fw = fac[:, None] * fac[None, :]
            GF = WWt - GA_np * fw               # Gram of W over the free rows
            v = M @ (WtZr_np[rows] * fac)
            N = np.eye(2 * kk2) - (M @ GF) / th
            v = scipy.linalg.solve(N, v)
            coef = np.zeros(2 * R)
            coef[rows] = v * fac
            zwv = torch.empty_like(x)
            lincomb_(H.HS, 2 * R, torch.from_numpy(coef.astype(np.float32)).to(dev), 0.0, None, zwv)
            du = -(rF / th) - (zwv / (th * th))
        else:
            du = -(rF / th)
        du = torch.where(free, du, torch.zeros_like(du))
        xbar = torch.minimum(torch.maximum(xcp + du, lo), hi)
        dirn = xbar - x
        # ------------------------------------------------ line search along x + a dirn
        a1 = 1.0
        if k == 0 or not H.order:
            dnorm2 = float(red.reduce(sums=[(dirn.double() ** 2).sum()])[0])
            a1 = min(1.0, 1.0 / math.sqrt(max(dnorm2, 1e-300)))
        cache = {}
        d0_box = [None]

        def phi(alpha):
            nonlocal nfev
            torch.add(x, dirn, alpha=float(alpha), out=xt)
            if dev_call is not None:
                lt, ga = dev_call(xt)
                ga = ga.clone()
            else:
                fl, ga = obj(xt)
                ga = ga.clone()
                lt = torch.tensor([fl], dtype=torch.float64)
            # directional derivative(s) summed over the ranks with the (global) loss: one copy
            parts = [(ga.double() * dirn.double()).sum()]
            if d0_box[0] is None:
                parts.append((g.double() * dirn.double()).sum())
            red2 = red.reduce(sums=parts, local=[lt.reshape(1)])
            fa = float(red2[-1])
            if d0_box[0] is None:
                d0_box[0] = float(red2[1])
            nfev += 1
            cache[alpha] = (fa, ga, float(red2[0]))
            return fa, float(red2[0])

        best = _line_search(phi, f, d0_box, a1, c1, c2, maxls)
        if d0_box[0] is not None and d0_box[0] >= 0:
            # the projected subspace step is not a descent direction: truncate instead
            ratio = torch.where(du > 0, (hi - xcp) / du, torch.where(du < 0, (lo - xcp) / du,
                                                                    torch.full_like(du, math.inf)))
            rmin_l = -ratio.min().double() if ratio.numel() else \
                torch.full((), -math.inf, dtype=torch.float64, device=dev)
            rmin = -float(red.reduce(maxes=[rmin_l])[0])
            dirn = xcp + min(1.0, rmin) * du - x
            cache.clear()
            d0_box[0] = None
            best = _line_search(phi, f, d0_box, a1, c1, c2, maxls)
        if best is None or best not in cache:
            cands = [(v[0], a) for a, v in cache.items() if v[0] < f]
            if not cands:
                status, message = 2, "ABNORMAL_TERMINATION_IN_LNSRCH"
                break
            best = min(cands)[1]
        f_new, g_new, _ = cache[best]
        q = H.spare()
        torch.mul(dirn, best, out=H.HS[q])
        torch.sub(g_new, g, out=H.HS[R + q])
        x.add_(H.HS[q])
        x.copy_(torch.minimum(torch.maximum(x, lo), hi))
        pending = q
        nit = k + 1
        f_old, f, g = f, f_new, g_new
        if hooks.active:
            hooks(k, f, None, (lambda: x) if not sharded else None, nfev=nfev)
        if (f_old - f) <= ftol * max(abs(f_old), abs(f), 1.0):
            status, message = 0, "CONVERGENCE: REL_REDUCTION_OF_F_<=_FACTR*EPSMCH"
            if callback is not None:
                run_callback(x)
            break
    host_calls = (getattr(comm, "host_collectives", 0) - host0) if comm is not None else 0
    red.check("L-BFGS-B")
    if getattr(obj, "check", None) is not None:
        obj.check("L-BFGS-B")  # the objective's own exchanges (engine: ZeRO two-shot, one-shot)
    xf = obj.full(x)
    if getattr(obj, "finalize", None) is not None:
        xf = obj.finalize(x)
    return scipy.optimize.OptimizeResult(
        x=xf, fun=f, jac=g, nit=nit, nfev=nfev, njev=nfev, status=status,
        success=status == 0, message=message, host_collectives=host_calls,
        reduction=red.describe())


def _cauchy_point(dd, p0, M, theta, tc, nfin, g, HS, rows, fac, red, K):
    """Generalized Cauchy point ``t*`` and ``c = W'(x^cp - x)`` (Byrd et al. 1995,
    algorithm CP), over the breakpoints in increasing order, in batches.

    ``tc``: this rank's breakpoints (+inf where none), ``nfin`` of them finite.  Each batch
    takes the next ``K`` of every rank (sorted on the device); across ranks the union is
    exact up to the smallest "largest gathered" breakpoint of the ranks that have more,
    and only that prefix is scanned (the rest waits for the next batch).  The scan of a
    batch is vectorised: the running ``p``, ``c``, ``f'`` and ``f''`` of the sequential
    algorithm are prefix sums over the sorted breakpoints (``_scan_batch``)."""
    dev = tc.device
    k2 = p0.size
    Mt = torch.as_tensor(M, dtype=torch.float64, device=dev)
    st = {"p": torch.as_tensor(p0, dtype=torch.float64, device=dev),
          "c": torch.zeros(k2, dtype=torch.float64, device=dev),
          "fp": -dd, "fpp": theta * dd - (float(p0 @ M @ p0) if k2 else 0.0), "told": 0.0}
    order = torch.argsort(tc)
    rows_t = torch.as_tensor(rows, dtype=torch.int64, device=dev)
    fac_t = torch.as_tensor(fac, dtype=torch.float64, device=dev)
    comm = None if red is None else red.comm
    multi = comm is not None and comm.size > 1
    # batch sizes: K if given, else geometric from 2^14 (the Cauchy point usually lies among
    # the first few thousand breakpoints, and a scan costs O(2k x batch) in fp64) up to
    # 2^16 per rank (several ranks: one all-gather per batch) or 2^20 (one rank)
    B_cap = int(K) if K is not None else (_B_CAP_MULTI if multi else 1 << 20)
    B = int(K) if K is not None else min(1 << 14, B_cap)
    ptr = 0
    while True:
        sel = order[ptr:ptr + B]
        tb = tc[sel].double()
        gb = g[sel].double()
        Wb = (HS[rows_t[:, None], sel[None, :]].double() * fac_t[:, None]) if k2 else \
            torch.zeros((0, sel.numel()), dtype=torch.float64, device=dev)
        left = nfin - ptr  # this rank's finite breakpoints not yet scanned
        if multi:
            rec = torch.full((B, 2 + k2), math.inf, dtype=torch.float64, device=dev)
            nb = sel.numel()
            rec[:nb, 0], rec[:nb, 1], rec[:nb, 2:] = tb, gb, Wb.T
            rec[nb:, 1:] = 0.0
            hdr = torch.tensor([[float(left)] + [0.0] * (1 + k2)], dtype=torch.float64, device=dev)
            mine = torch.cat([hdr, rec]).contiguous()
            allr = red.all_gather(mine)   # peer memory / RCCL: [W, 1 + B, 2 + k2]
            # one copy: every rank's count of unscanned breakpoints and its B-th breakpoint
            hdr = torch.stack([allr[:, 0, 0], allr[:, B, 0]], 1).cpu().numpy()
            lefts = hdr[:, 0]
            t_cut = math.inf
            for r in range(comm.size):
                if lefts[r] > B:
                    t_cut = min(t_cut, float(hdr[r, 1]))
            recs = allr[:, 1:].reshape(-1, 2 + k2)
            keep = recs[:, 0] <= t_cut
            recs = recs[keep & torch.isfinite(recs[:, 0])]
            recs = recs[torch.argsort(recs[:, 0], stable=True)]
            tb, gb, Wb = recs[:, 0], recs[:, 1], recs[:, 2:].T.contiguous()
            mine_used = int(((rec[:, 0] <= t_cut) & torch.isfinite(rec[:, 0])).sum().item())
            more = bool((lefts > B).any())
        else:
            fin = torch.isfinite(tb)
            tb, gb, Wb = tb[fin], gb[fin], Wb[:, fin]
            mine_used = sel.numel()
            more = left > B
        found, tstar, c = _scan_batch(st, tb, gb, Wb, Mt, theta)
        if found:
            return tstar, c
        ptr += mine_used
        B = min(B * 8, B_cap)
        if not more:
            dtmin = -st["fp"] / st["fpp"] if st["fpp"] > 0 else 0.0
            dtmin = max(dtmin, 0.0)
            c = st["c"] + dtmin * st["p"]
            return st["told"] + dtmin, c.cpu().numpy()


def _rowcumsum(X: torch.Tensor) -> torch.Tensor:
    """Inclusive cumulative sum along the last dim of a (R x N) tensor as ONE device-wide
    scan of the flattened data minus each row's start offset.  torch's per-row scan runs
    one block per row, so with R = 2k ~ 20 rows it used ~20 blocks of the GPU (565 us per
    call at N = 2^20, against ~0.1 ms here); fp64, so the offsets cost no accuracy."""
    if X.dim() == 1 or X.shape[0] == 1:
        return torch.cumsum(X, -1)
    c = torch.cumsum(X.reshape(-1), 0).reshape(X.shape)
    off = torch.cat([torch.zeros(1, dtype=c.dtype, device=c.device), c[:-1, -1]])
    return c - off[:, None]


def _gram(A: torch.Tensor, chunk: int = 8192) -> torch.Tensor:
    """``A @ A.T`` for a short, very wide fp64 ``A`` (2k x K): a batched product over column
    chunks, summed.  A single GEMM with M = N = 2k and K ~ 1e6-1e7 runs a 128x128 tile
    with no split of K (5.4 ms measured at K ~ 5e6)."""
    R, K = A.shape
    if K <= 4 * chunk:
        return A @ A.T
    nc = -(-K // chunk)
    Ap = torch.zeros((R, nc * chunk), dtype=A.dtype, device=A.device)
    Ap[:, :K] = A
    X = Ap.view(R, nc, chunk).permute(1, 0, 2)          # (nc, R, chunk), strided view
    return torch.bmm(X, X.transpose(1, 2)).sum(0)


def _scan_batch(st, t, g, W, M, theta):
    """One batch of the Cauchy-point scan (sorted breakpoints ``t``, gradient entries
    ``g``, columns ``W`` (2k x N) = rows of ``[Y, theta S]`` at the breakpoints).  Returns
    ``(True, t*, c)`` when the minimiser lies in a segment of this batch, else advances
    ``st`` past it and returns ``(False, None, None)``.  The 2k-vectors are kept as
    (2k x N) so every prefix sum runs along the contiguous dimension."""
    N = t.numel()
    if N == 0:
        return False, None, None
    told0 = st["told"]
    prev = torch.cat([torch.full((1,), told0, dtype=torch.float64, device=t.device), t[:-1]])
    dt = t - prev
    gw = W * g[None, :]
    P = st["p"][:, None] + _rowcumsum(gw) - gw               # p before breakpoint i
    Mw = M @ W                                               # M w_i (M symmetric)
    wMp = (Mw * P).sum(0)
    wMw = (Mw * W).sum(0)
    dfpp = -theta * g * g - 2 * g * wMp - g * g * wMw
    fpp_b = st["fpp"] + torch.cumsum(dfpp, 0) - dfpp          # f'' at the start of segment i
    Cp = st["c"][:, None] + _rowcumsum(P * dt[None, :])     # c after breakpoint i
    wMc = (Mw * Cp).sum(0)
    dfp = dt * fpp_b + g * g - theta * t * g * g - g * wMc
    fp_b = st["fp"] + torch.cumsum(dfp, 0) - dfp              # f' at the start of segment i
    dtmin = torch.where(fpp_b > 0, -fp_b / fpp_b, torch.full_like(fp_b, math.inf))
    stop = dtmin < dt
    # ONE host copy: the first stop index (or -1), the end-of-batch state, and -- formed on
    # the device at that index, used only when it is >= 0 -- t* and c (three copies fewer
    # per Cauchy point than reading t[j-1], dtmin[j] and c back one by one)
    jt = torch.argmax(stop.to(torch.int8))
    first = torch.where(stop.any(), jt.to(torch.float64),
                        torch.full((), -1.0, dtype=torch.float64, device=t.device))
    told_t = torch.where(jt > 0, t[(jt - 1).clamp(min=0)],
                         torch.full((), told0, dtype=torch.float64, device=t.device))
    dtm_t = dtmin[jt].clamp(min=0.0)
    c_prev = torch.where(jt > 0, Cp[:, (jt - 1).clamp(min=0)], st["c"])
    c_t = c_prev + dtm_t * P[:, jt]
    tail = torch.cat([torch.stack([first, fp_b[-1] + dfp[-1], fpp_b[-1] + dfpp[-1], t[-1],
                                   told_t + dtm_t]), c_t]).cpu().numpy()
    j = int(tail[0])
    if j >= 0:
        return True, float(tail[4]), tail[5:]
    st["p"] = P[:, -1] + gw[:, -1]
    st["c"] = Cp[:, -1]
    st["fp"], st["fpp"], st["told"] = float(tail[1]), float(tail[2]), float(tail[3])
    return False, None, None


def _line_search(phi, f0, d0_box, a1, c1, c2, maxls):
    """Strong-Wolfe search on (0, 1] (bracketing + zoom); ``d0_box[0]`` is filled by the
    first evaluation (the directional derivative at 0 travels with it)."""
    alpha = a1
    fa, da = phi(alpha)
    d0 = d0_box[0]
    if d0 >= 0:
        return None
    a_prev, f_prev, dphi_prev = 0.0, f0, d0
    for i in range(maxls):
        if i > 0:
            fa, da = phi(alpha)
        if not np.isfinite(fa) or fa > f0 + c1 * alpha * d0 or (i > 0 and fa >= f_prev):
            return _zoom(phi, a_prev, alpha, f_prev, fa, dphi_prev, da, f0, d0, c1, c2, maxls)
        if abs(da) <= -c2 * d0:
            return alpha
        if da >= 0 or alpha >= 1.0:
            if da >= 0:
                return _zoom(phi, alpha, a_prev, fa, f_prev, da, dphi_prev, f0, d0, c1, c2, maxls)
            return alpha  # the step to the projected point: accept (sufficient decrease holds)
        a_prev, f_prev, dphi_prev = alpha, fa, da
        alpha = min(1.0, alpha * 2.0)
    return None


def run_lbfgsb_device(loss_and_grad_fn, params, maxsteps: int = 100, param_bounds=None,
                      randkey=None, comm=None, history: int = 10, **kw):
    """Device L-BFGS-B for a generic ``loss_and_grad_fn(params[, randkey])`` (replicated)."""
    from ..utils.random import init_randkey
    from ..utils.tensors import as_param_tensor
    x0 = as_param_tensor(params)
    lo, hi = bounds_arrays(param_bounds, x0.numel())
    fkw = {} if randkey is None else {"randkey": init_randkey(randkey)}
    obj = BoxObjective(loss_and_grad_fn, x0, comm=comm, **fkw)
    return lbfgsb_minimize(obj, lo, hi, maxiter=maxsteps, m=history, **kw)


def bounds_arrays(param_bounds, n: int):
    """``(lo, hi)`` float arrays (+-inf for open sides) from a reference-style spec
    ``(ndim, 2)`` with ``None`` entries, or ``(None, None)``."""
    if param_bounds is None:
        return None, None
    if isinstance(param_bounds, (np.ndarray, torch.Tensor)):
        b = np.asarray(param_bounds.detach().cpu() if isinstance(param_bounds, torch.Tensor)
                       else param_bounds, dtype=np.float64).reshape(n, 2)
        b = np.where(np.isnan(b), np.array([-np.inf, np.inf]), b)
        return b[:, 0].astype(np.float32), b[:, 1].astype(np.float32)
    lo = np.full(n, -np.inf)
    hi = np.full(n, np.inf)
    for i, b in enumerate(param_bounds):
        if b is None:
            continue
        a, c = b
        if a is not None:
            lo[i] = float(a)
        if c is not None:
            hi[i] = float(c)
    return lo.astype(np.float32), hi.astype(np.float32)


def lbfgsb_minimize(*args, **kwargs):
    """See ``_lbfgsb_minimize_impl``; runs with the BLAS pools limited to one thread (the host-side
    compact-form solves are tiny; a spinning BLAS pool would slow the CPU evaluations)."""
    from ..utils.hooks import driver_guard
    from ..utils.tensors import blas_single_thread
    obj = args[0] if args else kwargs.get("obj")
    with driver_guard(getattr(obj, "comm", None)), blas_single_thread():
        return _lbfgsb_minimize_impl(*args, **kwargs)


lbfgsb_minimize.__doc__ = _lbfgsb_minimize_impl.__doc__
