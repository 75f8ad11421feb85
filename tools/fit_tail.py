"""Fit the normal-tail polynomial of the SMF forward kernel (rsqrt basis).

Scaled coordinate w (exp(-z^2/2) = exp2(-w^2), see csrc/common.h kWScale).  The upper
tail Q(|z|) = erfc(a)/2 with a = |w| sqrt(ln 2).  The kernel forms

    s = w^2 + c,   g = exp2(-s),   t = rsqrt(s),   Q ~= P(t) * g

so s is one packed fma, g one v_exp and t one v_rsq; no |w| (the abs and add of the
reciprocal basis disappear) and P(t) = 2^c erfcx(a)/2 is smooth on t in (0, 1/sqrt(c)],
linear at t -> 0 (the far tail).  Two contracts, fitted as linear programs (minimax):

  absolute: max |Q_fit - Q| over all w (weight g), the float32-erf class (~1.2e-7)
  relative: max |Q_fit / Q - 1| for w <= WMAX, P(0) = 0 enforced

The fitted coefficients are rounded to float32 and re-checked by a float32 emulation of
the kernel's Horner evaluation (per-operation rounding; v_rsq / v_exp modelled as
correctly rounded).  Usage: python tools/fit_tail.py [--scan] [--mode absolute|relative]
[--c C] [--deg D]
"""
import argparse

import numpy as np
from scipy.optimize import linprog
from scipy.special import erfcx, erfc

LN2 = np.log(2.0)


def target(w):
    """Q(w) in the scaled coordinate (float64)."""
    return 0.5 * erfc(w * np.sqrt(LN2))


def fit(c, deg, mode, wmax=9.5, n=6000):
    # sample densely in w (uniform in w and in t), map to x = t*sqrt(c) in (0, 1]
    w = np.unique(np.concatenate([np.linspace(0, wmax, n), np.sqrt(1.0 / np.linspace(1e-4, 1, n) ** 2 - 1) * np.sqrt(c)]))
    w = w[(w >= 0) & (w <= wmax)]
    s = w * w + c
    x = np.sqrt(c / s)                       # in (0, 1]
    f = 2.0 ** c * 0.5 * erfcx(w * np.sqrt(LN2))  # P target: Q / exp2(-s)
    if mode == "absolute":
        wt = 2.0 ** (-s)                     # error in Q
        j0 = 0
    else:
        wt = 1.0 / f                         # relative error
        j0 = 1                               # P(0) = 0
    J = np.arange(j0, deg + 1)
    A = x[:, None] ** J[None, :]
    m = len(J)
    # variables: a_j (m), e ; minimize e s.t. |wt (A a - f)| <= e
    Aw = A * wt[:, None]
    fw = f * wt
    A_ub = np.block([[Aw, -np.ones((len(x), 1))], [-Aw, -np.ones((len(x), 1))]])
    b_ub = np.concatenate([fw, -fw])
    cost = np.zeros(m + 1)
    cost[-1] = 1
    r = linprog(cost, A_ub=A_ub, b_ub=b_ub, bounds=[(None, None)] * m + [(0, None)], method="highs")
    assert r.status == 0, r.message
    a = r.x[:m]
    # back to the t basis: P(t) = sum a_j (sqrt(c) t)^j
    coef = np.zeros(deg + 1)
    coef[J] = a * np.sqrt(c) ** J
    return coef, r.x[-1]


def f32(v):
    return np.asarray(v, dtype=np.float64).astype(np.float32).astype(np.float64)


def emulate(coef, c, w):
    """float32 emulation of the kernel: s = fma(w, w, c); t = rsq(s); g = exp2(-s);
    Horner fmas in t; Q = P * g."""
    cf = f32(coef)
    w = f32(w)
    s = f32(w * w + f32(c))
    t = f32(1.0 / np.sqrt(s))
    g = f32(2.0 ** (-s))
    p = np.full_like(w, cf[-1])
    for k in range(len(cf) - 2, -1, -1):
        p = f32(p * t + cf[k])
    return p * g


def check(coef, c, mode, wmax=9.5):
    w = np.linspace(0, 14, 400001)
    q = target(w)
    qf = emulate(coef, c, w)
    absmax = np.max(np.abs(qf - q))
    m = w <= wmax
    rel = np.max(np.abs(qf[m] / q[m] - 1))
    # the assembled CDF Phi = pos + sign*Q must stay monotone and inside [0, 1]
    ok = np.all(qf >= 0) and np.all(qf <= 0.5 + 1e-7) and np.all(np.diff(qf) <= 1e-7)
    return absmax, rel, ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="absolute", choices=["absolute", "relative"])
    ap.add_argument("--c", type=float, default=None)
    ap.add_argument("--deg", type=int, default=None)
    ap.add_argument("--scan", action="store_true")
    a = ap.parse_args()
    if a.scan:
        for deg in range(3, 9):
            for c in (0.25, 0.5, 0.75, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0):
                try:
                    coef, e = fit(c, deg, a.mode)
                except AssertionError:
                    continue
                am, rel, ok = check(coef, c, a.mode)
                print(f"deg {deg} c {c:5.2f}: lp {e:.2e}  f32 abs {am:.2e} rel(w<=9.5) {rel:.2e} ok={ok}")
        return
    coef, e = fit(a.c, a.deg, a.mode)
    am, rel, ok = check(coef, a.c, a.mode)
    print(f"lp error {e:.3e}; float32 abs {am:.3e} rel {rel:.3e} ok={ok}")
    for k in range(len(coef) - 1, -1, -1):
        print(f"  c{k} = {float(np.float32(coef[k])).hex()}f  ({coef[k]:.9g})")


if __name__ == "__main__":
    main()
