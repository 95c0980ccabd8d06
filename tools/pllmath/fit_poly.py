#!/usr/bin/env python3
"""Near-minimax refit of the sin/cos kernels of pll_math.h with one coefficient fewer each.

sin r = r + r^3 P(z), cos r = 1 - z/2 + z^2 Q(z), z = r^2, |r| <= pi/4 (+ margin), with P, Q of
degree 4 (S1..S5, C1..C5), fitted by Lawson's iteratively re-weighted least squares on the
relative error of sin / cos (mpmath, 60 digits), then rounded to double; reports the maximum
relative error of the double-precision Estrin evaluation against mpmath.
  python tools/pllmath/fit_poly.py
"""
import mpmath as mp

mp.mp.dps = 60
R = mp.pi / 4 * (1 + mp.mpf(2) ** -20)
N = 400


def fit(kind):
    pts = [R * mp.cos(mp.pi * (i + 0.5) / (2 * N)) for i in range(N)]   # Chebyshev in r on (0, R]
    rows, rhs, wts = [], [], []
    for r in pts:
        z = r * r
        if kind == "sin":
            g = (mp.sin(r) - r) / (r * z)
            w = r * z / mp.sin(r)
        else:
            g = (mp.cos(r) - 1 + z / 2) / (z * z)
            w = z * z / mp.cos(r)
        rows.append([z ** k for k in range(5)])
        rhs.append(g)
        wts.append(w)
    lw = [mp.mpf(1) / N] * N
    coef = None
    for it in range(60):
        # weighted least squares: minimise sum lw_i * (w_i (A c - g))^2
        A = mp.matrix([[mp.sqrt(lw[i]) * wts[i] * rows[i][k] for k in range(5)] for i in range(N)])
        b = mp.matrix([mp.sqrt(lw[i]) * wts[i] * rhs[i] for i in range(N)])
        coef = mp.lu_solve(A.T * A, A.T * b)
        err = [abs(wts[i] * (sum(coef[k] * rows[i][k] for k in range(5)) - rhs[i])) for i in range(N)]
        s = sum(lw[i] * err[i] for i in range(N))
        lw = [lw[i] * err[i] / s for i in range(N)]
    return [coef[k] for k in range(5)], max(err)


def check(cs, cc, M=20000):
    import struct
    S = [float(c) for c in cs]
    C = [float(c) for c in cc]
    worst_s = worst_c = 0.0
    for i in range(M + 1):
        r = float(R * i / M) if i else 1e-9
        z = r * r
        z2 = z * z
        # Estrin as in pll_math.h
        sp = S[0] + z * S[1] + z2 * (S[2] + z * S[3]) + (z2 * z2) * S[4]
        sr = r + (r * z) * sp
        cp = C[0] + z * C[1] + z2 * (C[2] + z * C[3]) + (z2 * z2) * C[4]
        cr = (1.0 - 0.5 * z) + z2 * cp
        es = abs((mp.mpf(sr) - mp.sin(mp.mpf(r))) / mp.sin(mp.mpf(r)))
        ec = abs((mp.mpf(cr) - mp.cos(mp.mpf(r))) / mp.cos(mp.mpf(r)))
        worst_s, worst_c = max(worst_s, es), max(worst_c, ec)
    return worst_s, worst_c


if __name__ == "__main__":
    cs, es = fit("sin")
    cc, ec = fit("cos")
    print("sin: minimax rel err %.3e (2^%.2f)" % (float(es), float(mp.log(es, 2))))
    print("cos: minimax rel err %.3e (2^%.2f)" % (float(ec), float(mp.log(ec, 2))))
    for k, c in enumerate(cs):
        print("S%d = %r" % (k + 1, float(c)))
    for k, c in enumerate(cc):
        print("C%d = %r" % (k + 1, float(c)))
    ws, wc = check(cs, cc)
    print("double evaluation: sin rel err %.3e (2^%.2f), cos %.3e (2^%.2f)" %
          (float(ws), float(mp.log(ws, 2)), float(wc), float(mp.log(wc, 2))))
