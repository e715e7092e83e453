#!/usr/bin/env python3
"""Plaintext noise model of the two Paterson-Stockmeyer splits for the
doubled-sinc index check.

Both evaluators run on float64 slot values over the x grid the reference's
rotationIndexCheckN evaluates (x = j/(2N), j in [-(2N-2), N-1],
src/sort_algo.h:719-728), and add independent N(0, sigma^2) noise to the
output of every rescaled operation (products, ct x const, linear sums) —
the CKKS rescale/key-switch noise in slot units.  sigma = 0 reproduces the
plain polynomial (checked against numpy's chebval).

  * "engine": this engine's split (fhesort.cpp PSEval: power-of-two giant
    steps T_G, p = q T_G + r with T_{G+j} = 2 T_G T_j - T_{G-j}).
  * "openfhe": OpenFHE's EvalChebyshevSeriesPS / InnerEvalChebyshevPS with
    ComputeDegreesPS and LongDivisionChebyshev, restated in
    oracle/oracle_core.cpp (ps_openfhe) — k*(2^m - 1) padding with a monic
    T term, long division by T_{k 2^(m-1)}, the r - T_{k(2^(m-1)-1)} / q
    second division, and the final subtraction of T_{k(2^m - 1)}.

usage: ps_noise_model.py [N ...]   (prints one JSON line per N x split x sigma)
"""
import json
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(os.path.dirname(HERE), 'fhe-sorting_amd', 'data')


def coeffs(N):
    return np.fromfile(os.path.join(DATA, f'doubled_sinc_{N}.f64'), dtype='<f8')


class Noisy:
    """slot values of a batch of trials; every rescaled op adds sigma noise"""

    def __init__(self, sigma, rng, shape):
        self.sigma, self.rng, self.shape = sigma, rng, shape
        self.rescales = 0

    def noise(self, v):
        self.rescales += 1
        if self.sigma == 0:
            return v
        return v + self.rng.normal(0.0, self.sigma, self.shape)


def degree(c):
    nz = np.nonzero(np.asarray(c) != 0.0)[0]
    return int(nz[-1]) if len(nz) else 0


# ------------------------------------------------------------------ engine split
def ceil_log2(x):
    r = 0
    while (1 << r) < x:
        r += 1
    return r


def engine_eval(c, x, nz: Noisy, stats):
    s = np.array(c, dtype=np.float64)
    s[0] /= 2.0
    d = len(s) - 1
    D = max(1, ceil_log2(d + 1))
    bmax = (1 << D) - d
    lim = math.sqrt(2.0 * d)
    B = 1
    while B * 2 <= bmax and B * 2 <= lim:
        B *= 2
    beta = ceil_log2(B) + 1
    T = {1: x}
    for i in range(2, B + 1):
        a = 1 << (ceil_log2(i) - 1)
        b = i - a
        if a == b:
            t = nz.noise(T[a] * T[a])
            t = 2 * t - 1.0
        else:
            t = nz.noise(T[a] * T[b])
            t = 2 * t - T[a - b]
        T[i] = t

    def giant(G):
        if G in T:
            return T[G]
        h = giant(G // 2)
        T[G] = 2 * nz.noise(h * h) - 1.0
        return T[G]

    def split(a):
        d = len(a) - 1
        Dpp = beta + 1
        while (1 << Dpp) - B < d:
            Dpp += 1
        G = 1 << (Dpp - 1)
        while G > d:
            G >>= 1
        q = np.zeros(d - G + 1)
        r = np.array(a[:G], dtype=np.float64)
        q[0] = a[G]
        for j in range(1, d - G + 1):
            q[j] = 2.0 * a[G + j]
            r[G - j] -= a[G + j]
        return q, r, G

    def trim(a):
        a = np.array(a, dtype=np.float64)
        n = degree(a)
        return a[: n + 1]

    def leaf(a):
        acc = 0.0
        for i in range(1, len(a)):
            if a[i] != 0.0:
                acc = acc + a[i] * T[i]
        return nz.noise(acc) + a[0] if len(a) > 1 else a[0] + 0 * x

    def ev(a, depth):
        a = trim(a)
        d = len(a) - 1
        if d <= B:
            return leaf(a)
        q, r, G = split(a)
        stats.setdefault('q_max', []).append((depth, float(np.max(np.abs(q)))))
        qv = ev(q, depth + 1)
        r = trim(r)
        stats.setdefault('qval_max', []).append((depth, float(np.max(np.abs(qv)))))
        if len(r) == 1 and r[0] == 0.0:
            return nz.noise(qv * giant(G))
        if 1 <= len(r) - 1 <= B:  # folded remainder (mul_add_raw): one rescale
            raw = sum(r[i] * T[i] for i in range(1, len(r)) if r[i] != 0.0)
            return nz.noise(qv * giant(G) + raw) + r[0]
        return nz.noise(qv * giant(G)) + ev(r, depth)

    return ev(s, 0)


# ----------------------------------------------------------------- OpenFHE split
def compute_degrees_ps(n):
    """OpenFHE ComputeDegreesPS (ckksrns-utils.cpp): argmin over (k, m) of
    k + 2m + 2^(m-1) - 4 with k (2^m - 1) > n and |floor(log2 k) - sqn2| <= 1"""
    sqn2 = math.floor(math.log2(math.sqrt(n // 2)))
    best = None
    for k in range(1, n + 1):
        mmax = math.ceil(math.log2(n // k) + 1) + 1 if n // k > 0 else 1
        for m in range(1, mmax + 1):
            if n - k * ((1 << m) - 1) < 0 and abs(math.floor(math.log2(k)) - sqn2) <= 1:
                mult = k + 2 * m + (1 << (m - 1)) - 4
                if best is None or mult < best[0]:
                    best = (mult, k, m)
    return best[1], best[2]


def long_division_chebyshev(f, g):
    """OpenFHE LongDivisionChebyshev; polynomials in the c0/2 convention"""
    f = list(map(float, f))
    g = list(map(float, g))
    n, k = degree(f), degree(g)
    assert n == len(f) - 1 and k == len(g) - 1
    r = list(f)
    if n - k >= 0:
        q = [0.0] * (n - k + 1)
        while n - k > 0:
            q[n - k] = 2 * r[-1]
            if g[k] != 1.0:
                q[n - k] /= g[-1]
            d = [0.0] * (n + 1)
            if k == n - k:
                d[0] = 2 * g[n - k]
                for i in range(1, 2 * k + 1):
                    d[i] = g[abs(n - k - i)]
            elif k > n - k:
                d[0] = 2 * g[n - k]
                for i in range(1, k - (n - k) + 1):
                    d[i] = g[abs(n - k - i)] + g[n - k + i]
                for i in range(k - (n - k) + 1, n + 1):
                    d[i] = g[abs(i - n + k)]
            else:
                d[n - k] = g[0]
                for i in range(n - 2 * k, n + 1):
                    if i != n - k:
                        d[i] = g[abs(i - n + k)]
            if r[-1] != 1.0:
                d = [v * r[-1] for v in d]
            if g[-1] != 1.0:
                d = [v / g[-1] for v in d]
            r = [a - b for a, b in zip(r, d)]
            if len(r) > 1:
                n_old, n = n, degree(r)
                r = r[: n + 1]
                if n >= n_old:  # a non-finite or non-cancelling leading term: no progress
                    raise ArithmeticError('long_division_chebyshev: leading term did not cancel')
        if n == k:
            q[0] = r[-1]
            if g[-1] != 1.0:
                q[0] /= g[-1]
            d = list(g)
            if r[-1] != 1.0:
                d = [v * r[-1] for v in d]
            if g[-1] != 1.0:
                d = [v / g[-1] for v in d]
            r = [a - b for a, b in zip(r, d)]
            if len(r) > 1:
                n = degree(r)
                r = r[: n + 1]
        q[0] *= 2
    else:
        q = [0.0]
    return q, r


def openfhe_eval(c, x, nz: Noisy, stats):
    f2 = list(map(float, c))
    n = degree(f2)
    f2 = f2[: n + 1]
    k, m = compute_degrees_ps(n)
    stats['k'], stats['m'] = k, m
    T = [None] * k
    T[0] = x
    for i in range(2, k + 1):
        if not (i & (i - 1)):
            T[i - 1] = 2 * nz.noise(T[i // 2 - 1] ** 2) - 1.0
        elif i % 2 == 1:
            T[i - 1] = 2 * nz.noise(T[i // 2 - 1] * T[i // 2]) - T[0]
        else:
            T[i - 1] = 2 * nz.noise(T[i // 2 - 1] ** 2) - 1.0
    # AdjustLevelsAndDepthInPlace: T[0..k-2] brought to T[k-1]'s level (a
    # level-adjusting constant product for those that are below it)
    for i in range(k - 1):
        if ceil_log2(i + 1) < ceil_log2(k):
            T[i] = nz.noise(T[i])
    T2 = [T[-1]]
    for i in range(1, m):
        T2.append(2 * nz.noise(T2[-1] ** 2) - 1.0)
    T2km1 = T2[0]
    for i in range(1, m):
        T2km1 = 2 * nz.noise(T2km1 * T2[i]) - T2[0]

    def linear(w, leading=None):
        # EvalLinearWSumMutable over T[0..len(w)-1], one rescale
        acc = 0.0
        for i, wi in enumerate(w):
            if wi != 0.0:
                acc = acc + wi * T[i]
        return nz.noise(acc)

    def inner(coefficients, mm, depth, top):
        k2m2k = k * (1 << (mm - 1)) - k
        Tkm = [0.0] * (k2m2k + k + 1)
        Tkm[-1] = 1.0
        q, r = long_division_chebyshev(coefficients, Tkm)
        stats.setdefault('q_max', []).append((depth, float(np.max(np.abs(q)))))
        r2 = list(r)
        if k2m2k - degree(r) <= 0:
            r2[k2m2k] -= 1
            r2 = r2[: degree(r2) + 1]
        else:
            r2 = r2 + [0.0] * (k2m2k + 1 - len(r2))
            r2 = r2[: k2m2k + 1]
            r2[-1] = -1.0
        cq, cr = long_division_chebyshev(r2, q)
        stats.setdefault('c_max', []).append((depth, float(np.max(np.abs(cq)))))
        s2 = list(cr) + [0.0] * max(0, k2m2k + 1 - len(cr))
        s2 = s2[: k2m2k + 1]
        s2[-1] = 1.0
        dc = degree(cq)
        cu = None
        if dc >= 1:
            if dc == 1:
                cu = nz.noise(cq[1] * T[0]) if cq[1] != 1 else T[0]
            else:
                cu = linear([cq[i + 1] for i in range(dc)])
            cu = cu + cq[0] / 2
        # q
        if degree(q) > k:
            qu = inner(q, mm - 1, depth + 1, False)
        else:
            qc = list(q) + [0.0] * max(0, k - len(q))
            qc = qc[:k]
            if degree(qc) > 0:
                qu = linear([q[i + 1] for i in range(degree(qc))])
                if top:
                    qu = qu + 2 * T[k - 1]
                else:
                    s = T[k - 1]
                    for _ in range(int(math.log2(q[-1]))):
                        s = s + s
                    qu = qu + s
            else:
                if top:
                    qu = T[k - 1]
                    for _ in range(1, int(q[-1])):
                        qu = qu + T[k - 1]
                else:
                    s = T[k - 1]
                    for _ in range(int(math.log2(q[-1]))):
                        s = s + s
                    qu = s
            qu = qu + q[0] / 2
        stats.setdefault('qval_max', []).append((depth, float(np.max(np.abs(qu)))))
        # s
        if degree(s2) > k:
            su = inner(s2, mm - 1, depth + 1, False)
        else:
            sc = s2[:k] + [0.0] * max(0, k - len(s2))
            if degree(sc) > 0:
                su = linear([s2[i + 1] for i in range(degree(sc))]) + T[k - 1]
            else:
                su = T[k - 1]
            su = su + s2[0] / 2
        res = (T2[mm - 1] + cu) if cu is not None else (T2[mm - 1] + cq[0] / 2)
        res = nz.noise(res * qu)
        res = res + su
        return res

    k2m2k = k * (1 << (m - 1)) - k
    f2 = f2 + [0.0] * (2 * k2m2k + k + 1 - len(f2))
    f2[-1] = 1.0
    res = inner(f2, m, 0, True)
    return res - T2km1


def run(N, split, sigma, trials, seed=1):
    c = coeffs(N)
    j = np.arange(-(2 * N - 2), N, dtype=np.float64)
    x0 = j / (2 * N)
    rng = np.random.default_rng(seed)
    shape = (trials, len(x0))
    nz = Noisy(sigma, rng, shape)
    x = x0[None, :] + (rng.normal(0, sigma, shape) if sigma else 0.0)
    stats = {}
    out = (engine_eval if split == 'engine' else openfhe_eval)(c, x, nz, stats)
    exact = np.polynomial.chebyshev.chebval(x0, np.concatenate([[c[0] / 2], c[1:]]))
    err = np.abs(out - exact[None, :])
    res = dict(N=N, split=split, sigma=sigma, trials=trials, max_err=float(err.max()),
               rms_err=float(np.sqrt(np.mean(err ** 2))), rescales=nz.rescales // max(1, 1))
    for key in ('k', 'm'):
        if key in stats:
            res[key] = stats[key]
    for key in ('q_max', 'c_max', 'qval_max'):
        if key in stats:
            by = {}
            for dpt, v in stats[key]:
                by[dpt] = max(by.get(dpt, 0.0), v)
            res[key + '_by_level'] = {str(k): float(f'{v:.4g}') for k, v in sorted(by.items())}
    return res


if __name__ == '__main__':
    sizes = [int(a) for a in sys.argv[1:]] or [128, 256, 512, 1024]
    for N in sizes:
        for split in ('engine', 'openfhe'):
            r0 = run(N, split, 0.0, 1)
            print(json.dumps(r0), flush=True)
            for sigma in (2.0 ** -26, 2.0 ** -36):
                print(json.dumps(run(N, split, sigma, 4)), flush=True)
