"""Host check of the fp64 epilogue of the folded-constant MFMA sums
(kernels.hip fold_rows2_fp; DESIGN.md §5 "Folded-constant leaf sums").

The kernel folds eight int32 MFMA rows v_0..v_7 (|v_b| <= 448 * 2^14: 56 sources x
8 bytes of magnitude <= 128 times balanced digits <= 128) into
V = L0 + 2^32 L1 with L = v_0 + 2^8 v_1 + 2^16 (v_2 + 2^8 v_3), and reduces V + a
(a < q) modulo a prime q < 2^41 in fp64:
  b = L1 * 2^32 (exact), h = rint(b / q), r1 = fma(-h, q, b) (exact: |r1| < 1.5 q),
  t = r1 + L0 + a (an exact integer < 2^49), h2 = rint(t / q), r = fma(-h2, q, t),
  r += q if r < 0.
An fma whose exact result is representable returns it exactly, so the fmas are
modelled by exact integer arithmetic plus a representability assertion; the
roundings (the two products by 1/q and rint, round-half-even) are numpy's doubles.
Test infrastructure only; no GPU."""
import random

import numpy as np

VMAX = 448 * 2 ** 14


def _is_prime(n):
    if n < 2:
        return False
    for p in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for a in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def _fold_fp(v0, v1, q, a):
    p0 = int(np.int32(v0[0] + (v0[1] << 8)))
    q0 = int(np.int32(v0[2] + (v0[3] << 8)))
    p1 = int(np.int32(v1[0] + (v1[1] << 8)))
    q1 = int(np.int32(v1[2] + (v1[3] << 8)))
    L0 = np.float64(p0) + np.float64(q0) * 65536.0
    L1 = np.float64(p1) + np.float64(q1) * 65536.0
    assert int(L0) == p0 + q0 * 65536 and int(L1) == p1 + q1 * 65536  # exact
    qd = np.float64(q)
    qi = np.float64(1.0) / qd
    b = L1 * np.float64(4294967296.0)
    assert int(b) == int(L1) << 32  # exact power-of-two scaling
    h = np.rint(b * qi)
    r1 = int(b) - int(h) * q  # fma(-h, q, b)
    assert abs(r1) < 1.5 * q and float(r1) == r1
    t = np.float64(r1) + L0 + np.float64(a)
    assert int(t) == r1 + int(L0) + a  # exact
    h2 = np.rint(t * qi)
    r = int(t) - int(h2) * q  # fma(-h2, q, t)
    assert abs(r) <= q // 2 + 1
    return r + q if r < 0 else r


def test_fold_rows2_fp_is_the_exact_residue():
    rng = random.Random(20251018)
    primes = []
    while len(primes) < 24:
        bits = rng.choice((33, 36, 39, 40, 41))
        q = rng.randrange(2 ** (bits - 1), 2 ** bits) | 1
        if q < 2 ** 41 and _is_prime(q):
            primes.append(q)
    for trial in range(20000):
        q = primes[trial % len(primes)]
        if trial % 5 == 0:
            v0, v1 = [VMAX] * 4, [VMAX] * 4
        elif trial % 5 == 1:
            v0, v1 = [-VMAX] * 4, [-VMAX] * 4
        elif trial % 5 == 2:
            v0, v1 = [VMAX, -VMAX] * 2, [-VMAX, VMAX] * 2
        else:
            v0 = [rng.randint(-VMAX, VMAX) for _ in range(4)]
            v1 = [rng.randint(-VMAX, VMAX) for _ in range(4)]
        a = rng.randrange(q)
        L0 = v0[0] + (v0[1] << 8) + ((v0[2] + (v0[3] << 8)) << 16)
        L1 = v1[0] + (v1[1] << 8) + ((v1[2] + (v1[3] << 8)) << 16)
        assert _fold_fp(v0, v1, q, a) == (L0 + (L1 << 32) + a) % q
