#!/usr/bin/env python3
"""Generate the big-integer golden vectors under tests/golden/.

Everything here is computed from the mathematical definitions with Python
integers (no oracle code involved), so the fixtures pin the oracle's (and
through it the GPU engine's) conventions independently:

  ntt_golden.json        negacyclic NTT of a seeded vector, evaluated naively:
                         A[k] = a(psi^(2 brev(k) + 1)) mod q, plus the
                         negacyclic product a*b mod (X^n + 1, q)
  automorph_golden.json  coefficient-domain automorphism X -> X^g (with the
                         X^n = -1 sign flips) for a seeded vector
  sinc_golden.json       spot values of the doubled-sinc indicator
                         (src/comparison.h:57-78 with N -> 2N) on the lattice
                         k/(2N) used by rotationIndexCheckN

Run: python tests/golden/make_golden.py   (seconds)
"""
import json
import math
import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))


def is_prime(n):
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


def first_prime(bits, n):
    m2 = 2 * n
    c = ((1 << bits) - 1) // m2 * m2 + 1
    if c >= 1 << bits:
        c -= m2
    while not is_prime(c):
        c -= m2
    return c


def brev(x, bits):
    return int(format(x, f'0{bits}b')[::-1], 2) if bits else 0


def ntt_case(logN, seed):
    n = 1 << logN
    q = first_prime(60, n)
    g = 2
    while pow(g, (q - 1) // 2, q) != q - 1:
        g += 1
    psi = pow(g, (q - 1) // (2 * n), q)
    rng = random.Random(seed)
    a = [rng.randrange(q) for _ in range(n)]
    b = [rng.randrange(q) for _ in range(n)]
    A = []
    for k in range(n):
        root = pow(psi, 2 * brev(k, logN) + 1, q)
        acc, p = 0, 1
        for c in range(n):
            acc = (acc + a[c] * p) % q
            p = p * root % q
        A.append(acc)
    prod = [0] * n
    for i in range(n):
        for j in range(n):
            t = a[i] * b[j]
            if i + j < n:
                prod[i + j] = (prod[i + j] + t) % q
            else:
                prod[i + j - n] = (prod[i + j - n] - t) % q
    return dict(logN=logN, q=str(q), psi=str(psi), a=[str(v) for v in a], b=[str(v) for v in b],
                ntt_a=[str(v) for v in A], negacyclic_ab=[str(v) for v in prod])


def automorph_case(logN, k, seed):
    n = 1 << logN
    q = first_prime(60, n)
    g = pow(5, k % (n // 2), 2 * n)
    rng = random.Random(seed)
    a = [rng.randrange(q) for _ in range(n)]
    out = [0] * n
    for i in range(n):
        e = i * g % (2 * n)
        if e < n:
            out[e] = (out[e] + a[i]) % q
        else:
            out[e - n] = (out[e - n] - a[i]) % q
    return dict(logN=logN, k=k, galois=g, q=str(q), a=[str(v) for v in a], sigma_a=[str(v) for v in out])


def doubled_sinc(x, NN):
    def s(t):
        return 1.0 if abs(t) < 1e-10 else math.sin(math.pi * NN * t) / (math.pi * NN * t)
    return s(x) + s(x + 0.5)


def main():
    ntt = [ntt_case(4, 1), ntt_case(6, 2)]
    with open(os.path.join(HERE, 'ntt_golden.json'), 'w') as f:
        json.dump(ntt, f)
    aut = [automorph_case(5, k, 10 + k) for k in (1, 3, -1)]
    with open(os.path.join(HERE, 'automorph_golden.json'), 'w') as f:
        json.dump(aut, f)
    sinc = []
    for N in (8, 128):
        pts = [k / (2 * N) for k in range(-2 * N + 2, N)]
        sinc.append(dict(N=N, x=pts, f=[doubled_sinc(x, 2 * N) for x in pts]))
    with open(os.path.join(HERE, 'sinc_golden.json'), 'w') as f:
        json.dump(sinc, f)


if __name__ == '__main__':
    main()
