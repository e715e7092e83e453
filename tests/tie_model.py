"""Plaintext model of the reference's DirectSort on inputs with ties (test
infrastructure; verdict r4 item 1).

DirectSort never special-cases equal values:
  * Comparison::compare (src/comparison.cpp:4-21) is (sign(a - b) + 1) / 2 and
    the composite sign polynomials are odd, so compare(x, x) = 1/2 exactly;
  * constructRank (src/sort_algo.h:368-506) sums compare(x_i, x_j) over j and
    subtracts 1/2 for the self comparison: r_i = #{x_j < x_i} + (m - 1) / 2 for a
    value of multiplicity m;
  * rotationIndexCheckN (src/sort_algo.h:652-750) weighs element i into output
    slot k by the doubled sinc f(t) = sinc(2N t) + sinc(2N (t + 1/2))
    (src/comparison.h:57-78) at t = (i - r_i - s) / 2N, s the checking-vector
    shift (generateCheckingVectorN, src/sort_algo.h:272-286) that the blind
    rotation (blindRotationOptN, src/sort_algo.h:561-584) turns into
    k = (i - s) mod N, so the weight is
        sinc(k - r_i) + sinc(k - r_i + N)   (k <= i)
        sinc(k - r_i) + sinc(k - r_i - N)   (k >  i).
With distinct values r_i is an integer and the weight is 1 at k = r_i and 0
elsewhere: a sort.  A value of odd multiplicity m has an integer rank, so all m
copies land in the ONE slot r_i (m x the value there, zeros in the other m - 1
slots of its run); an even multiplicity gives a half-integer rank and the copies
spread over every slot with sinc tails (+-0.64, -0.21, +0.13, ... of the value).

The sign is the reference's composite polynomial evaluated exactly
(compositeSign, src/sign.cpp:8-158: g3 / f3 of degree 7, g4 the degree-27
Chebyshev series, f4 of degree 15), so near-ties the polynomial cannot resolve
are modelled too.  The engine's decryption follows this model to CKKS
precision; the model is not an oracle of the words (the CPU oracle is)."""
import numpy as np
from numpy.polynomial import chebyshev as _cheb

_G3 = (4589 / 1024, -16577 / 1024, 25614 / 1024, -12860 / 1024)
_F3 = (35 / 16, -35 / 16, 21 / 16, -5 / 16)
_G4 = (0.0, 1.077117252745569, 0.0, -0.36166113998402755, 0.0, 0.2137420717859748,
       0.0, -0.15635204788780485, 0.0, 0.11749645501187332, 0.0, -0.10074154666447852,
       0.0, 0.08002086947825496, 0.0, -0.07533558758484624, 0.0, 0.059514472116534836,
       0.0, -0.06146663712787884, 0.0, 0.04570084927999001, 0.0, -0.05403683682999072,
       0.0, 0.03364293851188723, 0.0, -0.054459493266273494)
_F4 = (3.14208984375, -7.33154296875, 13.19677734375, -15.71044921875, 12.21923828125, -5.99853515625,
       1.69189453125, -0.20947265625)


def _odd(c, t):
    return sum(ci * t ** (2 * i + 1) for i, ci in enumerate(c))


def composite_sign(t, n, dg, df):
    g = (lambda v: _odd(_G3, v)) if n == 3 else (lambda v: _cheb.chebval(v, _G4))
    f = (lambda v: _odd(_F3, v)) if n == 3 else (lambda v: _odd(_F4, v))
    t = np.asarray(t, dtype=np.float64)
    for _ in range(dg):
        t = g(t)
    for _ in range(df):
        t = f(t)
    return t


def ranks(x, cfg):
    x = np.asarray(x, dtype=np.float64)
    c = (composite_sign(x[:, None] - x[None, :], *cfg) + 1.0) / 2.0
    return c.sum(axis=1) - 0.5


def direct_sort(x, cfg):
    """The reference DirectSort's output slots for input x (len N) in plaintext."""
    x = np.asarray(x, dtype=np.float64)
    N = len(x)
    r = ranks(x, cfg)
    k = np.arange(N)[None, :]
    d = k - r[:, None]
    w = np.sinc(d) + np.sinc(d + np.where(k > np.arange(N)[:, None], -N, N))
    return x @ w
