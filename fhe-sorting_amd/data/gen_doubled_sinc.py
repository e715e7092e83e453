#!/usr/bin/env python3
"""Generate the doubled-sinc Chebyshev coefficient tables used by
rotationIndexCheckN (reference: src/sort_algo.h:725-728).

Recipe restated from utils/generate_cheb_doubled_coeffs.cpp:11-36 and
Sinc<2N>::doubled_sinc (src/comparison.h:57-78):
  * f(x) = sinc(2N x) + sinc(2N (x + 1/2)),  sinc(t) = sin(pi t)/(pi t), sinc(0)=1
  * Chebyshev interpolation at degree 13011 on [-1, 1] (OpenFHE
    EvalChebyshevCoefficients: T = degree+1 nodes cos(pi (j+1/2)/T),
    c_i = 2/T * sum_j f(x_j) cos(pi i (j+1/2)/T))
  * coefficients with |c| < 1e-8 are zeroed, trailing zeros dropped.
Output: doubled_sinc_<N>.f64 (little-endian float64), read by both the
engine (fhe-sorting_amd) and the CPU oracle so they evaluate identical
polynomials.
"""
import os
import sys

import numpy as np

DEGREE = 13011
THRESH = 1e-8
SIZES = [4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048]


def doubled_sinc(x, nn):
    def s(t):
        out = np.ones_like(t)
        nz = np.abs(t) >= 1e-10
        out[nz] = np.sin(np.pi * nn * t[nz]) / (np.pi * nn * t[nz])
        return out
    return s(x) + s(x + 0.5)


def coefficients(N):
    T = DEGREE + 1
    j = np.arange(T, dtype=np.float64)
    xs = np.cos(np.pi / T * (j + 0.5))
    f = doubled_sinc(xs, 2 * N)
    c = np.empty(T)
    for lo in range(0, T, 1024):
        i = np.arange(lo, min(T, lo + 1024), dtype=np.float64)[:, None]
        c[lo:lo + i.shape[0]] = (np.cos(np.pi / T * i * (j + 0.5)[None, :]) @ f)
    c *= 2.0 / T
    c[np.abs(c) < THRESH] = 0.0
    nz = np.nonzero(c)[0]
    return c[: nz[-1] + 1]


def main(outdir):
    for N in SIZES:
        c = coefficients(N)
        c.astype('<f8').tofile(os.path.join(outdir, f'doubled_sinc_{N}.f64'))
        print(N, len(c))


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.dirname(os.path.abspath(__file__)))
