#!/usr/bin/env python3
"""Generate the scaled-sinc Chebyshev coefficient tables (selectCoefficients<N>())
used by the hybrid sort's index check for N < 256 (reference:
src/sort_algo.h:963-968) and by the older rotationIndexCheck.

Recipe restated from utils/generate_cheb_coeffs.cpp:11-51 and
Sinc<2N>::scaled_sinc (src/comparison.h:27-34):
  * f(x) = sin(pi 2N x) / (pi 2N x), f(0) = 1 (|x| < 1e-10)
  * Chebyshev interpolation at degree 13011 on [-1, 1] (OpenFHE
    EvalChebyshevCoefficients, as in gen_doubled_sinc.py)
  * even coefficients with |c| < 1e-6 and every odd coefficient are zeroed,
    trailing zeros (|c| < 1e-15) dropped.
Output: scaled_sinc_<N>.f64 (little-endian float64), read by the engine and
the CPU oracle.
"""
import os
import sys

import numpy as np

DEGREE = 13011
EVEN_THRESH = 1e-6
TRAIL_THRESH = 1e-15
SIZES = [4, 8, 16, 32, 64, 128]


def scaled_sinc(x, nn):
    out = np.ones_like(x)
    nz = np.abs(x) >= 1e-10
    out[nz] = np.sin(np.pi * nn * x[nz]) / (np.pi * nn * x[nz])
    return out


def coefficients(N):
    T = DEGREE + 1
    j = np.arange(T, dtype=np.float64)
    xs = np.cos(np.pi / T * (j + 0.5))
    f = scaled_sinc(xs, 2 * N)
    c = np.empty(T)
    for lo in range(0, T, 1024):
        i = np.arange(lo, min(T, lo + 1024), dtype=np.float64)[:, None]
        c[lo:lo + i.shape[0]] = (np.cos(np.pi / T * i * (j + 0.5)[None, :]) @ f)
    c *= 2.0 / T
    c[1::2] = 0.0
    c[np.abs(c) < EVEN_THRESH] = 0.0
    nz = np.nonzero(np.abs(c) >= TRAIL_THRESH)[0]
    return c[: nz[-1] + 1]


def main(outdir):
    for N in SIZES:
        c = coefficients(N)
        c.astype('<f8').tofile(os.path.join(outdir, f'scaled_sinc_{N}.f64'))
        print(N, len(c))


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.dirname(os.path.abspath(__file__)))
