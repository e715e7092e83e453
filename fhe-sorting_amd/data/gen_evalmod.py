#!/usr/bin/env python3
"""Chebyshev coefficients of the bootstrapping EvalMod cosine.

CKKS bootstrapping (EvalBootstrap, called by the reference's k-way network at
src/k-way/EvalUtils.cpp:76 and by compositeSign's lazy bootstrap,
src/sign.cpp:164-170) removes the q0 * I(X) term of a mod-raised ciphertext
with a scaled sine: after CoeffsToSlots a slot holds u = t / (K q0), and

    g(u) = cos(2 pi (K u - 1/4) / 2^r)          on [-1, 1]

followed by r double-angle steps y <- 2 y^2 - 1 gives cos(2 pi (t/q0 - 1/4)) =
sin(2 pi t / q0).  This script writes the degree-d Chebyshev interpolant of g
in the evaluator's convention (p = c0/2 + sum_{i>=1} c_i T_i, as OpenFHE's
EvalChebyshevSeriesPS), so c0 is stored doubled.

The engine (csrc/algo/bootstrap.cpp) and the CPU oracle (oracle/oracle_boot.cpp)
both read the same file, so their plaintext constants agree bit for bit.

  K = 512 bounds |I| for a uniform-ternary secret (std of I ~ sqrt(h/12),
  h ~ 2n/3: about 60 at n = 2^16, max over the coefficients < 300);
  r = 6, d = 88: max |p - g| ~ 2e-13 on [-1, 1] (fp64 floor), 7 levels for the
  series (OpenFHE's PS depth band 60..119) + 6 for the double angles.

Output: evalmod_k512r6_88.f64 (89 little-endian doubles) next to this script.
"""
import os
import sys

import numpy as np
from numpy.polynomial import chebyshev as C


def coefficients(K=512, r=6, d=88):
    f = lambda u: np.cos(2.0 * np.pi * (K * u - 0.25) / 2.0 ** r)
    a = C.chebinterpolate(f, d)
    u = np.linspace(-1, 1, 200001)
    err = float(np.max(np.abs(C.chebval(u, a) - f(u))))
    c = a.copy()
    c[0] *= 2.0
    return c, err


def main():
    K, r, d = (int(x) for x in (sys.argv[1:4] if len(sys.argv) >= 4 else (512, 6, 88)))
    c, err = coefficients(K, r, d)
    here = os.path.dirname(os.path.abspath(__file__))
    path = os.path.join(here, f'evalmod_k{K}r{r}_{d}.f64')
    c.astype('<f8').tofile(path)
    print(f'{path}: {len(c)} coefficients, max interpolation error {err:.3e}')


if __name__ == '__main__':
    main()
