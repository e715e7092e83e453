#!/usr/bin/env python3
"""Bootstrap precision on one MI355X: ring 2^logN, depth 40, scale 2^59 (the
k-way context), slots s, level budget (be, bd), optional EvalMod parameters.
usage: boot_precision.py logN s be bd [K r degree correction_bits]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'fhe-sorting_amd'))
import fhesort as F  # noqa: E402

logN, s, be, bd = (int(a) for a in sys.argv[1:5])
K, r, deg, cb = (int(a) for a in sys.argv[5:9]) if len(sys.argv) >= 9 else (512, 6, 88, 11)
ctx = F.Context(logN, 40, 59, 60, 3, seed=77)
B = F.Bootstrapper(ctx, s, (be, bd), K=K, r=r, degree=deg, correction_bits=cb)
x = np.random.default_rng(s).uniform(0, 1, s)
errs = []
for lv in (39, 30):
    y = B.bootstrap(ctx.encrypt(x, s, level=lv))
    errs.append(float(np.max(np.abs(ctx.decrypt(y) - x))))
ctx.sync()
t0 = time.time()
for _ in range(5):
    y = B.bootstrap(ctx.encrypt(x, s, level=39))
ctx.sync()
print(json.dumps(dict(logN=logN, slots=s, budget=[be, bd], K=K, r=r, degree=deg, correction_bits=cb,
                      depth=B.depth, errs=errs,
                      ms_per_bootstrap=round((time.time() - t0) / 5 * 1e3, 2))), flush=True)
