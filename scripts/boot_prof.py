#!/usr/bin/env python3
"""Five bootstraps in config 4's context (ring 2^16, depth 40, scale 2^59, 4096
slots, levelBudget {5,5}) after one warm-up: a short program for rocprofv3."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'fhe-sorting_amd'))
import fhesort as F  # noqa: E402

ctx = F.Context(16, 40, 59, 60, 3, seed=5)
B = F.Bootstrapper(ctx, 4096, (5, 5))
x = ctx.encrypt(np.random.default_rng(1).uniform(0, 1, 4096), 4096, level=39)
B.bootstrap(x)
ctx.sync()
t = time.perf_counter()
for _ in range(5):
    y = B.bootstrap(x)
ctx.sync()
print(f'bootstrap {(time.perf_counter() - t) / 5 * 1e3:.2f} ms', flush=True)
