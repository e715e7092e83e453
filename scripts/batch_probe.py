#!/usr/bin/env python3
"""Per-member cost of a relinearised product and a rotation, single vs stacked
batches, in config 4's context (ring 2^16, depth 40, scale 2^59): how much a
batch of 2 saves over two single ciphertexts."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'fhe-sorting_amd'))
import fhesort as F  # noqa: E402

ctx = F.Context(16, 40, 59, 60, 3, seed=5)
ctx.gen_rotation_keys([1])
rng = np.random.default_rng(1)
out = {}
for level in (5, 20, 32):
    cts = [ctx.encrypt(rng.uniform(-1, 1, 4096), 4096, level=level) for _ in range(4)]
    for bsz in (1, 2, 4):
        x = cts[0] if bsz == 1 else ctx.stack(cts[:bsz])

        def tm(f, reps=40):
            f()
            ctx.sync()
            t = time.perf_counter()
            for _ in range(reps):
                f()
            ctx.sync()
            return (time.perf_counter() - t) / reps * 1e3

        out[f'l{level}_b{bsz}'] = dict(mul_ms=round(tm(lambda: ctx.mul(x, x)), 3),
                                      rot_ms=round(tm(lambda: ctx.rotate(x, 1)), 3))
        print(level, bsz, out[f'l{level}_b{bsz}'], flush=True)
print(json.dumps(out))
