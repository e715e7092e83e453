#!/usr/bin/env python3
"""k-way sort with bootstrapping on one MI355X (BASELINE config 4 shape).

KWaySort235Test's context (tests/k-way/KWaySort235Test.cpp:18-51,
src/kway_adapter.h:41-63): scale 2^59, first modulus 60 bits, depth 40,
levelBudget {4,4} (N <= 128) or {5,5}, CompositeSign(3, d_f, d_g) in the test's
argument order, rotations +-2^i < N plus the bootstrap keys.
usage: kway_boot_run.py k M [logN] [d_g]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'fhe-sorting_amd'))
import fhesort as F  # noqa: E402


def main():
    k, M = int(sys.argv[1]), int(sys.argv[2])
    logN = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    dgk = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    N = k ** M
    s = 1
    while s < N:
        s *= 2
    budget = (4, 4) if N <= 128 else (5, 5)
    t0 = time.time()
    ctx = F.Context(logN, 40, 59, 60, 3, seed=2025)
    B = F.Bootstrapper(ctx, s, budget)
    ctx.gen_rotation_keys(F.kway_rotation_indices(N))
    t1 = time.time()
    x = np.random.default_rng(N).permutation(N) * (1 - 1e-8) / N
    ct = ctx.encrypt(x, s)
    ctx.reset_counters()
    ctx.sync()
    t2 = time.time()
    out = ctx.kway_sort(ct, k, M, (3, 2, dgk), boot=B)
    ctx.sync()
    t3 = time.time()
    c = ctx.counters()
    err = float(np.max(np.abs(ctx.decrypt(out)[:N] - np.sort(x))))
    # one bootstrap on its own
    y = ctx.encrypt(x, s, level=39)
    ctx.sync()
    t4 = time.time()
    B.bootstrap(y)
    ctx.sync()
    t5 = time.time()
    print(json.dumps(dict(k=k, M=M, N=N, logN=logN, slots=s, budget=budget, boot_depth=B.depth,
                          boot_keys=len(B.rotations()) + 1, key_GB=round(ctx.key_bytes() / 2**30, 2),
                          setup_s=round(t1 - t0, 1), sort_s=round(t3 - t2, 2), one_bootstrap_s=round(t5 - t4, 3),
                          checklevel_bootstraps=ctx.kway_bootstraps, counters=c, max_abs_err=err,
                          out_level=out.level)), flush=True)


if __name__ == '__main__':
    main()
