#!/usr/bin/env python3
"""Time each bootstrapping stage on one MI355X (config 4's context: ring 2^16,
depth 40, scale 2^59, 4096 slots, levelBudget {5,5})."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'fhe-sorting_amd'))
import fhesort as F  # noqa: E402

logN, s = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (16, 4096)
ctx = F.Context(logN, 40, 59, 60, 3, seed=5)
B = F.Bootstrapper(ctx, s, (5, 5))
x = ctx.encrypt(np.random.default_rng(1).uniform(0, 1, s), s, level=39)
last = ctx.mul_const_to(x, 2.0 ** -11, 40)


def tm(f, reps=5):
    f()
    ctx.sync()
    t = time.perf_counter()
    for _ in range(reps):
        r = f()
    ctx.sync()
    return r, (time.perf_counter() - t) / reps * 1e3


raised, t_raise = tm(lambda: B.mod_raise(last))
traced = raised
t_trace = 0.0
cts, t_cts = tm(lambda: B.coeffs_to_slots(raised))
em, t_em = tm(lambda: B.eval_mod(cts))
_, t_stc = tm(lambda: B.slots_to_coeffs(em))
_, t_all = tm(lambda: B.bootstrap(x))
ctx.reset_counters()
B.bootstrap(x)
print(json.dumps(dict(logN=logN, slots=s, ms=dict(mod_raise=round(t_raise, 2), coeffs_to_slots=round(t_cts, 2),
                                                  eval_mod=round(t_em, 2), slots_to_coeffs=round(t_stc, 2),
                                                  whole=round(t_all, 2)),
                      counters=ctx.counters())), flush=True)
