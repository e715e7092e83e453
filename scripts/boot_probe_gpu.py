"""Localise a bootstrap failure: run the stages one by one on a given context
(logN depth scale dnum slots budget input_level), printing after each."""
import faulthandler
import os
import sys

faulthandler.enable()
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'fhe-sorting_amd'))
import numpy as np  # noqa: E402

import fhesort as F  # noqa: E402

logN, depth, scale, dnum, s, be, bd, lvl = (int(a) for a in sys.argv[1:9])
ctx = F.Context(logN, depth, scale, 60, dnum, seed=77)
print('ctx', ctx.nq, ctx.K, ctx.alpha, flush=True)
B = F.Bootstrapper(ctx, s, (be, bd))
print('keys, depth', B.depth, flush=True)
x = ctx.encrypt([0.1, 0.2, 0.3, 0.4], s, level=lvl)
r = B.mod_raise(ctx.level_adjust(x, depth - 1)) if False else None
for st, name in ((4, 'mod_raise'),):
    try:
        y = B.bootstrap(ctx.level_adjust(x, depth), st)
        print(name, 'ok level', y.level, flush=True)
    except Exception as e:
        print(name, 'error', e, flush=True)
y = B.bootstrap(x)
print('bootstrap ok level', y.level, ctx.decrypt(y)[:4], flush=True)
