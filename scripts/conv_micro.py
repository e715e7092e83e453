"""Basis-conversion microbenchmark (round 6): HIP events on the engine stream
around `iters` launches of one conversion at ring 2^16, 40-bit scaling (the
bench context), for the limb counts given.  The kernel form is chosen by the
environment (FHE_MODDOWN_FP, FHE_MODUP_FP, ...), read once per process."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'fhe-sorting_amd'))
import fhesort as F  # noqa: E402

L = int(os.environ.get('CONV_L', '39'))
ctx = F.Context(16, L, 40, 60, 3, seed=1)
tag = os.environ.get('CONV_TAG', '')
for name in sys.argv[1].split(','):
    for limbs in [int(x) for x in sys.argv[2].split(',')]:
        r = F.time_kernel(ctx, name, limbs, iters=20)
        print(json.dumps(dict(tag=tag, kernel=name, limbs=limbs, avg_us=round(r['avg_ms'] * 1e3, 2),
                              hbm_frac=round(r['bytes'] / r['avg_ms'] / 1e9 / 8.0, 3))), flush=True)
