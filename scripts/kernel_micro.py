"""Per-kernel microbenchmark (HIP events on the engine stream) at ring 2^16."""
import os, sys, json
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'fhe-sorting_amd'))
import fhesort as F
ctx = F.Context(16, 39, 50, 60, 3, seed=1)
for name in ('ntt_fwd', 'ks_inner', 'modup_convert'):
    for limbs in (40, 20):
        r = F.time_kernel(ctx, name, limbs, iters=20)
        print(json.dumps(dict(kernel=name, limbs=limbs, avg_us=round(r['avg_ms'] * 1e3, 2),
                              GBps=round(r['bytes'] / r['avg_ms'] / 1e6, 1))), flush=True)
