import os, sys, json
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'fhe-sorting_amd'))
import fhesort as F
ctx = F.Context(16, 39, 50, 60, 3, seed=1)
for spec in sys.argv[1:]:
    name, limbs = spec.split(':')
    r = F.time_kernel(ctx, name, int(limbs), iters=3)
    print(name, limbs, 'ok', r, flush=True)
