"""Forward NTT of 156 limbs (ring 2^16, ModUp shape at l=40) x20 through the
engine's time_kernel: a short program for rocprofv3 --pmc passes on k_ntt_*."""
import json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'fhe-sorting_amd'))
import fhesort as F
ctx = F.Context(16, 39, 50, 60, 3, seed=1)
r = F.time_kernel(ctx, 'ntt_fwd', 40, iters=20)
print(json.dumps(dict(avg_us=round(r['avg_ms'] * 1e3, 2), GBps=round(r['bytes'] / r['avg_ms'] / 1e6, 1))))
