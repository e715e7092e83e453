"""A/B timing of the NTT row passes: DPP lane-swap (FHE_NTT_ROW_SHFL=1, the
default) vs the LDS-exchange passes (=0).  Runs itself once per setting in a
child process (the switch is read once per process) and prints one JSON line
per (setting, kernel, limbs)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'fhe-sorting_amd'))

if len(sys.argv) > 1 and sys.argv[1] == 'child':
    import fhesort as F
    ctx = F.Context(16, 39, 50, 60, 3, seed=1)
    for name in ('ntt_inv_row32', 'ntt_fwd_row32', 'ntt_inv_row', 'ntt_fwd_row', 'ntt_inv', 'ntt_fwd'):
        for limbs in (40, 14):
            r = F.time_kernel(ctx, name, limbs, iters=20)
            print(json.dumps(dict(shfl=os.environ.get('FHE_NTT_ROW_SHFL', '1'), kernel=name, limbs=limbs,
                                  avg_us=round(r['avg_ms'] * 1e3, 2),
                                  GBps=round(r['bytes'] / r['avg_ms'] / 1e6, 1))), flush=True)
else:
    for v in ('0', '1', '2'):
        env = dict(os.environ, FHE_NTT_ROW_SHFL=v)
        subprocess.run([sys.executable, os.path.abspath(__file__), 'child'], env=env, check=True)
