"""GPU precision diagnostic: rank error, index-check error with exact ranks,
and end-to-end sort error for DirectSort, per scale size and ring.
usage: diag_precision.py N:scale_bits[:logN[:ps_split]] ...  (ps_split 1 = OpenFHE, 0 = power-of-two)"""
import os, sys, time, json
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'fhe-sorting_amd'))
import fhesort as F

def cfg_of(N):
    return (3, 2, 2) if N <= 16 else (3, 3, 2) if N <= 128 else (3, 4, 2) if N <= 512 else (3, 5, 2)

def run(N, sb, logN=16, split=1, cfg=None):
    depth, rots = F.size_parameters(N)
    cfg = cfg or cfg_of(N)
    c = F.Context(logN, depth, sb, 60, 3, seed=11, ps_split=split)
    c.gen_rotation_keys(rots)
    x = np.random.default_rng(20250704).permutation(N) / N
    ct = c.encrypt(x, N)
    exp = np.array([np.sum(x < v) for v in x], dtype=float)
    t = time.time()
    rank = c.direct_sort(ct, N, rots, cfg, mode=1)
    r = c.decrypt(rank)
    rk = c.encrypt(exp, N, level=rank.level)
    o1 = c.direct_sort(ct, N, rots, cfg, mode=2, rank=rk)
    o2 = c.direct_sort(ct, N, rots, cfg, mode=2, rank=rank)
    res = dict(N=N, scale_bits=sb, logN=logN, ps_split=split, cfg=cfg, rank_err=float(np.max(np.abs(r - exp))),
               check_exact_rank_err=float(np.max(np.abs(c.decrypt(o1) - np.sort(x)))),
               sort_err=float(np.max(np.abs(c.decrypt(o2) - np.sort(x)))), level=o2.level, depth=depth,
               secs=round(time.time() - t, 2))
    print(json.dumps(res), flush=True)
    c.close()

if __name__ == '__main__':
    for spec in sys.argv[1:]:
        f = [int(v) for v in spec.split(':')]
        run(f[0], f[1], f[2] if len(f) > 2 else 16, f[3] if len(f) > 3 else 1)
