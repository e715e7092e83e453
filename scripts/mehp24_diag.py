"""MEHP24 diagnostics at ring 2^17 (engine only): error of several shapes."""
import sys, time
import numpy as np
sys.path.insert(0, 'fhe-sorting_amd')
import fhesort as F


def run(N, sub, depth, dnum, cfg, logN=17, scale=40):
    rots = F.mehp24_rotation_indices(N, sub or 256)
    ctx = F.Context(logN, depth, scale, 60, dnum, seed=N)
    ctx.gen_rotation_keys(rots)
    x = np.random.default_rng(N).permutation(N) / N
    slots = N * N if sub == 0 else sub * sub
    ct = ctx.encrypt(x, slots)
    dg_i = (int(np.log2(N)) + 1) // 2
    ctx.sync()
    t = time.time()
    out = ctx.mehp24_sort(ct, N, cfg, dg_i, 2, sub)
    ctx.sync()
    dt = time.time() - t
    y = ctx.decrypt(out)[:N]
    print(f'N={N} sub={sub} depth={depth} dnum={dnum} cfg={cfg}: {dt:.2f}s level {out.level} '
          f'err {np.max(np.abs(y - np.sort(x))):.3g}', flush=True)


for spec in sys.argv[1:]:
    N, sub, depth, dnum, n, dg, df = map(int, spec.split(','))
    run(N, sub, depth, dnum, (n, dg, df))
