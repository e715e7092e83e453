"""MEHP24 sortLargeArrayFG / sortFG on one GPU at the reference's parameters
(ring 2^17, scale 2^40, tests/mehp24/Mehp24SortTest.cpp:26-143): wall time,
HMult count, max error vs np.sort, output level.  usage: mehp24_run.py N [depth]"""
import json, os, sys, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'fhe-sorting_amd'))
import fhesort as F

N = int(sys.argv[1])
if N <= 2048:
    p = F.mehp24_parameters(N)
else:  # beyond the reference table: same Cfg / dg_i rule, depth from argv
    p = dict(F.mehp24_parameters(2048))
    p['dg_i'] = (int(np.log2(N)) + 1) // 2
    p['rots'] = F.mehp24_rotation_indices(N, 256)
if len(sys.argv) > 2:
    p['depth'] = int(sys.argv[2])
levels = p['depth'] + 1
dnum = p['dnum']
t0 = time.time()
ctx = F.Context(p['log_ring'], levels, p['scale_bits'], 60, dnum, seed=N)
ctx.gen_rotation_keys(p['rots'])
x = np.random.default_rng(N).permutation(N) / N
slots = min(N * N, 1 << (p['log_ring'] - 1))
ct = ctx.encrypt_ext(x, slots)
ctx.sync()
setup = time.time() - t0
print(json.dumps({'N': N, 'setup_s': round(setup, 1), 'rots': len(p['rots']), 'depth': p['depth'], 'dnum': dnum}),
      flush=True)
ctx.reset_counters()
t = time.perf_counter()
out = ctx.mehp24_sort(ct, N, p['cfg'], p['dg_i'], p['df_i'], p['sub'])
ctx.sync()
dt = time.perf_counter() - t
for rep in range(int(os.environ.get('MEHP24_REPEAT', '1')) - 1):  # warm runs (pool cache populated)
    print(json.dumps({'pool': ctx.pool_stats()}), flush=True)
    t = time.perf_counter()
    out = ctx.mehp24_sort(ct, N, p['cfg'], p['dg_i'], p['df_i'], p['sub'])
    ctx.sync()
    dt = time.perf_counter() - t
    print(json.dumps({'repeat': rep + 1, 'sort_s': round(dt, 3)}), flush=True)
clock = os.environ.get('MEHP24_CLOCK')
if clock:  # a second, instrumented sort: per-kernel time
    print(json.dumps({'pool_after_first': ctx.pool_stats()}), flush=True)
    ctx.pool_trim()
    with F.KernelClock(ctx) as clk:
        ctx.mehp24_sort(ct, N, p['cfg'], p['dg_i'], p['df_i'], p['sub'])
    with open(clock, 'w') as f:
        json.dump(clk.stats, f, indent=1)
c = ctx.counters()
y = ctx.decrypt(out)[:N]
print(json.dumps({'N': N, 'sort_s': round(dt, 3), 'hmult': c['hmult'], 'keyswitch': c['keyswitch'],
                  'hmult_per_s': round(c['hmult'] / dt, 1), 'max_err': float(np.max(np.abs(y - np.sort(x)))),
                  'out_level': out.level, 'levels': levels,
                  'hbm_peak_gb': round(ctx.pool_stats()['peak'] / 1e9, 1)}), flush=True)
