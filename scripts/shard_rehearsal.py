"""Per-rank time of a sharded sort on one GPU: rank 0 of `world` with a no-op
all-reduce hook, i.e. the replicated work plus 1/world of the sharded batches --
the compute part of an N-GPU run (the collective itself excluded; the output of
this run is not a valid sort).  usage: shard_rehearsal.py [direct|mehp24] worlds..."""
import json, os, sys, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'fhe-sorting_amd'))
os.environ.setdefault('FHE_TIME_COLLECTIVES', '1')  # allreduce_ms beside the compute
import fhesort as F

kind = sys.argv[1]
worlds = [int(w) for w in sys.argv[2:]] or [1, 2, 4, 8]
import ctypes as C
_hip = C.CDLL('libamdhip64.so')
_hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
_last = {'hdr': None}


def noop(ptr, count, _user):
    """No exchange; a 4-word header (presence, level + 1, (level + 1)^2, limbs)
    with no local partial gets the one of the last partial seen (the partials
    of one phase share a level), so rank 0 proceeds as if another rank had
    contributed."""
    if count != 4:
        return
    h = (C.c_uint64 * 4)()
    _hip.hipMemcpy(h, C.cast(ptr, C.c_void_p), 32, 2)
    if h[0]:
        _last['hdr'] = tuple(h)
    elif _last['hdr']:
        for i in range(4):
            h[i] = _last['hdr'][i]
        _hip.hipMemcpy(C.cast(ptr, C.c_void_p), h, 32, 1)
if kind == 'direct':
    N = 1024
    depth, rots = F.size_parameters(N)
    ctx = F.Context(16, depth, 40, 60, 3, seed=1)  # the bench config: 40-bit scaling, OpenFHE PS split
    ctx.gen_rotation_keys(rots)
    x = np.random.default_rng(1).permutation(N) / N
    ct = ctx.encrypt(x, N)
    run = lambda sh: ctx.direct_sort(ct, N, rots, (3, 5, 2), shard=sh, allreduce=noop if sh[1] > 1 else None)
else:
    N = 4096
    p = F.mehp24_parameters(N)
    ctx = F.Context(p['log_ring'], p['depth'] + 1, p['scale_bits'], 60, p['dnum'], seed=1)
    ctx.gen_rotation_keys(p['rots'])
    x = np.random.default_rng(1).permutation(N) / N
    ct = ctx.encrypt_ext(x, p['sub'] * p['sub'])
    run = lambda sh: ctx.mehp24_sort(ct, N, p['cfg'], p['dg_i'], p['df_i'], p['sub'], shard=sh,
                                     allreduce=noop if sh[1] > 1 else None)
run((0, 1))  # warm: masks, pool
for w in worlds:
    lanes_list = [int(v) for v in os.environ.get('SHARD_LANES', '2,1' if kind == 'direct' else '1').split(',')]
    for lanes in lanes_list:
        ctx.set_sort_lanes(lanes)
        run((0, w))  # warm this shape (allocation pool)
        ctx.sync()
        t = time.perf_counter()
        run((0, w))
        ctx.sync()
        print(json.dumps({'kind': kind, 'world': w, 'lanes': lanes, 'rank0_s': round(time.perf_counter() - t, 4)}),
              flush=True)
clock = os.environ.get('SHARD_CLOCK')
if clock:  # per-kernel clock of rank 0 at the last world size, one lane
    ctx.set_sort_lanes(1)
    with F.KernelClock(ctx) as clk:
        run((0, worlds[-1]))
    with open(clock, 'w') as f:
        json.dump(clk.stats, f, indent=1)
