"""sort_hybrid on the GPU engine: bit-exact with the CPU oracle at test sizes
(identical keys) on every mask path (scaled-sinc PS, indicator (3,4,2) and
(3,5,2), two blocks), stacked and unstacked, sharded over two ranks; and the
reference test's own property (decrypted output == sorted input within 0.01,
output level == multDepth; tests/DirectSortHTest.cpp:181-221) at its
parameters (ring 2^17, its depth / rotation table) for N = 256 and 512.

All calls go through the C ABI (include/fhe_gpu.h) via fhesort.py.
"""
import numpy as np
import pytest

import fhesort as F
import pyoracle as O
from test_hybrid import REF_DEPTH, cfg_of, hybrid_rotations

pytestmark = pytest.mark.gpu


def same(gct, oct_):
    gi, oi = gct.info(), oct_.info()
    assert (gi['level'], gi['slots'], gi['limbs'], gi['scale']) == (oi['level'], oi['slots'], oi['limbs'], oi['scale'])
    gd, od = gct.data(), oct_.data()
    if not np.array_equal(gd, od):
        bad = np.argwhere(gd != od)
        raise AssertionError(f'{len(bad)} limb words differ, first at {bad[0].tolist()}')


@pytest.mark.parametrize('N,depth,max_array,mask,stack', [
    (8, 25, 256, 0, 32),     # scaled-sinc PS
    (16, 40, 256, 2, 32),    # indicator (3,4,2)
    (64, 45, 32, 3, 32),     # indicator (3,5,2), two blocks: four masks stacked
    (64, 45, 32, 3, 3),      # ... split into stacks of 3 + 1
])
def test_sort_hybrid_matches_oracle(N, depth, max_array, mask, stack):
    rots = hybrid_rotations(N, max_array)
    orc = O.Context(11, depth, 40, 60, 3, seed=21)
    orc.gen_rotation_keys(rots)
    gpu = F.Context(11, depth, 40, 60, 3, seed=21, keygen=False)
    gpu.load_keys_from(orc, rots)
    x = np.random.default_rng(N).permutation(N) / N
    ox = orc.encrypt(x, N)
    gpu.set_sort_stack(stack)
    try:
        g = gpu.sort_hybrid(gpu.from_oracle(ox), N, rots, cfg_of(N), max_array=max_array, mask=mask)
    finally:
        gpu.set_sort_stack(32)
    o = orc.sort_hybrid(ox, N, rots, cfg_of(N), max_array=max_array, mask=mask)
    same(g, o)
    assert np.max(np.abs(gpu.decrypt(g)[:N] - np.sort(x))) < 0.01


def test_sort_hybrid_two_ranks_match():
    """blocks b = rank mod 2, partial outputs summed through the all-reduce hook
    (here: a host-side sum of the two ranks' device buffers, run in turn)."""
    import ctypes as C
    N, depth, max_array = 64, 45, 32
    rots = hybrid_rotations(N, max_array)
    gpu = F.Context(11, depth, 40, 60, 3, seed=22)
    gpu.gen_rotation_keys(rots)
    x = np.random.default_rng(1).permutation(N) / N
    ct = gpu.encrypt(x, N)
    rank = gpu.direct_sort(ct, N, rots, cfg_of(N), mode=1)
    hip = C.CDLL('libamdhip64.so')
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    parts = {}

    def record(tag):
        def fn(ptr, count, _user):  # store this rank's partial, return the zero-padded sum later
            buf = np.empty(count, dtype=np.uint64)
            assert hip.hipMemcpy(buf.ctypes.data, C.cast(ptr, C.c_void_p), count * 8, 2) == 0
            parts.setdefault(tag, []).append(buf)
        return fn
    for r in (0, 1):
        gpu.sort_hybrid(ct, N, rots, cfg_of(N), mode=1, rank=rank, max_array=max_array, mask=3, shard=(r, 2),
                        allreduce=record(r))
    # replay rank 0 with the summed partials fed back in call order
    sums = [a + b for a, b in zip(parts[0], parts[1])]
    it = iter(sums)

    def feed(ptr, count, _user):
        s = next(it)
        assert s.size == count
        assert hip.hipMemcpy(C.cast(ptr, C.c_void_p), s.ctypes.data, count * 8, 1) == 0
    sharded = gpu.sort_hybrid(ct, N, rots, cfg_of(N), mode=1, rank=rank, max_array=max_array, mask=3, shard=(0, 2),
                              allreduce=feed)
    ref = gpu.sort_hybrid(ct, N, rots, cfg_of(N), mode=1, rank=rank, max_array=max_array, mask=3)
    same(sharded, ref)


@pytest.mark.parametrize('N', [256, 512])
def test_reference_parameters_sort_hybrid(N):
    depth, rots = F.hybrid_parameters(N)
    ctx = F.Context(17, depth, 40, 60, 3, seed=N)
    ctx.gen_rotation_keys(rots)
    x = np.random.default_rng(N).permutation(N) / N
    out = ctx.sort_hybrid(ctx.encrypt(x, N), N, rots, cfg_of(N))
    assert np.max(np.abs(ctx.decrypt(out)[:N] - np.sort(x))) < 0.01
    assert out.level == REF_DEPTH[N]
