"""k-way sorting network on the GPU engine (src/k-way/*, no bootstrapping):
bit-exact with the CPU oracle on identical keys for k = 2, 3 (N = 4, 8, 9), and
the reference test's property (decrypted == sorted input within 0.01,
tests/k-way/KWaySort5Test.cpp) for k = 5, N = 25.  A context too shallow for
the network fails with FHE_EDEPTH where the reference would bootstrap.

All calls go through the C ABI (include/fhe_gpu.h) via fhesort.py.
"""
import numpy as np
import pytest

import fhesort as F
import pyoracle as O
from test_gpu_hybrid import same

pytestmark = pytest.mark.gpu


def _dnum(depth):  # the engine takes digits of <= 16 primes: deep chains need more digits
    return -(-(depth + 1) // 15)


def _slots(N):
    s = 1
    while s < N:
        s *= 2
    return s


@pytest.mark.parametrize('k,M,depth,used', [(2, 2, 52, 48), (3, 2, 70, 67), (2, 3, 100, 96)])
def test_kway_matches_oracle(k, M, depth, used):
    N = k ** M
    rots = F.kway_rotation_indices(N)
    orc = O.Context(11, depth, 40, 60, _dnum(depth), seed=41)
    orc.gen_rotation_keys(rots)
    gpu = F.Context(11, depth, 40, 60, _dnum(depth), seed=41, keygen=False)
    gpu.load_keys_from(orc, rots)
    x = np.random.default_rng(N).permutation(N) * (1 - 1e-8) / N
    ox = orc.encrypt(x, _slots(N))
    g = gpu.kway_sort(gpu.from_oracle(ox), k, M, (3, 2, 2))
    o = orc.kway_sort(ox, k, M, (3, 2, 2))
    same(g, o)
    assert g.info()['level'] == used
    assert np.max(np.abs(gpu.decrypt(g)[:N] - np.sort(x))) < 0.01


def test_kway_five_way_sorts():
    k, M = 5, 2
    N = k ** M
    gpu = F.Context(11, 104, 40, 60, _dnum(104), seed=42)
    gpu.gen_rotation_keys(F.kway_rotation_indices(N))
    x = np.random.default_rng(7).permutation(N) * (1 - 1e-8) / N
    out = gpu.kway_sort(gpu.encrypt(x, _slots(N)), k, M, (3, 2, 2))
    assert out.info()['level'] == 100
    assert np.max(np.abs(gpu.decrypt(out)[:N] - np.sort(x))) < 0.01


def test_kway_too_shallow_is_edepth():
    gpu = F.Context(11, 30, 40, 60, 3, seed=43)
    gpu.gen_rotation_keys(F.kway_rotation_indices(4))
    ct = gpu.encrypt(np.array([0.5, 0.25, 0.75, 0.0]), 4)
    with pytest.raises(F.FheError) as e:
        gpu.kway_sort(ct, 2, 2, (3, 2, 2))
    assert e.value.code == 3  # FHE_EDEPTH


@pytest.mark.parametrize('kk', [1, 2, 3, 4, 5])
def test_sortutils_sorters_bit_exact(kk):
    """fcnL and the 2/3/4/5-sorters (src/k-way/SortUtils.cpp:5-208) on the GPU
    == the oracle word for word, and SortUtilsTest's known answers within 0.1
    (tests/k-way/SortUtilsTest.cpp:68-260; depth 50, 59-bit scaling)."""
    from test_kway import SORTUTILS_KATS
    _, xs, cs, expected = SORTUTILS_KATS[kk - 1]
    orc = O.Context(12, 50, 59, 60, 4, seed=16)
    gpu = F.Context(12, 50, 59, 60, 4, seed=16, keygen=False)
    gpu.load_keys_from(orc)
    ox = [orc.encrypt(np.array(v, dtype=float), 16) for v in xs]
    oc = [orc.encrypt(np.array(v, dtype=float), 16) for v in cs]
    oo = orc.kway_sorter(kk, ox, oc)
    go = gpu.kway_sorter(kk, [gpu.from_oracle(c) for c in ox], [gpu.from_oracle(c) for c in oc])
    for g, o, e in zip(go, oo, expected):
        assert np.array_equal(g.data(), o.data())
        assert np.max(np.abs(gpu.decrypt(g)[:len(e)] - e)) < 0.1


@pytest.fixture(scope='module')
def sorter_ctx():
    """SorterTest's context (tests/k-way/SorterTest.cpp:14-45): ring 2^12, depth
    59, scale 2^59, 16 slots, rotations +-1..15, bootstrapping {4,4}; dnum 4
    (60 Q primes in 3 digits would exceed the engine's 16 primes per digit)."""
    gpu = F.Context(12, 59, 59, 60, 4, seed=59)
    gpu.gen_rotation_keys([r for i in range(1, 16) for r in (i, -i)])
    boot = F.Bootstrapper(gpu, 16, (4, 4))
    yield gpu, boot
    gpu.close()


@pytest.mark.parametrize('k,M,x', [
    (2, 3, [0.5, 0.2, 0.8, 0.1, 0.3, 0.6, 0.4, 0.7]),  # TwoWaySorting
    (3, 1, [0.5, 0.2, 0.8]),                          # ThreeWaySorting
    (5, 1, [0.5, 0.3, 0.4, 0.1, 0.2]),                # FiveWaySorting
])
def test_sortertest_whole_sorters(sorter_ctx, k, M, x):
    """SorterTest's TwoWay/ThreeWay/FiveWaySorting (SorterTest.cpp:313-383):
    Sorter::sorter with CompositeSign(3, d_g = 5, d_f = 2) sorts within 0.1."""
    gpu, boot = sorter_ctx
    out = gpu.kway_sort(gpu.encrypt(x, 16), k, M, (3, 5, 2), boot=boot)
    got = gpu.decrypt(out)[:len(x)]
    assert np.max(np.abs(got - np.sort(x))) < 0.1, got
