"""k-way sorting network (src/k-way/*) without bootstrapping:
the stage schedule and slot layouts of the C-ABI (host code, no GPU) against
the reference's own known answers and against the CPU oracle, and the oracle's
network against the reference test's property.

Pins:
* tests/k-way/MaskingTest.cpp:98-103 -- getRotateDistance(2,1,0)=2,
  (3,1,1)=6, (4,2,2)=32, (5,1,3)=5; :48-63 -- sortType(5,3,0) = (0,0,0) and
  a middle stage with slope <= k/2+1; :65-87 -- genIndices entries in [0, k].
* The stage count M + M(M-1)/2 * ceil(k/2) (src/k-way/Sorter.cpp:290).
* tests/k-way/KWaySort{2,3,5}Test.cpp:170-185 -- decrypted output equals
  std::sort of the input within 0.01 (input getVectorWithMinDiff(N, 0, 1,
  (1-1e-8)/N): here a seeded permutation of k(1-1e-8)/N, same spacing).
The reference bootstraps between stages (EvalBootstrap, not built here), so
the networks run on a context deep enough for every stage (levels measured
below); no reference test pins ciphertexts or levels, so beyond these
properties the oracle is parity-unpinned.
"""
import numpy as np
import pytest

import fhesort as F
import pyoracle as O

KWAY_CASES = [(2, 2), (2, 3), (2, 4), (2, 5), (3, 2), (3, 3), (3, 4), (5, 2), (5, 3)]


def test_rotate_distance_reference_kats():
    for fn in (F.kway_rotate_distance, O.kway_rotate_distance):
        assert fn(2, 1, 0) == 2
        assert fn(3, 1, 1) == 6
        assert fn(4, 2, 2) == 32
        assert fn(5, 1, 3) == 5


def test_sort_type_reference_kats():
    assert F.kway_sort_type(5, 3, 0) == (0, 0, 0)
    m, log_dist, slope = F.kway_sort_type(5, 3, 5)
    assert m >= 0 and log_dist >= 0 and slope <= 5 // 2 + 1


@pytest.mark.parametrize('k,M', KWAY_CASES)
def test_schedule_matches_oracle(k, M):
    stages = F.kway_stage_count(k, M)
    assert stages == M + M * (M - 1) // 2 * ((k + 1) // 2)
    N = k ** M
    for s in range(stages):
        t = F.kway_sort_type(k, M, s)
        assert t == O.kway_sort_type(k, M, s)
        m, log_dist, slope = t
        assert m + log_dist < M and 0 <= slope <= (k + 1) // 2
        assert F.kway_rotate_distance(k, log_dist, slope) == O.kway_rotate_distance(k, log_dist, slope)
        g, p = F.kway_gen_indices(N, k, M, m, log_dist, slope)
        go, po = O.kway_gen_indices(N, k, M, m, log_dist, slope)
        assert np.array_equal(g, go) and np.array_equal(p, po)
        assert g.min() >= 0 and g.max() <= k and p.max() <= k
        assert np.all((g > 0) == (p > 0)) and np.all(p <= g)
    # the first stage of every network sorts groups of k adjacent-by-dist slots
    g, p = F.kway_gen_indices(N, k, M, *F.kway_sort_type(k, M, 0))
    assert np.all(g == k) and sorted(np.bincount(p)[1:]) == [N // k] * k


def test_gen_indices_masking_test_case():
    g, p = F.kway_gen_indices(32, 2, 2, 1, 1, 0)  # MaskingTest.cpp:65-87
    assert len(g) == 32 and g.min() >= 0 and g.max() <= 2 and p.min() >= 0 and p.max() <= 2


def test_rotation_indices():
    assert F.kway_rotation_indices(25) == [1, -1, 2, -2, 4, -4, 8, -8, 16, -16]


def _slots(N):
    s = 1
    while s < N:
        s *= 2
    return s


@pytest.mark.parametrize('k,M,depth,used', [(2, 2, 52, 48), (3, 2, 70, 67)])
def test_oracle_network_sorts(k, M, depth, used):
    N = k ** M
    ctx = O.Context(11, depth, 40, 60, 3, seed=3)
    ctx.gen_rotation_keys(F.kway_rotation_indices(N))
    x = np.random.default_rng(k * 10 + M).permutation(N) * (1 - 1e-8) / N
    out = ctx.kway_sort(ctx.encrypt(x, _slots(N)), k, M, (3, 2, 2))
    assert out.level == used
    assert np.max(np.abs(ctx.decrypt(out)[:N] - np.sort(x))) < 0.01


def test_oracle_network_needs_levels():
    """where the reference would bootstrap, a too-shallow context is an error"""
    ctx = O.Context(11, 30, 40, 60, 3, seed=3)
    ctx.gen_rotation_keys(F.kway_rotation_indices(4))
    ct = ctx.encrypt(np.array([0.5, 0.25, 0.75, 0.0]), 4)
    with pytest.raises(RuntimeError, match='no levels left'):
        ctx.kway_sort(ct, 2, 2, (3, 2, 2))


# ---- SortUtilsTest known answers (tests/k-way/SortUtilsTest.cpp:68-260):
# fcnL and the 2/3/4/5-sorters on plain-value inputs and given comparison
# bits, at the suite's depth 50 / 59-bit scaling (ring 2^12; dnum 4), within 0.1.
SORTUTILS_KATS = [
    # (kk, inputs, comparisons, expected outputs ascending)
    (1, [[2, 4, 6, 8], [1, 5, 3, 7]], [[1, 0, 1, 1]], [[2, 5, 6, 8]]),
    (2, [[5, 2, 8, 1], [3, 6, 4, 7]], [[1, 0, 1, 0]], [[3, 2, 4, 1], [5, 6, 8, 7]]),
    (3, [[5, 9, 3, 7], [2, 4, 8, 1], [6, 1, 4, 5]],
     [[1, 1, 0, 1], [0, 1, 0, 1], [0, 1, 1, 0]],
     [[2, 1, 3, 1], [5, 4, 4, 5], [6, 9, 8, 7]]),
    (4, [[9, 7, 5], [6, 4, 8], [3, 8, 2], [7, 2, 6]],
     [[1, 1, 0], [1, 0, 1], [1, 1, 0], [1, 0, 1], [0, 1, 1], [0, 1, 0]],
     [[3, 2, 2], [6, 4, 5], [7, 7, 6], [9, 8, 8]]),
    (5, [[9, 7, 5], [6, 4, 8], [3, 8, 2], [7, 2, 6], [5, 6, 4]],
     [[1, 1, 0], [1, 0, 1], [1, 1, 0], [1, 1, 1], [1, 0, 1], [0, 1, 1], [1, 0, 1], [0, 1, 0], [0, 1, 0],
      [1, 0, 1]],
     [[3, 2, 2], [5, 4, 4], [6, 6, 5], [7, 7, 6], [9, 8, 8]]),
]


@pytest.fixture(scope='module')
def sortutils_ctx():
    return O.Context(12, 50, 59, 60, 4, seed=16)


@pytest.mark.parametrize('kat', SORTUTILS_KATS, ids=['fcnL', 'twoSorter', 'threeSorter', 'fourSorter', 'fiveSorter'])
def test_sortutils_known_answers(sortutils_ctx, kat):
    c = sortutils_ctx
    kk, xs, cs, expected = kat
    enc = lambda v: c.encrypt(np.array(v, dtype=float), 16)
    outs = c.kway_sorter(kk, [enc(v) for v in xs], [enc(v) for v in cs])
    for o, e in zip(outs, expected):
        assert np.max(np.abs(c.decrypt(o)[:len(e)] - e)) < 0.1
