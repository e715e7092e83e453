"""CKKS bootstrapping on the GPU engine.

The reference bootstraps through OpenFHE (EvalBootstrapSetup / KeyGen /
EvalBootstrap, tests/k-way/KWaySort235Test.cpp:46-48) wherever the k-way
network runs out of levels (src/k-way/EvalUtils.cpp:59-86) and inside
compositeSign (src/sign.cpp:164-170).  Here:

* every stage (ModRaise, conjugation, CoeffsToSlots, EvalMod, SlotsToCoeffs)
  and the whole bootstrap are word-identical to the CPU oracle on identical
  keys (GPU key generation == oracle key generation for one seed);
* the bootstrapped ciphertext decrypts to its input (sparse slots 8..512);
* k-way networks that need bootstraps are bit-exact vs the oracle (N = 4) and
  meet the reference test's bound (max error < 0.01, KWaySort235Test.cpp:291)
  for k = 2, 3, 5.

All calls go through the C ABI (include/fhe_gpu.h) via fhesort.py.
"""
import numpy as np
import pytest

import fhesort as F
import pyoracle as O
from test_gpu_hybrid import same

pytestmark = pytest.mark.gpu


def _slots(N):
    s = 1
    while s < N:
        s *= 2
    return s


def _pair(logN, L, seed, slots, budget):
    orc = O.Context(logN, L, 59, 60, 3, seed=seed)
    gpu = F.Context(logN, L, 59, 60, 3, seed=seed)  # GPU keygen == oracle keygen (test_gpu_parity)
    ob = O.Bootstrapper(orc, slots, budget)
    gb = F.Bootstrapper(gpu, slots, budget)
    return orc, gpu, ob, gb


def test_bootstrap_stages_bit_exact():
    orc, gpu, ob, gb = _pair(11, 24, 51, 8, (2, 2))
    try:
        assert gb.rotations() == ob.rotations()
        assert gb.depth == ob.depth == 2 + 7 + 6 + 2
        x = np.random.default_rng(5).uniform(-1, 1, 8)
        ox = orc.encrypt(x, 8, level=orc.L - 3)
        gx = gpu.from_oracle(ox)
        same(gpu.conjugate(gx), orc.conjugate(ox))
        olast, glast = orc.mul_const_to(ox, 0.25, orc.L), gpu.mul_const_to(gx, 0.25, gpu.L)
        same(glast, olast)
        oraised, graised = ob.mod_raise(olast), gb.mod_raise(glast)
        same(graised, oraised)
        ocs, gcs = ob.coeffs_to_slots(oraised), gb.coeffs_to_slots(graised)
        same(gcs, ocs)
        oem, gem = ob.eval_mod(ocs), gb.eval_mod(gcs)
        same(gem, oem)
        same(gb.slots_to_coeffs(gem), ob.slots_to_coeffs(oem))
        gout, oout = gb.bootstrap(gx), ob.bootstrap(ox)
        same(gout, oout)
        assert gout.level == gb.depth
        assert np.max(np.abs(gpu.decrypt(gout) - x)) < 1e-5
    finally:
        gpu.close()


@pytest.mark.parametrize("slots,budget", [(8, (2, 1)), (64, (3, 2)), (512, (4, 4))])
def test_bootstrap_refreshes_levels(slots, budget):
    gpu = F.Context(11, 28, 59, 60, 3, seed=52)
    try:
        B = F.Bootstrapper(gpu, slots, budget)
        x = np.random.default_rng(slots).uniform(-1, 1, slots)
        ct = gpu.encrypt(x, slots, level=27)  # one level left, as checkLevelAndBoot leaves it
        out = B.bootstrap(ct)
        assert out.level == B.depth < 27
        assert np.max(np.abs(gpu.decrypt(out) - x)) < 1e-4
        again = B.bootstrap(gpu.mul(out, out))  # a bootstrapped ciphertext computes and bootstraps again
        assert np.max(np.abs(gpu.decrypt(again) - x * x)) < 1e-4
    finally:
        gpu.close()


def test_bootstrap_rejects_last_level_and_wrong_slots():
    gpu = F.Context(11, 24, 59, 60, 3, seed=53)
    try:
        B = F.Bootstrapper(gpu, 8, (2, 2))
        ct = gpu.encrypt(np.ones(8) * 0.5, 8, level=24)
        with pytest.raises(F.FheError):
            B.bootstrap(ct)  # OpenFHE cannot bootstrap at level == multDepth either (EvalUtils.cpp:63)
        with pytest.raises(F.FheError) as e:
            B.bootstrap(gpu.encrypt(np.ones(16) * 0.5, 16, level=20))
        assert e.value.code == F.FHE_EINVAL
    finally:
        gpu.close()


def test_kway_with_bootstrap_matches_oracle():
    k, M = 2, 2
    N = k ** M
    rots = F.kway_rotation_indices(N)
    orc, gpu, ob, gb = _pair(11, 26, 54, _slots(N), (2, 2))
    try:
        orc.gen_rotation_keys(rots)
        gpu.gen_rotation_keys(rots)
        x = np.random.default_rng(3).permutation(N) * (1 - 1e-8) / N
        ox = orc.encrypt(x, _slots(N))
        g = gpu.kway_sort(gpu.from_oracle(ox), k, M, (3, 2, 2), boot=gb)
        assert gpu.kway_bootstraps >= 1
        o = orc.kway_sort(ox, k, M, (3, 2, 2), boot=ob)
        same(g, o)
        assert np.max(np.abs(gpu.decrypt(g)[:N] - np.sort(x))) < 0.01
    finally:
        gpu.close()


def test_kway5_two_lanes_match_oracle():
    """k = 5: a stage's two comparisons (and their level-check bootstraps) run on
    two engine lanes at once (fhe_set_sort_lanes >= 2, the default); the words
    equal the oracle's sequential sorter and the one-lane run."""
    k, M = 5, 2
    N = k ** M
    rots = F.kway_rotation_indices(N)
    orc, gpu, ob, gb = _pair(11, 26, 54, _slots(N), (2, 2))
    try:
        orc.gen_rotation_keys(rots)
        gpu.gen_rotation_keys(rots)
        x = np.random.default_rng(5).permutation(N) * (1 - 1e-8) / N
        ox = orc.encrypt(x, _slots(N))
        gpu.set_sort_lanes(2)
        g2 = gpu.kway_sort(gpu.from_oracle(ox), k, M, (3, 2, 2), boot=gb)
        b2 = gpu.kway_bootstraps
        gpu.set_sort_lanes(1)
        g1 = gpu.kway_sort(gpu.from_oracle(ox), k, M, (3, 2, 2), boot=gb)
        assert b2 >= 1 and gpu.kway_bootstraps == b2
        same(g2, g1)
        o = orc.kway_sort(ox, k, M, (3, 2, 2), boot=ob)
        same(g2, o)
        assert np.max(np.abs(gpu.decrypt(g2)[:N] - np.sort(x))) < 0.01
    finally:
        gpu.close()


@pytest.mark.parametrize('k,M,cfg', [(2, 4, (3, 2, 2)), (3, 2, (3, 2, 2)), (5, 2, (3, 2, 3))])
def test_kway_with_bootstrap_sorts(k, M, cfg):
    N = k ** M
    s = _slots(N)
    gpu = F.Context(12, 30, 59, 60, 3, seed=55 + N)
    try:
        B = F.Bootstrapper(gpu, s, (2, 2))
        gpu.gen_rotation_keys(F.kway_rotation_indices(N))
        x = np.random.default_rng(N).permutation(N) * (1 - 1e-8) / N
        out = gpu.kway_sort(gpu.encrypt(x, s), k, M, cfg, boot=B)
        assert gpu.kway_bootstraps >= 1
        assert np.max(np.abs(gpu.decrypt(out)[:N] - np.sort(x))) < 0.01
    finally:
        gpu.close()


def test_config4_kway_k5_n3125_ring16():
    """BASELINE config 4: k = 5, N = 3125 (KWaySort235Test's commented-out
    case, tests/k-way/KWaySort235Test.cpp:88,213-218) at ring 2^16 with the
    reference context (depth 40, scale 2^59, levelBudget {5,5}, d_g = 5)."""
    k, M = 5, 5
    N = k ** M
    gpu = F.Context(16, 40, 59, 60, 3, seed=2025)
    try:
        B = F.Bootstrapper(gpu, 4096, (5, 5))
        assert B.depth == 23
        gpu.gen_rotation_keys(F.kway_rotation_indices(N))
        x = np.random.default_rng(N).permutation(N) * (1 - 1e-8) / N
        out = gpu.kway_sort(gpu.encrypt(x, 4096), k, M, (3, 2, 5), boot=B)
        assert gpu.kway_bootstraps > 20
        err = np.abs(gpu.decrypt(out)[:N] - np.sort(x))
        assert np.max(err) < 0.01 and np.sum(err >= 0.01) == 0  # KWaySort235Test.cpp:291-292
    finally:
        gpu.close()


# KWaySort235Test's size table (tests/k-way/KWaySort235Test.cpp:68-222): N, k, M,
# d_f, d_g; run at ring 2^16 (config 4's ring) with the test's context otherwise
# (depth 40, scale 2^59, levelBudget {4,4} for N <= 128, else {5,5}) and its
# assertions (max error < 0.01, no slot >= 0.01).  N = 3125 is
# test_config4_kway_k5_n3125_ring16.
KWAY235 = [(4, 2, 2, 2, 2), (8, 2, 3, 2, 2), (9, 3, 2, 2, 2), (16, 2, 4, 2, 2), (25, 5, 2, 2, 3),
           (27, 3, 3, 2, 3), (32, 2, 5, 2, 3), (64, 2, 6, 2, 3), (81, 3, 4, 2, 3), (125, 5, 3, 2, 3),
           (128, 2, 7, 2, 4), (243, 3, 5, 2, 4), (256, 2, 8, 2, 4), (512, 2, 9, 2, 4), (625, 5, 4, 2, 5),
           (729, 3, 6, 2, 5), (1024, 2, 10, 2, 5), (2048, 2, 11, 2, 5), (2187, 3, 7, 2, 5)]


@pytest.fixture(scope='module')
def kway_ctx():
    gpu = F.Context(16, 40, 59, 60, 3, seed=235)
    gpu.gen_rotation_keys(F.kway_rotation_indices(2187))  # +-2^i < 2187 covers every N here
    boots = {}
    yield gpu, boots
    for b in boots.values():
        b.close()
    gpu.close()


@pytest.mark.parametrize('N,k,M,d_f,d_g', KWAY235)
def test_kway235_sizes(kway_ctx, N, k, M, d_f, d_g):
    gpu, boots = kway_ctx
    assert k ** M == N
    s = _slots(N)
    budget = (4, 4) if N <= 128 else (5, 5)
    if (s, budget) not in boots:
        boots[(s, budget)] = F.Bootstrapper(gpu, s, budget)
    x = np.random.default_rng(N).permutation(N) * (1 - 1e-8) / N  # getVectorWithMinDiff(N, 0, 1, (1-1e-8)/N)
    out = gpu.kway_sort(gpu.encrypt(x, s), k, M, (3, d_f, d_g), boot=boots[(s, budget)])
    err = np.abs(gpu.decrypt(out)[:N] - np.sort(x))
    assert np.max(err) < 0.01 and np.sum(err >= 0.01) == 0  # KWaySort235Test.cpp:291-292
