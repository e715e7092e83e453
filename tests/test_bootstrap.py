"""CPU checks of the bootstrapping spec on the oracle (oracle/oracle_boot.cpp).

* a bootstrap returns the input message at level depth (sparse slots, ring
  2^11, the reference's 59-bit scaling primes, src/kway_adapter.h:44-46);
* the level bookkeeping: input needs one spare level (OpenFHE cannot
  bootstrap at level == multDepth, src/k-way/EvalUtils.cpp:63), the slots must
  match the setup's;
* the k-way network bootstraps where EvalUtils::checkLevelAndBoot does and
  still meets KWaySort235Test's bound (max error < 0.01).
The GPU engine is checked word for word against this in test_gpu_bootstrap.py.
"""
import numpy as np
import pytest

import pyoracle as O


@pytest.fixture(scope='module')
def ctx():
    return O.Context(11, 24, 59, 60, 3, seed=61)


def test_bootstrap_recovers_the_message(ctx):
    B = O.Bootstrapper(ctx, 8, (2, 2))
    assert B.depth == 2 + 7 + 6 + 2  # CtS + PS(degree 88) + 6 double angles + StC
    x = np.random.default_rng(1).uniform(-1, 1, 8)
    for level in (0, 10, ctx.L - 1):
        out = B.bootstrap(ctx.encrypt(x, 8, level=level))
        assert out.level == B.depth and out.slots == 8
        assert np.max(np.abs(ctx.decrypt(out) - x)) < 1e-5


def test_bootstrap_rotation_set(ctx):
    B = O.Bootstrapper(ctx, 8, (2, 2), keygen=False)
    r = B.rotations()
    assert r == sorted(set(r)) and all(0 < k < 16 or k % 8 == 0 for k in r)
    # partial trace over the n/2s = 128 copies of the 8 slots: its 7 doubling steps
    # three at a time as hoisted sums, x + sum_{0<j<2^c} rot(x, j 2^b0 8), so the
    # keys are j 8 (j < 8), j 64 (j < 8) and 512
    trace = sorted({j * (8 << b0) for b0, c in ((0, 3), (3, 3), (6, 1)) for j in range(1, 1 << c)})
    assert [k for k in r if k >= 16] == [k for k in trace if k >= 16]


def test_bootstrap_level_and_slot_checks(ctx):
    B = O.Bootstrapper(ctx, 8, (2, 2))
    with pytest.raises(RuntimeError, match='no level left'):
        B.bootstrap(ctx.encrypt(np.ones(8) * 0.5, 8, level=ctx.L))
    with pytest.raises(RuntimeError, match='slots'):
        B.bootstrap(ctx.encrypt(np.ones(16) * 0.5, 16, level=3))
    with pytest.raises(RuntimeError, match='slots must be'):
        O.Bootstrapper(ctx, 1024, (2, 2), keygen=False)  # > n/4


def test_kway_bootstraps_where_levels_run_out():
    k, M = 2, 2
    N = k ** M
    c = O.Context(11, 26, 59, 60, 3, seed=62)
    B = O.Bootstrapper(c, N, (2, 2))
    c.gen_rotation_keys([1, -1, 2, -2])
    x = np.random.default_rng(2).permutation(N) * (1 - 1e-8) / N
    c.reset_counters()
    out = c.kway_sort(c.encrypt(x, N), k, M, (3, 2, 2), boot=B)
    assert np.max(np.abs(c.decrypt(out)[:N] - np.sort(x))) < 0.01
    assert out.level >= B.depth  # the output went through at least one bootstrap
