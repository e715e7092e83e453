"""MEHP24 sort on the GPU engine: bit-exact with the CPU oracle at test sizes
(identical keys), and the reference test's own property (decrypted output ==
sorted input within 0.01, tests/mehp24/Mehp24SortTest.cpp:144-185) at the
reference's parameters (ring 2^17, scale 2^40, its depth table).

All calls go through the C ABI (include/fhe_gpu.h) via fhesort.py.
"""
import numpy as np
import pytest

import fhesort as F
import pyoracle as O

pytestmark = pytest.mark.gpu

LOGN, DEPTH = 11, 35
ROTS = sorted(set(O.mehp24_rotation_indices(4)) | set(O.mehp24_rotation_indices(8)) |
              set(O.mehp24_rotation_indices(8, 4)) | set(O.mehp24_rotation_indices(16, 4)))


@pytest.fixture(scope='module')
def pair():
    orc = O.Context(LOGN, DEPTH, 40, 60, 3, seed=9)
    orc.gen_rotation_keys(ROTS)
    gpu = F.Context(LOGN, DEPTH, 40, 60, 3, seed=9, keygen=False)
    gpu.load_keys_from(orc, ROTS)
    return orc, gpu


def same(gct, oct_):
    gi, oi = gct.info(), oct_.info()
    assert (gi['level'], gi['slots'], gi['limbs'], gi['scale']) == (oi['level'], oi['slots'], oi['limbs'], oi['scale'])
    gd, od = gct.data(), oct_.data()
    if not np.array_equal(gd, od):
        bad = np.argwhere(gd != od)
        raise AssertionError(f'{len(bad)} limb words differ, first at {bad[0].tolist()}')


def test_encrypt_ext_matches_oracle():
    """Same seed, same encryption counter: identical ciphertexts."""
    orc = O.Context(LOGN, 4, 40, 60, 3, seed=8)
    gpu = F.Context(LOGN, 4, 40, 60, 3, seed=8)
    x = np.random.default_rng(8).uniform(-1, 1, 64)
    o = orc.encrypt_ext(x, 64)
    g = gpu.encrypt_ext(x, 64)
    assert o.level == g.level == 1
    same(g, o)
    assert np.max(np.abs(gpu.decrypt(g) - x)) < 1e-8


def test_indicator_adv_matches_oracle(pair):
    orc, gpu = pair
    v = np.array([-3.0, -1.0, 0.0, 0.2, 1.0, 2.0, -0.1, 3.0])
    o = orc.encrypt(v, 16)
    ro = orc.mehp24_indicator(o, 4.0, 2, 2)
    rg = gpu.mehp24_indicator(gpu.from_oracle(o), 4.0, 2, 2)
    same(rg, ro)


@pytest.mark.parametrize('N,sub,stack', [(4, 0, 32), (8, 0, 32), (8, 4, 32), (8, 4, 1), (16, 4, 5)])
def test_sort_matches_oracle(pair, N, sub, stack):
    """sortFG (sub 0) and sortLargeArrayFG with parts of 4 values; stack 1 runs
    every compare / indicator alone, 5 splits them into uneven stacks."""
    orc, gpu = pair
    cfg = (3, 2, 2) if N <= 16 else (3, 3, 2)
    dg_i = (int(np.log2(N)) + 1) // 2
    x = np.random.default_rng(N + sub).permutation(N) / N
    o = orc.encrypt(x, N * N if sub == 0 else sub * sub)
    gpu.set_sort_stack(stack)
    try:
        rg = gpu.mehp24_sort(gpu.from_oracle(o), N, cfg, dg_i, 2, sub)
    finally:
        gpu.set_sort_stack(32)
    ro = orc.mehp24_sort(o, N, cfg, dg_i, 2, sub)
    same(rg, ro)
    y = gpu.decrypt(rg)[:N]
    assert np.max(np.abs(y - np.sort(x))) < 0.01


def _full(N):
    p = F.mehp24_parameters(N)
    ctx = F.Context(p['log_ring'], p['depth'] + 1, p['scale_bits'], 60, p['dnum'], seed=N)
    ctx.gen_rotation_keys(p['rots'])
    x = np.random.default_rng(N).permutation(N) / N  # getVectorWithMinDiff(N, 0, 1, 1/N)
    slots = min(N * N, 1 << (p['log_ring'] - 1))
    out = ctx.mehp24_sort(ctx.encrypt_ext(x, slots), N, p['cfg'], p['dg_i'], p['df_i'], p['sub'])
    y = ctx.decrypt(out)[:N]
    return x, y, out


@pytest.mark.parametrize('N', [16, 256, 512, 4096])
def test_reference_parameters_sort(N):
    """The reference test at its own parameters: N=16 and N=256 (sortFG) and
    N=512 (sortLargeArrayFG, two parts of 256) at ring 2^17, input encrypted
    FLEXIBLEAUTOEXT-style (OpenFHE's default, which the reference runs under);
    N=4096 is BASELINE config 5 (16 parts of 256, ~15 s on one MI355X)."""
    x, y, out = _full(N)
    err = np.max(np.abs(y - np.sort(x)))
    assert err < 0.01, err
    assert out.level <= F.mehp24_parameters(N)['depth'] + 1


def test_full_slot_ops_match_oracle():
    """slots = n/2 (the reference packs N*N = 65536 values at ring 2^17):
    encryption, every MEHP24 rotation for N=32, masks and a product, bit-exact."""
    N = 32
    rots = O.mehp24_rotation_indices(N)
    orc = O.Context(LOGN, 12, 40, 60, 3, seed=4)
    orc.gen_rotation_keys(rots)
    gpu = F.Context(LOGN, 12, 40, 60, 3, seed=4, keygen=False)
    gpu.load_keys_from(orc, rots)
    x = np.random.default_rng(2).uniform(-1, 1, N * N)
    o = orc.encrypt(x, N * N)
    g = gpu.from_oracle(o)
    assert np.max(np.abs(gpu.decrypt(g) - x)) < 1e-6
    for k in rots:
        try:
            same(gpu.rotate(g, k), orc.rotate(o, k))
        except AssertionError as e:
            raise AssertionError(f'rotation {k}: {e}')
    mask = (np.arange(N * N) % N == 0).astype(float)
    same(gpu.mul_plain(g, gpu.encode(mask, N * N, 0)), orc.mul_plain(o, orc.encode(mask, N * N, 0)))
    same(gpu.mul(g, g), orc.mul(o, o))


def test_full_slot_sort_matches_oracle():
    N = 32
    rots = O.mehp24_rotation_indices(N)
    orc = O.Context(LOGN, 42, 40, 60, 3, seed=6)
    orc.gen_rotation_keys(rots)
    gpu = F.Context(LOGN, 42, 40, 60, 3, seed=6, keygen=False)
    gpu.load_keys_from(orc, rots)
    x = np.random.default_rng(N).permutation(N) / N
    o = orc.encrypt(x, N * N)
    rg = gpu.mehp24_sort(gpu.from_oracle(o), N, (3, 3, 2), 3, 2)
    same(rg, orc.mehp24_sort(o, N, (3, 3, 2), 3, 2))
