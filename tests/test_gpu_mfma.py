"""The i8-MFMA sums of products (kernels.hip: k_leaf_sums_mfma, k_modup_mfma,
k_moddown_rescale_mfma; fhe_set_mfma_sums) against the CPU oracle.

The build default runs the PS linear sums on MFMA and the basis conversions on
the 64-bit VALU kernels (the MFMA conversions are word-identical
and measured slower); these tests switch every MFMA form on and require the same words as the oracle -- PS linear sums of
up to 10 leaves and 32 baby steps, ModUp digits of 1..22 primes (one to three
64-byte K steps), the fused ModDown+rescale with 3..16 special primes, at rings
2^12 and 2^16.  All calls go through the C ABI (include/fhe_gpu.h).
"""
import numpy as np
import pytest

import fhesort as F
import pyoracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def mfma_on():
    prev = F.set_mfma_sums(7)
    yield
    F.set_mfma_sums(prev)


def same(gct, oct_):
    gi, oi = gct.info(), oct_.info()
    assert (gi['level'], gi['limbs'], gi['scale']) == (oi['level'], oi['limbs'], oi['scale'])
    gd, od = gct.data(), oct_.data()
    if not np.array_equal(gd, od):
        bad = np.argwhere(gd != od)
        raise AssertionError(f'{len(bad)} limb words differ, first at {bad[0].tolist()}')


def test_mask_query_and_set():
    assert F.set_mfma_sums(-1) == 7
    assert F.set_mfma_sums(1) == 7
    assert F.set_mfma_sums(-1) == 1


@pytest.mark.parametrize('mask', [7, 0])
@pytest.mark.parametrize('split', [F.PS_SPLIT_OPENFHE, F.PS_SPLIT_ENGINE])
@pytest.mark.parametrize('deg', [7, 70, 200])
def test_chebyshev_ps_mfma(deg, split, mask):
    """Paterson-Stockmeyer leaves through k_leaf_sums_mfma (mask 7) and the
    VALU k_linear_sum_multi (mask 0): word-identical to the oracle."""
    F.set_mfma_sums(mask)
    L = 10 if deg <= 119 else 11
    orc = O.Context(12, L, 40, 60, 3, seed=9, ps_split=split)
    gpu = F.Context(12, L, 40, 60, 3, seed=9, keygen=False, ps_split=split)
    gpu.load_keys_from(orc)
    ox = orc.encrypt(np.linspace(-1, 1, 16), 16)
    # a well-conditioned series (coefficients decaying like 1/i^2): OpenFHE's
    # division tree takes it (a slowly decaying one could fall back
    # to the power-of-two split and run the same path twice)
    c = np.random.default_rng(deg).normal(size=deg + 1) / (1 + np.arange(deg + 1)) ** 2
    if deg >= 5:
        assert F.cheb_ps_uses_openfhe(c)
    out = gpu.cheb(gpu.from_oracle(ox), c)
    same(out, orc.cheb(ox, c))
    assert out.level == ox.level + F.cheb_ps_depth(deg, split)


@pytest.mark.parametrize('L', [12, 65])
def test_modup_moddown_products_rotations_mfma(L):
    """ModUp at full and partial digits (alpha 3 at L=12, 22 at L=65), ModDown,
    relinearised products down the chain (the fused ModDown+rescale) and
    rotations: word-identical to the oracle."""
    rots = [1, -3]
    orc = O.Context(12, L, 40, 60, 3, seed=L + 1)
    orc.gen_rotation_keys(rots)
    gpu = F.Context(12, L, 40, 60, 3, seed=L + 1, keygen=False)
    gpu.load_keys_from(orc, rots)
    rng = np.random.default_rng(L)
    alpha = orc.alpha
    for ell in sorted({L + 1, 2 * alpha, alpha + 1, alpha, 7, 1}):
        if ell > L + 1:
            continue
        d = np.stack([rng.integers(0, int(q), size=orc.n, dtype=np.uint64) for q in orc.primes[:ell]])
        assert np.array_equal(orc.modup(d), gpu.modup(d)), f'modup differs at ell={ell}'
    a, b = rng.uniform(-1, 1, 16), rng.uniform(-1, 1, 16)
    oa, ob = orc.encrypt(a, 16), orc.encrypt(b, 16)
    ga, gb = gpu.from_oracle(oa), gpu.from_oracle(ob)
    oc, gc = oa, ga
    for i in range(L - 2):
        oc, gc = orc.mul(oc, ob), gpu.mul(gc, gb)
        if i % 7 == 0:
            same(gc, oc)
            for k in rots:
                same(gpu.rotate(gc, k), orc.rotate(oc, k))
    same(gc, oc)


def test_ring16_products_mfma():
    """Ring 2^16 (full 256-coefficient blocks, chunked target groups): stacked
    products word-identical to the oracle with every MFMA form on."""
    orc = O.Context(16, 8, 40, 60, 3, seed=16)
    gpu = F.Context(16, 8, 40, 60, 3, seed=16, keygen=False)
    gpu.load_keys_from(orc, [])
    rng = np.random.default_rng(16)
    xs = [orc.encrypt(rng.uniform(-1, 1, 64), 64) for _ in range(3)]
    gx = [gpu.from_oracle(x) for x in xs]
    oc, gc = xs[0], gx[0]
    for _ in range(6):
        oc, gc = orc.mul(oc, xs[1]), gpu.mul(gc, gx[1])
    same(gc, oc)
    st = gpu.mul(gpu.stack(gx), gx[2])
    for m in range(3):
        same(gpu.member(st, m), orc.mul(xs[m], xs[2]))


def test_leaf_sums_4096_blocks_ring16_stack32():
    """k_leaf_sums_mfma (or k_leaf_sums_fold) at the width the bench runs it: ring 2^16 and a
    32-member stack (64 segments), so the launches take the 4096-coefficient
    blocks (kernels.hip ew_linear_sum_multi: n / 4096 x limbs x segments >= 2048),
    passes of more than 8 baby steps (KS >= 2) and more than 4 leaves (NG >= 2):
    a degree-848 series, the doubled sinc's degree at N = 128.  Every member
    word-identical to the oracle's series on that member (four distinct inputs,
    each stacked eight times)."""
    L = 12
    orc = O.Context(16, L, 40, 60, 3, seed=61)
    gpu = F.Context(16, L, 40, 60, 3, seed=61, keygen=False)
    gpu.load_keys_from(orc, [])
    rng = np.random.default_rng(61)
    xs = [orc.encrypt(rng.uniform(-1, 1, 64), 64) for _ in range(4)]
    c = rng.normal(size=849) / (1 + np.arange(849)) ** 2
    assert F.cheb_ps_uses_openfhe(c)
    st = gpu.stack([gpu.from_oracle(xs[m % 4]) for m in range(32)])
    with F.KernelClock(gpu) as clk:
        out = gpu.cheb(st, c)
    shapes = [tuple(int(v) for v in k.split('<')[1].rstrip('>').split(','))
              for k in clk.stats if k.startswith(('k_leaf_sums_mfma<', 'k_leaf_sums_fold<'))]
    assert any(ks >= 2 and ng >= 2 for ks, ng in shapes), f'leaf-sum launches: {sorted(clk.stats)}'
    ref = [orc.cheb(x, c) for x in xs]
    for m in range(32):
        same(gpu.member(out, m), ref[m % 4])


def test_kernel_clock_bytes_are_algorithmic():
    """The live clock the bench's roofline reads: a ciphertext add at level l of
    ring 2^12 books exactly 3 x 2 x (l+1) x n x 8 algorithmic bytes (two inputs,
    one output, two polynomials) on one k_add launch, and no kernel of an HMult
    claims more than 10 TB/s (the JSON once appended a stray digit to every byte
    count, a 10x error)"""
    L = 6
    orc = O.Context(12, L, 40, 60, 3, seed=62)
    gpu = F.Context(12, L, 40, 60, 3, seed=62, keygen=False)
    gpu.load_keys_from(orc, [])
    rng = np.random.default_rng(62)
    x = gpu.from_oracle(orc.encrypt(rng.uniform(-1, 1, 64), 64))
    y = gpu.from_oracle(orc.encrypt(rng.uniform(-1, 1, 64), 64))
    with F.KernelClock(gpu) as clk:
        gpu.add(x, y)
    st = clk.stats
    assert st['k_add']['launches'] == 1
    assert st['k_add']['bytes'] == 3 * 2 * x.info()['limbs'] * 4096 * 8
    with F.KernelClock(gpu) as clk:
        gpu.mul(x, y)
    for k, v in clk.stats.items():
        assert v['bytes'] > 0 and v['bytes'] / (v['ms'] * 1e-3) < 10e12, (k, v)
