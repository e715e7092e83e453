"""The folded-constant MFMA conversions on every path, forced through their
environment switches (kernels.hip k_modup_fold, k_moddown_rescale_fold;
DESIGN.md §5 "Folded-constant conversions").  The switches are read once per
process, so the checks run in one child process with FHE_MODUP_FOLD=1 (every
ModUp digit, alpha 3 / 14 / 22) and FHE_MODDOWN_FOLD=1 (the HMult tail's
ModDown+rescale, K = 3 / 14 / 22 special primes): ModUp outputs, chains of
relinearised products, rotations and a stacked product are word-identical to
the CPU oracle.  The default build keeps ModUp folded only above 16 sources and
ModDown on the VALU, so without this test those forms would run only in A/B
measurements."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

CHILD = r'''
import sys
import numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
import fhesort as F
import pyoracle as O

def same(g, o, what):
    gi, oi = g.info(), o.info()
    assert (gi['level'], gi['limbs'], gi['scale']) == (oi['level'], oi['limbs'], oi['scale']), what
    assert np.array_equal(g.data(), o.data()), what

for logn, L in ((12, 12), (12, 40), (12, 65), (14, 20)):
    rots = [1, -3]
    orc = O.Context(logn, L, 40, 60, 3, seed=L + logn)
    orc.gen_rotation_keys(rots)
    gpu = F.Context(logn, L, 40, 60, 3, seed=L + logn, keygen=False)
    gpu.load_keys_from(orc, rots)
    rng = np.random.default_rng(L)
    alpha = orc.alpha
    for ell in sorted({L + 1, 2 * alpha, alpha + 1, alpha, 7, 1}):
        if ell > L + 1:
            continue
        d = np.stack([rng.integers(0, int(q), size=orc.n, dtype=np.uint64) for q in orc.primes[:ell]])
        assert np.array_equal(orc.modup(d), gpu.modup(d)), f'modup logN={logn} L={L} ell={ell}'
    xs = [orc.encrypt(rng.uniform(-1, 1, 16), 16) for _ in range(3)]
    gx = [gpu.from_oracle(x) for x in xs]
    oc, gc = xs[0], gx[0]
    for i in range(min(L - 2, 12)):
        oc, gc = orc.mul(oc, xs[1]), gpu.mul(gc, gx[1])
        if i % 4 == 0:
            same(gc, oc, f'product {i} logN={logn} L={L}')
            for k in rots:
                same(gpu.rotate(gc, k), orc.rotate(oc, k), f'rotation {k} logN={logn} L={L}')
    same(gc, oc, f'chain logN={logn} L={L}')
    with F.KernelClock(gpu) as clk:
        st = gpu.mul(gpu.stack(gx), gx[2])
    names = set(k.split('<')[0] for k in clk.stats)
    assert {'k_modup_fold', 'k_moddown_rescale_fold'} <= names, sorted(names)
    for m in range(3):
        same(gpu.member(st, m), orc.mul(xs[m], xs[2]), f'stacked member {m} logN={logn} L={L}')
    print('ok', logn, L, alpha, flush=True)
print('ALLOK')
'''


def test_folded_conversions_forced_on():
    env = dict(os.environ, FHE_MODUP_FOLD='1', FHE_MODDOWN_FOLD='1')
    r = subprocess.run([sys.executable, '-c', CHILD, os.path.join(REPO, 'fhe-sorting_amd'), os.path.join(REPO, 'oracle')],
                       env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0 and 'ALLOK' in r.stdout, f'rc={r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-3000:]}'
