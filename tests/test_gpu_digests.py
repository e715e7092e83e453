"""Full-size DirectSort pinned bit-exact against the CPU oracle through
committed digests.

tests/golden/make_digests.py ran the oracle once in the build container on the
BASELINE configurations and stored SHA-256 digests of the encrypted input, the
constructRank output (mode 1) and the sorted output.  Here the GPU engine
generates its keys and encrypts from the same seed (GPU keygen/encryption are
word-identical to the oracle's, test_gpu_parity.py::test_keygen_and_encrypt_
parity) and must reproduce every digest, the level (== multDepth,
tests/DirectSortTest.cpp:128) and the decrypted error bound (0.01,
tests/DirectSortTest.cpp:169).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import fhesort as F

pytestmark = pytest.mark.gpu

DB = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'sort_digests.json')))


def digest(words):
    return hashlib.sha256(np.ascontiguousarray(words, dtype='<u8').tobytes()).hexdigest()


@pytest.mark.parametrize('name', sorted(DB))
def test_direct_sort_matches_oracle_digest(name):
    c = DB[name]
    N = c['N']
    depth, rots = F.size_parameters(N)
    assert depth == c['depth'] and [int(r) for r in rots] == c['rotations']
    # records made before the OpenFHE split became the default carry ps_split 0
    ctx = F.Context(c['logN'], depth, c['scale_bits'], 60, c['dnum'], seed=c['seed'],
                    ps_split=c.get('ps_split', F.PS_SPLIT_ENGINE))
    try:
        ctx.gen_rotation_keys(rots)
        x = np.random.default_rng(c['seed']).permutation(N) / N
        ct = ctx.encrypt(x, N)
        assert digest(ct.data()) == c['input_sha256'], 'GPU encryption differs from the oracle run'
        out = ctx.direct_sort(ct, N, rots, tuple(c['cfg']))
        assert out.level == c['level'] == depth
        assert out.info()['scale'] == c['scale']
        assert digest(out.data()) == c['sha256'], 'sorted ciphertext differs from the oracle word for word'
        y = ctx.decrypt(out)[:N]
        err = float(np.max(np.abs(y - np.sort(x))))
        assert err == pytest.approx(c['max_abs_err'], rel=1e-9, abs=1e-12) and err < 0.01
        rank = ctx.direct_sort(ct, N, rots, tuple(c['cfg']), mode=1)
        assert rank.level == c['rank_level']
        assert digest(rank.data()) == c['rank_sha256'], 'constructRank output differs from the oracle'
    finally:
        ctx.close()
