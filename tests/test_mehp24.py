"""MEHP24 (Mazzone et al.) sort on the CPU oracle, and the host-side parameter
logic of the engine's C-ABI (no GPU needed).

The reference's own check (tests/mehp24/Mehp24SortTest.cpp:144-185) is the
decrypted output against std::sort of the input, max error < 0.01; its
parameter table (depth per N, CompositeSign config, dg_i/df_i, sortFG vs
sortLargeArrayFG) is pinned below.  The reference ships no MEHP24 golden
ciphertexts, so oracle parity beyond that property is unpinned; the GPU tests
(test_gpu_mehp24.py) hold the engine bit-exact to this oracle.
"""
import numpy as np
import pytest

import fhesort as F
import pyoracle as O

# tests/mehp24/Mehp24SortTest.cpp:33-64 (depth), 117-128 (Cfg, dg_i, df_i), 136-143 (N > 256 splits)
REF_TABLE = {4: 31, 8: 35, 16: 35, 32: 42, 64: 42, 128: 46, 256: 49, 512: 57, 1024: 60, 2048: 64}


def ref_rotation_indices(N, sub=256):
    """mehp24::utils::getRotationIndices (src/mehp24/mehp24_utils.cpp:197-225)
    restated from its loop structure, duplicates and 0 removed."""
    out, sz = [], N
    if N > sub:
        for i in range(N // sub):
            out += [i * sub, -i * sub]
        sz = sub
    lg = int(np.log2(sz))
    for i in range(lg):
        t = sz * (sz - 1) // (1 << (i + 1))
        out += [1 << i, -(1 << i), -(1 << (lg + i)), t, -t]
    res = []
    for k in out:
        if k != 0 and k not in res:
            res.append(k)
    return res


def test_rotation_indices_known_answer():
    assert O.mehp24_rotation_indices(4) == [1, -1, -4, 6, -6, 2, -2, -8, 3, -3]
    for N in (4, 8, 64, 256, 512, 2048):
        assert O.mehp24_rotation_indices(N) == ref_rotation_indices(N)
        assert F.mehp24_rotation_indices(N) == ref_rotation_indices(N)
    assert F.mehp24_rotation_indices(16, 4) == ref_rotation_indices(16, 4) == O.mehp24_rotation_indices(16, 4)


@pytest.mark.parametrize('N', sorted(REF_TABLE))
def test_parameters_match_reference_test(N):
    p = F.mehp24_parameters(N)
    assert p['depth'] == REF_TABLE[N] and p['log_ring'] == 17 and p['scale_bits'] == 40
    assert p['cfg'] == (3, 2 if N <= 16 else 3 if N <= 128 else 4 if N <= 512 else 5, 2)
    assert p['dg_i'] == (int(np.log2(N)) + 1) // 2 and p['df_i'] == 2
    assert p['sub'] == (0 if N <= 256 else 256)
    assert p['rots'] == ref_rotation_indices(N)
    assert p['dnum'] == 3  # OpenFHE's default digit count, which the reference leaves in place


def test_parameters_4096_extension():
    """N=4096 (BASELINE config 5) is beyond the reference table (which ends at
    2048); it keeps 2048's Cfg (3,5,2), dg_i = 6 and depth, parts of 256."""
    p, q = F.mehp24_parameters(4096), F.mehp24_parameters(2048)
    assert (p['depth'], p['cfg'], p['dg_i'], p['df_i'], p['sub']) == (q['depth'], q['cfg'], 6, 2, 256)
    assert p['rots'] == ref_rotation_indices(4096)


def test_parameters_reject_bad_n():
    with pytest.raises(F.FheError):
        F.mehp24_parameters(12)


def _sort(N, sub, logN=11, depth=35, seed=3):
    cfg = (3, 2, 2) if N <= 16 else (3, 3, 2)
    dg_i = (int(np.log2(N)) + 1) // 2
    orc = O.Context(logN, depth, 40, 60, 3, seed=seed)
    orc.gen_rotation_keys(O.mehp24_rotation_indices(N, sub or 256))
    x = np.random.default_rng(seed).permutation(N) / N  # getVectorWithMinDiff(N, 0, 1, 1/N)
    ct = orc.encrypt(x, N * N if sub == 0 else sub * sub)
    out = orc.mehp24_sort(ct, N, cfg, dg_i, 2, sub)
    return x, orc.decrypt(out)[:N], out


def test_oracle_sort_fg_single():
    x, y, out = _sort(4, 0)
    assert np.max(np.abs(y - np.sort(x))) < 0.01
    assert out.level <= 31


def test_oracle_sort_large_array_split():
    """sortLargeArrayFG path (split, multi-ciphertext sortFG, combine) with
    parts of 4 values instead of 256, so it runs at ring 2^11."""
    x, y, _ = _sort(8, 4)
    assert np.max(np.abs(y - np.sort(x))) < 0.01


def test_oracle_indicator_adv():
    orc = O.Context(11, 20, 40, 60, 3, seed=1)
    v = np.array([-3.0, -2.0, -1.0, -0.2, 0.0, 0.1, 1.0, 2.0, 3.0, 0.25])  # ranks minus targets: integers
    r = orc.decrypt(orc.mehp24_indicator(orc.encrypt(v, 16), 4.0, 2, 2))[:len(v)]
    want = (np.abs(v) < 0.5).astype(float)
    assert np.max(np.abs(r - want)) < 0.05, r
