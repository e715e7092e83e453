"""Device-side CKKS encoding (csrc/device/encode.hip, verdict r3 item 7): the
special inverse FFT restated in fp64 on the GPU, the rounding, RNS split and
NTT -- word-identical to the host encoder and to the CPU oracle's, at rings
2^12 and 2^16.  The DirectSort masks and checking vectors (src/sort_algo.h:
206-233 mask_vector, 272-286 checking_vector, 289-306 vector_rotate) are
generated on the device too; a sort that re-encodes them all at its start
(fhe_set_mask_cache(0), the reference's per-sort encoding) gives the same words
as the cached one and as the oracle.  All calls go through the C ABI."""
import numpy as np
import pytest

import fhesort as F
import pyoracle as O

pytestmark = pytest.mark.gpu


def mask_vector(num_slots, N, k):  # src/sort_algo.h:206-233
    v = np.zeros(num_slots)
    v[k * N:(k + 1) * N] = 1.0
    return v


def vector_rotate(v, r):  # src/sort_algo.h:289-306 (left rotation by r)
    return np.roll(v, -r)


def checking_vector(num_slots, N, k):  # src/sort_algo.h:272-286
    return np.array([(k + i // N) % N for i in range(num_slots)], dtype=np.float64)


@pytest.mark.parametrize('logN', [12, 16])
def test_device_encode_matches_host_and_oracle(logN):
    L = 6
    orc = O.Context(logN, L, 40, 60, 3, seed=5, keygen=False)
    gpu = F.Context(logN, L, 40, 60, 3, seed=5, keygen=False)
    rng = np.random.default_rng(logN)
    n = 1 << logN
    for slots in (4, 64, n // 2):
        for level in (0, 3, L):
            v = rng.uniform(-1, 1, slots)
            want = orc.encode(v, slots, level).data()
            assert np.array_equal(gpu.encode(v, slots, level).data(), want)
            got = gpu.encode_device(v, slots, level).data()
            if not np.array_equal(got, want):
                bad = np.argwhere(got != want)
                raise AssertionError(f'slots {slots} level {level}: {len(bad)} words differ, first {bad[0].tolist()}')
    # values that round at half-integers and large magnitudes (scale 2^40)
    v = np.array([0.5 / 2 ** 40, -0.5 / 2 ** 40, 1.0, -1.0, 3.75, 1e3, -1e3, 0.0])
    assert np.array_equal(gpu.encode_device(v, 8, 1).data(), orc.encode(v, 8, 1).data())


@pytest.mark.parametrize('logN,N', [(12, 16), (16, 1024)])
def test_device_masks_match_host_encoder(logN, N):
    """kind 0 (mask_vector rotated by r, positive and negative r) and kind 1
    (checking_vector) at several levels in one batch == fhe_pt_encode of the
    restated vectors"""
    L = 8
    gpu = F.Context(logN, L, 40, 60, 3, seed=6, keygen=False)
    num_slots = min(N * N, (1 << logN) // 2)
    parts = num_slots // N
    specs = [(0, 0, 0, 2), (0, parts - 1, 5, 2), (0, 1, -3, 4), (0, parts // 2, -(N // 2), 7),
             (1, 0, 0, 3), (1, N // 2, 0, 3), (1, N - 1, 0, 8), (0, 1, num_slots - 1, 0)]
    pts = gpu.encode_masks(specs, num_slots, N)
    for (kind, k, r, level), pt in zip(specs, pts):
        v = vector_rotate(mask_vector(num_slots, N, k), r) if kind == 0 else checking_vector(num_slots, N, k)
        want = gpu.encode(v, num_slots, level).data()
        assert np.array_equal(pt.data(), want), (kind, k, r, level)


def test_per_sort_masks_sort_matches_cached_and_oracle():
    """DirectSort N=64 at ring 2^11 (4 stacked batches, 2 lanes): with the masks
    re-encoded on the device at the start of every sort the output words equal
    the cached sort's and the oracle's, sort after sort"""
    N, cfg = 64, (3, 3, 2)
    depth, rots = O.size_parameters(N)
    orc = O.Context(11, depth, 40, 60, 3, seed=7)
    orc.gen_rotation_keys(rots)
    gpu = F.Context(11, depth, 40, 60, 3, seed=7, keygen=False)
    gpu.load_keys_from(orc, rots)
    gpu.set_sort_lanes(2)
    x = np.random.default_rng(66).permutation(N) / N
    ox = orc.encrypt(x, N)
    gx = gpu.from_oracle(ox)
    want = orc.direct_sort(ox, N, rots, cfg).data()
    cached = gpu.direct_sort(gx, N, rots, cfg).data()
    assert np.array_equal(cached, want)
    gpu.set_mask_cache(False)
    for _ in range(2):
        assert np.array_equal(gpu.direct_sort(gx, N, rots, cfg).data(), want)
    gpu.set_mask_cache(True)
