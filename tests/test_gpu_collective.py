"""Collectives and key state on the GPU engine.

* RCCL on hardware: a world-1 communicator is legal on one GPU, so
  fhe_comm_init + fhe_ct_allreduce (ncclAllReduce, u64 sum + mod-q reduce) and
  a DirectSort whose rank/index-check partials go through the RCCL hook
  (src/sort_algo.h:489-490, 740-741 -> ncclAllReduce) run here; the results
  must equal the communicator-free ones word for word.
* The all-reduce protocol's guards: a world whose u64 residue sum could wrap is
  refused before any work, a peer at another level fails every rank before the
  data collective, an exception inside a Python hook reaches the caller.
* Keys loaded after a sort reach every lane engine (forks share one key set).
"""
import ctypes as C

import numpy as np
import pytest

import fhesort as F
import pyoracle as O

pytestmark = pytest.mark.gpu

N, LOGN = 64, 11


def _ctx(seed=31, lanes=1):
    depth, rots = F.size_parameters(N)
    ctx = F.Context(LOGN, depth, 40, 60, 3, seed=seed)
    ctx.gen_rotation_keys(rots)
    ctx.set_sort_stack(2)
    ctx.set_sort_lanes(lanes)
    return ctx, rots


def test_rccl_world1_ct_allreduce_and_sort():
    ctx, rots = _ctx()
    x = np.random.default_rng(5).permutation(N) / N
    ct = ctx.encrypt(x, N)
    ref = ctx.direct_sort(ct, N, rots, (3, 3, 2))        # no communicator
    a = ctx.encrypt(np.linspace(-0.5, 0.5, N), N)
    b = ctx.encrypt(np.linspace(0.25, -0.25, N), N)
    st = ctx.stack([a, b])
    words = lambda: [ctx.member(st, m).data().copy() for m in (0, 1)]
    before = words()
    ctx.comm_init(F.Context.comm_unique_id(), 0, 1)
    ctx.ct_allreduce(st)                                 # ncclAllReduce over both members
    assert all(np.array_equal(x, y) for x, y in zip(words(), before)), 'world-1 all-reduce must be the identity'
    out = ctx.direct_sort(ct, N, rots, (3, 3, 2), shard=(0, 1))  # partials through RCCL
    assert np.array_equal(out.data(), ref.data()), 'RCCL-reduced sort differs from the plain sort'
    with pytest.raises(F.FheError):
        ctx.direct_sort(ct, N, rots, (3, 3, 2), shard=(0, 2))  # communicator world is 1


def test_world_beyond_u64_bound_is_refused():
    ctx, rots = _ctx()
    ct = ctx.encrypt(np.linspace(0, 1, N, endpoint=False), N)
    with pytest.raises(F.FheError, match='overflow') as e:
        ctx.direct_sort(ct, N, rots, (3, 3, 2), shard=(0, 17), allreduce=lambda p, n, u: None)
    assert e.value.code == F.FHE_EINVAL


def test_comm_init_refuses_worlds_beyond_u64_bound():
    """fhe_comm_init checks world * q_max < 2^64 (and the rank) before RCCL is
    touched, so fhe_ct_allreduce never runs a wrapping u64 sum."""
    ctx, _ = _ctx()
    uid = F.Context.comm_unique_id()
    with pytest.raises(F.FheError, match='overflow') as e:
        ctx.comm_init(uid, 0, 17)
    assert e.value.code == F.FHE_EINVAL
    with pytest.raises(F.FheError) as e:
        ctx.comm_init(uid, 1, 1)
    assert e.value.code == F.FHE_EINVAL


def test_mismatched_partial_levels_fail_before_data_allreduce():
    ctx, rots = _ctx()
    ct = ctx.encrypt(np.random.default_rng(2).permutation(N) / N, N)
    hip = C.CDLL('libamdhip64.so')
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    counts = []

    def peer_at_other_level(ptr, count, _user):
        counts.append(int(count))
        h = np.empty(count, dtype=np.uint64)
        assert hip.hipMemcpy(h.ctypes.data, C.cast(ptr, C.c_void_p), count * 8, 2) == 0
        if count == 4 and h[0] == 1:
            l1 = int(h[1]) + 1
            h += np.array([1, l1, l1 * l1, int(h[3]) - 1], dtype=np.uint64)
            assert hip.hipMemcpy(C.cast(ptr, C.c_void_p), h.ctypes.data, count * 8, 1) == 0
    with pytest.raises(F.FheError, match='differ in level'):
        ctx.direct_sort(ct, N, rots, (3, 3, 2), shard=(0, 2), allreduce=peer_at_other_level)
    assert counts and all(c == 4 for c in counts)


def test_exception_in_hook_propagates():
    ctx, rots = _ctx()
    ct = ctx.encrypt(np.random.default_rng(3).permutation(N) / N, N)

    class Boom(Exception):
        pass

    def failing(ptr, count, _user):
        raise Boom('transport down')
    with pytest.raises(Boom):
        ctx.direct_sort(ct, N, rots, (3, 3, 2), shard=(0, 2), allreduce=failing)


def test_keys_loaded_after_a_sort_reach_every_lane():
    """Sort with 2 lanes on keys A, load keys B (secret included), sort again:
    bit-exact with the oracle on keys B (the lane engines share the key set)."""
    depth, rots = F.size_parameters(N)
    x = np.random.default_rng(9).permutation(N) / N
    gpu = F.Context(LOGN, depth, 40, 60, 3, seed=41, keygen=False)
    for seed in (41, 42):
        orc = O.Context(LOGN, depth, 40, 60, 3, seed=seed)
        orc.gen_rotation_keys(rots)
        gpu.load_keys_from(orc, rots)
        gpu.set_sort_stack(1)
        gpu.set_sort_lanes(2)
        ox = orc.encrypt(x, N)
        gout = gpu.direct_sort(gpu.from_oracle(ox), N, rots, (3, 3, 2))
        oout = orc.direct_sort(ox, N, rots, (3, 3, 2))
        assert np.array_equal(gout.data(), oout.data()), f'keys of seed {seed}: GPU differs from the oracle'


@pytest.mark.parametrize('shard', [(0, 0), (2, 2), (-1, 2), (3, 2)])
def test_bad_shard_arguments_are_refused(shard):
    """1 <= shard_world and 0 <= shard_rank < shard_world are
    checked before any work (shard_world 0 used to divide by zero in the batch
    assignment), for the rank sort, the hybrid sort and MEHP24."""
    ctx, rots = _ctx()
    ct = ctx.encrypt(np.random.default_rng(4).permutation(N) / N, N)
    hook = lambda p, n, u: None
    with pytest.raises(F.FheError) as e:
        ctx.direct_sort(ct, N, rots, (3, 3, 2), shard=shard, allreduce=hook)
    assert e.value.code == F.FHE_EINVAL
    ok = ctx.direct_sort(ct, N, rots, (3, 3, 2))  # the cached sorter is unharmed
    assert np.max(np.abs(ctx.decrypt(ok)[:N] - np.sort(ctx.decrypt(ct)[:N]))) < 0.01


def test_bootstrap_correction_bits_bounded():
    """correction bits outside 1..40 are refused (70 used to
    overflow the SlotsToCoeffs factor and hang setup); 0 selects the default 10."""
    ctx = F.Context(11, 30, 59, 60, 3, seed=8)
    for bits in (41, 70, -3):
        with pytest.raises(F.FheError) as e:
            F.Bootstrapper(ctx, 8, (2, 2), correction_bits=bits, keygen=False)
        assert e.value.code == F.FHE_EINVAL
