"""Batched giant-step rotations (round 4): RotationComposerN::rotateMembers, the
form DirectSort's blindRotationOptN / vecRotsOpt now take
(src/sort_algo.h:326-366, 561-584).  Member m of a stacked batch rotated by its
own amount through the same keyed steps as the composer's rotate() -- zero,
keyed, composed, negative and wrapping amounts, members whose step lists differ
in length -- must give, word for word, the member-wise rotations.  Through the C
ABI (fhe_compose_rotate_members)."""
import numpy as np
import pytest

import fhesort as F

pytestmark = pytest.mark.gpu

KEYS = [1, 2, 4, 8, 16, 32, 64, -1, -2, -4, -8, -16, -32, -64]


@pytest.mark.parametrize('algo', [0, 2])  # NAF, BINARY
def test_rotate_members_equals_member_wise(algo):
    N, slots = 128, 128
    ctx = F.Context(12, 6, 40, 60, 3, seed=31)
    ctx.gen_rotation_keys(KEYS)
    rng = np.random.default_rng(31)
    amounts = [0, 1, 3, -5, 100, 127, -64, 77]
    cts = [ctx.encrypt(rng.uniform(-1, 1, slots), slots) for _ in amounts]
    st = ctx.stack(cts)
    got = ctx.compose_rotate_members(st, N, KEYS, algo, amounts)
    for m, (c, r) in enumerate(zip(cts, amounts)):
        want = ctx.compose_rotate(c, N, KEYS, algo, r).data()
        assert np.array_equal(ctx.member(got, m).data(), want), (m, r)
    # one member: the plain path
    one = ctx.compose_rotate_members(ctx.stack(cts[:1]), N, KEYS, algo, [37])
    assert np.array_equal(ctx.member(one, 0).data(), ctx.compose_rotate(cts[0], N, KEYS, algo, 37).data())
