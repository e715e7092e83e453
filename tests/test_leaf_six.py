"""The six-digit row layout of the folded leaf sums (kernels.hip k_leaf_sums_fold,
FHE_LEAF_SIX, round 6) rests on two host-checkable facts, restated here: (1) the
balanced base-256 digits 6 and 7 of every constant d < 2^41 (an FP-class prime's
canonical residue) are zero, and the six digits still rebuild d; (2) the pair
layout -- blocks 3p + g hold group g's digits 0-3 at row 4 ta + b, block 3p + 2
holds both groups' digits 4-5 at row 4 ta + 2 g + b - 4 -- places every
(group, output, digit) of a pair on its own row, and the lane group that holds
output ta's digits 0-3 (rows 4 ta .. 4 ta + 3 of the group's block) also holds its
digits 4-5 (rows 4 ta + 2 g, + 1 of block 3p + 2), so the fold needs no cross-lane
data.  The GPU side (word-identical sums) is tests/test_gpu_mfma.py and the
digest tests.  No GPU."""
import numpy as np


def balanced_digits(c):
    """kernels.hip balanced_digits: 8 signed base-256 digits of c < 2^60."""
    out, v = [], int(c)
    for _ in range(8):
        dig = v & 255
        if dig >= 128:
            dig -= 256
        v = (v - dig) >> 8
        out.append(dig)
    assert v == 0
    return out


def test_fp_constants_have_six_digits():
    rng = np.random.default_rng(41)
    edge = [0, 1, 127, 128, 255, 256, (1 << 40) - 1, 1 << 40, (1 << 41) - 1, (1 << 41) - 129,
            int('7f' * 5, 16), int('80' * 5, 16), int('ff' * 5, 16)]
    vals = edge + [int(x) for x in rng.integers(0, 1 << 41, size=20000, dtype=np.int64)]
    for d in vals:
        e = balanced_digits(d)
        assert e[6] == 0 and e[7] == 0, (d, e)
        assert sum(b * 256 ** k for k, b in enumerate(e[:6])) == d
    # a 60-bit prime's residues need all eight (the integer class keeps eight rows)
    assert any(balanced_digits(d)[6] != 0 for d in [(1 << 59) + 12345, (1 << 55) - 3])


def test_pair_layout_is_a_bijection_and_lane_local():
    seen = {}
    for g in range(2):          # group within the pair
        for ta in range(4):     # output within the group
            for b in range(6):  # digit
                blk = g if b < 4 else 2
                row = 4 * ta + b if b < 4 else 4 * ta + 2 * g + (b - 4)
                assert 0 <= row < 16
                assert (blk, row) not in seen
                seen[(blk, row)] = (g, ta, b)
                # the MFMA result layout: lane group lg holds rows 4 lg .. 4 lg + 3
                assert row // 4 == ta
    assert len(seen) == 48  # three full 16-row blocks
    # the fold's second operand for group g: rows 2g, 2g + 1 of the lane's four
    for g in range(2):
        for ta in range(4):
            assert [seen[(2, 4 * ta + 2 * g + k)][2] for k in range(2)] == [4, 5]
