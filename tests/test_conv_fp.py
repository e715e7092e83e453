"""The fp64 basis conversions (kernels.hip k_moddown_rescale_fp and k_modup_fp,
round 6) are
exact: tests/conv_fp_check.cpp replays the kernel's fp64 arithmetic on the
engine's own tables (host::make_level_tables, g++ -ffp-contract=off, correctly
rounded fma()) and compares every output with exact 128-bit integers, at the
contexts the sorts run (the bench's ring 2^16 / depth 39 / 40-bit, MEHP24's ring
2^17 / depth 64 with K = 16, the CLI's ring 2^17 / depth 44, BASELINE config 2),
with the halfway-reduction form forced as well.  A 59-bit context (k-way) has no
fp targets.  The GPU side of the same claim: every HMult parity and digest test
runs the kernel.  Test infrastructure only; no GPU."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
HOST = os.path.join(HERE, '..', 'fhe-sorting_amd', 'csrc', 'host', 'hostmath.cpp')


@pytest.fixture(scope='module')
def exe(tmp_path_factory):
    out = tmp_path_factory.mktemp('convfp') / 'conv_fp_check'
    try:
        subprocess.run(['g++', '-O2', '-std=c++17', '-ffp-contract=off', '-o', str(out),
                        os.path.join(HERE, 'conv_fp_check.cpp'), HOST, '-lm'], check=True, capture_output=True)
    except (OSError, subprocess.CalledProcessError) as e:
        pytest.skip(f'no host C++ compiler: {e}')
    return str(out)


@pytest.mark.parametrize('cfg,mid', [((16, 39, 40, 3), 0), ((17, 65, 40, 3), 0), ((17, 44, 40, 3), 0),
                                     ((16, 30, 40, 3), 0), ((12, 20, 40, 3), 0), ((16, 40, 59, 3), -1)])
def test_conversions_fp_exact(exe, cfg, mid):
    for seed, force in ((1, 0), (2, 1)):
        r = subprocess.run([exe, *map(str, cfg), '1500', str(seed), str(force)], capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0 and r.stdout.startswith('ok'), r.stdout + r.stderr
        f = r.stdout.split()  # ok <mid> <checked> K=<K> modup <mid> <checked>
        for got, n in ((int(f[1]), int(f[2])), (int(f[5]), int(f[6]))):
            if mid < 0:
                assert got == -1
            else:
                assert got == (1 if force else mid) and n > 0
