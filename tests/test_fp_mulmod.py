"""The fp64 NTT arithmetic (ntt.hip fp_mulmod / fp_reduce / fp_in / fp_out, the
FP launches for primes < 2^41) is exact at the bounds DESIGN.md §5 derives:
checked on the host against 128-bit integers (tests/fp_mulmod_check.c, gcc,
-ffp-contract=off, correctly rounded fma()).  The GPU side of the same claim is
every ring-2^16/2^17 parity and digest test, which runs the FP passes."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def test_fp_mulmod_exact(tmp_path):
    exe = tmp_path / 'fp_mulmod_check'
    try:
        subprocess.run(['gcc', '-O2', '-ffp-contract=off', '-o', str(exe), os.path.join(HERE, 'fp_mulmod_check.c'),
                        '-lm'], check=True, capture_output=True)
    except (OSError, subprocess.CalledProcessError) as e:
        pytest.skip(f'no host C compiler: {e}')
    for seed in (1, 2, 3):
        out = subprocess.run([str(exe), '600000', str(seed)], capture_output=True, text=True, timeout=300)
        assert out.returncode == 0 and out.stdout.startswith('ok'), out.stdout + out.stderr
