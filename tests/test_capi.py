"""CPU checks of the drop-in boundary: the HIP library loads, exports every
symbol include/fhe_gpu.h declares, and its pure-host entry points
(Decomposer, size parameters) agree with the oracle and the reference's
tables.  No GPU compute is issued here.
"""
import ctypes
import re
import subprocess

import numpy as np
import pytest

import fhesort as F
import pyoracle as O


def declared_symbols():
    src = open(F.HEADER).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(fhe_[a-z0-9_]+)\s*\(', src)))


def test_header_declares_the_boundary():
    names = declared_symbols()
    for must in ('fhe_ctx_create', 'fhe_ctx_load_keys', 'fhe_ct_upload', 'fhe_ct_download', 'fhe_mul_relin',
                 'fhe_rotate', 'fhe_rotate_hoisted', 'fhe_cheb_ps', 'fhe_sign_composite', 'fhe_compare',
                 'fhe_indicator', 'fhe_direct_sort', 'fhe_comm_init', 'fhe_ct_allreduce', 'fhe_ntt', 'fhe_modup',
                 'fhe_moddown', 'fhe_automorph'):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(F.LIB_PATH)
    missing = [n for n in declared_symbols() if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(['nm', '-D', '--defined-only', F.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r' T (fhe_[a-z0-9_]+)', out))
    assert set(declared_symbols()) <= exported


def test_library_has_gfx950_code_objects():
    data = open(F.LIB_PATH, 'rb').read()
    assert b'gfx950' in data
    assert b'k_ntt_fwd' in data and b'k_ntt_inv' in data and b'k_ks_inner' in data


def test_binding_loads_without_gpu():
    F.lib()  # binds every signature; no HIP call issued


@pytest.mark.parametrize('N', [4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048])
def test_size_parameters_match_oracle(N):
    assert F.size_parameters(N) == O.size_parameters(N)


def test_decomposer_matches_oracle():
    rng = np.random.default_rng(0)
    for N in (128, 1024):
        _, rots = O.size_parameters(N)
        for r in rng.integers(1, 4 * N, size=40):
            for algo in (F.NAF, F.BNAF, F.BINARY):
                assert F.decompose(N, rots, int(r), N * N // 2, algo) == O.decompose(N, rots, int(r), N * N // 2, algo)


def test_errors_cross_as_status_codes():
    with pytest.raises(F.FheError) as e:
        F.size_parameters(3)
    assert e.value.code == F.FHE_EINVAL


def test_binding_declares_every_entry_point():
    """Every C-ABI function has a ctypes signature in fhesort.py: without one ctypes
    passes Python ints as 32-bit C ints and truncates handle pointers (a missing
    entry once segfaulted a GPU test)."""
    missing = [f for f in declared_symbols() if f not in F._SIGS]
    assert not missing, missing


def test_secure_sampler_block_matches_rfc8439():
    """The secure sampler (seed 0: secret, errors and encryption randomness) is
    ChaCha20; its block function reproduces RFC 8439 §2.3.2's test vector."""
    key = np.frombuffer(bytes(range(32)), dtype='<u4')
    nonce = np.frombuffer(bytes.fromhex('000000090000004a00000000'), dtype='<u4')
    want = bytes.fromhex('10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e'
                         'd2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e')
    assert F.prng_block(key, 1, nonce).astype('<u4').tobytes() == want

