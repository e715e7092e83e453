"""Wire format (csrc/wire/wire.hpp; the file boundary of the reference's CLI,
src/sort.h:31-102) on the CPU: the library's header / checksum validation
against files written by the independent restatement in tests/wire_spec.py,
the error codes for damaged files, and the client's depth rule."""
import json
import os

import numpy as np
import pytest

import fhesort as F
import wire_spec as W


def _client():
    import importlib.util
    spec = importlib.util.spec_from_file_location('fhe_client', os.path.join(os.path.dirname(F.__file__), 'client.py'))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _ct_file(tmp_path, name='ct.bin', n=16, limbs=3):
    rng = np.random.default_rng(3)
    words = rng.integers(0, 1 << 59, size=(2, limbs, n), dtype=np.uint64)
    body = W.ciphertext_body(2, 8, 2.0 ** 50, words)
    p = tmp_path / name
    p.write_bytes(W.pack('ciphertext', 0x1234, 4, 5, 2, body))
    return p, words


@pytest.mark.parametrize('nbody', [0, 1, 2, 3, 4, 5, 17, (1 << 20) + 3])
def test_checksum_agrees_for_every_body_length(tmp_path, nbody):
    # the library hashes the header words, then the body in 8-MiB chunks, keeping
    # word j on lane j mod 4 across calls; the restatement hashes in one go
    body = np.arange(nbody, dtype=np.uint64) * np.uint64(0x9e3779b97f4a7c15)
    p = tmp_path / 'b.bin'
    p.write_bytes(W.pack('secret_key', 1, 4, 1, 1, body))
    assert F.wire_inspect(str(p))['body_words'] == nbody


@pytest.mark.parametrize('n,limbs', [(16, 1), (16, 3), (8, 5)])
def test_inspect_accepts_restated_files(tmp_path, n, limbs):
    p, _ = _ct_file(tmp_path, n=n, limbs=limbs)
    info = F.wire_inspect(str(p))
    assert info['kind'] == 'ciphertext'
    assert info['version'] == W.VERSION
    assert info['params_id'] == 0x1234
    assert (info['log_n'], info['nq'], info['K']) == (4, 5, 2)
    assert info['body_words'] == 5 + 2 * limbs * n


def test_every_kind_round_trips_through_inspect(tmp_path):
    for kind in W.KINDS:
        p = tmp_path / f'{kind}.bin'
        p.write_bytes(W.pack(kind, 7, 12, 3, 1, np.arange(11, dtype=np.uint64)))
        assert F.wire_inspect(str(p))['kind'] == kind


def test_damaged_files_are_rejected_with_eio(tmp_path):
    p, _ = _ct_file(tmp_path)
    raw = bytearray(p.read_bytes())
    cases = {
        'flipped body bit': raw[:80] + bytes([raw[80] ^ 1]) + raw[81:],
        'flipped header word': raw[:24] + bytes([raw[24] ^ 4]) + raw[25:],
        'truncated': raw[:-8],
        'extra bytes': raw + b'\0' * 8,
        'bad magic': b'X' + raw[1:],
        'short': raw[:20],
    }
    for what, data in cases.items():
        q = tmp_path / 'bad.bin'
        q.write_bytes(bytes(data))
        with pytest.raises(F.FheError) as e:
            F.wire_inspect(str(q))
        assert e.value.code == F.FHE_EIO, what
    with pytest.raises(F.FheError) as e:
        F.wire_inspect(str(tmp_path / 'missing.bin'))
    assert e.value.code == F.FHE_EIO


def test_wrong_version_is_rejected(tmp_path):
    data = bytearray(W.pack('ciphertext', 1, 4, 5, 2, np.zeros(4, dtype=np.uint64)))
    w = np.frombuffer(bytes(data), dtype=np.uint64).copy()
    w[1] = 2 | (5 << 32)
    w[-1] = W.checksum(w[1:-1])
    q = tmp_path / 'v2.bin'
    q.write_bytes(w.tobytes())
    with pytest.raises(F.FheError) as e:
        F.wire_inspect(str(q))
    assert e.value.code == F.FHE_EIO and 'version' in str(e.value)


def test_restated_parser_reads_what_it_wrote(tmp_path):
    p, words = _ct_file(tmp_path)
    level, slots, limbs, scale, got = W.ciphertext(p.read_bytes(), 16)
    assert (level, slots, limbs, scale) == (2, 8, 3, 2.0 ** 50)
    assert np.array_equal(got, words)


def test_cli_depth_rule():
    """client.required_depth: getSizeParameters' depth re-sized to the CLI's
    CompositeSign(4, 3, 3).  N = 8 -> 39 was found as the smallest depth the CPU
    oracle's DirectSort<8> completes with at (4, 3, 3) (it ends at level 39,
    like (3, 2, 2) ends at the table's 24); N = 128 -> 42."""
    c = _client()
    assert c.required_depth(8, (3, 2, 2)) == 24
    assert c.required_depth(8, (4, 3, 3)) == 39
    assert c.required_depth(128, (3, 3, 2)) == 30
    assert c.required_depth(128, (4, 3, 3)) == 42
    assert c.cli_rotations(128) == c.MAIN_ROTATIONS
    assert c.cli_rotations(8) == F.size_parameters(8)[1]


def test_setup_rotations_cover_the_cli():
    """advisor r5: `setup --config X` keys X's indexes_for_rotation_key for N = 128,
    plus every rotation bin/fhesort uses that X lacks (the CLI's set is fixed,
    sort_cli.cpp), so the sort never meets a missing key."""
    c = _client()
    rots, added = c.setup_rotations(128, {'indexes_for_rotation_key': c.MAIN_ROTATIONS})
    assert rots == list(c.MAIN_ROTATIONS) and added == []
    short = list(c.MAIN_ROTATIONS)[:5] + [12345]
    rots, added = c.setup_rotations(128, {'indexes_for_rotation_key': short})
    assert set(c.MAIN_ROTATIONS) <= set(rots) and 12345 in rots
    assert added == [r for r in c.MAIN_ROTATIONS if r not in short]
    rots, added = c.setup_rotations(8, {'indexes_for_rotation_key': [1]})
    assert rots == c.cli_rotations(8) and added == []


def test_client_defaults_are_the_reference_config(tmp_path):
    """Verdict r4 item 1: client.py setup defaults to src/config.json's context
    (ring 131072, multDepth 44, scale 40, batch 128, main.cpp's rotations) and
    reads another config file of that format; encrypt --testcase takes the
    reference's testcase format and divides by 255 (inputOver255)."""
    c = _client()
    ref = c.REFERENCE_CONFIG
    assert (ref['ring_dimension'], ref['mult_depth'], ref['scale_mod_size'], ref['batch_size']) == (131072, 44, 40, 128)
    assert ref['indexes_for_rotation_key'] == c.MAIN_ROTATIONS and c.load_config(None) == ref
    assert c.required_depth(128, (4, 3, 3)) <= ref['mult_depth']
    cfg = tmp_path / 'config.json'
    cfg.write_text(json.dumps({'mult_depth': 40, 'ring_dimension': 65536, 'scale_mod_size': 50}))
    assert c.load_config(str(cfg))['ring_dimension'] == 65536
    tc = tmp_path / 'testcase.json'
    tc.write_text(json.dumps([{'scheme': 'CKKS', 'runs': [{'input': [{'name': 'input', 'value': [2.34, 245.67]}],
                                                          'output': []}]}]))
    assert np.array_equal(c.testcase_values(str(tc)), [2.34, 245.67])


def test_cli_binary_fails_like_the_reference(tmp_path):
    """main.cpp / SortContext::initCC: a missing context file -> message, exit 1."""
    import subprocess
    exe = os.path.join(os.path.dirname(F.__file__), 'bin', 'fhesort')
    assert os.path.exists(exe), 'bin/fhesort not built (run __graft_entry__.build())'
    r = subprocess.run([exe, '--cc', str(tmp_path / 'none.bin')], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1
    assert 'Could not deserialize cryptocontext file' in r.stderr


def test_context_with_absurd_parameters_is_refused(tmp_path):
    """A context file drives allocations: ring 2^40 or depth 10^6 are refused
    before any engine is built (FHE_EINVAL), no GPU needed."""
    for log_n, depth in ((40, 10), (12, 1000000)):
        body = np.array([log_n, depth, 50, 60, 3, 1, 2, 3, 5], dtype=np.uint64)
        p = tmp_path / f'cc_{log_n}_{depth}.bin'
        p.write_bytes(W.pack('context', 1, log_n, depth + 1, 1, body))
        h = F.C.c_void_p()
        rc = F.lib().fhe_deserialize_context(str(p).encode(), 0, F.C.byref(h))
        assert rc == F.FHE_EINVAL and not h.value
        assert 'out of range' in F.lib().fhe_last_error().decode()
