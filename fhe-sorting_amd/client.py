"""Client side of the competition CLI (bin/fhesort, the reference's
src/main.cpp + src/sort.h): produces the files the CLI reads and reads the one
it writes.  The reference ships no such tool -- its harness hands the CLI an
OpenFHE context, keys and ciphertext -- so this is the engine's equivalent of
that harness, in the engine's wire format (csrc/wire/wire.hpp).

  python fhe-sorting_amd/client.py setup   --dir D [--config src/config.json] [--n 128] [--sign 4,3,3] ...
  python fhe-sorting_amd/client.py encrypt --dir D --values v.npy|--testcase T.json|--random SEED [--n 128] --output x.bin
  python fhe-sorting_amd/client.py decrypt --dir D --input y.bin [--n 128] [--output y.npy]
  bin/fhesort --cc D/cc.bin --key_pub D/key_pub.bin --key_mult D/key_mult.bin \\
              --key_rot D/key_rot.bin --input x.bin --output y.bin

setup writes cc.bin, key_pub.bin, key_mult.bin, key_rot.bin (what the CLI
loads) and key_sec.bin (kept by the client for decrypt).  Its defaults are the
reference CLI's context, src/config.json:1-9 (REFERENCE_CONFIG: ring 131072,
multDepth 44, 40-bit scaling, batch 128, main.cpp's 21 rotations); --config
reads another file of that format, --log-n / --depth / --scale-bits override.
encrypt --testcase reads the reference's src/testcase.json format
(runs[0].input[].value) and divides by 255, constructRank's inputOver255
normalisation (src/sort_algo.h:419-421).
"""
import json
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import fhesort as F  # noqa: E402

# main.cpp:38-40: the rotation set the CLI sorts N = 128 with
MAIN_ROTATIONS = [-1, -2, -4, -8, -16, -32, 1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384]
# src/config.json:1-9, the context the reference CLI runs in
REFERENCE_CONFIG = {'indexes_for_rotation_key': MAIN_ROTATIONS, 'mult_depth': 44, 'ring_dimension': 131072,
                    'scale_mod_size': 40, 'batch_size': 128, 'enable_bootstrapping': False}
TESTCASE_SCALE = 255.0  # inputOver255 (src/sort_algo.h:419-421)
# sign-composite depth per round: g_n / f_n polynomial depths (src/sign.cpp:8-158:
# g3, f3 degree 7; g4 degree 27 in PS form, f4 degree 15)
_G, _F = {3: 3, 4: 5}, {3: 3, 4: 4}
FILES = {'cc': 'cc.bin', 'pub': 'key_pub.bin', 'mult': 'key_mult.bin', 'rot': 'key_rot.bin', 'sec': 'key_sec.bin'}


def cli_rotations(N):
    """The rotation set bin/fhesort uses for N (sort_cli.cpp)."""
    return list(MAIN_ROTATIONS) if N == 128 else F.size_parameters(N)[1]


def setup_rotations(N, conf):
    """The rotation keys `setup` generates: the config's indexes_for_rotation_key
    for N = 128 (src/main.cpp's context), else bin/fhesort's set for N -- always
    including every rotation bin/fhesort uses (sort_cli.cpp), so a config with a
    different list cannot leave the CLI without a key at sort time (advisor r5).
    Returns (rotations, the CLI rotations the config lacked)."""
    need = cli_rotations(N)
    if N == 128 and conf.get('indexes_for_rotation_key'):
        rots = [int(r) for r in conf['indexes_for_rotation_key']]
        have = set(rots)
        added = [r for r in need if r not in have]
        return rots + added, added
    return list(need), []


def table_sign_config(N):
    """DirectSortTest's CompositeSign per N (tests/DirectSortTest.cpp:104-112),
    the configuration getSizeParameters' depth is sized for."""
    return (3, 2, 2) if N <= 16 else (3, 3, 2) if N <= 128 else (3, 4, 2) if N <= 512 else (3, 5, 2)


def sign_depth(cfg):
    n, dg, df = cfg
    if n not in _G:
        raise ValueError(f'sign depth for n = {n} unknown: pass --depth')
    return dg * _G[n] + df * _F[n]


def required_depth(N, cfg):
    """getSizeParameters' depth (sort_algo.h:87-201) re-sized from the test's
    sign configuration to `cfg` (the CLI's CompositeSign(4, 3, 3) at N = 128: 42)."""
    return F.size_parameters(N)[0] - sign_depth(table_sign_config(N)) + sign_depth(cfg)


def _path(d, k):
    return os.path.join(d, FILES[k])


def load_config(path):
    """a reference config.json (src/config.json's keys); REFERENCE_CONFIG if None"""
    if not path:
        return dict(REFERENCE_CONFIG)
    c = json.load(open(path))
    missing = [k for k in ('mult_depth', 'ring_dimension', 'scale_mod_size') if k not in c]
    if missing:
        raise SystemExit(f'{path}: missing {missing}')
    if c.get('enable_bootstrapping'):
        raise SystemExit(f'{path}: bootstrapping contexts are not supported by the CLI')
    return c


def setup(a):
    cfg = tuple(int(x) for x in a.sign.split(','))
    conf = load_config(a.config)
    ring = int(conf['ring_dimension'])
    if ring & (ring - 1):
        raise SystemExit(f'ring_dimension {ring} is not a power of two')
    log_n = a.log_n or ring.bit_length() - 1
    scale_bits = a.scale_bits or int(conf['scale_mod_size'])
    depth = a.depth or int(conf['mult_depth'])
    need = required_depth(a.n, cfg)
    if depth < need:
        raise SystemExit(f'depth {depth} < {need} needed by DirectSort<{a.n}> with CompositeSign{cfg}')
    os.makedirs(a.dir, exist_ok=True)
    ctx = F.Context(log_n, depth, scale_bits, 60, 3, seed=a.seed, device=a.device)
    rots, added = setup_rotations(a.n, conf)
    if added:
        print(f'setup: the config\'s indexes_for_rotation_key lacks {len(added)} rotation(s) bin/fhesort uses '
              f'for N = {a.n} ({added[:8]}{"..." if len(added) > 8 else ""}); their keys are generated too')
    ctx.gen_rotation_keys(rots)
    ctx.serialize(_path(a.dir, 'cc'))
    ctx.serialize_public_key(_path(a.dir, 'pub'))
    ctx.serialize_eval_mult_key(_path(a.dir, 'mult'))
    ctx.serialize_eval_automorphism_key(_path(a.dir, 'rot'))
    ctx.serialize_secret_key(_path(a.dir, 'sec'))
    print(f'setup: ring 2^{log_n}, depth {depth}, scale 2^{scale_bits}, sign {cfg}, '
          f'{len(rots)} rotations -> {a.dir}')
    ctx.close()


def _client_ctx(a, secret=False):
    ctx = F.Context.deserialize(_path(a.dir, 'cc'), a.device)
    ctx.deserialize_public_key(_path(a.dir, 'pub'))
    if secret:
        ctx.deserialize_secret_key(_path(a.dir, 'sec'))
    return ctx


def testcase_values(path):
    """the input values of a reference testcase file (src/testcase.json format)"""
    run = json.load(open(path))[0]['runs'][0]
    return np.array([v for e in run['input'] for v in (e['value'] if isinstance(e, dict) else [e])], dtype=np.float64)


def encrypt(a):
    if a.testcase:
        v = testcase_values(a.testcase) / TESTCASE_SCALE
    elif a.values:
        v = np.load(a.values) if a.values.endswith('.npy') else np.loadtxt(a.values)
    else:
        v = np.random.default_rng(a.random).permutation(a.n) / a.n
    v = np.asarray(v, dtype=np.float64).ravel()
    if len(v) != a.n:
        raise SystemExit(f'{len(v)} values for --n {a.n}')
    ctx = _client_ctx(a)
    ctx.serialize_ciphertext(ctx.encrypt(v, a.n), a.output)
    ctx.close()


def decrypt(a):
    ctx = _client_ctx(a, secret=True)
    y = ctx.decrypt(ctx.deserialize_ciphertext(a.input))[:a.n]
    if a.output:
        np.save(a.output, y)
    else:
        print(' '.join(f'{x:.6f}' for x in y))
    ctx.close()


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split('\n\n')[0])
    sub = p.add_subparsers(dest='cmd', required=True)
    for name in ('setup', 'encrypt', 'decrypt'):
        s = sub.add_parser(name)
        s.add_argument('--dir', required=True)
        s.add_argument('--n', type=int, default=128)
        s.add_argument('--device', type=int, default=0)
        if name == 'setup':
            s.add_argument('--config', default=None,
                           help='a reference config.json (default: src/config.json\'s values, REFERENCE_CONFIG)')
            s.add_argument('--log-n', type=int, default=0, help='override the config\'s ring dimension')
            s.add_argument('--scale-bits', type=int, default=0, help='override scale_mod_size')
            s.add_argument('--sign', default='4,3,3')
            s.add_argument('--depth', type=int, default=0, help='override mult_depth')
            s.add_argument('--seed', type=int, default=0,
                           help='0 (default): keys from the OS CSPRNG; nonzero: reproducible keys, for tests only')
        elif name == 'encrypt':
            g = s.add_mutually_exclusive_group(required=True)
            g.add_argument('--values')
            g.add_argument('--testcase', help='a reference testcase.json (values / 255)')
            g.add_argument('--random', type=int)
            s.add_argument('--output', required=True)
        else:
            s.add_argument('--input', required=True)
            s.add_argument('--output')
    a = p.parse_args(argv)
    {'setup': setup, 'encrypt': encrypt, 'decrypt': decrypt}[a.cmd](a)


if __name__ == '__main__':
    main()
