#!/usr/bin/env python3
"""Full-size DirectSort digests from the CPU oracle (test infrastructure).

The oracle (oracle/, a CPU restatement of the reference's algorithm) sorts the
BASELINE configurations once, here in the build container, and the SHA-256 of
the output ciphertext's limb words is committed to tests/golden/sort_digests.json
together with its level, scale and decrypted error.  tests/test_gpu_digests.py
repeats the same sort on the GPU from the same seeds -- GPU key generation and
encryption are word-identical to the oracle's (test_gpu_parity.py::
test_keygen_and_encrypt_parity) -- and compares digests, so the headline
configuration is pinned bit-exact at full size without running the oracle on
the GPU box.

Cases:
  config1   N=8,    ring 2^17, depth 24, scale 40, keys {1,2,4,6,8,16,32,64},
            CompositeSign(3,2,2) -- the shipped DirectSortTest instantiation
            (tests/DirectSortTest.cpp:24-31,105-106,175; src/sort_algo.h:99-102)
  config2   N=128,  ring 2^16, depth 30, scale 40, CompositeSign(3,3,2)
  config3   N=1024, ring 2^16, depth 39, scale 50, CompositeSign(3,5,2) -- the
            round-2 bench workload
  *_of      the same with OpenFHE's Paterson-Stockmeyer split (round 3's
            default) and 40-bit scaling throughout; config3_of is the bench
            workload
Each case pins the sorted output (level multDepth, one limb) and the
constructRank output (mode 1: the rank ciphertext, many limbs).

Input: x = default_rng(20250704).permutation(N) / N (getVectorWithMinDiff's
distribution, tests/utils.h:28-51).  Keys: context seed 20250704.

Run: python tests/golden/make_digests.py [case ...]   (config3 takes ~1 h on 8
cores and ~30 GB of host memory for its rotation keys)
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, '..', '..'))
sys.path.insert(0, os.path.join(REPO, 'oracle'))

SEED = 20250704
CASES = {
    # rounds 1-2: the power-of-two Paterson-Stockmeyer split (ps_split 0)
    'config1': dict(N=8, logN=17, depth=24, scale_bits=40, dnum=3, cfg=(3, 2, 2), ps_split=0),
    'config2': dict(N=128, logN=16, depth=30, scale_bits=40, dnum=3, cfg=(3, 3, 2), ps_split=0),
    'config3': dict(N=1024, logN=16, depth=39, scale_bits=50, dnum=3, cfg=(3, 5, 2), ps_split=0),
    # round 3: OpenFHE's split (the default), the reference's 40-bit scaling for every N
    'config1_of': dict(N=8, logN=17, depth=24, scale_bits=40, dnum=3, cfg=(3, 2, 2), ps_split=1),
    'config2_of': dict(N=128, logN=16, depth=30, scale_bits=40, dnum=3, cfg=(3, 3, 2), ps_split=1),
    'config3_of': dict(N=1024, logN=16, depth=39, scale_bits=40, dnum=3, cfg=(3, 5, 2), ps_split=1),
}
OUT = os.path.join(HERE, 'sort_digests.json')


def digest(words):
    return hashlib.sha256(np.ascontiguousarray(words, dtype='<u8').tobytes()).hexdigest()


def run(name):
    import pyoracle as O
    c = CASES[name]
    N = c['N']
    depth, rots = O.size_parameters(N)
    assert depth == c['depth'], (depth, c['depth'])
    t0 = time.time()
    orc = O.Context(c['logN'], depth, c['scale_bits'], 60, c['dnum'], seed=SEED, ps_split=c['ps_split'])
    orc.gen_rotation_keys(rots)
    x = np.random.default_rng(SEED).permutation(N) / N
    ct = orc.encrypt(x, N)
    t1 = time.time()
    out = orc.direct_sort(ct, N, rots, c['cfg'])
    t2 = time.time()
    rank = orc.direct_sort(ct, N, rots, c['cfg'], mode=1)  # constructRank alone: more limbs pinned
    rinfo = rank.info()
    info = out.info()
    y = orc.decrypt(out)[:N]
    rec = dict(c, cfg=list(c['cfg']), seed=SEED, input='default_rng(seed).permutation(N) / N',
               rotations=[int(r) for r in rots], level=int(info['level']), limbs=int(info['limbs']),
               scale=float(info['scale']), sha256=digest(out.data()),
               input_sha256=digest(ct.data()),
               rank_sha256=digest(rank.data()), rank_level=int(rinfo['level']), rank_limbs=int(rinfo['limbs']),
               max_abs_err=float(np.max(np.abs(y - np.sort(x)))),
               oracle_setup_s=round(t1 - t0, 1), oracle_sort_s=round(t2 - t1, 1),
               oracle_threads=int(O.lib().orc_num_threads()))
    print(name, json.dumps(rec)[:400], flush=True)
    return rec


def main():
    names = sys.argv[1:] or list(CASES)
    db = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for n in names:
        db[n] = run(n)
        with open(OUT, 'w') as f:
            json.dump(db, f, indent=1, sort_keys=True)


if __name__ == '__main__':
    main()
