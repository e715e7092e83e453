#!/usr/bin/env python3
"""Digest of the reference CLI's own configuration on its only held input (test
infrastructure; verdict r4 item 1).

The reference's competition CLI (src/main.cpp:9-44, src/sort.h:15-103) sorts
DirectSort<128> with CompositeSign(4, 3, 3) over main.cpp's 21 rotations in the
context of src/config.json: ring 131072, multDepth 44, scaling 40 bits, batch
128.  Its one held input is src/testcase.json's 128 values in [2.34, 245.67],
35 distinct; the harness normalises them by 255 (constructRank's
"inputOver255", src/sort_algo.h:419-421).  The fixture's "output" is NOT used:
it has 121 entries and its multiset differs from the input's (13 extra 245.67,
several values short), so it is not the sort of the input.

Here the CPU oracle runs that sort once (keys and encryption from SEED, ps_split
OpenFHE) and the SHA-256 of the encrypted input and of the sorted output words
go to tests/golden/cli_digest.json together with the 128 input values (data,
so the GPU box needs nothing from /root/reference), the output's level and
scale and the decryption.  tests/test_gpu_wire.py::test_cli_reference_context
repeats it through bin/fhesort on the GPU and compares.

Run: python tests/golden/make_cli_digest.py   (build container; ~8 GB of host
memory for the ring-2^17 rotation keys)
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
sys.path.insert(0, os.path.join(REPO, 'tests'))

SEED = 20250704
LOGN, DEPTH, SCALE, DNUM, N = 17, 44, 40, 3, 128  # src/config.json:1-9
CFG = (4, 3, 3)  # src/sort.h:93
ROTATIONS = [-1, -2, -4, -8, -16, -32, 1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384]
OUT = os.path.join(HERE, 'cli_digest.json')
TESTCASE = '/root/reference/src/testcase.json'


def digest(words):
    return hashlib.sha256(np.ascontiguousarray(words, dtype='<u8').tobytes()).hexdigest()


def testcase_values():
    run = json.load(open(TESTCASE))[0]['runs'][0]
    vals = [v for e in run['input'] for v in (e['value'] if isinstance(e, dict) else [e])]
    assert len(vals) == N, len(vals)
    return [float(v) for v in vals]


def main():
    import pyoracle as O
    import tie_model
    vals = testcase_values()
    x = np.array(vals) / 255.0
    t0 = time.time()
    orc = O.Context(LOGN, DEPTH, SCALE, 60, DNUM, seed=SEED, ps_split=1)
    orc.gen_rotation_keys(ROTATIONS)
    ct = orc.encrypt(x, N)
    t1 = time.time()
    out = orc.direct_sort(ct, N, ROTATIONS, CFG)
    t2 = time.time()
    info = out.info()
    y = orc.decrypt(out)[:N]
    model = tie_model.direct_sort(x, CFG)
    rec = dict(N=N, logN=LOGN, depth=DEPTH, scale_bits=SCALE, dnum=DNUM, cfg=list(CFG), rotations=ROTATIONS,
               seed=SEED, ps_split=1, input_values=vals, input='input_values / 255',
               input_sha256=digest(ct.data()), sha256=digest(out.data()), level=int(info['level']),
               limbs=int(info['limbs']), scale=float(info['scale']), decrypted=[float(v) for v in y],
               max_abs_dev_from_tie_model=float(np.max(np.abs(y - model))),
               max_abs_dev_from_sorted=float(np.max(np.abs(y - np.sort(x)))),
               oracle_setup_s=round(t1 - t0, 1), oracle_sort_s=round(t2 - t1, 1),
               oracle_threads=int(O.lib().orc_num_threads()))
    with open(OUT, 'w') as f:
        json.dump(rec, f, indent=1, sort_keys=True)
    print({k: v for k, v in rec.items() if k not in ('input_values', 'decrypted')})


if __name__ == '__main__':
    main()
