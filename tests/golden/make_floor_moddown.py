"""What the exact centred ModDown buys at the hot path's own configuration
(verdict r5 item 7; DESIGN.md §2 "Numeric specification").

This build's ModDown rounds x / P to nearest (an exact centred base conversion);
OpenFHE's ApproxModDown floors it through the plain fast base conversion, with a
0..K overshoot.  The oracle can run either (Context.set_moddown_floor).  This
script runs BASELINE config 2 -- DirectSort N=128 at ring 2^16, depth 30, the
reference's 40-bit scaling primes, CompositeSign(3,3,2) (src/sort_algo.h:117-123,
tests/DirectSortTest.cpp:107-108) -- on the CPU oracle with both forms, same keys
and input, and records the decrypted error of each against DirectSortTest's 0.01
bound (tests/DirectSortTest.cpp:169).  ~7 minutes on 8 threads; the result is
committed as floor_moddown.json and checked by tests/test_oracle.py.
usage: python tests/golden/make_floor_moddown.py [N logN]"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', '..', 'oracle'))
import numpy as np  # noqa: E402
import pyoracle as O  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
logN = int(sys.argv[2]) if len(sys.argv) > 2 else 16
CFG = (3, 3, 2)
depth, rots = O.size_parameters(N)
t0 = time.time()
orc = O.Context(logN, depth, 40, 60, 3, seed=2)
orc.gen_rotation_keys(rots)
x = np.random.default_rng(20250704).permutation(N) / N
rows = []
for floor in (0, 1):
    orc.set_moddown_floor(floor)
    ox = orc.encrypt(x, N)
    t = time.time()
    y = orc.direct_sort(ox, N, rots, CFG)
    err = float(np.max(np.abs(orc.decrypt(y)[:N] - np.sort(x))))
    rows.append({'moddown': 'floor (OpenFHE ApproxModDown)' if floor else 'centred (this build)', 'floor': floor,
                 'max_abs_err': err, 'bound': 0.01, 'passes': err < 0.01, 'level': y.level, 'sort_s': round(time.time() - t, 1)})
    print(json.dumps(rows[-1]), flush=True)
out = {'config': {'N': N, 'log_ring': logN, 'depth': depth, 'scale_bits': 40, 'sign': list(CFG), 'seed': 2,
                  'input': 'permutation(N) / N, numpy default_rng(20250704)',
                  'threads': int(O.lib().orc_num_threads())},
       'runs': rows, 'total_s': round(time.time() - t0, 1)}
if N == 128 and logN == 16:
    with open(os.path.join(HERE, 'floor_moddown.json'), 'w') as f:
        json.dump(out, f, indent=1)
print(json.dumps(out))
