#!/usr/bin/env python3
"""NTT pass throughput on device memory (fhe_ntt_dev): `limbs` primes x `segs`
segments per call, forward and inverse, rings 2^16 and 2^17."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'fhe-sorting_amd'))
import fhesort as F  # noqa: E402

hip = C.CDLL('libamdhip64.so')
hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
hip.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
out = []
for logN, limbs, segs in ((17, 32, 32), (16, 32, 32), (17, 32, 1), (16, 32, 1)):
    ctx = F.Context(logN, limbs, 40, 60, 3, seed=1, keygen=False)
    n = 1 << logN
    p = C.c_void_p()
    assert hip.hipMalloc(C.byref(p), limbs * segs * n * 8) == 0
    assert hip.hipMemset(p, 0, limbs * segs * n * 8) == 0
    for inv in (False, True):
        f = lambda: ctx.ntt_dev(p.value, 0, limbs, inverse=inv, segments=segs, seg_stride=limbs * n)
        f()
        ctx.sync()
        reps = 20
        t = time.perf_counter()
        for _ in range(reps):
            f()
        ctx.sync()
        dt = (time.perf_counter() - t) / reps
        gbs = 2 * 2 * limbs * segs * n * 8 / dt / 1e9  # two passes, read + write each
        r = dict(logN=logN, limbs=limbs, segs=segs, inverse=inv, ms=round(dt * 1e3, 3), GBps_2pass=round(gbs, 1))
        print(json.dumps(r), flush=True)
