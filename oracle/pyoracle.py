"""ctypes binding of the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — never by the product path.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, 'build', 'liboracle.so')
COEFF_DIR = os.path.join(REPO, 'fhe-sorting_amd', 'data')

_lib = None


def build():
    subprocess.check_call(['make', '-s', '-C', HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, ip, dp, u64p = C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_double), C.POINTER(C.c_uint64)
        PP = C.POINTER(C.c_void_p)
        sig = {
            'orc_last_error': (C.c_char_p, []),
            'orc_ctx_new': (vp, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64]),
            'orc_ctx_free': (None, [vp]),
            'orc_set_ps_split': (C.c_int, [vp, C.c_int]),
            'orc_set_moddown_floor': (C.c_int, [vp, C.c_int]),
            'orc_cheb_ps_depth': (C.c_int, [C.c_int, C.c_int]),
            'orc_params': (C.c_int, [vp, u64p, ip, ip, ip, dp]),
            'orc_keygen': (C.c_int, [vp]),
            'orc_gen_rotation_keys': (C.c_int, [vp, ip, C.c_int]),
            'orc_secret_ntt': (C.c_int, [vp, u64p]),
            'orc_secret_coeff': (C.c_int, [vp, C.POINTER(C.c_int64)]),
            'orc_public_key': (C.c_int, [vp, u64p]),
            'orc_relin_key': (C.c_int, [vp, u64p]),
            'orc_rot_key': (C.c_uint64, [vp, C.c_int, u64p]),
            'orc_encode': (vp, [vp, dp, C.c_int, C.c_int, C.c_int]),
            'orc_pt_data': (C.c_int, [vp, u64p]),
            'orc_pt_free': (None, [vp]),
            'orc_encrypt': (vp, [vp, dp, C.c_int, C.c_int, C.c_int]),
            'orc_encrypt_ext': (vp, [vp, dp, C.c_int, C.c_int]),
            'orc_decrypt': (C.c_int, [vp, vp, dp]),
            'orc_ct_free': (None, [vp]),
            'orc_ct_info': (C.c_int, [vp, ip, ip, dp, ip]),
            'orc_ct_data': (C.c_int, [vp, u64p]),
            'orc_ct_from': (vp, [vp, u64p, C.c_int, C.c_int, C.c_int, C.c_double]),
            'orc_ct_set_slots': (C.c_int, [vp, C.c_int]),
            'orc_add': (vp, [vp, vp, vp]),
            'orc_sub': (vp, [vp, vp, vp]),
            'orc_mul': (vp, [vp, vp, vp]),
            'orc_square': (vp, [vp, vp]),
            'orc_negate': (vp, [vp, vp]),
            'orc_add_const': (vp, [vp, vp, C.c_double]),
            'orc_mul_const': (vp, [vp, vp, C.c_double]),
            'orc_mul_const_to': (vp, [vp, vp, C.c_double, C.c_int]),
            'orc_mul_int': (vp, [vp, vp, C.c_int64]),
            'orc_level_adjust': (vp, [vp, vp, C.c_int]),
            'orc_rescale': (vp, [vp, vp]),
            'orc_rotate': (vp, [vp, vp, C.c_int]),
            'orc_mul_plain': (vp, [vp, vp, vp]),
            'orc_mul_plain_sum': (vp, [vp, C.POINTER(vp), C.POINTER(vp), C.c_int]),
            'orc_add_plain': (vp, [vp, vp, vp]),
            'orc_rotate_hoisted': (C.c_int, [vp, vp, ip, C.c_int, C.POINTER(vp)]),
            'orc_linear_sum_to': (vp, [vp, C.POINTER(vp), dp, C.c_int, C.c_int]),
            'orc_cheb': (vp, [vp, vp, dp, C.c_int, C.c_double, C.c_double]),
            'orc_sign': (vp, [vp, vp, C.c_int, C.c_int, C.c_int]),
            'orc_compare': (vp, [vp, vp, vp, C.c_int, C.c_int, C.c_int]),
            'orc_indicator': (vp, [vp, vp, C.c_double, C.c_int, C.c_int, C.c_int]),
            'orc_compose_rotate': (vp, [vp, vp, C.c_int, ip, C.c_int, C.c_int, C.c_int]),
            'orc_direct_sort': (vp, [vp, vp, vp, C.c_int, ip, C.c_int, C.c_int, C.c_int, C.c_int,
                                     C.c_int, C.c_int, C.c_int, vp, vp]),
            'orc_size_parameters': (C.c_int, [C.c_int, ip, ip, C.c_int]),
            'orc_sort_hybrid': (vp, [vp, vp, vp, C.c_int, ip, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                     C.c_int]),
            'orc_mehp24_sort': (vp, [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
            'orc_mehp24_sort_sharded': (vp, [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                             C.c_int, C.c_int, vp, vp]),
            'orc_mehp24_indicator': (vp, [vp, vp, C.c_double, C.c_int, C.c_int]),
            'orc_mehp24_rotation_indices': (C.c_int, [C.c_int, C.c_int, ip, C.c_int]),
            'orc_kway_sort': (vp, [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int]),
            'orc_kway_sorter': (C.c_int, [vp, C.c_int, PP, C.c_int, PP, C.c_int, PP]),
            'orc_kway_sort_type': (C.c_int, [C.c_int, C.c_int, C.c_int, ip]),
            'orc_kway_gen_indices': (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, ip, ip]),
            'orc_kway_rotate_distance': (C.c_int, [C.c_int, C.c_int, C.c_int]),
            'orc_decompose': (C.c_int, [C.c_int, ip, C.c_int, C.c_int, C.c_int, C.c_int, ip, ip, C.c_int]),
            'orc_set_coeff_dir': (None, [C.c_char_p]),
            'orc_doubled_sinc': (C.c_int, [C.c_int, dp, C.c_int]),
            'orc_ntt': (C.c_int, [vp, C.c_int, u64p, C.c_int]),
            'orc_psi': (C.c_uint64, [vp, C.c_int]),
            'orc_automorph_perm': (C.c_int, [C.c_int, C.c_uint64, C.POINTER(C.c_uint32)]),
            'orc_galois': (C.c_uint64, [C.c_int, C.c_int]),
            'orc_modup': (C.c_int, [vp, u64p, C.c_int, u64p]),
            'orc_moddown': (C.c_int, [vp, u64p, C.c_int, u64p]),
            'orc_counters': (C.c_int, [vp, u64p]),
            'orc_reset_counters': (None, [vp]),
            'orc_num_threads': (C.c_int, []),
            'orc_boot_new': (vp, [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
            'orc_boot_free': (None, [vp]),
            'orc_boot_keygen': (C.c_int, [vp]),
            'orc_boot_depth': (C.c_int, [vp]),
            'orc_boot_rotations': (C.c_int, [vp, ip, C.c_int]),
            'orc_bootstrap': (vp, [vp, vp, C.c_int]),
            'orc_conjugate': (vp, [vp, vp]),
            'orc_gen_galois_keys': (C.c_int, [vp, u64p, C.c_int]),
            'orc_galois_key': (C.c_uint64, [vp, C.c_uint64, u64p]),
            'orc_encode_complex': (vp, [vp, dp, dp, C.c_int, C.c_int, C.c_int, C.c_double]),
            'orc_kway_sort_boot': (vp, [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, vp]),
            'orc_compare_boot': (vp, [vp, vp, vp, C.c_int, C.c_int, C.c_int, vp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        L.orc_set_coeff_dir(COEFF_DIR.encode())
        _lib = L
    return _lib


ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_uint64), C.c_uint64, C.c_void_p)


class _Hook:
    """ctypes wrapper of a Python all-reduce callback f(dev_ptr, count, user):
    an exception inside it is recorded and reported as a non-zero return (the
    C side then aborts the sort); the caller re-raises it after the C call."""

    def __init__(self, f):
        self.exc = None

        def call(ptr, count, user):
            try:
                r = f(ptr, count, user)
                return 0 if r is None else int(r)
            except BaseException as e:  # noqa: BLE001 -- must not unwind through C
                self.exc = e
                return 1
        self.fn = ALLREDUCE_FN(call) if f else None

    def ptr(self):
        return C.cast(self.fn, C.c_void_p) if self.fn else None

    def reraise(self, err):
        if self.exc is not None:
            raise self.exc from err
        raise err


def _u64(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint64))


def _dbl(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _int(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


def _check(ptr):
    if not ptr:
        raise RuntimeError('oracle: ' + lib().orc_last_error().decode())
    return ptr


class Ct:
    def __init__(self, ctx, h):
        self.ctx, self.h = ctx, _check(h)

    def __del__(self):
        try:
            lib().orc_ct_free(self.h)
        except Exception:
            pass

    def info(self):
        lv, sl, lm = C.c_int(), C.c_int(), C.c_int()
        sc = C.c_double()
        lib().orc_ct_info(self.h, C.byref(lv), C.byref(sl), C.byref(sc), C.byref(lm))
        return dict(level=lv.value, slots=sl.value, scale=sc.value, limbs=lm.value)

    @property
    def level(self):
        return self.info()['level']

    @property
    def slots(self):
        return self.info()['slots']

    def set_slots(self, s):
        lib().orc_ct_set_slots(self.h, s)

    def data(self):
        inf = self.info()
        out = np.empty((2, inf['limbs'], self.ctx.n), dtype=np.uint64)
        lib().orc_ct_data(self.h, _u64(out))
        return out

    def decrypt(self):
        return self.ctx.decrypt(self)


class Pt:
    def __init__(self, ctx, h, level):
        self.ctx, self.h, self.level = ctx, _check(h), level

    def __del__(self):
        try:
            lib().orc_pt_free(self.h)
        except Exception:
            pass

    def data(self):
        limbs = self.ctx.nq - self.level
        out = np.empty((limbs, self.ctx.n), dtype=np.uint64)
        lib().orc_pt_data(self.h, _u64(out))
        return out


def cheb_ps_depth(degree, split=1):
    """levels a degree-d Chebyshev series consumes under the given PS split"""
    return int(lib().orc_cheb_ps_depth(int(degree), int(split)))


class Context:
    def __init__(self, logN, L, scale_bits=40, first_bits=60, dnum=3, seed=1, keygen=True, ps_split=1):
        self.logN, self.n, self.L = logN, 1 << logN, L
        self.h = _check(lib().orc_ctx_new(logN, L, scale_bits, first_bits, dnum, seed))
        nq, K, alpha = C.c_int(), C.c_int(), C.c_int()
        lib().orc_params(self.h, None, C.byref(nq), C.byref(K), C.byref(alpha), None)
        self.nq, self.K, self.alpha = nq.value, K.value, alpha.value
        self.primes = np.empty(self.nq + self.K, dtype=np.uint64)
        self.delta = np.empty(L + 1)
        lib().orc_params(self.h, _u64(self.primes), None, None, None, _dbl(self.delta))
        self.params = dict(logN=logN, L=L, scale_bits=scale_bits, first_bits=first_bits, dnum=dnum, seed=seed)
        self.set_ps_split(ps_split)
        if keygen:
            self.keygen()

    def __del__(self):
        try:
            lib().orc_ctx_free(self.h)
        except Exception:
            pass

    def set_ps_split(self, split):
        """1: OpenFHE's EvalChebyshevSeriesPS split (default); 0: power-of-two split"""
        if lib().orc_set_ps_split(self.h, int(split)) != 0:
            raise ValueError('ps split must be 0 or 1')
        self.ps_split = int(split)

    def set_moddown_floor(self, floor):
        """1: OpenFHE's ApproxModDown (the flooring fast base conversion); 0: the
        exact centred ModDown this build specifies (the default)"""
        if lib().orc_set_moddown_floor(self.h, int(floor)) != 0:
            raise ValueError('moddown floor must be 0 or 1')

    # keys -------------------------------------------------------------
    def keygen(self):
        if lib().orc_keygen(self.h) != 0:
            raise RuntimeError(lib().orc_last_error().decode())

    def gen_rotation_keys(self, rots):
        r = np.asarray(rots, dtype=np.int32)
        if lib().orc_gen_rotation_keys(self.h, _int(r), len(r)) != 0:
            raise RuntimeError(lib().orc_last_error().decode())

    @property
    def digits(self):
        return (self.nq + self.alpha - 1) // self.alpha

    def secret_ntt(self):
        out = np.empty((self.nq + self.K, self.n), dtype=np.uint64)
        lib().orc_secret_ntt(self.h, _u64(out))
        return out

    def secret_coeff(self):
        out = np.empty(self.n, dtype=np.int64)
        lib().orc_secret_coeff(self.h, out.ctypes.data_as(C.POINTER(C.c_int64)))
        return out

    def public_key(self):
        out = np.empty((2, self.nq, self.n), dtype=np.uint64)
        lib().orc_public_key(self.h, _u64(out))
        return out

    def relin_key(self):
        out = np.empty((self.digits, 2, self.nq + self.K, self.n), dtype=np.uint64)
        lib().orc_relin_key(self.h, _u64(out))
        return out

    def rot_key(self, k):
        out = np.empty((self.digits, 2, self.nq + self.K, self.n), dtype=np.uint64)
        g = lib().orc_rot_key(self.h, int(k), _u64(out))
        return (g, out) if g else (0, None)

    # objects ----------------------------------------------------------
    def encode(self, v, slots, level=0):
        v = np.ascontiguousarray(v, dtype=np.float64)
        return Pt(self, lib().orc_encode(self.h, _dbl(v), len(v), slots, level), level)

    def encrypt(self, v, slots=None, level=0):
        v = np.ascontiguousarray(v, dtype=np.float64)
        slots = slots or len(v)
        return Ct(self, lib().orc_encrypt(self.h, _dbl(v), len(v), slots, level))

    def encrypt_ext(self, v, slots=None):
        v = np.ascontiguousarray(v, dtype=np.float64)
        return Ct(self, lib().orc_encrypt_ext(self.h, _dbl(v), len(v), slots or len(v)))

    def decrypt(self, ct):
        out = np.empty(ct.slots)
        if lib().orc_decrypt(self.h, ct.h, _dbl(out)) < 0:
            raise RuntimeError(lib().orc_last_error().decode())
        return out

    def ct_from(self, data, level, slots, scale=None):
        data = np.ascontiguousarray(data, dtype=np.uint64)
        limbs = data.shape[1]
        scale = self.delta[level] if scale is None else scale
        return Ct(self, lib().orc_ct_from(self.h, _u64(data), limbs, level, slots, scale))

    # ops ----------------------------------------------------------------
    def add(self, a, b): return Ct(self, lib().orc_add(self.h, a.h, b.h))
    def sub(self, a, b): return Ct(self, lib().orc_sub(self.h, a.h, b.h))
    def mul(self, a, b): return Ct(self, lib().orc_mul(self.h, a.h, b.h))
    def square(self, a): return Ct(self, lib().orc_square(self.h, a.h))
    def negate(self, a): return Ct(self, lib().orc_negate(self.h, a.h))
    def add_const(self, a, k): return Ct(self, lib().orc_add_const(self.h, a.h, k))
    def mul_const(self, a, k): return Ct(self, lib().orc_mul_const(self.h, a.h, k))
    def mul_const_to(self, a, k, t): return Ct(self, lib().orc_mul_const_to(self.h, a.h, k, t))
    def mul_int(self, a, k): return Ct(self, lib().orc_mul_int(self.h, a.h, k))
    def level_adjust(self, a, t): return Ct(self, lib().orc_level_adjust(self.h, a.h, t))
    def rescale(self, a): return Ct(self, lib().orc_rescale(self.h, a.h))
    def rotate(self, a, k): return Ct(self, lib().orc_rotate(self.h, a.h, k))
    def mul_plain(self, a, p): return Ct(self, lib().orc_mul_plain(self.h, a.h, p.h))

    def mul_plain_sum(self, cts, pts):
        ca = (C.c_void_p * len(cts))(*[c.h for c in cts])
        pa = (C.c_void_p * len(pts))(*[p.h for p in pts])
        return Ct(self, lib().orc_mul_plain_sum(self.h, ca, pa, len(cts)))
    def add_plain(self, a, p): return Ct(self, lib().orc_add_plain(self.h, a.h, p.h))

    def rotate_hoisted(self, a, ks):
        ks = np.asarray(ks, dtype=np.int32)
        outs = (C.c_void_p * len(ks))()
        if lib().orc_rotate_hoisted(self.h, a.h, _int(ks), len(ks), outs) != 0:
            raise RuntimeError(lib().orc_last_error().decode())
        return [Ct(self, outs[i]) for i in range(len(ks))]

    def linear_sum_to(self, xs, cs, target):
        arr = (C.c_void_p * len(xs))(*[x.h for x in xs])
        cs = np.ascontiguousarray(cs, dtype=np.float64)
        return Ct(self, lib().orc_linear_sum_to(self.h, arr, _dbl(cs), len(xs), target))

    def cheb(self, a, coeffs, lo=-1.0, hi=1.0):
        c = np.ascontiguousarray(coeffs, dtype=np.float64)
        return Ct(self, lib().orc_cheb(self.h, a.h, _dbl(c), len(c), lo, hi))

    def sign(self, a, n, dg, df): return Ct(self, lib().orc_sign(self.h, a.h, n, dg, df))
    def compare(self, a, b, n, dg, df): return Ct(self, lib().orc_compare(self.h, a.h, b.h, n, dg, df))
    def indicator(self, a, c, n, dg, df): return Ct(self, lib().orc_indicator(self.h, a.h, c, n, dg, df))

    def compose_rotate(self, a, N, rots, algo, rotation):
        r = np.asarray(rots, dtype=np.int32)
        return Ct(self, lib().orc_compose_rotate(self.h, a.h, N, _int(r), len(r), algo, rotation))

    def direct_sort(self, x, N, rots, cfg, mode=0, rank=None, shard=(0, 1), allreduce=None):
        r = np.asarray(rots, dtype=np.int32)
        hk = _Hook(allreduce)
        h = lib().orc_direct_sort(self.h, x.h, rank.h if rank is not None else None, N, _int(r), len(r),
                                  cfg[0], cfg[1], cfg[2], mode, shard[0], shard[1], hk.ptr(), None)
        try:
            return Ct(self, h)
        except RuntimeError as e:
            hk.reraise(e)

    def sort_hybrid(self, x, N, rots, cfg, mode=0, rank=None, max_array=256, mask=0):
        """DirectSort::sort_hybrid (mode 0) or rotationIndexCheckHybrid(rank, x) (mode 1)."""
        r = np.asarray(rots, dtype=np.int32)
        return Ct(self, lib().orc_sort_hybrid(self.h, x.h, rank.h if rank is not None else None, N, _int(r), len(r),
                                              cfg[0], cfg[1], cfg[2], mode, max_array, mask))

    def mehp24_sort(self, x, N, cfg, dg_i, df_i, sub=0, shard=(0, 1), allreduce=None):
        if shard == (0, 1) and allreduce is None:
            return Ct(self, lib().orc_mehp24_sort(self.h, x.h, N, sub, cfg[0], cfg[1], cfg[2], dg_i, df_i))
        hk = _Hook(allreduce)
        h = lib().orc_mehp24_sort_sharded(self.h, x.h, N, sub, cfg[0], cfg[1], cfg[2], dg_i, df_i,
                                          shard[0], shard[1], hk.ptr(), None)
        try:
            return Ct(self, h)
        except RuntimeError as e:
            hk.reraise(e)

    def mehp24_indicator(self, a, b, dg, df):
        return Ct(self, lib().orc_mehp24_indicator(self.h, a.h, b, dg, df))

    def kway_sort(self, x, k, M, cfg, boot=None):
        """k-way network; cfg = (n, dg, df) with n = 3; boot: a Bootstrapper (checkLevelAndBoot)"""
        if boot is None:
            return Ct(self, lib().orc_kway_sort(self.h, x.h, k, M, cfg[1], cfg[2]))
        return Ct(self, lib().orc_kway_sort_boot(self.h, x.h, k, M, cfg[1], cfg[2], boot.h))

    def compare_boot(self, a, b, n, dg, df, boot):
        """Comparison::compare with compositeSign's lazy bootstrap (src/sign.cpp:164-170)"""
        return Ct(self, lib().orc_compare_boot(self.h, a.h, b.h, n, dg, df, boot.h))

    def conjugate(self, a): return Ct(self, lib().orc_conjugate(self.h, a.h))

    def gen_galois_keys(self, gs):
        g = np.asarray(gs, dtype=np.uint64)
        if lib().orc_gen_galois_keys(self.h, _u64(g), len(g)) != 0:
            raise RuntimeError(lib().orc_last_error().decode())

    def galois_key(self, g):
        out = np.empty((self.digits, 2, self.nq + self.K, self.n), dtype=np.uint64)
        r = lib().orc_galois_key(self.h, int(g), _u64(out))
        return out if r else None

    def encode_complex(self, v, slots, level, scale=None):
        v = np.asarray(v, dtype=np.complex128)
        re, im = np.ascontiguousarray(v.real), np.ascontiguousarray(v.imag)
        scale = self.delta[level] if scale is None else scale
        return Pt(self, lib().orc_encode_complex(self.h, _dbl(re), _dbl(im), len(v), slots, level, scale), level)

    def kway_sorter(self, kk, xs, cmps):
        """SortUtils::fcnL (kk = 1) or the kk-sorter (kk = 2..5): ascending outputs."""
        xa = (C.c_void_p * len(xs))(*[x.h for x in xs])
        ca = (C.c_void_p * len(cmps))(*[c.h for c in cmps])
        nout = 1 if kk == 1 else kk
        outs = (C.c_void_p * nout)()
        if lib().orc_kway_sorter(self.h, kk, xa, len(xs), ca, len(cmps), outs) != 0:
            raise RuntimeError(lib().orc_last_error().decode())
        return [Ct(self, outs[i]) for i in range(nout)]

    # kernel level -----------------------------------------------------
    def ntt(self, prime_index, data, inverse=False):
        d = np.ascontiguousarray(data, dtype=np.uint64).copy()
        lib().orc_ntt(self.h, prime_index, _u64(d), 1 if inverse else 0)
        return d

    def psi(self, prime_index):
        return lib().orc_psi(self.h, prime_index)

    def modup(self, d):
        d = np.ascontiguousarray(d, dtype=np.uint64)
        ell = d.shape[0]
        digits = (ell + self.alpha - 1) // self.alpha
        out = np.empty((digits, ell + self.K, self.n), dtype=np.uint64)
        lib().orc_modup(self.h, _u64(d), ell, _u64(out))
        return out

    def moddown(self, x):
        x = np.ascontiguousarray(x, dtype=np.uint64)
        ell = x.shape[0] - self.K
        out = np.empty((ell, self.n), dtype=np.uint64)
        lib().orc_moddown(self.h, _u64(x), ell, _u64(out))
        return out

    def counters(self):
        out = np.zeros(6, dtype=np.uint64)
        lib().orc_counters(self.h, _u64(out))
        return dict(zip(['hmult', 'keyswitch', 'rotations', 'rescale', 'ptmult', 'constmult'], map(int, out)))

    def reset_counters(self):
        lib().orc_reset_counters(self.h)


class Bootstrapper:
    """EvalBootstrapSetup(levelBudget={budget_enc, budget_dec}, slots) +
    EvalBootstrapKeyGen + EvalBootstrap (oracle_boot.cpp)."""

    def __init__(self, ctx, slots, budget=(4, 4), K=512, r=6, degree=88, correction_bits=10, keygen=True):
        self.ctx = ctx
        self.cfg = dict(slots=slots, budget=tuple(budget), K=K, r=r, degree=degree, correction_bits=correction_bits)
        self.h = _check(lib().orc_boot_new(ctx.h, slots, budget[0], budget[1], K, r, degree, correction_bits))
        if keygen:
            self.keygen()

    def __del__(self):
        try:
            lib().orc_boot_free(self.h)
        except Exception:
            pass

    def keygen(self):
        if lib().orc_boot_keygen(self.h) != 0:
            raise RuntimeError(lib().orc_last_error().decode())

    @property
    def depth(self):
        return lib().orc_boot_depth(self.h)

    def rotations(self):
        out = np.zeros(4096, dtype=np.int32)
        m = lib().orc_boot_rotations(self.h, _int(out), 4096)
        return [int(x) for x in out[:m]]

    def bootstrap(self, x, stage=0):
        return Ct(self.ctx, lib().orc_bootstrap(self.h, x.h, stage))

    def mod_raise(self, x): return self.bootstrap(x, 4)
    def coeffs_to_slots(self, x): return self.bootstrap(x, 1)
    def eval_mod(self, x): return self.bootstrap(x, 2)
    def slots_to_coeffs(self, x): return self.bootstrap(x, 3)


def automorph_perm(logN, g):
    out = np.empty(1 << logN, dtype=np.uint32)
    lib().orc_automorph_perm(logN, g, out.ctypes.data_as(C.POINTER(C.c_uint32)))
    return out


def galois(logN, k):
    return lib().orc_galois(logN, k)


def size_parameters(N):
    d = C.c_int()
    rots = np.zeros(512, dtype=np.int32)
    m = lib().orc_size_parameters(N, C.byref(d), _int(rots), 512)
    if m < 0:
        raise ValueError(lib().orc_last_error().decode())
    return d.value, [int(x) for x in rots[:m]]


def mehp24_rotation_indices(N, sub=256):
    rots = np.zeros(1024, dtype=np.int32)
    m = lib().orc_mehp24_rotation_indices(N, sub, _int(rots), 1024)
    if m < 0:
        raise ValueError(lib().orc_last_error().decode())
    return [int(x) for x in rots[:m]]


def kway_sort_type(k, M, stage):
    out = np.zeros(3, dtype=np.int32)
    if lib().orc_kway_sort_type(k, M, stage, _int(out)) < 0:
        raise ValueError(lib().orc_last_error().decode())
    return tuple(int(v) for v in out)


def kway_gen_indices(num_slots, k, M, m, log_dist, slope):
    g = np.zeros(num_slots, dtype=np.int32)
    p = np.zeros(num_slots, dtype=np.int32)
    if lib().orc_kway_gen_indices(num_slots, k, M, m, log_dist, slope, _int(g), _int(p)) < 0:
        raise ValueError(lib().orc_last_error().decode())
    return g, p


def kway_rotate_distance(k, log_dist, slope):
    return int(lib().orc_kway_rotate_distance(k, log_dist, slope))


def decompose(N, rots, rotation, wrapN, algo):
    r = np.asarray(rots, dtype=np.int32)
    vals = np.zeros(128, dtype=np.int32)
    sizes = np.zeros(128, dtype=np.int32)
    m = lib().orc_decompose(N, _int(r), len(r), rotation, wrapN, algo, _int(vals), _int(sizes), 128)
    return [(int(vals[i]), int(sizes[i])) for i in range(m)]


def doubled_sinc(N):
    m = lib().orc_doubled_sinc(N, None, 0)
    out = np.empty(m)
    lib().orc_doubled_sinc(N, _dbl(out), m)
    return out


NAF, BNAF, BINARY = 0, 1, 2
