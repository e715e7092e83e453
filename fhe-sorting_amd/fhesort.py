"""Python binding of the MI355X engine (lib/libfhesort.so, C ABI in
include/fhe_gpu.h).

This is the host-side handle the tests and bench.py use.  There is no CPU
fallback: if the HIP library is missing or no GPU is visible, constructing a
Context raises.  Method names mirror the reference API where one exists
(compare, indicator, sign_composite, direct_sort, ...).
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('FHE_LIB') or os.path.join(HERE, 'lib', 'libfhesort.so')  # FHE_LIB: A/B builds
COEFF_DIR = os.path.join(HERE, 'data')
HEADER = os.path.join(os.path.dirname(HERE), 'include', 'fhe_gpu.h')
PS_SPLIT_ENGINE, PS_SPLIT_OPENFHE = 0, 1  # fhe_set_ps_split (include/fhe_gpu.h)

FHE_OK, FHE_EINVAL, FHE_ENOKEY, FHE_EDEPTH, FHE_EHIP, FHE_ENOMEM, FHE_EINTERNAL, FHE_ENOCOMM, FHE_EIO = range(9)
NAF, BNAF, BINARY = 0, 1, 2


class FheError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f'fhe error {code}: {msg}')
        self.code = code


class NoKeyError(FheError):
    pass


class Params(C.Structure):
    _fields_ = [('log_n', C.c_int), ('mult_depth', C.c_int), ('scale_bits', C.c_int), ('first_bits', C.c_int),
                ('dnum', C.c_int), ('seed', C.c_uint64)]


_lib = None
vp, ip, dp, u64p = C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_double), C.POINTER(C.c_uint64)
PP = C.POINTER(C.c_void_p)
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

_SIGS = {
    'fhe_last_error': (C.c_char_p, []),
    'fhe_ctx_create': (C.c_int, [C.POINTER(Params), C.c_int, PP]),
    'fhe_ctx_destroy': (C.c_int, [vp]),
    'fhe_ctx_info': (C.c_int, [vp, ip, ip, ip, u64p, dp]),
    'fhe_set_coeff_dir': (C.c_int, [C.c_char_p]),
    'fhe_keygen': (C.c_int, [vp]),
    'fhe_gen_rotation_keys': (C.c_int, [vp, ip, C.c_int]),
    'fhe_ctx_load_secret': (C.c_int, [vp, u64p]),
    'fhe_ctx_load_public': (C.c_int, [vp, u64p]),
    'fhe_ctx_load_keys': (C.c_int, [vp, u64p, ip, C.POINTER(u64p), C.c_int]),
    'fhe_key_bytes': (C.c_uint64, [vp]),
    'fhe_encrypt': (C.c_int, [vp, dp, C.c_int, C.c_int, C.c_int, PP]),
    'fhe_encrypt_ext': (C.c_int, [vp, dp, C.c_int, C.c_int, PP]),
    'fhe_decrypt': (C.c_int, [vp, vp, dp]),
    'fhe_ct_upload': (C.c_int, [vp, u64p, C.c_int, C.c_int, C.c_int, C.c_double, PP]),
    'fhe_ct_download': (C.c_int, [vp, vp, u64p]),
    'fhe_ct_info': (C.c_int, [vp, ip, ip, dp, ip]),
    'fhe_ct_set_slots': (C.c_int, [vp, C.c_int]),
    'fhe_ct_free': (C.c_int, [vp]),
    'fhe_pt_encode': (C.c_int, [vp, dp, C.c_int, C.c_int, C.c_int, PP]),
    'fhe_pt_upload': (C.c_int, [vp, u64p, C.c_int, C.c_int, C.c_int, C.c_double, PP]),
    'fhe_pt_free': (C.c_int, [vp]),
    'fhe_add': (C.c_int, [vp, vp, vp, PP]),
    'fhe_sub': (C.c_int, [vp, vp, vp, PP]),
    'fhe_negate': (C.c_int, [vp, vp, PP]),
    'fhe_add_const': (C.c_int, [vp, vp, C.c_double, PP]),
    'fhe_mul_const': (C.c_int, [vp, vp, C.c_double, PP]),
    'fhe_mul_const_to': (C.c_int, [vp, vp, C.c_double, C.c_int, PP]),
    'fhe_mul_int': (C.c_int, [vp, vp, C.c_int64, PP]),
    'fhe_level_adjust': (C.c_int, [vp, vp, C.c_int, PP]),
    'fhe_rescale': (C.c_int, [vp, vp, PP]),
    'fhe_mul_plain': (C.c_int, [vp, vp, vp, PP]),
    'fhe_add_plain': (C.c_int, [vp, vp, vp, PP]),
    'fhe_mul_relin': (C.c_int, [vp, vp, vp, PP]),
    'fhe_square_relin': (C.c_int, [vp, vp, PP]),
    'fhe_rotate': (C.c_int, [vp, vp, C.c_int, PP]),
    'fhe_rotate_hoisted': (C.c_int, [vp, vp, ip, C.c_int, PP]),
    'fhe_linear_sum_to': (C.c_int, [vp, PP, dp, C.c_int, C.c_int, PP]),
    'fhe_cheb_ps': (C.c_int, [vp, vp, dp, C.c_int, C.c_double, C.c_double, PP]),
    'fhe_sign_composite': (C.c_int, [vp, vp, C.c_int, C.c_int, C.c_int, PP]),
    'fhe_compare': (C.c_int, [vp, vp, vp, C.c_int, C.c_int, C.c_int, PP]),
    'fhe_indicator': (C.c_int, [vp, vp, C.c_double, C.c_int, C.c_int, C.c_int, PP]),
    'fhe_compose_rotate': (C.c_int, [vp, vp, C.c_int, ip, C.c_int, C.c_int, C.c_int, PP]),
    'fhe_compose_rotate_members': (C.c_int, [vp, vp, C.c_int, ip, C.c_int, C.c_int, ip, C.c_int, PP]),
    'fhe_decompose': (C.c_int, [C.c_int, ip, C.c_int, C.c_int, C.c_int, C.c_int, ip, ip, C.c_int]),
    'fhe_rotation_tree_create': (C.c_int, [vp, C.c_int, ip, C.c_int, C.c_int, PP]),
    'fhe_rotation_tree_build': (C.c_int, [vp, C.c_int, C.c_int]),
    'fhe_rotation_tree_rotate': (C.c_int, [vp, vp, C.c_int, PP]),
    'fhe_rotation_tree_stats': (C.c_int, [vp, C.POINTER(C.c_uint64)]),
    'fhe_rotation_tree_destroy': (None, [vp]),
    'fhe_size_parameters': (C.c_int, [C.c_int, ip, ip, C.c_int]),
    'fhe_direct_sort': (C.c_int, [vp, vp, vp, C.c_int, ip, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                  C.c_int, C.c_int, vp, vp, PP]),
    'fhe_sort_hybrid': (C.c_int, [vp, vp, vp, C.c_int, ip, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                  C.c_int, C.c_int, C.c_int, vp, vp, PP]),
    'fhe_hybrid_parameters': (C.c_int, [C.c_int, ip, ip, C.c_int]),
    'fhe_mehp24_parameters': (C.c_int, [C.c_int, ip, ip, ip, ip, ip, ip, ip, ip, ip, C.c_int]),
    'fhe_mehp24_rotation_indices': (C.c_int, [C.c_int, C.c_int, ip, C.c_int]),
    'fhe_mehp24_sort': (C.c_int, [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, PP]),
    'fhe_mehp24_sort_sharded': (C.c_int, [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                          C.c_int, C.c_int, vp, vp, PP]),
    'fhe_mehp24_indicator': (C.c_int, [vp, vp, C.c_double, C.c_int, C.c_int, PP]),
    'fhe_kway_sort': (C.c_int, [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, PP]),
    'fhe_kway_sorter': (C.c_int, [vp, C.c_int, PP, C.c_int, PP, C.c_int, PP]),
    'fhe_kway_sort_boot': (C.c_int, [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, vp, C.POINTER(C.c_int), PP]),
    'fhe_boot_create': (C.c_int, [vp, vp, PP]),
    'fhe_boot_destroy': (C.c_int, [vp]),
    'fhe_boot_keygen': (C.c_int, [vp]),
    'fhe_boot_rotation_indices': (C.c_int, [vp, C.POINTER(C.c_int32), C.c_int]),
    'fhe_boot_depth': (C.c_int, [vp]),
    'fhe_bootstrap': (C.c_int, [vp, vp, PP]),
    'fhe_check_level_and_boot': (C.c_int, [vp, vp, C.c_int, vp, C.POINTER(C.c_int), PP]),
    'fhe_bootstrap_stage': (C.c_int, [vp, vp, C.c_int, PP]),
    'fhe_conjugate': (C.c_int, [vp, vp, PP]),
    'fhe_gen_galois_keys': (C.c_int, [vp, u64p, C.c_int]),
    'fhe_ctx_load_galois_key': (C.c_int, [vp, C.c_uint64, u64p]),
    'fhe_pt_encode_complex': (C.c_int, [vp, dp, dp, C.c_int, C.c_int, C.c_int, C.c_double, PP]),
    'fhe_kway_sort_type': (C.c_int, [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                     C.POINTER(C.c_int)]),
    'fhe_kway_stage_count': (C.c_int, [C.c_int, C.c_int]),
    'fhe_kway_rotate_distance': (C.c_int, [C.c_int, C.c_int, C.c_int]),
    'fhe_kway_gen_indices': (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                       C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    'fhe_kway_rotation_indices': (C.c_int, [C.c_int, C.POINTER(C.c_int32), C.c_int]),
    'fhe_comm_get_unique_id': (C.c_int, [C.POINTER(C.c_uint8)]),
    'fhe_comm_init': (C.c_int, [vp, C.POINTER(C.c_uint8), C.c_int, C.c_int]),
    'fhe_comm_destroy': (C.c_int, [vp]),
    'fhe_ct_allreduce': (C.c_int, [vp, vp]),
    'fhe_ntt': (C.c_int, [vp, u64p, C.c_int, C.c_int, C.c_int]),
    'fhe_modup': (C.c_int, [vp, u64p, C.c_int, u64p]),
    'fhe_moddown': (C.c_int, [vp, u64p, C.c_int, u64p]),
    'fhe_automorph': (C.c_int, [vp, u64p, C.c_int, C.c_uint64, u64p]),
    'fhe_counters': (C.c_int, [vp, u64p]),
    'fhe_collective_stats': (C.c_int, [vp, u64p]),
    'fhe_region_marker': (C.c_int, [vp, C.c_int]),
    'fhe_set_mask_cache': (C.c_int, [vp, C.c_int]),
    'fhe_pt_limbs': (C.c_int, [vp]),
    'fhe_pt_download': (C.c_int, [vp, vp, u64p]),
    'fhe_pt_encode_device': (C.c_int, [vp, dp, C.c_int, C.c_int, C.c_int, PP]),
    'fhe_pt_encode_masks': (C.c_int, [vp, C.POINTER(C.c_int32), C.c_int, C.c_int, C.c_int, PP]),
    'fhe_reset_counters': (C.c_int, [vp]),
    'fhe_sync': (C.c_int, [vp]),
    'fhe_stream': (vp, [vp]),
    'fhe_time_kernel': (C.c_int, [vp, C.c_char_p, C.c_int, C.c_int, dp, dp]),
    'fhe_kernel_clock_start': (C.c_int, [vp]),
    'fhe_set_sort_stack': (C.c_int, [vp, C.c_int]),
    'fhe_set_sort_lanes': (C.c_int, [vp, C.c_int]),
    'fhe_set_ps_split': (C.c_int, [vp, C.c_int]),
    'fhe_ntt_dev': (C.c_int, [vp, vp, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_int, vp]),
    'fhe_automorph_dev': (C.c_int, [vp, vp, C.c_int, C.c_uint64, vp, vp]),
    'fhe_host_stats': (C.c_int, [dp]),
    'fhe_set_mfma_sums': (C.c_int, [C.c_int]),
    'fhe_host_stats_reset': (C.c_int, []),
    'fhe_prng_block': (C.c_int, [C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    'fhe_get_ps_split': (C.c_int, [vp]),
    'fhe_cheb_ps_depth': (C.c_int, [C.c_int, C.c_int]),
    'fhe_cheb_ps_plan': (C.c_int, [C.POINTER(C.c_double), C.c_int]),
    'fhe_pool_trim': (C.c_int, [vp]),
    'fhe_pool_stats': (C.c_int, [vp, u64p, u64p, u64p]),
    'fhe_ct_stack': (C.c_int, [vp, C.POINTER(C.c_void_p), C.c_int, C.POINTER(C.c_void_p)]),
    'fhe_mul_plain_sum': (C.c_int, [vp, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.c_int,
                                    C.POINTER(C.c_void_p)]),
    'fhe_ct_member': (C.c_int, [vp, vp, C.c_int, C.POINTER(C.c_void_p)]),
    'fhe_ct_sum_members': (C.c_int, [vp, vp, C.POINTER(C.c_void_p)]),
    'fhe_kernel_clock_stop': (C.c_int, [vp, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    'fhe_wire_inspect': (C.c_int, [C.c_char_p, vp]),
    'fhe_serialize_context': (C.c_int, [vp, C.c_char_p]),
    'fhe_deserialize_context': (C.c_int, [C.c_char_p, C.c_int, C.POINTER(C.c_void_p)]),
    'fhe_serialize_ciphertext': (C.c_int, [vp, vp, C.c_char_p]),
    'fhe_deserialize_ciphertext': (C.c_int, [vp, C.c_char_p, C.POINTER(C.c_void_p)]),
    'fhe_deserialize_eval_automorphism_key': (C.c_int, [vp, C.c_char_p, C.POINTER(C.c_int)]),
    **{f'fhe_{d}serialize_{k}': (C.c_int, [vp, C.c_char_p])
       for d in ('', 'de') for k in ('public_key', 'secret_key', 'eval_mult_key')},
    'fhe_serialize_eval_automorphism_key': (C.c_int, [vp, C.c_char_p]),
}


class WireInfo(C.Structure):
    _fields_ = [('kind', C.c_uint32), ('version', C.c_uint32), ('params_id', C.c_uint64), ('log_n', C.c_uint64),
                ('nq', C.c_uint64), ('K', C.c_uint64), ('body_words', C.c_uint64)]


WIRE_KINDS = {1: 'context', 2: 'public_key', 3: 'eval_mult_key', 4: 'eval_automorphism_key', 5: 'ciphertext',
              6: 'secret_key'}


def set_mfma_sums(mask):
    """Process-wide choice of the i8-MFMA sums-of-products kernels (1 PS linear
    sums, 2 ModUp, 4 ModDown+rescale; fhe_set_mfma_sums).  mask < 0 only
    queries.  Returns the previous mask.  The output words do not change."""
    return lib().fhe_set_mfma_sums(int(mask))


def wire_inspect(path):
    """Header of a wire file (csrc/wire/wire.hpp) after its checksum is verified;
    host only, no GPU needed."""
    i = WireInfo()
    _chk(lib().fhe_wire_inspect(os.fsencode(path), C.byref(i)))
    return {'kind': WIRE_KINDS.get(i.kind, i.kind), 'version': i.version, 'params_id': i.params_id,
            'log_n': i.log_n, 'nq': i.nq, 'K': i.K, 'body_words': i.body_words}


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f'MI355X engine library missing: {LIB_PATH} (run __graft_entry__.build())')
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        L.fhe_set_coeff_dir(COEFF_DIR.encode())
        _lib = L
    return _lib


def _chk(rc):
    if rc != FHE_OK:
        msg = lib().fhe_last_error().decode()
        if rc == FHE_ENOKEY:
            raise NoKeyError(rc, msg)
        raise FheError(rc, msg)


def _u64(a):
    return a.ctypes.data_as(u64p)


def _dbl(a):
    return a.ctypes.data_as(dp)


def _int(a):
    return a.ctypes.data_as(ip)


class RotationTree:
    """Handle over fhe_rotation_tree_*: build(start, end), rotate(ct, k), stats()."""

    def __init__(self, ctx, N, rots, algo=0):
        r = np.asarray(rots, dtype=np.int32)
        out = C.c_void_p()
        _chk(lib().fhe_rotation_tree_create(ctx.h, N, _int(r), len(r), algo, C.byref(out)))
        self.ctx, self.h = ctx, out.value

    def __del__(self):
        try:
            if self.h:
                lib().fhe_rotation_tree_destroy(self.h)
        except Exception:
            pass

    def build(self, start, end):
        _chk(lib().fhe_rotation_tree_build(self.h, start, end))

    def rotate(self, a, rotation):
        out = C.c_void_p()
        _chk(lib().fhe_rotation_tree_rotate(self.h, a.h, rotation, C.byref(out)))
        return Ct(self.ctx, out.value)

    def stats(self):
        v = (C.c_uint64 * 5)()
        _chk(lib().fhe_rotation_tree_stats(self.h, v))
        return dict(zip(('fast', 'normal', 'total', 'cache_hits', 'cache_misses'), (int(x) for x in v)))


class BootParams(C.Structure):
    """fhe_boot_params (include/fhe_gpu.h)"""
    _fields_ = [('slots', C.c_int), ('level_budget_enc', C.c_int), ('level_budget_dec', C.c_int),
                ('K', C.c_int), ('r', C.c_int), ('degree', C.c_int), ('correction_bits', C.c_int)]


class Bootstrapper:
    """EvalBootstrapSetup(levelBudget, {0, 0}, slots) / EvalBootstrapKeyGen /
    EvalBootstrap on the GPU (fhe_boot_*; tests/k-way/KWaySort235Test.cpp:46-48)."""

    def __init__(self, ctx, slots, budget=(4, 4), K=512, r=6, degree=88, correction_bits=10, keygen=True):
        p = BootParams(slots, budget[0], budget[1], K, r, degree, correction_bits)
        out = C.c_void_p()
        _chk(lib().fhe_boot_create(ctx.h, C.byref(p), C.byref(out)))
        self.ctx, self.h = ctx, out.value
        ctx._boots.append(self)
        if keygen:
            self.keygen()

    def close(self):
        if getattr(self, 'h', None):
            lib().fhe_boot_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def keygen(self):
        _chk(lib().fhe_boot_keygen(self.h))

    @property
    def depth(self):
        return lib().fhe_boot_depth(self.h)

    def rotations(self):
        out = np.zeros(4096, dtype=np.int32)
        m = lib().fhe_boot_rotation_indices(self.h, out.ctypes.data_as(C.POINTER(C.c_int32)), 4096)
        if m < 0:
            _chk(-m)
        return [int(x) for x in out[:m]]

    def bootstrap(self, x, stage=0):
        out = C.c_void_p()
        _chk(lib().fhe_bootstrap_stage(self.h, x.h, stage, C.byref(out)))
        return Ct(self.ctx, out.value)

    def mod_raise(self, x): return self.bootstrap(x, 4)
    def coeffs_to_slots(self, x): return self.bootstrap(x, 1)
    def eval_mod(self, x): return self.bootstrap(x, 2)
    def slots_to_coeffs(self, x): return self.bootstrap(x, 3)


class Ct:
    def __init__(self, ctx, h):
        self.ctx, self.h = ctx, h

    def __del__(self):
        try:
            if self.h:
                lib().fhe_ct_free(self.h)
        except Exception:
            pass

    def info(self):
        lv, sl, lm, sc = C.c_int(), C.c_int(), C.c_int(), C.c_double()
        _chk(lib().fhe_ct_info(self.h, C.byref(lv), C.byref(sl), C.byref(sc), C.byref(lm)))
        return dict(level=lv.value, slots=sl.value, scale=sc.value, limbs=lm.value)

    @property
    def level(self):
        return self.info()['level']

    @property
    def slots(self):
        return self.info()['slots']

    def set_slots(self, s):
        _chk(lib().fhe_ct_set_slots(self.h, s))

    def data(self):
        inf = self.info()
        out = np.empty((2, inf['limbs'], self.ctx.n), dtype=np.uint64)
        _chk(lib().fhe_ct_download(self.ctx.h, self.h, _u64(out)))
        return out

    def decrypt(self):
        return self.ctx.decrypt(self)


class Pt:
    def __init__(self, ctx, h):
        self.ctx, self.h = ctx, h

    def data(self):
        """the plaintext's words [limbs][n] (NTT form)"""
        out = np.empty((lib().fhe_pt_limbs(self.h), self.ctx.n), dtype=np.uint64)
        _chk(lib().fhe_pt_download(self.ctx.h, self.h, _u64(out)))
        return out

    def __del__(self):
        try:
            if self.h:
                lib().fhe_pt_free(self.h)
        except Exception:
            pass


class Context:
    """One engine on one GPU (`device`).  seed 0 (the default): the secret, the
    errors and the encryption randomness come from the OS CSPRNG; a nonzero seed
    makes keys and encryptions reproducible (tests, oracle parity) and must not
    be used to protect data."""

    def __init__(self, logN, L, scale_bits=40, first_bits=60, dnum=3, seed=0, device=0, keygen=True, _handle=None,
                 ps_split=None):
        self.logN, self.n, self.L = logN, 1 << logN, L
        self._boots = []
        if _handle is None:
            p = Params(logN, L, scale_bits, first_bits, dnum, seed)
            h = C.c_void_p()
            _chk(lib().fhe_ctx_create(C.byref(p), device, C.byref(h)))
            _handle = h
        self.h = _handle
        nq, K, alpha = C.c_int(), C.c_int(), C.c_int()
        _chk(lib().fhe_ctx_info(self.h, C.byref(nq), C.byref(K), C.byref(alpha), None, None))
        self.nq, self.K, self.alpha = nq.value, K.value, alpha.value
        self.primes = np.empty(self.nq + self.K, dtype=np.uint64)
        self.delta = np.empty(L + 1)
        _chk(lib().fhe_ctx_info(self.h, None, None, None, _u64(self.primes), _dbl(self.delta)))
        if ps_split is not None:
            self.set_ps_split(ps_split)
        if keygen:
            self.keygen()

    # ---- wire format (src/sort.h:31-74, 97-102: Serial::*ToFile, Serialize/DeserializeEval*Key)
    @classmethod
    def deserialize(cls, path, device=0):
        """Serial::DeserializeFromFile(path, cc): a context with no keys."""
        info = wire_inspect(path)
        h = C.c_void_p()
        _chk(lib().fhe_deserialize_context(os.fsencode(path), device, C.byref(h)))
        return cls(int(info['log_n']), int(info['nq']) - 1, keygen=False, _handle=h)

    def serialize(self, path):
        _chk(lib().fhe_serialize_context(self.h, os.fsencode(path)))

    def serialize_public_key(self, path): _chk(lib().fhe_serialize_public_key(self.h, os.fsencode(path)))
    def deserialize_public_key(self, path): _chk(lib().fhe_deserialize_public_key(self.h, os.fsencode(path)))
    def serialize_secret_key(self, path): _chk(lib().fhe_serialize_secret_key(self.h, os.fsencode(path)))
    def deserialize_secret_key(self, path): _chk(lib().fhe_deserialize_secret_key(self.h, os.fsencode(path)))
    def serialize_eval_mult_key(self, path): _chk(lib().fhe_serialize_eval_mult_key(self.h, os.fsencode(path)))
    def deserialize_eval_mult_key(self, path): _chk(lib().fhe_deserialize_eval_mult_key(self.h, os.fsencode(path)))

    def serialize_eval_automorphism_key(self, path):
        _chk(lib().fhe_serialize_eval_automorphism_key(self.h, os.fsencode(path)))

    def deserialize_eval_automorphism_key(self, path):
        n = C.c_int()
        _chk(lib().fhe_deserialize_eval_automorphism_key(self.h, os.fsencode(path), C.byref(n)))
        return n.value

    def serialize_ciphertext(self, ct, path):
        _chk(lib().fhe_serialize_ciphertext(self.h, ct.h, os.fsencode(path)))

    def deserialize_ciphertext(self, path):
        h = C.c_void_p()
        _chk(lib().fhe_deserialize_ciphertext(self.h, os.fsencode(path), C.byref(h)))
        return Ct(self, h.value)

    def close(self):
        for b in getattr(self, '_boots', []):  # bootstrappers refer to the context
            b.close()
        if getattr(self, 'h', None):
            lib().fhe_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def digits(self):
        return (self.nq + self.alpha - 1) // self.alpha

    def _new(self, fn, *args):
        out = C.c_void_p()
        _chk(fn(self.h, *args, C.byref(out)))
        return Ct(self, out.value)

    # keys ---------------------------------------------------------------
    def keygen(self):
        _chk(lib().fhe_keygen(self.h))

    def gen_rotation_keys(self, rots):
        r = np.asarray(rots, dtype=np.int32)
        _chk(lib().fhe_gen_rotation_keys(self.h, _int(r), len(r)))

    def load_keys_from(self, orc, rots=()):
        """Upload the CPU oracle's secret/public/relin/rotation keys (parity tests)."""
        s = np.ascontiguousarray(orc.secret_ntt())
        _chk(lib().fhe_ctx_load_secret(self.h, _u64(s)))
        pk = np.ascontiguousarray(orc.public_key())
        _chk(lib().fhe_ctx_load_public(self.h, _u64(pk)))
        rl = np.ascontiguousarray(orc.relin_key())
        keys, idx = [], []
        for k in rots:
            g, key = orc.rot_key(k)
            if g:
                keys.append(np.ascontiguousarray(key))
                idx.append(k)
        arr = (u64p * max(1, len(keys)))(*[_u64(k) for k in keys])
        ia = np.asarray(idx, dtype=np.int32)
        _chk(lib().fhe_ctx_load_keys(self.h, _u64(rl), _int(ia), arr, len(keys)))

    def load_galois_keys_from(self, orc, gs):
        """Upload the oracle's keys of galois elements gs (conjugation: 2n - 1)."""
        for g in gs:
            key = orc.galois_key(g)
            if key is not None:
                _chk(lib().fhe_ctx_load_galois_key(self.h, int(g), _u64(np.ascontiguousarray(key))))

    def gen_galois_keys(self, gs):
        g = np.asarray(gs, dtype=np.uint64)
        _chk(lib().fhe_gen_galois_keys(self.h, _u64(g), len(g)))

    def key_bytes(self):
        return lib().fhe_key_bytes(self.h)

    def encode_complex(self, v, slots, level, scale=None):
        v = np.asarray(v, dtype=np.complex128)
        re, im = np.ascontiguousarray(v.real), np.ascontiguousarray(v.imag)
        scale = self.delta[level] if scale is None else scale
        out = C.c_void_p()
        _chk(lib().fhe_pt_encode_complex(self.h, _dbl(re), _dbl(im), len(v), slots, level, scale, C.byref(out)))
        return Pt(self, out.value)

    def conjugate(self, a): return self._new(lib().fhe_conjugate, a.h)

    # objects ------------------------------------------------------------
    def encode(self, v, slots, level=0):
        v = np.ascontiguousarray(v, dtype=np.float64)
        out = C.c_void_p()
        _chk(lib().fhe_pt_encode(self.h, _dbl(v), len(v), slots, level, C.byref(out)))
        return Pt(self, out.value)

    def encode_device(self, v, slots, level=0):
        """fhe_pt_encode_device: encode(v) on the device, word for word"""
        v = np.ascontiguousarray(v, dtype=np.float64)
        out = C.c_void_p()
        _chk(lib().fhe_pt_encode_device(self.h, _dbl(v), len(v), slots, level, C.byref(out)))
        return Pt(self, out.value)

    def encode_masks(self, specs, num_slots, N):
        """fhe_pt_encode_masks: specs = [(kind, k, r, level), ...] -> plaintexts"""
        sp = np.ascontiguousarray(np.asarray(specs, dtype=np.int32).reshape(-1, 4))
        outs = (C.c_void_p * len(sp))()
        _chk(lib().fhe_pt_encode_masks(self.h, sp.ctypes.data_as(C.POINTER(C.c_int32)), len(sp), num_slots, N, outs))
        return [Pt(self, outs[i]) for i in range(len(sp))]

    def set_mask_cache(self, cache):
        """True (default): masks encoded once per context; False: re-encoded on the
        device at the start of every sort (the reference's per-sort encoding)"""
        _chk(lib().fhe_set_mask_cache(self.h, 1 if cache else 0))

    def upload_pt(self, data, level, slots, scale=None):
        data = np.ascontiguousarray(data, dtype=np.uint64)
        scale = self.delta[level] if scale is None else scale
        out = C.c_void_p()
        _chk(lib().fhe_pt_upload(self.h, _u64(data), data.shape[0], level, slots, scale, C.byref(out)))
        return Pt(self, out.value)

    def encrypt(self, v, slots=None, level=0):
        v = np.ascontiguousarray(v, dtype=np.float64)
        return self._new(lib().fhe_encrypt, _dbl(v), len(v), slots or len(v), level)

    def encrypt_ext(self, v, slots=None):
        """FLEXIBLEAUTOEXT-style encryption (lands at level 1, noise / q_L)."""
        v = np.ascontiguousarray(v, dtype=np.float64)
        return self._new(lib().fhe_encrypt_ext, _dbl(v), len(v), slots or len(v))

    def decrypt(self, ct):
        out = np.empty(ct.slots)
        _chk(lib().fhe_decrypt(self.h, ct.h, _dbl(out)))
        return out

    def upload(self, data, level, slots, scale=None):
        data = np.ascontiguousarray(data, dtype=np.uint64)
        scale = self.delta[level] if scale is None else scale
        return self._new(lib().fhe_ct_upload, _u64(data), data.shape[1], level, slots, scale)

    def from_oracle(self, oct):
        inf = oct.info()
        return self.upload(oct.data(), inf['level'], inf['slots'], inf['scale'])

    # ops ----------------------------------------------------------------
    def add(self, a, b): return self._new(lib().fhe_add, a.h, b.h)
    def sub(self, a, b): return self._new(lib().fhe_sub, a.h, b.h)
    def negate(self, a): return self._new(lib().fhe_negate, a.h)
    def add_const(self, a, k): return self._new(lib().fhe_add_const, a.h, k)
    def mul_const(self, a, k): return self._new(lib().fhe_mul_const, a.h, k)
    def mul_const_to(self, a, k, t): return self._new(lib().fhe_mul_const_to, a.h, k, t)
    def mul_int(self, a, k): return self._new(lib().fhe_mul_int, a.h, k)
    def level_adjust(self, a, t): return self._new(lib().fhe_level_adjust, a.h, t)
    def rescale(self, a): return self._new(lib().fhe_rescale, a.h)
    def mul_plain(self, a, p): return self._new(lib().fhe_mul_plain, a.h, p.h)
    def add_plain(self, a, p): return self._new(lib().fhe_add_plain, a.h, p.h)
    def mul(self, a, b): return self._new(lib().fhe_mul_relin, a.h, b.h)
    def square(self, a): return self._new(lib().fhe_square_relin, a.h)
    def rotate(self, a, k): return self._new(lib().fhe_rotate, a.h, k)

    def rotate_hoisted(self, a, ks):
        ks = np.asarray(ks, dtype=np.int32)
        outs = (C.c_void_p * len(ks))()
        _chk(lib().fhe_rotate_hoisted(self.h, a.h, _int(ks), len(ks), outs))
        return [Ct(self, outs[i]) for i in range(len(ks))]

    def stack(self, xs):
        arr = (C.c_void_p * len(xs))(*[x.h for x in xs])
        out = C.c_void_p()
        _chk(lib().fhe_ct_stack(self.h, arr, len(xs), C.byref(out)))
        return Ct(self, out.value)

    def mul_plain_sum(self, cts, pts):
        ca = (C.c_void_p * len(cts))(*[c.h for c in cts])
        pa = (C.c_void_p * len(pts))(*[p.h for p in pts])
        out = C.c_void_p()
        _chk(lib().fhe_mul_plain_sum(self.h, ca, pa, len(cts), C.byref(out)))
        return Ct(self, out.value)

    def member(self, a, m): return self._new(lib().fhe_ct_member, a.h, m)
    def sum_members(self, a): return self._new(lib().fhe_ct_sum_members, a.h)

    def linear_sum_to(self, xs, cs, target):
        arr = (C.c_void_p * len(xs))(*[x.h for x in xs])
        cs = np.ascontiguousarray(cs, dtype=np.float64)
        return self._new(lib().fhe_linear_sum_to, arr, _dbl(cs), len(xs), target)

    def cheb(self, a, coeffs, lo=-1.0, hi=1.0):
        c = np.ascontiguousarray(coeffs, dtype=np.float64)
        return self._new(lib().fhe_cheb_ps, a.h, _dbl(c), len(c), lo, hi)

    def sign(self, a, n, dg, df): return self._new(lib().fhe_sign_composite, a.h, n, dg, df)
    def compare(self, a, b, n, dg, df): return self._new(lib().fhe_compare, a.h, b.h, n, dg, df)
    def indicator(self, a, c, n, dg, df): return self._new(lib().fhe_indicator, a.h, c, n, dg, df)

    def rotation_tree(self, N, rots, algo=0):
        """RotationTree<N>(cc, rots, algo) (src/rotation.h:240-358); algo 0 = NAF."""
        return RotationTree(self, N, rots, algo)

    def compose_rotate(self, a, N, rots, algo, rotation):
        r = np.asarray(rots, dtype=np.int32)
        return self._new(lib().fhe_compose_rotate, a.h, N, _int(r), len(r), algo, rotation)

    def compose_rotate_members(self, a, N, rots, algo, rotations):
        """member m of the batch `a` rotated by rotations[m], steps batched across members"""
        r = np.asarray(rots, dtype=np.int32)
        k = np.asarray(rotations, dtype=np.int32)
        return self._new(lib().fhe_compose_rotate_members, a.h, N, _int(r), len(r), algo, _int(k), len(k))

    def direct_sort(self, x, N, rots, cfg, mode=0, rank=None, shard=(0, 1), allreduce=None):
        r = np.asarray(rots, dtype=np.int32)
        hk = _Hook(allreduce)
        try:
            return self._new(lib().fhe_direct_sort, x.h, rank.h if rank is not None else None, N, _int(r), len(r),
                             cfg[0], cfg[1], cfg[2], mode, shard[0], shard[1], hk.ptr(), None)
        except FheError as e:
            hk.reraise(e)

    def sort_hybrid(self, x, N, rots, cfg, mode=0, rank=None, max_array=256, mask=0, shard=(0, 1), allreduce=None):
        """DirectSort::sort_hybrid (mode 0) or rotationIndexCheckHybrid(rank, x) (mode 1)."""
        r = np.asarray(rots, dtype=np.int32)
        hk = _Hook(allreduce)
        try:
            return self._new(lib().fhe_sort_hybrid, x.h, rank.h if rank is not None else None, N, _int(r), len(r),
                             cfg[0], cfg[1], cfg[2], mode, max_array, mask, shard[0], shard[1], hk.ptr(), None)
        except FheError as e:
            hk.reraise(e)

    def mehp24_sort(self, x, N, cfg, dg_i, df_i, sub=0, shard=(0, 1), allreduce=None):
        """mehp24::sortFG (sub 0; x holds N values in N*N slots) or
        sortLargeArrayFG with parts of `sub` values (x in sub*sub slots).
        shard=(rank, world): the pair compares and indicators are split over
        ranks and combined by `allreduce` (or RCCL after comm_init)."""
        if shard == (0, 1) and allreduce is None:
            return self._new(lib().fhe_mehp24_sort, x.h, N, sub, cfg[0], cfg[1], cfg[2], dg_i, df_i)
        hk = _Hook(allreduce)
        try:
            return self._new(lib().fhe_mehp24_sort_sharded, x.h, N, sub, cfg[0], cfg[1], cfg[2], dg_i, df_i,
                             shard[0], shard[1], hk.ptr(), None)
        except FheError as e:
            hk.reraise(e)

    def mehp24_indicator(self, x, b, dg, df):
        return self._new(lib().fhe_mehp24_indicator, x.h, b, dg, df)

    def kway_sort(self, x, k, M, cfg, boot=None):
        """kwaySort::Sorter::sorter via KWayAdapter<k^M>::sort; cfg = (3, dg, df).
        boot: a Bootstrapper (checkLevelAndBoot + compositeSign's lazy bootstrap);
        the number of checkLevelAndBoot bootstraps is left in self.kway_bootstraps."""
        if boot is None:
            return self._new(lib().fhe_kway_sort, x.h, k, M, cfg[1], cfg[2])
        nb = C.c_int()
        out = self._new(lib().fhe_kway_sort_boot, x.h, k, M, cfg[1], cfg[2], boot.h, C.byref(nb))
        self.kway_bootstraps = nb.value
        return out

    def check_level_and_boot(self, x, need, boot=None):
        """EvalUtils::checkLevelAndBoot: (ciphertext, booted)."""
        b = C.c_int()
        out = self._new(lib().fhe_check_level_and_boot, x.h, need, boot.h if boot is not None else None, C.byref(b))
        return out, bool(b.value)

    def kway_sorter(self, kk, xs, cmps):
        """SortUtils::fcnL (kk = 1) or the kk-sorter (kk = 2..5): ascending outputs."""
        xa = (C.c_void_p * len(xs))(*[x.h for x in xs])
        ca = (C.c_void_p * len(cmps))(*[c.h for c in cmps])
        nout = 1 if kk == 1 else kk
        outs = (C.c_void_p * nout)()
        _chk(lib().fhe_kway_sorter(self.h, kk, xa, len(xs), ca, len(cmps), outs))
        return [Ct(self, outs[i]) for i in range(nout)]

    # multi-GPU -----------------------------------------------------------
    @staticmethod
    def comm_unique_id():
        buf = (C.c_uint8 * 128)()
        _chk(lib().fhe_comm_get_unique_id(buf))
        return bytes(buf)

    def comm_init(self, uid, rank, world):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        _chk(lib().fhe_comm_init(self.h, buf, rank, world))

    def pool_trim(self):
        _chk(lib().fhe_pool_trim(self.h))

    def pool_stats(self):
        v = [C.c_uint64() for _ in range(3)]
        _chk(lib().fhe_pool_stats(self.h, *[C.byref(x) for x in v]))
        return {'live': v[0].value, 'cached': v[1].value, 'peak': v[2].value}

    def set_sort_lanes(self, m):
        _chk(lib().fhe_set_sort_lanes(self.h, m))

    def set_ps_split(self, split):
        """PS_SPLIT_OPENFHE (default) or PS_SPLIT_ENGINE (fhe_set_ps_split)"""
        _chk(lib().fhe_set_ps_split(self.h, int(split)))

    @property
    def ps_split(self):
        return int(lib().fhe_get_ps_split(self.h))

    def set_sort_stack(self, m):
        _chk(lib().fhe_set_sort_stack(self.h, m))

    def ct_allreduce(self, ct):
        _chk(lib().fhe_ct_allreduce(self.h, ct.h))

    # kernel level -------------------------------------------------------
    def ntt(self, prime_index, data, inverse=False):
        d = np.ascontiguousarray(data, dtype=np.uint64).copy()
        limbs = 1 if d.ndim == 1 else d.shape[0]
        _chk(lib().fhe_ntt(self.h, _u64(d), prime_index, limbs, 1 if inverse else 0))
        return d

    def ntt_dev(self, dev_ptr, first_prime, limbs, inverse=False, segments=1, seg_stride=0, stream=None):
        """fhe_ntt_dev: in place on device memory, enqueued on `stream` (hipStream_t
        as an int, None = the context stream); returns without synchronising"""
        _chk(lib().fhe_ntt_dev(self.h, C.c_void_p(dev_ptr), first_prime, limbs, segments, seg_stride,
                               1 if inverse else 0, C.c_void_p(stream) if stream else None))

    def automorph_dev(self, dev_in, limbs, galois, dev_out, stream=None):
        _chk(lib().fhe_automorph_dev(self.h, C.c_void_p(dev_in), limbs, galois, C.c_void_p(dev_out),
                                     C.c_void_p(stream) if stream else None))

    def modup(self, d):
        d = np.ascontiguousarray(d, dtype=np.uint64)
        ell = d.shape[0]
        digits = (ell + self.alpha - 1) // self.alpha
        out = np.empty((digits, ell + self.K, self.n), dtype=np.uint64)
        _chk(lib().fhe_modup(self.h, _u64(d), ell, _u64(out)))
        return out

    def moddown(self, x):
        x = np.ascontiguousarray(x, dtype=np.uint64)
        ell = x.shape[0] - self.K
        out = np.empty((ell, self.n), dtype=np.uint64)
        _chk(lib().fhe_moddown(self.h, _u64(x), ell, _u64(out)))
        return out

    def automorph(self, x, g):
        x = np.ascontiguousarray(x, dtype=np.uint64)
        out = np.empty_like(x)
        _chk(lib().fhe_automorph(self.h, _u64(x), x.shape[0], g, _u64(out)))
        return out

    def counters(self):
        out = np.zeros(7, dtype=np.uint64)
        _chk(lib().fhe_counters(self.h, _u64(out)))
        return dict(zip(['hmult', 'keyswitch', 'rotations', 'rescale', 'ptmult', 'constmult', 'opbytes'],
                        map(int, out)))

    def collective_stats(self):
        """{'allreduce_s': host seconds inside the sharded sorts' partial-sum
        exchanges since reset_counters(), 'allreduce_calls': their count}"""
        out = np.zeros(2, dtype=np.uint64)
        _chk(lib().fhe_collective_stats(self.h, _u64(out)))
        return {'allreduce_s': int(out[0]) * 1e-9, 'allreduce_calls': int(out[1])}

    def region_marker(self, begin):
        """k_region_begin / k_region_end on the context stream (profiling)"""
        _chk(lib().fhe_region_marker(self.h, 1 if begin else 0))

    def reset_counters(self):
        _chk(lib().fhe_reset_counters(self.h))

    def sync(self):
        _chk(lib().fhe_sync(self.h))

    def stream(self):
        return lib().fhe_stream(self.h)


def time_kernel(ctx, name, limbs, iters=20):
    ms, b = C.c_double(), C.c_double()
    _chk(lib().fhe_time_kernel(ctx.h, name.encode(), limbs, iters, C.byref(ms), C.byref(b)))
    return {'name': name, 'avg_ms': ms.value, 'bytes': b.value}


class KernelClock:
    """Live per-launch clock over real work (HIP events on the engine stream
    around every NTT pass): `with KernelClock(ctx) as k: ...; k.stats`."""

    def __init__(self, ctx):
        self.ctx, self.stats = ctx, None

    def __enter__(self):
        _chk(lib().fhe_kernel_clock_start(self.ctx.h))
        return self

    def __exit__(self, *exc):
        import json
        need = C.c_size_t()
        buf = C.create_string_buffer(1 << 20)
        _chk(lib().fhe_kernel_clock_stop(self.ctx.h, buf, len(buf), C.byref(need)))
        if need.value > len(buf):
            raise FheError(FHE_EINTERNAL, 'kernel clock report truncated')
        self.stats = json.loads(buf.value.decode())
        return False


def host_stats(reset=False):
    """process-wide host costs (fhe_host_stats): encodes, encode s, pool-miss mallocs, malloc s"""
    out = np.zeros(4)
    _chk(lib().fhe_host_stats(_dbl(out)))
    if reset:
        _chk(lib().fhe_host_stats_reset())
    return {'encodes': int(out[0]), 'encode_s': round(float(out[1]), 4), 'mallocs': int(out[2]),
            'malloc_s': round(float(out[3]), 4)}


def prng_block(key, counter, nonce):
    """ChaCha20 block of the secure sampler (fhe_prng_block), 16 u32 words"""
    k = np.ascontiguousarray(key, dtype=np.uint32)
    nn = np.ascontiguousarray(nonce, dtype=np.uint32)
    out = np.zeros(16, dtype=np.uint32)
    P32 = C.POINTER(C.c_uint32)
    _chk(lib().fhe_prng_block(k.ctypes.data_as(P32), int(counter), nn.ctypes.data_as(P32), out.ctypes.data_as(P32)))
    return out


def cheb_ps_uses_openfhe(coeffs):
    """True iff the OpenFHE split evaluates these coefficients with its division
    tree (fhe_cheb_ps_plan; False: the power-of-two fallback)"""
    c = np.ascontiguousarray(coeffs, dtype=np.float64)
    r = lib().fhe_cheb_ps_plan(c.ctypes.data_as(C.POINTER(C.c_double)), len(c))
    if r < 0:
        raise FheError(-r, lib().fhe_last_error().decode())
    return r == 1


def cheb_ps_depth(degree, split=PS_SPLIT_OPENFHE):
    """levels a degree-d Chebyshev series consumes under `split` (fhe_cheb_ps_depth)"""
    r = lib().fhe_cheb_ps_depth(int(degree), int(split))
    if r < 0:
        raise FheError(-r, lib().fhe_last_error().decode())
    return r


def size_parameters(N):
    d = C.c_int()
    rots = np.zeros(512, dtype=np.int32)
    m = lib().fhe_size_parameters(N, C.byref(d), _int(rots), 512)
    if m < 0:
        raise FheError(-m, lib().fhe_last_error().decode())
    return d.value, [int(x) for x in rots[:m]]


def mehp24_parameters(N):
    """The reference MEHP24 test's parameters for N (Mehp24SortTest.cpp:26-128)."""
    v = [C.c_int() for _ in range(7)]
    cfg = np.zeros(3, dtype=np.int32)
    rots = np.zeros(1024, dtype=np.int32)
    m = lib().fhe_mehp24_parameters(N, *(C.byref(x) for x in v[:4]), _int(cfg), *(C.byref(x) for x in v[4:]),
                                    _int(rots), 1024)
    if m < 0:
        raise FheError(-m, lib().fhe_last_error().decode())
    depth, log_ring, scale, dnum, dg_i, df_i, sub = (x.value for x in v)
    return dict(depth=depth, log_ring=log_ring, scale_bits=scale, dnum=dnum, cfg=tuple(int(c) for c in cfg), dg_i=dg_i,
                df_i=df_i, sub=sub, rots=[int(x) for x in rots[:m]])


def hybrid_parameters(N):
    """The hybrid sort test's (depth, rotations) for N (tests/DirectSortHTest.cpp:23-104)."""
    d = C.c_int()
    rots = np.zeros(256, dtype=np.int32)
    m = lib().fhe_hybrid_parameters(N, C.byref(d), _int(rots), 256)
    if m < 0:
        raise FheError(-m, lib().fhe_last_error().decode())
    return d.value, [int(x) for x in rots[:m]]


def mehp24_rotation_indices(N, sub=256):
    rots = np.zeros(1024, dtype=np.int32)
    m = lib().fhe_mehp24_rotation_indices(N, sub, _int(rots), 1024)
    if m < 0:
        raise FheError(-m, lib().fhe_last_error().decode())
    return [int(x) for x in rots[:m]]


def kway_rotation_indices(N):
    rots = np.zeros(64, dtype=np.int32)
    m = lib().fhe_kway_rotation_indices(N, _int(rots), 64)
    if m < 0:
        raise FheError(-m, lib().fhe_last_error().decode())
    return [int(x) for x in rots[:m]]


def kway_stage_count(k, M):
    return int(lib().fhe_kway_stage_count(k, M))


def kway_sort_type(k, M, stage):
    v = [C.c_int() for _ in range(3)]
    _chk(lib().fhe_kway_sort_type(k, M, stage, *[C.byref(a) for a in v]))
    return tuple(a.value for a in v)


def kway_rotate_distance(k, log_dist, slope):
    return int(lib().fhe_kway_rotate_distance(k, log_dist, slope))


def kway_gen_indices(num_slots, k, M, m, log_dist, slope):
    g = np.zeros(num_slots, dtype=np.int32)
    p = np.zeros(num_slots, dtype=np.int32)
    _chk(lib().fhe_kway_gen_indices(num_slots, k, M, m, log_dist, slope, _int(g), _int(p)))
    return g, p


def decompose(N, rots, rotation, wrapN, algo):
    r = np.asarray(rots, dtype=np.int32)
    vals = np.zeros(128, dtype=np.int32)
    sizes = np.zeros(128, dtype=np.int32)
    m = lib().fhe_decompose(N, _int(r), len(r), rotation, wrapN, algo, _int(vals), _int(sizes), 128)
    if m < 0:
        raise FheError(-m, lib().fhe_last_error().decode())
    return [(int(vals[i]), int(sizes[i])) for i in range(m)]
