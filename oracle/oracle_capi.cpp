// CPU ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h header).
// Plain C entry points so the Python tests (ctypes) can drive the oracle and
// compare it limb-for-limb with the GPU engine.  Errors never cross the ABI
// as exceptions: functions return NULL / -1 and orc_last_error() explains.
#include <cstring>
#include <memory>
#include <string>
#ifdef _OPENMP
#include <omp.h>
#endif

#include <stdexcept>

#include "oracle.h"

using namespace oracle;

namespace {
thread_local std::string g_err;
struct CtH {
    CtPtr p;
};
struct PtH {
    Plaintext p;
};
template <class F>
auto guard(F &&f, decltype(f()) fail) -> decltype(f()) {
    try {
        return f();
    } catch (const std::exception &e) {
        g_err = e.what();
        return fail;
    } catch (...) {
        g_err = "unknown error";
        return fail;
    }
}
CtH *wrap(CtPtr p) { return new CtH{std::move(p)}; }
SignConfig cfg3(int n, int dg, int df) {
    SignConfig c;
    c.n = n;
    c.dg = dg;
    c.df = df;
    return c;
}
}  // namespace

extern "C" {

const char *orc_last_error() { return g_err.c_str(); }

void *orc_ctx_new(int logN, int L, int scale_bits, int first_bits, int dnum, uint64_t seed) {
    return guard([&]() -> void * { return new Context(make_params(logN, L, scale_bits, first_bits, dnum), seed); },
                 (void *)nullptr);
}
void orc_ctx_free(void *c) { delete static_cast<Context *>(c); }
int orc_cheb_ps_depth(int degree, int split) {
    return guard([&]() { return cheb_ps_depth_split(degree, split); }, -1);
}
// Paterson-Stockmeyer split (1 = OpenFHE's, 0 = power-of-two), as fhe_set_ps_split
int orc_set_ps_split(void *c, int split) {
    if (split != 0 && split != 1) return -1;
    static_cast<Context *>(c)->ps_split = split;
    return 0;
}

// ModDown form: 1 = OpenFHE's flooring fast conversion, 0 = the exact centred one
int orc_set_moddown_floor(void *c, int floor) {
    if (floor != 0 && floor != 1) return -1;
    static_cast<Context *>(c)->moddown_floor = floor;
    return 0;
}
int orc_params(void *c, uint64_t *primes, int *nq, int *K, int *alpha, double *delta) {
    auto *cc = static_cast<Context *>(c);
    if (primes) std::memcpy(primes, cc->P.primes.data(), cc->P.primes.size() * 8);
    if (nq) *nq = (int)cc->P.nq();
    if (K) *K = cc->P.K;
    if (alpha) *alpha = cc->P.alpha;
    if (delta) std::memcpy(delta, cc->P.delta.data(), cc->P.delta.size() * 8);
    return 0;
}

int orc_keygen(void *c) {
    return guard([&]() { static_cast<Context *>(c)->keygen(); return 0; }, -1);
}
int orc_gen_rotation_keys(void *c, const int *rots, int nrot) {
    return guard([&]() {
        static_cast<Context *>(c)->gen_rotation_keys(std::vector<int>(rots, rots + nrot));
        return 0;
    }, -1);
}
int orc_secret_ntt(void *c, uint64_t *out) {
    auto *cc = static_cast<Context *>(c);
    std::memcpy(out, cc->s_ntt.data(), cc->s_ntt.size() * 8);
    return 0;
}
int orc_secret_coeff(void *c, int64_t *out) {
    auto *cc = static_cast<Context *>(c);
    std::memcpy(out, cc->s_coeff.data(), cc->s_coeff.size() * 8);
    return 0;
}
int orc_public_key(void *c, uint64_t *out) {
    auto *cc = static_cast<Context *>(c);
    std::memcpy(out, cc->pk.data(), cc->pk.size() * 8);
    return 0;
}
int orc_relin_key(void *c, uint64_t *out) {
    auto *cc = static_cast<Context *>(c);
    std::memcpy(out, cc->relin.data.data(), cc->relin.data.size() * 8);
    return cc->relin.digits;
}
// returns the galois element of the key, 0 if absent
uint64_t orc_rot_key(void *c, int k, uint64_t *out) {
    auto *cc = static_cast<Context *>(c);
    uint64_t g = galois_for_rotation(cc->P.logN, k);
    auto it = cc->rotkeys.find(g);
    if (it == cc->rotkeys.end()) return 0;
    if (out) std::memcpy(out, it->second.data.data(), it->second.data.size() * 8);
    return g;
}

// ------------------------------------------------------------ objects -----
void *orc_encode(void *c, const double *v, int len, int slots, int level) {
    return guard([&]() -> void * {
        auto *cc = static_cast<Context *>(c);
        return new PtH{cc->encode(std::vector<double>(v, v + len), slots, level)};
    }, (void *)nullptr);
}
int orc_pt_data(void *p, uint64_t *out) {
    auto *pt = static_cast<PtH *>(p);
    std::memcpy(out, pt->p.m.data(), pt->p.m.size() * 8);
    return (int)pt->p.limbs;
}
void orc_pt_free(void *p) { delete static_cast<PtH *>(p); }

void *orc_encrypt(void *c, const double *v, int len, int slots, int level) {
    return guard([&]() -> void * {
        auto *cc = static_cast<Context *>(c);
        return wrap(cc->encrypt(std::vector<double>(v, v + len), slots, level));
    }, (void *)nullptr);
}
void *orc_encrypt_ext(void *c, const double *v, int len, int slots) {
    return guard([&]() -> void * {
        return wrap(static_cast<Context *>(c)->encrypt_ext(std::vector<double>(v, v + len), slots));
    }, (void *)nullptr);
}
int orc_decrypt(void *c, void *ct, double *out) {
    return guard([&]() {
        auto *cc = static_cast<Context *>(c);
        auto v = cc->decrypt(*static_cast<CtH *>(ct)->p);
        std::memcpy(out, v.data(), v.size() * 8);
        return (int)v.size();
    }, -1);
}
void orc_ct_free(void *ct) { delete static_cast<CtH *>(ct); }
int orc_ct_info(void *ct, int *level, int *slots, double *scale, int *limbs) {
    auto &p = *static_cast<CtH *>(ct)->p;
    if (level) *level = p.level;
    if (slots) *slots = p.slots;
    if (scale) *scale = p.scale;
    if (limbs) *limbs = (int)p.limbs;
    return 0;
}
int orc_ct_data(void *ct, uint64_t *out) {
    auto &p = *static_cast<CtH *>(ct)->p;
    std::memcpy(out, p.c.data(), p.c.size() * 8);
    return 0;
}
void *orc_ct_from(void *c, const uint64_t *data, int limbs, int level, int slots, double scale) {
    auto *cc = static_cast<Context *>(c);
    auto p = std::make_shared<Ciphertext>();
    p->limbs = (size_t)limbs;
    p->level = level;
    p->slots = slots;
    p->scale = scale;
    p->c.assign(data, data + 2 * (size_t)limbs * cc->P.n);
    return wrap(p);
}
int orc_ct_set_slots(void *ct, int slots) {
    static_cast<CtH *>(ct)->p->slots = slots;
    return 0;
}

// ----------------------------------------------------------------- ops ----
#define CTX static_cast<Context *>(c)
#define CT(x) (*static_cast<CtH *>(x)->p)
void *orc_add(void *c, void *a, void *b) { return guard([&]() -> void * { return wrap(CTX->add(CT(a), CT(b))); }, (void *)nullptr); }
void *orc_sub(void *c, void *a, void *b) { return guard([&]() -> void * { return wrap(CTX->sub(CT(a), CT(b))); }, (void *)nullptr); }
void *orc_mul(void *c, void *a, void *b) { return guard([&]() -> void * { return wrap(CTX->mul(CT(a), CT(b))); }, (void *)nullptr); }
void *orc_square(void *c, void *a) { return guard([&]() -> void * { return wrap(CTX->square(CT(a))); }, (void *)nullptr); }
void *orc_negate(void *c, void *a) { return guard([&]() -> void * { return wrap(CTX->negate(CT(a))); }, (void *)nullptr); }
void *orc_add_const(void *c, void *a, double k) { return guard([&]() -> void * { return wrap(CTX->add_const(CT(a), k)); }, (void *)nullptr); }
void *orc_mul_const(void *c, void *a, double k) { return guard([&]() -> void * { return wrap(CTX->mul_const(CT(a), k)); }, (void *)nullptr); }
void *orc_mul_const_to(void *c, void *a, double k, int t) { return guard([&]() -> void * { return wrap(CTX->mul_const_to(CT(a), k, t)); }, (void *)nullptr); }
void *orc_mul_int(void *c, void *a, int64_t k) { return guard([&]() -> void * { return wrap(CTX->mul_int(CT(a), k)); }, (void *)nullptr); }
void *orc_level_adjust(void *c, void *a, int t) { return guard([&]() -> void * { return wrap(CTX->level_adjust(CT(a), t)); }, (void *)nullptr); }
void *orc_rescale(void *c, void *a) { return guard([&]() -> void * { return wrap(CTX->rescale(CT(a))); }, (void *)nullptr); }
void *orc_rotate(void *c, void *a, int k) { return guard([&]() -> void * { return wrap(CTX->rotate(CT(a), k)); }, (void *)nullptr); }
void *orc_mul_plain(void *c, void *a, void *p) {
    return guard([&]() -> void * { return wrap(CTX->mul_plain(CT(a), static_cast<PtH *>(p)->p)); }, (void *)nullptr);
}
void *orc_mul_plain_sum(void *c, void *const *as, void *const *ps, int m) {
    return guard([&]() -> void * {
        std::vector<const Ciphertext *> a;
        std::vector<const Plaintext *> p;
        for (int i = 0; i < m; ++i) {
            a.push_back(&CT(as[i]));
            p.push_back(&static_cast<PtH *>(ps[i])->p);
        }
        return wrap(CTX->mul_plain_sum(a, p));
    }, (void *)nullptr);
}
void *orc_add_plain(void *c, void *a, void *p) {
    return guard([&]() -> void * { return wrap(CTX->add_plain(CT(a), static_cast<PtH *>(p)->p)); }, (void *)nullptr);
}
int orc_rotate_hoisted(void *c, void *a, const int *ks, int m, void **outs) {
    return guard([&]() {
        std::vector<long> kk(ks, ks + m);
        auto v = CTX->rotate_hoisted(CT(a), kk);
        for (int i = 0; i < m; ++i) outs[i] = wrap(v[i]);
        return 0;
    }, -1);
}
void *orc_linear_sum_to(void *c, void **xs, const double *cs, int m, int target) {
    return guard([&]() -> void * {
        std::vector<const Ciphertext *> v;
        for (int i = 0; i < m; ++i) v.push_back(static_cast<CtH *>(xs[i])->p.get());
        return wrap(CTX->linear_sum_to(v, std::vector<double>(cs, cs + m), target));
    }, (void *)nullptr);
}
void *orc_cheb(void *c, void *a, const double *coeffs, int nc, double lo, double hi) {
    return guard([&]() -> void * {
        return wrap(cheb_series_ps(*CTX, CT(a), std::vector<double>(coeffs, coeffs + nc), lo, hi));
    }, (void *)nullptr);
}
void *orc_sign(void *c, void *a, int n, int dg, int df) {
    return guard([&]() -> void * { return wrap(sign(*CTX, CT(a), SignFunc::CompositeSign, cfg3(n, dg, df))); },
                 (void *)nullptr);
}
void *orc_compare(void *c, void *a, void *b, int n, int dg, int df) {
    return guard([&]() -> void * {
        return wrap(compare(*CTX, CT(a), CT(b), SignFunc::CompositeSign, cfg3(n, dg, df)));
    }, (void *)nullptr);
}
void *orc_indicator(void *c, void *a, double k, int n, int dg, int df) {
    return guard([&]() -> void * {
        return wrap(indicator(*CTX, CT(a), k, SignFunc::CompositeSign, cfg3(n, dg, df)));
    }, (void *)nullptr);
}
void *orc_compose_rotate(void *c, void *a, int N, const int *rots, int nrot, int algo, int rotation) {
    return guard([&]() -> void * {
        RotationComposer rc(*CTX, N, std::vector<int>(rots, rots + nrot), (DecomposeAlgo)algo);
        return wrap(rc.rotate(CT(a), rotation));
    }, (void *)nullptr);
}

typedef int (*orc_allreduce_fn)(uint64_t *data, uint64_t count, void *user);

// mode: 0 = sort, 1 = constructRank, 2 = rotationIndexCheckN(rank=b)
void *orc_direct_sort(void *c, void *x, void *rank, int N, const int *rots, int nrot, int n, int dg, int df,
                      int mode, int shard_rank, int shard_world, orc_allreduce_fn fn, void *user) {
    return guard([&]() -> void * {
        DirectSort ds(*CTX, N, std::vector<int>(rots, rots + nrot));
        ds.shard_rank = shard_rank;
        ds.shard_world = shard_world;
        if (fn) ds.allreduce = [fn, user](uint64_t *d, size_t cnt) {
            if (fn(d, (uint64_t)cnt, user) != 0) throw std::runtime_error("allreduce hook failed");
        };
        auto cfg = cfg3(n, dg, df);
        if (mode == 1) return wrap(ds.constructRank(CT(x), SignFunc::CompositeSign, cfg));
        if (mode == 2) return wrap(ds.rotationIndexCheckN(CT(rank), CT(x)));
        return wrap(ds.sort(CT(x), SignFunc::CompositeSign, cfg));
    }, (void *)nullptr);
}

// sort_hybrid (mode 0) / rotationIndexCheckHybrid(rank, x) (mode 1),
// src/sort_algo.h:893-1064; max_array = maxArraySize (256), mask_mode 0 = by N
void *orc_sort_hybrid(void *c, void *x, void *rank, int N, const int *rots, int nrot, int n, int dg, int df,
                      int mode, int max_array, int mask_mode) {
    return guard([&]() -> void * {
        DirectSort ds(*CTX, N, std::vector<int>(rots, rots + nrot));
        ds.hybrid_max_array = max_array;
        ds.hybrid_mask = mask_mode;
        if (mode == 1) return wrap(ds.rotationIndexCheckHybrid(CT(rank), CT(x)));
        return wrap(ds.sort_hybrid(CT(x), SignFunc::CompositeSign, cfg3(n, dg, df)));
    }, (void *)nullptr);
}

// MEHP24: sub == 0 -> sortFG on one ciphertext; otherwise sortLargeArrayFG
// with parts of `sub` values (mehp24_sort.h sortFG / sortLargeArrayFG)
void *orc_mehp24_sort_sharded(void *c, void *x, int N, int sub, int n, int dg, int df, int dg_i, int df_i,
                              int shard_rank, int shard_world, orc_allreduce_fn fn, void *user) {
    return guard([&]() -> void * {
        auto cfg = cfg3(n, dg, df);
        if (sub == 0) return wrap(mehp24::sort_fg(*CTX, CT(x), N, SignFunc::CompositeSign, cfg, dg_i, df_i));
        Shard sh;
        sh.rank = shard_rank;
        sh.world = shard_world;
        if (fn) sh.allreduce = [fn, user](uint64_t *d, size_t cnt) {
            if (fn(d, (uint64_t)cnt, user) != 0) throw std::runtime_error("allreduce hook failed");
        };
        return wrap(mehp24::sort_large_fg(*CTX, CT(x), N, sub, SignFunc::CompositeSign, cfg, dg_i, df_i, sh));
    }, (void *)nullptr);
}
void *orc_mehp24_sort(void *c, void *x, int N, int sub, int n, int dg, int df, int dg_i, int df_i) {
    return orc_mehp24_sort_sharded(c, x, N, sub, n, dg, df, dg_i, df_i, 0, 1, nullptr, nullptr);
}
void *orc_mehp24_indicator(void *c, void *a, double b, int dg, int df) {
    return guard([&]() -> void * { return wrap(mehp24::indicator_adv(*CTX, CTX->clone(CT(a)), b, dg, df)); },
                 (void *)nullptr);
}
int orc_mehp24_rotation_indices(int N, int sub, int *rots, int maxr) {
    return guard([&]() {
        auto r = mehp24::rotation_indices(N, sub);
        int m = std::min((int)r.size(), maxr);
        for (int i = 0; i < m; ++i) rots[i] = r[i];
        return (int)r.size();
    }, -1);
}

// k-way network (src/k-way/Sorter.cpp:289-404), CompositeSign(3, dg, df)
void *orc_kway_sort(void *c, void *x, int k, int M, int dg, int df) {
    return guard([&]() -> void * { return wrap(kway::sort(*CTX, CT(x), k, M, cfg3(3, dg, df))); },
                 (void *)nullptr);
}
// kk = 1: fcnL(x0, x1, s0); kk = 2..5: the kk-sorter; outs[] receives 1 or kk handles
int orc_kway_sorter(void *c, int kk, void **x, int nx, void **s, int ns, void **outs) {
    return guard([&]() -> int {
        std::vector<CtPtr> xv, sv;
        for (int i = 0; i < nx; ++i) xv.push_back(CTX->clone(CT(x[i])));
        for (int i = 0; i < ns; ++i) sv.push_back(CTX->clone(CT(s[i])));
        auto o = kway::sorter(*CTX, kk, xv, sv);
        for (size_t i = 0; i < o.size(); ++i) outs[i] = wrap(o[i]);
        return 0;
    }, -1);
}

// ------------------------------------------------- bootstrapping ----------
// EvalBootstrapSetup(levelBudget, {0,0}, slots) + EvalBootstrapKeyGen +
// EvalBootstrap (tests/k-way/KWaySort235Test.cpp:46-48, EvalUtils.cpp:76)
void *orc_boot_new(void *c, int slots, int budget_enc, int budget_dec, int K, int r, int degree,
                   int correction_bits) {
    return guard([&]() -> void * {
        BootConfig b;
        b.slots = slots;
        b.budget_enc = budget_enc;
        b.budget_dec = budget_dec;
        b.K = K;
        b.r = r;
        b.degree = degree;
        b.correction_bits = correction_bits;
        return new Bootstrapper(*CTX, b);
    }, (void *)nullptr);
}
void orc_boot_free(void *b) { delete static_cast<Bootstrapper *>(b); }
int orc_boot_keygen(void *b) {
    return guard([&]() { static_cast<Bootstrapper *>(b)->keygen(); return 0; }, -1);
}
int orc_boot_depth(void *b) { return static_cast<Bootstrapper *>(b)->depth(); }
int orc_boot_rotations(void *b, int *out, int maxr) {
    auto r = static_cast<Bootstrapper *>(b)->rotation_indices();
    for (int i = 0; i < std::min((int)r.size(), maxr); ++i) out[i] = r[i];
    return (int)r.size();
}
// stage: 0 = full bootstrap, 1 = CoeffsToSlots (input: a raised ciphertext),
// 2 = EvalMod, 3 = SlotsToCoeffs, 4 = ModRaise (context op)
void *orc_bootstrap(void *b, void *x, int stage) {
    return guard([&]() -> void * {
        auto *B = static_cast<Bootstrapper *>(b);
        switch (stage) {
            case 1: return wrap(B->coeffs_to_slots(CT(x)));
            case 2: return wrap(B->eval_mod(CT(x)));
            case 3: return wrap(B->slots_to_coeffs(CT(x)));
            case 4: return wrap(B->cc.mod_raise(CT(x)));
            default: return wrap(B->bootstrap(CT(x)));
        }
    }, (void *)nullptr);
}
void *orc_conjugate(void *c, void *a) { return guard([&]() -> void * { return wrap(CTX->conjugate(CT(a))); }, (void *)nullptr); }
int orc_gen_galois_keys(void *c, const uint64_t *gs, int m) {
    return guard([&]() { CTX->gen_galois_keys(std::vector<uint64_t>(gs, gs + m)); return 0; }, -1);
}
// key of galois element g (0 if absent, else g)
uint64_t orc_galois_key(void *c, uint64_t g, uint64_t *out) {
    auto it = CTX->rotkeys.find(g);
    if (it == CTX->rotkeys.end()) return 0;
    if (out) std::memcpy(out, it->second.data.data(), it->second.data.size() * 8);
    return g;
}
void *orc_encode_complex(void *c, const double *re, const double *im, int len, int slots, int level, double scale) {
    return guard([&]() -> void * {
        std::vector<std::complex<double>> v;
        for (int i = 0; i < len; ++i) v.emplace_back(re[i], im[i]);
        return new PtH{CTX->encode_complex(v, slots, level, scale)};
    }, (void *)nullptr);
}
// k-way sort / compare with a bootstrapper (b may be NULL: no bootstrapping)
void *orc_kway_sort_boot(void *c, void *x, int k, int M, int dg, int df, void *b) {
    return guard([&]() -> void * {
        auto cfg = cfg3(3, dg, df);
        if (b) cfg.boot = [b](const Ciphertext &ct) { return static_cast<Bootstrapper *>(b)->bootstrap(ct); };
        return wrap(kway::sort(*CTX, CT(x), k, M, cfg));
    }, (void *)nullptr);
}
void *orc_compare_boot(void *c, void *a, void *bb, int n, int dg, int df, void *b) {
    return guard([&]() -> void * {
        auto cfg = cfg3(n, dg, df);
        if (b) cfg.boot = [b](const Ciphertext &ct) { return static_cast<Bootstrapper *>(b)->bootstrap(ct); };
        return wrap(compare(*CTX, CT(a), CT(bb), SignFunc::CompositeSign, cfg));
    }, (void *)nullptr);
}

int orc_kway_sort_type(int k, int M, int stage, int *out3) {
    return guard([&]() {
        if (k < 2 || M < 1 || stage < 0 || stage >= kway::stage_count(k, M)) throw std::invalid_argument("stage");
        kway::sort_type(k, stage, out3[0], out3[1], out3[2]);
        return 0;
    }, -1);
}
int orc_kway_gen_indices(int ns, int k, int M, int m, int log_dist, int slope, int *grp, int *pos) {
    return guard([&]() {
        std::vector<int> g, p;
        kway::gen_indices(ns, k, M, m, log_dist, slope, g, p);
        std::copy(g.begin(), g.end(), grp);
        std::copy(p.begin(), p.end(), pos);
        return 0;
    }, -1);
}
int orc_kway_rotate_distance(int k, int log_dist, int slope) { return (int)kway::rotate_distance(k, log_dist, slope); }

int orc_size_parameters(int N, int *multDepth, int *rots, int maxr) {
    return guard([&]() {
        std::vector<int> r;
        direct_sort_size_parameters(N, *multDepth, r);
        int m = std::min((int)r.size(), maxr);
        for (int i = 0; i < m; ++i) rots[i] = r[i];
        return (int)r.size();
    }, -1);
}

int orc_decompose(int N, const int *rots, int nrot, int rotation, int wrapN, int algo, int *values, int *sizes,
                  int maxsteps) {
    return guard([&]() {
        Decomposer d(N, std::vector<int>(rots, rots + nrot));
        auto s = d.decompose(rotation, wrapN, (DecomposeAlgo)algo);
        int m = std::min((int)s.size(), maxsteps);
        for (int i = 0; i < m; ++i) {
            values[i] = s[i].value;
            sizes[i] = s[i].stepSize;
        }
        return (int)s.size();
    }, -1);
}

void orc_set_coeff_dir(const char *dir) { set_coefficient_dir(dir); }
int orc_doubled_sinc(int N, double *out, int maxn) {
    return guard([&]() {
        const auto &v = doubled_sinc_coefficients(N);
        int m = std::min((int)v.size(), maxn);
        if (out) std::memcpy(out, v.data(), m * 8);
        return (int)v.size();
    }, -1);
}

// ------------------------------------------------------- kernel-level -----
int orc_ntt(void *c, int prime_index, uint64_t *data, int inverse) {
    auto *cc = CTX;
    if (inverse)
        ntt_inverse(data, cc->tab[prime_index], cc->P.n);
    else
        ntt_forward(data, cc->tab[prime_index], cc->P.n);
    return 0;
}
uint64_t orc_psi(void *c, int prime_index) { return CTX->tab[prime_index].psi; }
int orc_automorph_perm(int logN, uint64_t g, uint32_t *out) {
    auto p = automorphism_perm(logN, g);
    std::memcpy(out, p.data(), p.size() * 4);
    return 0;
}
uint64_t orc_galois(int logN, int k) { return galois_for_rotation(logN, k); }
int orc_modup(void *c, const uint64_t *d, int ell, uint64_t *ext) {
    std::vector<uint64_t> e;
    CTX->modup(d, (size_t)ell, e);
    std::memcpy(ext, e.data(), e.size() * 8);
    return (int)(e.size() / CTX->P.n);
}
int orc_moddown(void *c, const uint64_t *in, int ell, uint64_t *out) {
    CTX->moddown(in, (size_t)ell, out);
    return 0;
}
int orc_counters(void *c, uint64_t *out) {
    auto &t = CTX->ctr;
    out[0] = t.hmult;
    out[1] = t.keyswitch;
    out[2] = t.rotations;
    out[3] = t.rescale;
    out[4] = t.ptmult;
    out[5] = t.constmult;
    return 0;
}
void orc_reset_counters(void *c) { CTX->ctr = OpCounters(); }
int orc_num_threads() {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
}
