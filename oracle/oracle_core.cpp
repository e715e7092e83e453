// CPU ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h header).
//
// RNS-CKKS core: primes, negacyclic NTT, canonical-embedding encoder,
// seeded sampling, key generation, encryption and the homomorphic operations
// that OpenFHE provides to the reference (EvalAdd/EvalSub/EvalMult/
// EvalRotate/rescale).  Spec: DESIGN.md §3.  Every routine is plain scalar
// C++ (OpenMP over limbs only); it is the checker for the HIP kernels.
#include "oracle.h"

#include <algorithm>
#include <cassert>
#include <cmath>
#include <complex>
#include <cstring>
#include <stdexcept>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace oracle {

// ============================================================== modular ====
Modulus::Modulus(u64 q_) : q(q_) {
    k = 64 - __builtin_clzll(q);
    u128 two2k = (u128)1 << (2 * k);
    mu = (u64)(two2k / q);
}

u64 mod_reduce128(u128 z, const Modulus &m) {
    // Barrett: z < q^2 <= 2^(2k); mu = floor(2^(2k)/q)
    u64 t = (u64)(z >> (m.k - 1));
    u64 qh = (u64)(((u128)t * m.mu) >> (m.k + 1));
    u64 r = (u64)z - qh * m.q;
    while (r >= m.q) r -= m.q;
    return r;
}
u64 mod_mul(u64 a, u64 b, const Modulus &m) { return mod_reduce128((u128)a * b, m); }
u64 mod_pow(u64 a, u64 e, const Modulus &m) {
    u64 r = 1 % m.q;
    a %= m.q;
    while (e) {
        if (e & 1) r = mod_mul(r, a, m);
        a = mod_mul(a, a, m);
        e >>= 1;
    }
    return r;
}
u64 mod_inv(u64 a, const Modulus &m) { return mod_pow(a % m.q, m.q - 2, m); }
u64 signed_to_mod(i64 v, u64 q) {
    if (v >= 0) return (u64)v % q;
    u64 r = (u64)(-(v + 1)) % q;  // avoid overflow at INT64_MIN
    r = (r + 1) % q;
    return r == 0 ? 0 : q - r;
}
u64 i128_to_mod(i128 v, u64 q) {
    if (v >= 0) return (u64)((u128)v % q);
    u128 r = (u128)(-(v + 1)) % q;
    r = (r + 1) % q;
    return r == 0 ? 0 : (u64)(q - r);
}
ScaledConst scaled_const(double x) {
    if (!std::isfinite(x)) throw std::invalid_argument("scaled constant is not finite");
    if (std::fabs(x) <= 0x1p62) return ScaledConst{std::llround(x), 0};
    const int sh = (int)std::ceil(std::log2(std::fabs(x))) - 62;
    return ScaledConst{std::llround(std::ldexp(x, -sh)), sh};
}

static u64 powmod_plain(u64 a, u64 e, u64 q) {
    u128 r = 1, b = a % q;
    while (e) {
        if (e & 1) r = (r * b) % q;
        b = (b * b) % q;
        e >>= 1;
    }
    return (u64)r;
}
bool is_prime(u64 n) {
    if (n < 2) return false;
    static const u64 small[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    for (u64 p : small) {
        if (n % p == 0) return n == p;
    }
    u64 d = n - 1;
    int s = 0;
    while ((d & 1) == 0) {
        d >>= 1;
        ++s;
    }
    for (u64 a : small) {
        u64 x = powmod_plain(a, d, n);
        if (x == 1 || x == n - 1) continue;
        bool comp = true;
        for (int r = 1; r < s; ++r) {
            x = (u64)(((u128)x * x) % n);
            if (x == n - 1) {
                comp = false;
                break;
            }
        }
        if (comp) return false;
    }
    return true;
}

// =============================================================== params ====
Params make_params(int logN, int L, int scale_bits, int first_bits, int dnum) {
    Params P;
    P.logN = logN;
    P.n = (size_t)1 << logN;
    P.L = L;
    P.dnum = dnum;
    P.scale_bits = scale_bits;
    P.first_bits = first_bits;
    const u64 m2 = 2 * (u64)P.n;
    std::vector<u64> q;
    std::set<u64> used;
    // first prime: largest prime < 2^first_bits, == 1 mod 2n
    u64 c = (((u64)1 << first_bits) - 1) / m2 * m2 + 1;
    if (c >= ((u64)1 << first_bits)) c -= m2;
    while (!is_prime(c)) c -= m2;
    q.push_back(c);
    used.insert(c);
    u64 q0 = c;
    // scaling primes, chosen greedily from the top level down so that the
    // canonical scale Delta_l (Delta_{l+1} = Delta_l^2 / q_{L-l}) stays at
    // 2^scale_bits: q_{L-l} = the unused NTT prime closest to Delta_l.
    auto closest_prime = [&](double target) -> u64 {
        u64 t = (u64)target;
        u64 lo = (t / m2) * m2 + 1;
        if (lo > t) lo -= m2;
        u64 hi = lo + m2;
        for (;;) {
            bool take_lo = (double)(t - lo) <= (double)(hi - t);
            u64 c = take_lo ? lo : hi;
            if (is_prime(c) && !used.count(c)) return c;
            if (take_lo)
                lo -= m2;
            else
                hi += m2;
        }
    };
    q.resize(L + 1);
    if (L >= 1) {
        double d = std::ldexp(1.0, scale_bits);
        q[L] = closest_prime(d);
        used.insert(q[L]);
        d = (double)q[L];
        for (int l = 0; l + 1 < L; ++l) {
            d = d * d / (double)q[L - l];
            q[L - l - 1] = closest_prime(d);
            used.insert(q[L - l - 1]);
        }
    }
    P.alpha = (L + 1 + dnum - 1) / dnum;
    // K special primes: enough bits to cover the largest digit product
    double maxbits = 0;
    for (int j = 0; j * P.alpha < L + 1; ++j) {
        double b = 0;
        for (int i = j * P.alpha; i < std::min((j + 1) * P.alpha, L + 1); ++i) b += std::log2((double)q[i]);
        maxbits = std::max(maxbits, b);
    }
    // P must exceed every digit product by the ModUp overshoot (the extended
    // digit is exact only up to a multiple < alpha of Q_j): with P ~ Q_j the
    // key-switch noise grows alpha-fold (measured: 10x at alpha 13, 40-bit scale)
    P.K = (int)std::ceil((maxbits + std::log2((double)P.alpha)) / 60.0);
    u64 p = q0;
    for (int k = 0; k < P.K; ++k) {
        do { p -= m2; } while (!is_prime(p) || used.count(p));
        q.push_back(p);
        used.insert(p);
    }
    P.primes = q;
    P.delta.resize(L + 1);
    P.delta[0] = (double)q[L];
    for (int l = 0; l < L; ++l) P.delta[l + 1] = P.delta[l] * P.delta[l] / (double)q[L - l];
    return P;
}

// ================================================================== NTT ====
static inline uint32_t bitrev(uint32_t x, int bits) {
    uint32_t r = 0;
    for (int i = 0; i < bits; ++i) {
        r = (r << 1) | (x & 1);
        x >>= 1;
    }
    return r;
}

NTTTable make_ntt_table(u64 q, int logN) {
    NTTTable t;
    t.mod = Modulus(q);
    size_t n = (size_t)1 << logN;
    // psi = g^((q-1)/2n), g = smallest quadratic non-residue
    u64 g = 2;
    while (mod_pow(g, (q - 1) / 2, t.mod) != q - 1) ++g;
    t.psi = mod_pow(g, (q - 1) / (2 * n), t.mod);
    u64 psi_inv = mod_inv(t.psi, t.mod);
    t.fwd.resize(n);
    t.fwd_shoup.resize(n);
    t.inv.resize(n);
    t.inv_shoup.resize(n);
    std::vector<u64> pw(n), pwi(n);
    pw[0] = 1;
    pwi[0] = 1;
    for (size_t i = 1; i < n; ++i) {
        pw[i] = mod_mul(pw[i - 1], t.psi, t.mod);
        pwi[i] = mod_mul(pwi[i - 1], psi_inv, t.mod);
    }
    for (size_t k = 0; k < n; ++k) {
        uint32_t r = bitrev((uint32_t)k, logN);
        t.fwd[k] = pw[r];
        t.inv[k] = pwi[r];
        t.fwd_shoup[k] = shoup_pre(t.fwd[k], q);
        t.inv_shoup[k] = shoup_pre(t.inv[k], q);
    }
    t.ninv = mod_inv(n % q, t.mod);
    t.ninv_shoup = shoup_pre(t.ninv, q);
    return t;
}

// Cooley-Tukey, natural -> bit-reversed; a[k] = a(psi^(2 brev(k) + 1))
void ntt_forward(u64 *a, const NTTTable &t, size_t n) {
    const u64 q = t.mod.q;
    size_t tt = n;
    for (size_t m = 1; m < n; m <<= 1) {
        tt >>= 1;
        for (size_t i = 0; i < m; ++i) {
            const size_t j1 = 2 * i * tt;
            const u64 W = t.fwd[m + i], Wp = t.fwd_shoup[m + i];
            for (size_t j = j1; j < j1 + tt; ++j) {
                u64 U = a[j];
                u64 V = mul_shoup(a[j + tt], W, Wp, q);
                a[j] = mod_add(U, V, q);
                a[j + tt] = mod_sub(U, V, q);
            }
        }
    }
}

// Gentleman-Sande, bit-reversed -> natural, includes n^-1
void ntt_inverse(u64 *a, const NTTTable &t, size_t n) {
    const u64 q = t.mod.q;
    size_t tt = 1;
    for (size_t m = n >> 1; m >= 1; m >>= 1) {
        size_t j1 = 0;
        for (size_t i = 0; i < m; ++i) {
            const u64 W = t.inv[m + i], Wp = t.inv_shoup[m + i];
            for (size_t j = j1; j < j1 + tt; ++j) {
                u64 U = a[j], V = a[j + tt];
                a[j] = mod_add(U, V, q);
                a[j + tt] = mul_shoup(mod_sub(U, V, q), W, Wp, q);
            }
            j1 += 2 * tt;
        }
        tt <<= 1;
    }
    for (size_t j = 0; j < n; ++j) a[j] = mul_shoup(a[j], t.ninv, t.ninv_shoup, q);
}

std::vector<uint32_t> automorphism_perm(int logN, u64 g) {
    size_t n = (size_t)1 << logN;
    u64 m2 = 2 * n;
    std::vector<uint32_t> perm(n);
    for (size_t k = 0; k < n; ++k) {
        u64 i = bitrev((uint32_t)k, logN);
        u64 e = ((2 * i + 1) * g) % m2;
        u64 ip = (e - 1) / 2;
        perm[k] = bitrev((uint32_t)ip, logN);
    }
    return perm;
}

u64 galois_for_rotation(int logN, long k) {
    long half = 1L << (logN - 1);
    long kk = ((k % half) + half) % half;
    u64 m2 = (u64)1 << (logN + 1);
    u64 g = 1;
    for (long i = 0; i < kk; ++i) g = (g * 5) % m2;
    return g;
}

// ================================================================= PRNG ====
SplitMix64::SplitMix64(u64 seed, u64 tag) : s(seed ^ (tag * 0xD1B54A32D192ED03ULL)) { next(); }
u64 SplitMix64::next() {
    s += 0x9E3779B97F4A7C15ULL;
    u64 z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
u64 sample_uniform_mod(SplitMix64 &g, u64 q) {
    int bits = 64 - __builtin_clzll(q);
    for (;;) {
        u64 r = g.next() >> (64 - bits);
        if (r < q) return r;
    }
}
int sample_ternary(SplitMix64 &g) {
    u64 r = g.next() % 3;
    return r == 0 ? 0 : (r == 1 ? 1 : -1);
}
int sample_cbd(SplitMix64 &g) {
    const u64 mask = (1ULL << 21) - 1;
    u64 a = g.next(), b = g.next();
    return __builtin_popcountll(a & mask) - __builtin_popcountll(b & mask);
}

// ============================================================== encoder ====
using cd = std::complex<double>;

struct EncTables {
    size_t n = 0;
    std::vector<cd> ksi;       // exp(2 pi i k / M), k = 0..M
    std::vector<u64> rotGroup; // 5^j mod M
};
static const EncTables &enc_tables(size_t n) {
    static std::map<size_t, EncTables> cache;
#pragma omp critical(oracle_enc_tables)
    {
        if (!cache.count(n)) {
            EncTables t;
            t.n = n;
            size_t M = 2 * n;
            t.ksi.resize(M + 1);
            for (size_t k = 0; k <= M; ++k) {
                double ang = 2.0 * M_PI * (double)k / (double)M;
                t.ksi[k] = cd(std::cos(ang), std::sin(ang));
            }
            t.rotGroup.resize(n / 2);
            u64 g = 1;
            for (size_t j = 0; j < n / 2; ++j) {
                t.rotGroup[j] = g;
                g = (g * 5) % M;
            }
            cache[n] = std::move(t);
        }
    }
    return cache.at(n);
}
static void bitrev_inplace(std::vector<cd> &v) {
    size_t n = v.size();
    for (size_t i = 1, j = 0; i < n; ++i) {
        size_t bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) std::swap(v[i], v[j]);
    }
}
static void emb_inv(std::vector<cd> &vals, const EncTables &T) {
    const size_t slots = vals.size(), M = 2 * T.n;
    for (size_t len = slots; len >= 1; len >>= 1) {
        for (size_t i = 0; i < slots; i += len) {
            size_t lenh = len >> 1, lenq = len << 2, gap = M / lenq;
            for (size_t j = 0; j < lenh; ++j) {
                size_t idx = (lenq - (T.rotGroup[j] % lenq)) * gap;
                cd u = vals[i + j] + vals[i + j + lenh];
                cd v = vals[i + j] - vals[i + j + lenh];
                v *= T.ksi[idx];
                vals[i + j] = u;
                vals[i + j + lenh] = v;
            }
        }
    }
    bitrev_inplace(vals);
    for (auto &x : vals) x /= (double)slots;
}
static void emb(std::vector<cd> &vals, const EncTables &T) {
    const size_t slots = vals.size(), M = 2 * T.n;
    bitrev_inplace(vals);
    for (size_t len = 2; len <= slots; len <<= 1) {
        for (size_t i = 0; i < slots; i += len) {
            size_t lenh = len >> 1, lenq = len << 2, gap = M / lenq;
            for (size_t j = 0; j < lenh; ++j) {
                size_t idx = (T.rotGroup[j] % lenq) * gap;
                cd u = vals[i + j];
                cd v = vals[i + j + lenh];
                v *= T.ksi[idx];
                vals[i + j] = u + v;
                vals[i + j + lenh] = u - v;
            }
        }
    }
}

// ============================================================== context ====
Context::Context(const Params &p, u64 seed_) : P(p), seed(seed_) {
    tab.resize(P.nall());
#pragma omp parallel for
    for (size_t i = 0; i < P.nall(); ++i) tab[i] = make_ntt_table(P.primes[i], P.logN);
}

Plaintext Context::encode(const std::vector<double> &v, int slots, int level) const {
    return encode_scaled(v, slots, level, P.delta[level]);
}
Plaintext Context::encode_scaled(const std::vector<double> &v, int slots, int level, double scale) const {
    std::vector<cd> z;
    for (size_t i = 0; i < v.size() && i < (size_t)std::max(slots, 0); ++i) z.push_back(cd(v[i], 0));
    return encode_complex(z, slots, level, scale);
}
Plaintext Context::encode_complex(const std::vector<cd> &v, int slots, int level, double scale, bool ext) const {
    const size_t n = P.n;
    if (slots <= 0 || (slots & (slots - 1)) || (size_t)slots > n / 2)
        throw std::invalid_argument("encode: slots must be a power of two <= n/2");
    const EncTables &T = enc_tables(n);
    std::vector<cd> vals(slots, cd(0, 0));
    for (size_t i = 0; i < v.size() && i < (size_t)slots; ++i) vals[i] = v[i];
    emb_inv(vals, T);
    const size_t gap = n / (2 * (size_t)slots);
    std::vector<i64> coef(n, 0);
    auto rnd = [](double x) -> i64 {
        if (!(std::fabs(x) < 9.2e18)) throw std::overflow_error("encode: scaled coefficient exceeds 63 bits");
        return std::llround(x);
    };
    for (size_t i = 0; i < (size_t)slots; ++i) {
        coef[i * gap] = rnd(vals[i].real() * scale);
        coef[i * gap + n / 2] = rnd(vals[i].imag() * scale);
    }
    Plaintext pt;
    pt.level = level;
    pt.slots = slots;
    pt.scale = scale;
    const size_t ell = P.limbs_at(level);
    pt.limbs = ext ? ell + P.K : ell;
    pt.m.assign(pt.limbs * n, 0);
#pragma omp parallel for
    for (size_t l = 0; l < pt.limbs; ++l) {
        const size_t pi = l < ell ? l : P.nq() + (l - ell);
        u64 *d = pt.m.data() + l * n;
        for (size_t k = 0; k < n; ++k) d[k] = signed_to_mod(coef[k], P.primes[pi]);
        ntt_forward(d, tab[pi], n);
    }
    return pt;
}

std::vector<double> Context::decode(const std::vector<u64> &m0, int slots, double scale) const {
    const size_t n = P.n;
    const u64 q0 = P.primes[0];
    const EncTables &T = enc_tables(n);
    const size_t gap = n / (2 * (size_t)slots);
    auto centered = [&](u64 x) -> double {
        return x > q0 / 2 ? -(double)(q0 - x) : (double)x;
    };
    std::vector<cd> vals(slots);
    for (size_t i = 0; i < (size_t)slots; ++i)
        vals[i] = cd(centered(m0[i * gap]) / scale, centered(m0[i * gap + n / 2]) / scale);
    emb(vals, T);
    std::vector<double> out(slots);
    for (size_t i = 0; i < (size_t)slots; ++i) out[i] = vals[i].real();
    return out;
}

void Context::keygen() {
    const size_t n = P.n, na = P.nall(), nq = P.nq();
    SplitMix64 gs(seed, 1);
    s_coeff.resize(n);
    for (size_t k = 0; k < n; ++k) s_coeff[k] = sample_ternary(gs);
    s_ntt.assign(na * n, 0);
#pragma omp parallel for
    for (size_t l = 0; l < na; ++l) {
        u64 *d = s_ntt.data() + l * n;
        for (size_t k = 0; k < n; ++k) d[k] = signed_to_mod(s_coeff[k], P.primes[l]);
        ntt_forward(d, tab[l], n);
    }
    // public key over Q
    pk.assign(2 * nq * n, 0);
    SplitMix64 ga(seed, 2), ge(seed, 3);
    std::vector<i64> e(n);
    for (size_t k = 0; k < n; ++k) e[k] = sample_cbd(ge);
    for (size_t l = 0; l < nq; ++l) {
        u64 *a = pk.data() + (nq + l) * n;
        for (size_t k = 0; k < n; ++k) a[k] = sample_uniform_mod(ga, P.primes[l]);
    }
#pragma omp parallel for
    for (size_t l = 0; l < nq; ++l) {
        const u64 q = P.primes[l];
        std::vector<u64> el(n);
        for (size_t k = 0; k < n; ++k) el[k] = signed_to_mod(e[k], q);
        ntt_forward(el.data(), tab[l], n);
        u64 *b = pk.data() + l * n;
        const u64 *a = pk.data() + (nq + l) * n;
        const u64 *s = s_ntt.data() + l * n;
        for (size_t k = 0; k < n; ++k)
            b[k] = mod_add(mod_sub(0, mod_mul(a[k], s[k], tab[l].mod), q), el[k], q);
    }
    // relinearisation key: s' = s^2
    std::vector<u64> s2(nq * n);
    for (size_t l = 0; l < nq; ++l)
        for (size_t k = 0; k < n; ++k)
            s2[l * n + k] = mod_mul(s_ntt[l * n + k], s_ntt[l * n + k], tab[l].mod);
    gen_switch_key(s2, relin, 0);
}

void Context::gen_switch_key(const std::vector<u64> &sp, SwitchKey &out, u64 kid) {
    const size_t n = P.n, na = P.nall(), nq = P.nq();
    const int digits = (int)((nq + P.alpha - 1) / P.alpha);
    out.digits = digits;
    out.data.assign((size_t)digits * 2 * na * n, 0);
    // P mod q_i
    std::vector<u64> Pmod(nq);
    for (size_t i = 0; i < nq; ++i) {
        u64 acc = 1 % P.primes[i];
        for (int k = 0; k < P.K; ++k) acc = mod_mul(acc, P.primes[nq + k] % P.primes[i], tab[i].mod);
        Pmod[i] = acc;
    }
    for (int j = 0; j < digits; ++j) {
        u64 *bj = out.data.data() + ((size_t)j * 2 + 0) * na * n;
        u64 *aj = out.data.data() + ((size_t)j * 2 + 1) * na * n;
        SplitMix64 ga(seed, 0x100000ULL + kid * 16 + 2 * j), ge(seed, 0x100000ULL + kid * 16 + 2 * j + 1);
        for (size_t l = 0; l < na; ++l)
            for (size_t k = 0; k < n; ++k) aj[l * n + k] = sample_uniform_mod(ga, P.primes[l]);
        std::vector<i64> e(n);
        for (size_t k = 0; k < n; ++k) e[k] = sample_cbd(ge);
        const size_t lo = (size_t)j * P.alpha, hi = std::min(nq, (size_t)(j + 1) * P.alpha);
#pragma omp parallel for
        for (size_t l = 0; l < na; ++l) {
            const u64 q = P.primes[l];
            std::vector<u64> el(n);
            for (size_t k = 0; k < n; ++k) el[k] = signed_to_mod(e[k], q);
            ntt_forward(el.data(), tab[l], n);
            const u64 *s = s_ntt.data() + l * n;
            for (size_t k = 0; k < n; ++k) {
                u64 v = mod_add(mod_sub(0, mod_mul(aj[l * n + k], s[k], tab[l].mod), q), el[k], q);
                if (l >= lo && l < hi) v = mod_add(v, mod_mul(Pmod[l], sp[l * n + k], tab[l].mod), q);
                bj[l * n + k] = v;
            }
        }
    }
}

void Context::gen_rotation_keys(const std::vector<int> &rot) {
    std::vector<u64> gs;
    for (int k : rot) gs.push_back(galois_for_rotation(P.logN, k));
    gen_galois_keys(gs);
}

void Context::gen_galois_keys(const std::vector<u64> &gs) {
    const size_t n = P.n, nq = P.nq();
    for (u64 g : gs) {
        if (g == 1 || rotkeys.count(g)) continue;
        auto perm = automorphism_perm(P.logN, g);
        std::vector<u64> sp(nq * n);
        for (size_t l = 0; l < nq; ++l)
            for (size_t kk = 0; kk < n; ++kk) sp[l * n + kk] = s_ntt[l * n + perm[kk]];
        gen_switch_key(sp, rotkeys[g], g);
    }
}

bool Context::has_rotation_key(long k) const { return rotkeys.count(galois_for_rotation(P.logN, k)) > 0; }

CtPtr Context::encrypt_pt(const Plaintext &pt) {
    const size_t n = P.n, nq = P.nq(), ell = pt.limbs;
    u64 cnt = enc_counter++;
    SplitMix64 gv(seed, 0x80000000ULL + 3 * cnt), g0(seed, 0x80000000ULL + 3 * cnt + 1),
        g1(seed, 0x80000000ULL + 3 * cnt + 2);
    std::vector<i64> v(n), e0(n), e1(n);
    for (size_t k = 0; k < n; ++k) v[k] = sample_ternary(gv);
    for (size_t k = 0; k < n; ++k) e0[k] = sample_cbd(g0);
    for (size_t k = 0; k < n; ++k) e1[k] = sample_cbd(g1);
    auto ct = std::make_shared<Ciphertext>();
    ct->level = pt.level;
    ct->slots = pt.slots;
    ct->scale = pt.scale;
    ct->limbs = ell;
    ct->c.assign(2 * ell * n, 0);
#pragma omp parallel for
    for (size_t l = 0; l < ell; ++l) {
        const u64 q = P.primes[l];
        std::vector<u64> vv(n), ee0(n), ee1(n);
        for (size_t k = 0; k < n; ++k) {
            vv[k] = signed_to_mod(v[k], q);
            ee0[k] = signed_to_mod(e0[k], q);
            ee1[k] = signed_to_mod(e1[k], q);
        }
        ntt_forward(vv.data(), tab[l], n);
        ntt_forward(ee0.data(), tab[l], n);
        ntt_forward(ee1.data(), tab[l], n);
        const u64 *b = pk.data() + l * n, *a = pk.data() + (nq + l) * n;
        u64 *c0 = ct->c.data() + l * n, *c1 = ct->c.data() + (ell + l) * n;
        const u64 *m = pt.m.data() + l * n;
        for (size_t k = 0; k < n; ++k) {
            c0[k] = mod_add(mod_add(mod_mul(vv[k], b[k], tab[l].mod), ee0[k], q), m[k], q);
            c1[k] = mod_add(mod_mul(vv[k], a[k], tab[l].mod), ee1[k], q);
        }
    }
    return ct;
}

CtPtr Context::encrypt(const std::vector<double> &v, int slots, int level) {
    return encrypt_pt(encode(v, slots, level));
}

// Fresh encryption one level up, as OpenFHE's FLEXIBLEAUTOEXT (its default
// CKKS scaling technique, which the reference's tests run under): the message
// is encoded at scale Delta_1 on the level-0 basis and multiplied by the top
// prime q_L (scale Delta_1 q_L), encrypted, and rescaled by q_L -- the
// encryption noise is divided by q_L and the result sits at level 1 with the
// canonical scale Delta_1.
CtPtr Context::encrypt_ext(const std::vector<double> &v, int slots) {
    if (P.L < 1) throw std::runtime_error("encrypt_ext: needs one extra level");
    Plaintext pt = encode_scaled(v, slots, 0, P.delta[1]);
    const size_t n = P.n;
    const u64 qL = P.primes[P.nq() - 1];
#pragma omp parallel for
    for (size_t l = 0; l < pt.limbs; ++l) {
        const u64 kv = qL % P.primes[l];
        u64 *d = pt.m.data() + l * n;
        for (size_t k = 0; k < n; ++k) d[k] = mod_mul(d[k], kv, tab[l].mod);
    }
    pt.scale = P.delta[1] * (double)qL;
    CtPtr r = rescale(*encrypt_pt(pt));
    r->scale = P.delta[1];
    return r;
}

std::vector<double> Context::decrypt(const Ciphertext &ct) {
    // m = c0 + c1 s on the first one or two limbs; two limbs -> CRT lift mod q0 q1
    const size_t n = P.n;
    const size_t L2 = ct.limbs >= 2 ? 2 : 1;
    std::vector<u64> m(L2 * n);
    const u64 *c0 = ct.poly(0, n), *c1 = ct.poly(1, n);
    for (size_t l = 0; l < L2; ++l) {
        for (size_t k = 0; k < n; ++k)
            m[l * n + k] = mod_add(c0[l * n + k], mod_mul(c1[l * n + k], s_ntt[l * n + k], tab[l].mod), P.primes[l]);
        ntt_inverse(m.data() + l * n, tab[l], n);
    }
    if (L2 == 1) return decode(m, ct.slots, ct.scale);
    const u64 q0 = P.primes[0], q1 = P.primes[1];
    const u64 q0inv = mod_inv(q0 % q1, tab[1].mod);
    const u128 Q = (u128)q0 * q1;
    std::vector<double> lifted(n);
    for (size_t k = 0; k < n; ++k) {
        const u64 a0 = m[k], a1 = m[n + k];
        const u64 t = mod_mul(mod_sub(a1, a0 % q1, q1), q0inv, tab[1].mod);
        const u128 x = (u128)a0 + (u128)q0 * t;
        lifted[k] = x > Q / 2 ? -(double)(Q - x) : (double)x;
    }
    return decode_real(lifted, ct.slots, ct.scale);
}

std::vector<double> Context::decode_real(const std::vector<double> &m, int slots, double scale) const {
    const size_t n = P.n;
    const EncTables &T = enc_tables(n);
    const size_t gap = n / (2 * (size_t)slots);
    std::vector<cd> vals(slots);
    for (size_t i = 0; i < (size_t)slots; ++i) vals[i] = cd(m[i * gap] / scale, m[i * gap + n / 2] / scale);
    emb(vals, T);
    std::vector<double> out(slots);
    for (size_t i = 0; i < (size_t)slots; ++i) out[i] = vals[i].real();
    return out;
}

// ================================================================== ops ====
static CtPtr make_ct(int level, int slots, double scale, size_t limbs, size_t n) {
    auto c = std::make_shared<Ciphertext>();
    c->level = level;
    c->slots = slots;
    c->scale = scale;
    c->limbs = limbs;
    c->c.assign(2 * limbs * n, 0);
    return c;
}

CtPtr Context::clone(const Ciphertext &a) const { return std::make_shared<Ciphertext>(a); }

CtPtr Context::drop_to(const Ciphertext &a, int level) const {
    if (level < a.level) throw std::invalid_argument("drop_to: cannot raise level");
    const size_t n = P.n, ell = P.limbs_at(level);
    auto r = make_ct(level, a.slots, a.scale, ell, n);
    for (int i = 0; i < 2; ++i) std::memcpy(r->poly(i, n), a.poly(i, n), ell * n * sizeof(u64));
    return r;
}

void Context::match_levels(CtPtr &a, CtPtr &b) {
    if (a->level < b->level) a = level_adjust(*a, b->level);
    else if (b->level < a->level) b = level_adjust(*b, a->level);
}

CtPtr Context::add(const Ciphertext &a0, const Ciphertext &b0) {
    CtPtr a = clone(a0), b = std::make_shared<Ciphertext>(b0);
    match_levels(a, b);
    const size_t n = P.n, ell = a->limbs;
#pragma omp parallel for
    for (size_t l = 0; l < ell; ++l)
        for (int i = 0; i < 2; ++i) {
            u64 *x = a->poly(i, n) + l * n;
            const u64 *y = b->poly(i, n) + l * n;
            for (size_t k = 0; k < n; ++k) x[k] = mod_add(x[k], y[k], P.primes[l]);
        }
    return a;
}

CtPtr Context::sub(const Ciphertext &a0, const Ciphertext &b0) {
    CtPtr a = clone(a0), b = std::make_shared<Ciphertext>(b0);
    match_levels(a, b);
    const size_t n = P.n, ell = a->limbs;
#pragma omp parallel for
    for (size_t l = 0; l < ell; ++l)
        for (int i = 0; i < 2; ++i) {
            u64 *x = a->poly(i, n) + l * n;
            const u64 *y = b->poly(i, n) + l * n;
            for (size_t k = 0; k < n; ++k) x[k] = mod_sub(x[k], y[k], P.primes[l]);
        }
    return a;
}

void Context::add_inplace(CtPtr &acc, const Ciphertext &b) {
    if (!acc) {
        acc = clone(b);
        return;
    }
    acc = add(*acc, b);
}

CtPtr Context::negate(const Ciphertext &a) const {
    auto r = clone(a);
    const size_t n = P.n;
    for (size_t l = 0; l < a.limbs; ++l)
        for (int i = 0; i < 2; ++i) {
            u64 *x = r->poly(i, n) + l * n;
            for (size_t k = 0; k < n; ++k) x[k] = mod_sub(0, x[k], P.primes[l]);
        }
    return r;
}

CtPtr Context::add_plain(const Ciphertext &a, const Plaintext &p) const {
    if (p.level != a.level) throw std::invalid_argument("add_plain: level mismatch");
    auto r = clone(a);
    const size_t n = P.n;
    for (size_t l = 0; l < a.limbs; ++l) {
        u64 *x = r->poly(0, n) + l * n;
        const u64 *y = p.m.data() + l * n;
        for (size_t k = 0; k < n; ++k) x[k] = mod_add(x[k], y[k], P.primes[l]);
    }
    return r;
}
CtPtr Context::sub_plain(const Ciphertext &a, const Plaintext &p) const {
    if (p.level != a.level) throw std::invalid_argument("sub_plain: level mismatch");
    auto r = clone(a);
    const size_t n = P.n;
    for (size_t l = 0; l < a.limbs; ++l) {
        u64 *x = r->poly(0, n) + l * n;
        const u64 *y = p.m.data() + l * n;
        for (size_t k = 0; k < n; ++k) x[k] = mod_sub(x[k], y[k], P.primes[l]);
    }
    return r;
}
CtPtr Context::plain_sub(const Plaintext &p, const Ciphertext &a) const {
    auto r = negate(a);
    const size_t n = P.n;
    for (size_t l = 0; l < a.limbs; ++l) {
        u64 *x = r->poly(0, n) + l * n;
        const u64 *y = p.m.data() + l * n;
        for (size_t k = 0; k < n; ++k) x[k] = mod_add(x[k], y[k], P.primes[l]);
    }
    return r;
}

CtPtr Context::add_const(const Ciphertext &a, double c) const {
    auto r = clone(a);
    const size_t n = P.n;
    const ScaledConst K = scaled_const(c * a.scale);
    for (size_t l = 0; l < a.limbs; ++l) {
        u64 kv = K.mod(P.primes[l]);
        u64 *x = r->poly(0, n) + l * n;
        for (size_t k = 0; k < n; ++k) x[k] = mod_add(x[k], kv, P.primes[l]);
    }
    return r;
}

CtPtr Context::mul_int(const Ciphertext &a, i64 K) const { return mul_int(a, ScaledConst{K, 0}); }
CtPtr Context::mul_int(const Ciphertext &a, const ScaledConst &K) const {
    auto r = clone(a);
    const size_t n = P.n;
#pragma omp parallel for
    for (size_t l = 0; l < a.limbs; ++l) {
        u64 kv = K.mod(P.primes[l]);
        for (int i = 0; i < 2; ++i) {
            u64 *x = r->poly(i, n) + l * n;
            for (size_t k = 0; k < n; ++k) x[k] = mod_mul(x[k], kv, tab[l].mod);
        }
    }
    return r;
}

// multiply by round(c * Delta_t * q_{L-t+1} / scale) at level t-1 and rescale
CtPtr Context::mul_const_to(const Ciphertext &a, double c, int target) {
    if (target <= a.level) throw std::invalid_argument("mul_const_to: target must exceed level");
    ctr.constmult++;
    auto d = drop_to(a, target - 1);
    const double qd = (double)P.primes[P.L - target + 1];
    const ScaledConst K = scaled_const(c * P.delta[target] * qd / a.scale);
    auto m = mul_int(*d, K);
    auto r = rescale(*m);
    r->scale = P.delta[target];
    return r;
}
CtPtr Context::mul_const(const Ciphertext &a, double c) { return mul_const_to(a, c, a.level + 1); }

CtPtr Context::level_adjust(const Ciphertext &a, int target) {
    if (target == a.level) return clone(a);
    return mul_const_to(a, 1.0, target);
}

CtPtr Context::mul_plain(const Ciphertext &a, const Plaintext &p) {
    if (p.level != a.level) throw std::invalid_argument("mul_plain: level mismatch");
    ctr.ptmult++;
    auto r = clone(a);
    const size_t n = P.n;
#pragma omp parallel for
    for (size_t l = 0; l < a.limbs; ++l) {
        const u64 *y = p.m.data() + l * n;
        for (int i = 0; i < 2; ++i) {
            u64 *x = r->poly(i, n) + l * n;
            for (size_t k = 0; k < n; ++k) x[k] = mod_mul(x[k], y[k], tab[l].mod);
        }
    }
    auto out = rescale(*r);
    out->scale = P.delta[a.level + 1];
    return out;
}

CtPtr Context::mul_plain_sum(const std::vector<const Ciphertext *> &a, const std::vector<const Plaintext *> &p) {
    if (a.empty() || a.size() != p.size()) throw std::invalid_argument("mul_plain_sum: bad operand lists");
    const int level = a[0]->level;
    for (size_t i = 0; i < a.size(); ++i)
        if (a[i]->level != level || p[i]->level != level)
            throw std::invalid_argument("mul_plain_sum: level mismatch");
    ctr.ptmult += a.size();
    auto r = make_ct(level, a[0]->slots, a[0]->scale, a[0]->limbs, P.n);
    const size_t n = P.n;
#pragma omp parallel for
    for (size_t l = 0; l < a[0]->limbs; ++l) {
        const Modulus &m = tab[l].mod;
        for (int c = 0; c < 2; ++c) {
            u64 *o = r->poly(c, n) + l * n;
            for (size_t k = 0; k < n; ++k) {
                u64 acc = 0;
                for (size_t i = 0; i < a.size(); ++i)
                    acc = mod_add(acc, mod_mul(a[i]->poly(c, n)[l * n + k], p[i]->m[l * n + k], m), m.q);
                o[k] = acc;
            }
        }
    }
    auto out = rescale(*r);
    out->scale = P.delta[level + 1];
    return out;
}

// --------------------------------------------------------- key switching ---
// ModUp (HYBRID): for each digit j of the level-ell basis, extend the digit's
// residues to every other prime of Q_ell u P by fast basis conversion.
void Context::modup(const u64 *d, size_t ell, std::vector<u64> &ext) const {
    const size_t n = P.n, nq = P.nq(), K = P.K, alpha = P.alpha;
    const size_t digits = (ell + alpha - 1) / alpha;
    const size_t W = ell + K;
    ext.assign(digits * W * n, 0);
    std::vector<u64> coef(ell * n);
    std::memcpy(coef.data(), d, ell * n * sizeof(u64));
#pragma omp parallel for
    for (size_t l = 0; l < ell; ++l) ntt_inverse(coef.data() + l * n, tab[l], n);
    auto prime_of = [&](size_t t) { return t < ell ? t : nq + (t - ell); };
    for (size_t j = 0; j < digits; ++j) {
        const size_t lo = j * alpha, hi = std::min(ell, (j + 1) * alpha);
        // QHatInv_i mod q_i, and QHat_i mod t
        std::vector<u64> qhinv(hi - lo);
        for (size_t i = lo; i < hi; ++i) {
            u64 prod = 1;
            for (size_t s = lo; s < hi; ++s)
                if (s != i) prod = mod_mul(prod, P.primes[s] % P.primes[i], tab[i].mod);
            qhinv[i - lo] = mod_inv(prod, tab[i].mod);
        }
#pragma omp parallel for
        for (size_t t = 0; t < W; ++t) {
            u64 *out = ext.data() + (j * W + t) * n;
            if (t >= lo && t < hi) {
                std::memcpy(out, d + t * n, n * sizeof(u64));
                continue;
            }
            const size_t pt = prime_of(t);
            const Modulus &mt = tab[pt].mod;
            std::vector<u64> qhat(hi - lo);
            for (size_t i = lo; i < hi; ++i) {
                u64 prod = 1;
                for (size_t s = lo; s < hi; ++s)
                    if (s != i) prod = mod_mul(prod, P.primes[s] % mt.q, mt);
                qhat[i - lo] = prod;
            }
            for (size_t k = 0; k < n; ++k) {
                u64 acc = 0;
                for (size_t i = lo; i < hi; ++i) {
                    u64 y = mod_mul(coef[i * n + k], qhinv[i - lo], tab[i].mod);
                    acc = mod_add(acc, mod_mul(y % mt.q, qhat[i - lo], mt), mt.q);
                }
                out[k] = acc;
            }
            ntt_forward(out, tab[pt], n);
        }
    }
}

// ModDown: (x - FastBaseConv_{P->Q}(x mod P)) * P^-1 mod q_i, NTT form in/out
void Context::moddown(const u64 *in, size_t ell, u64 *out) const {
    const size_t n = P.n, nq = P.nq(), K = P.K;
    std::vector<u64> pc(K * n);
    std::memcpy(pc.data(), in + ell * n, K * n * sizeof(u64));
    for (size_t k = 0; k < K; ++k) ntt_inverse(pc.data() + k * n, tab[nq + k], n);
    std::vector<u64> phinv(K);
    for (size_t k = 0; k < K; ++k) {
        u64 prod = 1;
        const Modulus &mk = tab[nq + k].mod;
        for (size_t s = 0; s < K; ++s)
            if (s != k) prod = mod_mul(prod, P.primes[nq + s] % mk.q, mk);
        phinv[k] = mod_inv(prod, mk);
    }
    for (size_t k = 0; k < K; ++k)
        for (size_t c = 0; c < n; ++c) pc[k * n + c] = mod_mul(pc[k * n + c], phinv[k], tab[nq + k].mod);
#pragma omp parallel for
    for (size_t i = 0; i < ell; ++i) {
        const Modulus &mi = tab[i].mod;
        std::vector<u64> phat(K);
        u64 Pm = 1;
        for (size_t k = 0; k < K; ++k) {
            u64 prod = 1;
            for (size_t s = 0; s < K; ++s)
                if (s != k) prod = mod_mul(prod, P.primes[nq + s] % mi.q, mi);
            phat[k] = prod;
            Pm = mod_mul(Pm, P.primes[nq + k] % mi.q, mi);
        }
        u64 Pinv = mod_inv(Pm, mi);
        // centred exact conversion: x mod P = sum_k y_k Phat_k - v P, v =
        // round(sum_k y_k / p_k) in fp64 (k ascending), so the result is
        // round(x / P); a plain fast conversion floors with a 0..K overshoot,
        // a biased error that s turns into a few large slot errors
        const u64 Pq = Pm;
        std::vector<u64> conv(n);
        for (size_t c = 0; c < n; ++c) {
            u64 acc = 0;
            double t = 0.0;
            for (size_t k = 0; k < K; ++k) {
                acc = mod_add(acc, mod_mul(pc[k * n + c] % mi.q, phat[k], mi), mi.q);
                t = t + (double)pc[k * n + c] * (1.0 / (double)P.primes[nq + k]);
            }
            const u64 v = moddown_floor ? 0 : (u64)(t + 0.5);
            conv[c] = mod_sub(acc, mod_mul(v, Pq, mi), mi.q);
        }
        ntt_forward(conv.data(), tab[i], n);
        const u64 *x = in + i * n;
        u64 *o = out + i * n;
        for (size_t c = 0; c < n; ++c) o[c] = mod_mul(mod_sub(x[c], conv[c], mi.q), Pinv, mi);
    }
}

// inner product with the key (optionally reading ext through an automorphism
// permutation), then ModDown of both accumulators: out01 = [2][ell][n]
void Context::keyswitch_core(const std::vector<u64> &ext, size_t ell, const SwitchKey &key,
                             const std::vector<uint32_t> *perm, std::vector<u64> &out01) const {
    const size_t n = P.n, W = ell + P.K;
    std::vector<u64> acc(2 * W * n, 0);
    keyswitch_acc(ext, ell, key, perm, acc);
    out01.assign(2 * ell * n, 0);
    moddown(acc.data(), ell, out01.data());
    moddown(acc.data() + W * n, ell, out01.data() + ell * n);
}

void Context::keyswitch_acc(const std::vector<u64> &ext, size_t ell, const SwitchKey &key,
                            const std::vector<uint32_t> *perm, std::vector<u64> &acc) const {
    const size_t n = P.n, nq = P.nq(), na = P.nall(), K = P.K, alpha = P.alpha;
    const size_t digits = (ell + alpha - 1) / alpha, W = ell + K;
    if (acc.size() != 2 * W * n) throw std::invalid_argument("keyswitch_acc: accumulator size");
#pragma omp parallel for
    for (size_t t = 0; t < W; ++t) {
        const size_t pt = t < ell ? t : nq + (t - ell);
        const Modulus &m = tab[pt].mod;
        u64 *a0 = acc.data() + t * n, *a1 = acc.data() + (W + t) * n;
        for (size_t j = 0; j < digits; ++j) {
            const u64 *e = ext.data() + (j * W + t) * n;
            const u64 *kb = key.data.data() + ((j * 2 + 0) * na + pt) * n;
            const u64 *ka = key.data.data() + ((j * 2 + 1) * na + pt) * n;
            for (size_t c = 0; c < n; ++c) {
                u64 x = perm ? e[(*perm)[c]] : e[c];
                a0[c] = mod_add(a0[c], mod_mul(x, kb[c], m), m.q);
                a1[c] = mod_add(a1[c], mod_mul(x, ka[c], m), m.q);
            }
        }
    }
}

void Context::rescale_poly(const u64 *in, size_t ell, u64 *out) const {
    const size_t n = P.n;
    const size_t last = ell - 1;
    const u64 ql = P.primes[last];
    std::vector<u64> c(in + last * n, in + ell * n);
    ntt_inverse(c.data(), tab[last], n);
#pragma omp parallel for
    for (size_t i = 0; i < last; ++i) {
        const u64 qi = P.primes[i];
        const Modulus &mi = tab[i].mod;
        const u64 qlmod = ql % qi;
        const u64 qlinv = mod_inv(qlmod, mi);
        std::vector<u64> t(n);
        for (size_t k = 0; k < n; ++k) {
            u64 v = c[k] % qi;
            if (c[k] > ql / 2) v = mod_sub(v, qlmod, qi);  // centred lift of the last residue
            t[k] = v;
        }
        ntt_forward(t.data(), tab[i], n);
        const u64 *x = in + i * n;
        u64 *o = out + i * n;
        for (size_t k = 0; k < n; ++k) o[k] = mod_mul(mod_sub(x[k], t[k], qi), qlinv, mi);
    }
}

CtPtr Context::rescale(const Ciphertext &a) {
    if (a.level >= P.L) throw std::runtime_error("rescale: no levels left");
    ctr.rescale++;
    const size_t n = P.n, ell = a.limbs;
    auto r = make_ct(a.level + 1, a.slots, a.scale / (double)P.primes[ell - 1], ell - 1, n);
    for (int i = 0; i < 2; ++i) rescale_poly(a.poly(i, n), ell, r->poly(i, n));
    return r;
}

CtPtr Context::mul(const Ciphertext &a0, const Ciphertext &b0) { return mul_add(a0, b0, {}, {}); }

// a*b + sum_i c_i x_i with ONE rescale: the linear sum is formed at the
// product's pre-rescale scale Delta_{l}^2 = Delta_{l+1} q_removed (the same
// integer constants linear_sum_to(xs, c, l+1) uses) and added to the tensor
// before relinearisation; rescale(a*b + sum) then lands at Delta_{l+1}.
// OpenFHE's Paterson-Stockmeyer also rescales such sums lazily.
CtPtr Context::mul_add(const Ciphertext &a0, const Ciphertext &b0, const std::vector<const Ciphertext *> &xs,
                       const std::vector<double> &cs) {
    CtPtr a = clone(a0), b = std::make_shared<Ciphertext>(b0);
    match_levels(a, b);
    ctr.hmult++;
    ctr.keyswitch++;
    const size_t n = P.n, ell = a->limbs;
    auto t = make_ct(a->level, a->slots, a->scale * b->scale, ell, n);
    std::vector<u64> d2(ell * n);
    const bool sq = (&a0 == &b0);
#pragma omp parallel for
    for (size_t l = 0; l < ell; ++l) {
        const Modulus &m = tab[l].mod;
        const u64 q = m.q;
        const u64 *x0 = a->poly(0, n) + l * n, *x1 = a->poly(1, n) + l * n;
        const u64 *y0 = b->poly(0, n) + l * n, *y1 = b->poly(1, n) + l * n;
        u64 *o0 = t->poly(0, n) + l * n, *o1 = t->poly(1, n) + l * n, *o2 = d2.data() + l * n;
        for (size_t k = 0; k < n; ++k) {
            o0[k] = mod_mul(x0[k], y0[k], m);
            if (sq) {
                u64 p = mod_mul(x0[k], y1[k], m);
                o1[k] = mod_add(p, p, q);
            } else {
                o1[k] = mod_add(mod_mul(x0[k], y1[k], m), mod_mul(x1[k], y0[k], m), q);
            }
            o2[k] = mod_mul(x1[k], y1[k], m);
        }
    }
    if (!xs.empty()) {
        const int target = a->level + 1;
        const double qd = (double)P.primes[P.L - target + 1];
        std::vector<std::vector<u64>> Kmod(xs.size(), std::vector<u64>(ell));
        for (size_t i = 0; i < xs.size(); ++i) {
            if (xs[i]->level > a->level) throw std::invalid_argument("mul_add: summand level too high");
            const ScaledConst K = scaled_const(cs[i] * P.delta[target] * qd / xs[i]->scale);
            for (size_t l = 0; l < ell; ++l) Kmod[i][l] = K.mod(P.primes[l]);
        }
        ctr.constmult += xs.size();
#pragma omp parallel for
        for (size_t l = 0; l < ell; ++l) {
            const Modulus &m = tab[l].mod;
            for (int p = 0; p < 2; ++p) {
                u64 *o = t->poly(p, n) + l * n;
                for (size_t i = 0; i < xs.size(); ++i) {
                    const u64 *x = xs[i]->poly(p, n) + l * n;
                    for (size_t k = 0; k < n; ++k) o[k] = mod_add(o[k], mod_mul(x[k], Kmod[i][l], m), m.q);
                }
            }
        }
    }
    std::vector<u64> ext, ks;
    modup(d2.data(), ell, ext);
    keyswitch_core(ext, ell, relin, nullptr, ks);
#pragma omp parallel for
    for (size_t l = 0; l < ell; ++l)
        for (int i = 0; i < 2; ++i) {
            u64 *x = t->poly(i, n) + l * n;
            const u64 *y = ks.data() + (i * ell + l) * n;
            for (size_t k = 0; k < n; ++k) x[k] = mod_add(x[k], y[k], P.primes[l]);
        }
    auto r = rescale(*t);
    r->scale = P.delta[a->level + 1];
    return r;
}

CtPtr Context::square(const Ciphertext &a) { return mul(a, a); }

std::vector<CtPtr> Context::rotate_hoisted(const Ciphertext &a, const std::vector<long> &ks) {
    std::vector<u64> gs;
    for (long k : ks) gs.push_back(galois_for_rotation(P.logN, k));
    return apply_galois_hoisted(a, gs);
}

CtPtr Context::conjugate(const Ciphertext &a) { return apply_galois_hoisted(a, {2 * (u64)P.n - 1})[0]; }

std::vector<CtPtr> Context::apply_galois_hoisted(const Ciphertext &a, const std::vector<u64> &gs) {
    const size_t n = P.n, ell = a.limbs;
    std::vector<CtPtr> outs;
    std::vector<u64> ext;
    bool have_ext = false;
    for (u64 g : gs) {
        if (g == 1) {
            outs.push_back(clone(a));
            continue;
        }
        auto it = rotkeys.find(g);
        if (it == rotkeys.end()) throw std::out_of_range("rotate: no rotation key for galois element " + std::to_string(g));
        if (!have_ext) {
            modup(a.poly(1, n), ell, ext);
            have_ext = true;
        }
        ctr.keyswitch++;
        ctr.rotations++;
        auto perm = automorphism_perm(P.logN, g);
        std::vector<u64> ksout;
        keyswitch_core(ext, ell, it->second, &perm, ksout);
        auto r = make_ct(a.level, a.slots, a.scale, ell, n);
        for (size_t l = 0; l < ell; ++l) {
            const u64 q = P.primes[l];
            const u64 *c0 = a.poly(0, n) + l * n;
            u64 *o0 = r->poly(0, n) + l * n, *o1 = r->poly(1, n) + l * n;
            const u64 *k0 = ksout.data() + l * n, *k1 = ksout.data() + (ell + l) * n;
            for (size_t c = 0; c < n; ++c) {
                o0[c] = mod_add(c0[perm[c]], k0[c], q);
                o1[c] = k1[c];
            }
        }
        outs.push_back(r);
    }
    return outs;
}

CtPtr Context::rotate(const Ciphertext &a, long k) { return rotate_hoisted(a, {k})[0]; }

CtPtr Context::rotate_sum_hoisted(const Ciphertext &x, const std::vector<long> &ks) {
    if (ks.empty()) return clone(x);
    const size_t n = P.n, ell = x.limbs, W = ell + P.K;
    std::vector<u64> ext, acc(2 * W * n, 0), c0(ell * n, 0);
    modup(x.poly(1, n), ell, ext);
    for (long k : ks) {
        const u64 g = galois_for_rotation(P.logN, k);
        auto it = rotkeys.find(g);
        if (g == 1 || it == rotkeys.end())
            throw std::out_of_range("rotate_sum_hoisted: no rotation key for index " + std::to_string(k));
        ctr.keyswitch++;
        ctr.rotations++;
        const auto perm = automorphism_perm(P.logN, g);
        keyswitch_acc(ext, ell, it->second, &perm, acc);
        for (size_t t = 0; t < ell; ++t)
            for (size_t c = 0; c < n; ++c)
                c0[t * n + c] = mod_add(c0[t * n + c], x.poly(0, n)[t * n + perm[c]], P.primes[t]);
    }
    auto r = make_ct(x.level, x.slots, x.scale, ell, n);
    moddown(acc.data(), ell, r->poly(0, n));
    moddown(acc.data() + W * n, ell, r->poly(1, n));
    for (size_t t = 0; t < ell; ++t)
        for (size_t c = 0; c < n; ++c) {
            u64 &o0 = r->poly(0, n)[t * n + c], &o1 = r->poly(1, n)[t * n + c];
            o0 = mod_add(mod_add(o0, c0[t * n + c], P.primes[t]), x.poly(0, n)[t * n + c], P.primes[t]);
            o1 = mod_add(o1, x.poly(1, n)[t * n + c], P.primes[t]);
        }
    return r;
}

CtPtr Context::linear_transform_ext(const Ciphertext &x, const std::vector<long> &baby,
                                    const std::vector<LtGiant> &giants) {
    const size_t n = P.n, nq = P.nq(), K = P.K, ell = x.limbs, W = ell + K;
    if (x.level >= P.L) throw std::runtime_error("linear_transform_ext: no levels left");
    auto prime = [&](size_t t) { return t < ell ? t : nq + (t - ell); };
    std::vector<u64> Pq(ell);  // P mod q_t
    for (size_t t = 0; t < ell; ++t) {
        u64 v = 1;
        for (size_t k = 0; k < K; ++k) v = mod_mul(v, P.primes[nq + k] % P.primes[t], tab[t].mod);
        Pq[t] = v;
    }
    // babies over Q u P: (P sigma(c0), 0) + <sigma(ext), key>, or (P c0, P c1) unrotated
    std::vector<u64> ext;
    modup(x.poly(1, n), ell, ext);
    std::vector<std::vector<u64>> B(baby.size());
    for (size_t b = 0; b < baby.size(); ++b) {
        auto &acc = B[b];
        acc.assign(2 * W * n, 0);
        const u64 g = galois_for_rotation(P.logN, baby[b]);
        std::vector<uint32_t> perm;
        if (g == 1) {
            for (size_t t = 0; t < ell; ++t)
                for (int c = 0; c < 2; ++c)
                    for (size_t k = 0; k < n; ++k)
                        acc[(c * W + t) * n + k] = mod_mul(x.poly(c, n)[t * n + k], Pq[t], tab[t].mod);
            continue;
        }
        auto it = rotkeys.find(g);
        if (it == rotkeys.end()) throw std::out_of_range("linear_transform_ext: no rotation key for " + std::to_string(baby[b]));
        ctr.keyswitch++;
        ctr.rotations++;
        perm = automorphism_perm(P.logN, g);
        keyswitch_acc(ext, ell, it->second, &perm, acc);
        for (size_t t = 0; t < ell; ++t)
            for (size_t k = 0; k < n; ++k)
                acc[t * n + k] = mod_add(acc[t * n + k], mod_mul(x.poly(0, n)[t * n + perm[k]], Pq[t], tab[t].mod),
                                         P.primes[t]);
    }
    // inner sums over Q u P
    auto inner = [&](const LtGiant &G) {
        std::vector<u64> r(2 * W * n, 0);
        for (size_t j = 0; j < G.baby.size(); ++j) {
            const auto &b = B[(size_t)G.baby[j]];
            const Plaintext &pt = *G.pts[j];
            if (pt.limbs != W) throw std::invalid_argument("linear_transform_ext: plaintexts must be extended");
            ctr.ptmult++;
#pragma omp parallel for
            for (size_t t = 0; t < W; ++t) {
                const Modulus &m = tab[prime(t)].mod;
                for (int c = 0; c < 2; ++c)
                    for (size_t k = 0; k < n; ++k) {
                        u64 &o = r[(c * W + t) * n + k];
                        o = mod_add(o, mod_mul(b[(c * W + t) * n + k], pt.m[t * n + k], m), m.q);
                    }
            }
        }
        return r;
    };
    std::vector<u64> acc(2 * W * n, 0), c0(ell * n, 0);
    for (const LtGiant &G : giants)
        if (G.shift == 0) acc = inner(G);
    for (const LtGiant &G : giants) {
        if (G.shift == 0) continue;
        const auto in = inner(G);
        auto q = make_ct(x.level, x.slots, x.scale, ell, n);  // ModDown of the giant's inner sum
        moddown(in.data(), ell, q->poly(0, n));
        moddown(in.data() + W * n, ell, q->poly(1, n));
        const u64 g = galois_for_rotation(P.logN, G.shift);
        auto it = rotkeys.find(g);
        if (g == 1 || it == rotkeys.end())
            throw std::out_of_range("linear_transform_ext: no rotation key for " + std::to_string(G.shift));
        ctr.keyswitch++;
        ctr.rotations++;
        const auto perm = automorphism_perm(P.logN, g);
        std::vector<u64> e2;
        modup(q->poly(1, n), ell, e2);
        keyswitch_acc(e2, ell, it->second, &perm, acc);
        for (size_t t = 0; t < ell; ++t)
            for (size_t k = 0; k < n; ++k)
                c0[t * n + k] = mod_add(c0[t * n + k], q->poly(0, n)[t * n + perm[k]], P.primes[t]);
    }
    auto r = make_ct(x.level, x.slots, x.scale, ell, n);
    moddown(acc.data(), ell, r->poly(0, n));
    moddown(acc.data() + W * n, ell, r->poly(1, n));
    for (size_t t = 0; t < ell; ++t)
        for (size_t k = 0; k < n; ++k)
            r->poly(0, n)[t * n + k] = mod_add(r->poly(0, n)[t * n + k], c0[t * n + k], P.primes[t]);
    auto out = rescale(*r);
    out->scale = P.delta[x.level + 1];
    return out;
}

CtPtr Context::mod_raise(const Ciphertext &a) {
    if (a.limbs != 1) throw std::invalid_argument("mod_raise: input must be at the last level (one limb)");
    const size_t n = P.n, nq = P.nq();
    const u64 q0 = P.primes[0];
    auto r = make_ct(0, a.slots, P.delta[0], nq, n);
    for (int i = 0; i < 2; ++i) {
        std::vector<u64> c(a.poly(i, n), a.poly(i, n) + n);
        ntt_inverse(c.data(), tab[0], n);
        std::vector<i64> t(n);
        for (size_t k = 0; k < n; ++k) t[k] = c[k] > q0 / 2 ? (i64)c[k] - (i64)q0 : (i64)c[k];
#pragma omp parallel for
        for (size_t l = 0; l < nq; ++l) {
            u64 *o = r->poly(i, n) + l * n;
            for (size_t k = 0; k < n; ++k) o[k] = signed_to_mod(t[k], P.primes[l]);
            ntt_forward(o, tab[l], n);
        }
    }
    return r;
}

CtPtr Context::linear_sum_to(const std::vector<const Ciphertext *> &xs, const std::vector<double> &c,
                             int target) {
    const size_t n = P.n;
    const size_t ell = P.limbs_at(target - 1);
    auto acc = make_ct(target - 1, xs.empty() ? 0 : xs[0]->slots, 0, ell, n);
    const double qd = (double)P.primes[P.L - target + 1];
    std::vector<std::vector<u64>> Kmod(xs.size(), std::vector<u64>(ell));
    for (size_t i = 0; i < xs.size(); ++i) {
        if (xs[i]->level > target - 1) throw std::invalid_argument("linear_sum_to: input level too high");
        const ScaledConst K = scaled_const(c[i] * P.delta[target] * qd / xs[i]->scale);
        for (size_t l = 0; l < ell; ++l) Kmod[i][l] = K.mod(P.primes[l]);
    }
    ctr.constmult += xs.size();
#pragma omp parallel for
    for (size_t l = 0; l < ell; ++l) {
        const Modulus &m = tab[l].mod;
        for (int p = 0; p < 2; ++p) {
            u64 *o = acc->poly(p, n) + l * n;
            for (size_t i = 0; i < xs.size(); ++i) {
                const u64 *x = xs[i]->poly(p, n) + l * n;
                const u64 kv = Kmod[i][l];
                for (size_t k = 0; k < n; ++k) o[k] = mod_add(o[k], mod_mul(x[k], kv, m), m.q);
            }
        }
    }
    auto r = rescale(*acc);
    r->scale = P.delta[target];
    return r;
}

CtPtr Context::trivial_const(double c, int level, int slots) const {
    const size_t n = P.n, ell = P.limbs_at(level);
    auto r = make_ct(level, slots, P.delta[level], ell, n);
    const ScaledConst K = scaled_const(c * P.delta[level]);
    for (size_t l = 0; l < ell; ++l) {
        u64 kv = K.mod(P.primes[l]);
        u64 *x = r->poly(0, n) + l * n;
        for (size_t k = 0; k < n; ++k) x[k] = kv;
    }
    return r;
}
CtPtr Context::zero_like(int level, int slots) const {
    return make_ct(level, slots, P.delta[level], P.limbs_at(level), P.n);
}

}  // namespace oracle
