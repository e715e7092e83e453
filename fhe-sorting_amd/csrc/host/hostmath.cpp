// Host-side precomputation for the MI355X RNS-CKKS engine (see hostmath.hpp).
#include "hostmath.hpp"

#include <sys/random.h>

#include <cerrno>
#include <cstring>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <complex>
#include <mutex>
#include <set>
#include <stdexcept>

namespace fhe {
namespace host {

// ------------------------------------------------------------ arithmetic --
Modulus::Modulus(u64 q_) : q(q_) {
    k = 64 - __builtin_clzll(q);
    mu = (u64)(((u128)1 << (2 * k)) / q);
}
u64 mulmod(u64 a, u64 b, const Modulus &m) {
    const u128 z = (u128)a * b;
    const u64 t = (u64)(z >> (m.k - 1));
    const u64 qh = (u64)(((u128)t * m.mu) >> (m.k + 1));
    u64 r = (u64)z - qh * m.q;
    while (r >= m.q) r -= m.q;
    return r;
}
u64 powmod(u64 a, u64 e, const Modulus &m) {
    u64 r = 1 % m.q;
    a %= m.q;
    for (; e; e >>= 1) {
        if (e & 1) r = mulmod(r, a, m);
        a = mulmod(a, a, m);
    }
    return r;
}
u64 invmod(u64 a, const Modulus &m) { return powmod(a, m.q - 2, m); }
u64 shoup(u64 w, u64 q) { return (u64)(((u128)w << 64) / q); }
u64 to_mod(i64 v, u64 q) {
    if (v >= 0) return (u64)v % q;
    const u64 r = (u64)(-(v + 1)) % q;
    const u64 s = (r + 1) % q;
    return s ? q - s : 0;
}
bool is_prime(u64 n) {
    if (n < 2) return false;
    static const u64 bases[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    for (u64 p : bases)
        if (n % p == 0) return n == p;
    u64 d = n - 1;
    int s = 0;
    for (; !(d & 1); d >>= 1) ++s;
    auto pw = [n](u64 b, u64 e) {
        u128 r = 1, x = b % n;
        for (; e; e >>= 1) {
            if (e & 1) r = r * x % n;
            x = x * x % n;
        }
        return (u64)r;
    };
    for (u64 a : bases) {
        u64 x = pw(a, d);
        if (x == 1 || x == n - 1) continue;
        bool witness = true;
        for (int r = 1; r < s && witness; ++r) {
            x = (u64)((u128)x * x % n);
            if (x == n - 1) witness = false;
        }
        if (witness) return false;
    }
    return true;
}

// ---------------------------------------------------------------- params --
Params make_params(int logN, int L, int scale_bits, int first_bits, int dnum) {
    if (logN < 4 || logN > 17) throw std::invalid_argument("logN out of range [4,17]");
    // every prime < 2^60 keeps the 30-bit split sums of the basis conversions
    // and linear sums exact (16 products of 30-bit halves per 64-bit partial);
    // scaling primes are the primes nearest 2^scale_bits, so scale_bits <= 59
    if (scale_bits < 20 || scale_bits > 59 || first_bits > 60 || first_bits <= scale_bits)
        throw std::invalid_argument("unsupported modulus sizes");
    Params P;
    P.logN = logN;
    P.n = (size_t)1 << logN;
    P.L = L;
    P.dnum = dnum;
    P.scale_bits = scale_bits;
    P.first_bits = first_bits;
    const u64 m2 = 2 * (u64)P.n;
    std::set<u64> used;
    std::vector<u64> q(L + 1);
    // q_0: largest NTT prime below 2^first_bits
    u64 c = ((((u64)1 << first_bits) - 1) / m2) * m2 + 1;
    if (c >= ((u64)1 << first_bits)) c -= m2;
    while (!is_prime(c)) c -= m2;
    q[0] = c;
    used.insert(c);
    // q_L .. q_1: greedy closest primes keep Delta_l == 2^scale_bits (no drift)
    auto nearest = [&](double target) {
        const u64 t = (u64)target;
        u64 lo = (t / m2) * m2 + 1;
        if (lo > t) lo -= m2;
        u64 hi = lo + m2;
        for (;;) {
            const bool below = (double)(t - lo) <= (double)(hi - t);
            const u64 cand = below ? lo : hi;
            if (is_prime(cand) && !used.count(cand)) return cand;
            if (below)
                lo -= m2;
            else
                hi += m2;
        }
    };
    if (L >= 1) {
        double d = std::ldexp(1.0, scale_bits);
        q[L] = nearest(d);
        used.insert(q[L]);
        d = (double)q[L];
        for (int l = 0; l + 1 < L; ++l) {
            d = d * d / (double)q[L - l];
            q[L - l - 1] = nearest(d);
            used.insert(q[L - l - 1]);
        }
    }
    P.alpha = (L + 1 + dnum - 1) / dnum;
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
    u64 p = q[0];
    for (int k = 0; k < P.K; ++k) {
        do {
            p -= m2;
        } while (!is_prime(p) || used.count(p));
        q.push_back(p);
        used.insert(p);
    }
    P.primes = q;
    P.delta.resize(L + 1);
    P.delta[0] = (double)q[L];
    for (int l = 0; l < L; ++l) P.delta[l + 1] = P.delta[l] * P.delta[l] / (double)q[L - l];
    return P;
}

// ------------------------------------------------------------------- NTT --
static uint32_t brev(uint32_t x, int bits) {
    uint32_t r = 0;
    for (int i = 0; i < bits; ++i, x >>= 1) r = (r << 1) | (x & 1);
    return r;
}
NttTable make_ntt_table(u64 q, int logN) {
    const Modulus m(q);
    const size_t n = (size_t)1 << logN;
    NttTable t;
    u64 g = 2;
    while (powmod(g, (q - 1) / 2, m) != q - 1) ++g;  // smallest non-residue
    t.psi = powmod(g, (q - 1) / (2 * n), m);
    const u64 psii = invmod(t.psi, m);
    std::vector<u64> pw(n), pwi(n);
    pw[0] = pwi[0] = 1;
    for (size_t i = 1; i < n; ++i) {
        pw[i] = mulmod(pw[i - 1], t.psi, m);
        pwi[i] = mulmod(pwi[i - 1], psii, m);
    }
    t.fwd.resize(n);
    t.fwd_s.resize(n);
    t.inv.resize(n);
    t.inv_s.resize(n);
    for (size_t k = 0; k < n; ++k) {
        const uint32_t r = brev((uint32_t)k, logN);
        t.fwd[k] = pw[r];
        t.inv[k] = pwi[r];
        t.fwd_s[k] = shoup(t.fwd[k], q);
        t.inv_s[k] = shoup(t.inv[k], q);
    }
    t.ninv = invmod(n % q, m);
    t.ninv_s = shoup(t.ninv, q);
    return t;
}
std::vector<uint32_t> automorphism_perm(int logN, u64 g) {
    const size_t n = (size_t)1 << logN;
    const u64 m2 = 2 * (u64)n;
    std::vector<uint32_t> perm(n);
    for (size_t k = 0; k < n; ++k) {
        const u64 i = brev((uint32_t)k, logN);
        const u64 e = ((2 * i + 1) * g) % m2;
        perm[k] = brev((uint32_t)((e - 1) / 2), logN);
    }
    return perm;
}
u64 galois_for_rotation(int logN, long k) {
    const long half = 1L << (logN - 1);
    const long r = ((k % half) + half) % half;
    const u64 m2 = (u64)1 << (logN + 1);
    u64 g = 1;
    for (long i = 0; i < r; ++i) g = g * 5 % m2;
    return g;
}

// --------------------------------------------------------------- encoder --
namespace {
using cd = std::complex<double>;
struct Emb {
    std::vector<cd> ksi;
    std::vector<u64> rot;
};
const Emb &emb_tables(size_t n) {
    static std::mutex mu;
    static std::map<size_t, Emb> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(n);
    if (it != cache.end()) return it->second;
    Emb e;
    const size_t M = 2 * n;
    e.ksi.resize(M + 1);
    for (size_t k = 0; k <= M; ++k) {
        const double ang = 2.0 * M_PI * (double)k / (double)M;
        e.ksi[k] = cd(std::cos(ang), std::sin(ang));
    }
    e.rot.resize(n / 2);
    u64 g = 1;
    for (size_t j = 0; j < n / 2; ++j, g = g * 5 % M) e.rot[j] = g;
    return cache[n] = std::move(e);
}
void bit_reverse(std::vector<cd> &v) {
    const size_t n = v.size();
    for (size_t i = 1, j = 0; i < n; ++i) {
        size_t bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) std::swap(v[i], v[j]);
    }
}
// inverse special FFT: slot values -> (real, imag) coefficient halves
// (lq is a power of two: rot % lq is rot & (lq - 1); the twiddle of butterfly j
// of a stage is the same for every block i, so it is looked up once per stage.
// The floating-point operations and their order are unchanged, so the encoder
// stays bit-identical to the oracle's.)
void special_ifft(std::vector<cd> &v, const Emb &E, size_t n) {
    const size_t S = v.size(), M = 2 * n;
    std::vector<cd> tw(S / 2 + 1);
    for (size_t len = S; len >= 1; len >>= 1) {
        const size_t h = len >> 1, lq = len << 2, gap = M / lq;
        for (size_t j = 0; j < h; ++j) tw[j] = E.ksi[(lq - (E.rot[j] & (lq - 1))) * gap];
        for (size_t i = 0; i < S; i += len) {
            for (size_t j = 0; j < h; ++j) {
                cd u = v[i + j] + v[i + j + h];
                cd w = v[i + j] - v[i + j + h];
                w *= tw[j];
                v[i + j] = u;
                v[i + j + h] = w;
            }
        }
    }
    bit_reverse(v);
    for (auto &x : v) x /= (double)S;
}
void special_fft(std::vector<cd> &v, const Emb &E, size_t n) {
    const size_t S = v.size(), M = 2 * n;
    bit_reverse(v);
    std::vector<cd> tw(S / 2 + 1);
    for (size_t len = 2; len <= S; len <<= 1) {
        const size_t h = len >> 1, lq = len << 2, gap = M / lq;
        for (size_t j = 0; j < h; ++j) tw[j] = E.ksi[(E.rot[j] & (lq - 1)) * gap];
        for (size_t i = 0; i < S; i += len) {
            for (size_t j = 0; j < h; ++j) {
                cd u = v[i + j];
                cd w = v[i + j + h];
                w *= tw[j];
                v[i + j] = u + w;
                v[i + j + h] = u - w;
            }
        }
    }
}
}  // namespace

void embedding_tables(size_t n, std::vector<double> &ksi, std::vector<uint32_t> &rot) {
    const Emb &E = emb_tables(n);
    ksi.resize(2 * E.ksi.size());
    for (size_t k = 0; k < E.ksi.size(); ++k) {
        ksi[2 * k] = E.ksi[k].real();
        ksi[2 * k + 1] = E.ksi[k].imag();
    }
    rot.assign(E.rot.begin(), E.rot.end());
}

std::vector<i64> encode_coeffs(const std::vector<double> &v, size_t n, int slots, double scale) {
    std::vector<cd> z;
    for (size_t i = 0; i < v.size() && i < (size_t)std::max(slots, 0); ++i) z.push_back(cd(v[i], 0));
    return encode_coeffs_complex(z, n, slots, scale);
}

std::vector<i64> encode_coeffs_complex(const std::vector<std::complex<double>> &v, size_t n, int slots,
                                       double scale) {
    if (slots <= 0 || (slots & (slots - 1)) || (size_t)slots > n / 2)
        throw std::invalid_argument("encode: slots must be a power of two <= n/2");
    const Emb &E = emb_tables(n);
    std::vector<cd> z(slots, cd(0, 0));
    for (size_t i = 0; i < v.size() && i < (size_t)slots; ++i) z[i] = v[i];
    special_ifft(z, E, n);
    const size_t gap = n / (2 * (size_t)slots);
    std::vector<i64> coef(n, 0);
    auto rnd = [](double x) -> i64 {
        if (!(std::fabs(x) < 9.2e18)) throw std::overflow_error("encode: scaled coefficient exceeds 63 bits");
        return std::llround(x);
    };
    for (size_t i = 0; i < (size_t)slots; ++i) {
        coef[i * gap] = rnd(z[i].real() * scale);
        coef[i * gap + n / 2] = rnd(z[i].imag() * scale);
    }
    return coef;
}

std::vector<double> decode_coeffs(const u64 *m0, const u64 *m1, size_t n, u64 q0, u64 q1, int slots,
                                  double scale) {
    const Emb &E = emb_tables(n);
    const size_t gap = n / (2 * (size_t)slots);
    // centred lift mod q0 (one limb) or mod q0*q1 (two limbs, CRT)
    const Modulus M1(q1 ? q1 : 3);
    const u64 q0inv = q1 ? invmod(q0 % q1, M1) : 0;
    const u128 Q = (u128)q0 * (q1 ? q1 : 1);
    auto centred = [&](size_t k) -> double {
        if (!q1) {
            const u64 x = m0[k];
            return x > q0 / 2 ? -(double)(q0 - x) : (double)x;
        }
        const u64 a0 = m0[k], a1 = m1[k];
        const u64 t = mulmod((a1 + q1 - a0 % q1) % q1, q0inv, M1);
        const u128 x = (u128)a0 + (u128)q0 * t;
        return x > Q / 2 ? -(double)(Q - x) : (double)x;
    };
    std::vector<cd> z(slots);
    for (size_t i = 0; i < (size_t)slots; ++i)
        z[i] = cd(centred(i * gap) / scale, centred(i * gap + n / 2) / scale);
    special_fft(z, E, n);
    std::vector<double> out(slots);
    for (size_t i = 0; i < (size_t)slots; ++i) out[i] = z[i].real();
    return out;
}

SConst scaled_const(double x) {
    if (!std::isfinite(x)) throw std::invalid_argument("scaled constant is not finite");
    const double ax = std::fabs(x);
    if (ax <= 0x1p62) return SConst{std::llround(x), 0};
    const int sh = (int)std::ceil(std::log2(ax)) - 62;
    return SConst{std::llround(std::ldexp(x, -sh)), sh};
}
SConst const_to_target(double c, double delta_target, u64 q_dropped, double scale_in) {
    return scaled_const(c * delta_target * (double)q_dropped / scale_in);
}
SConst const_at_scale(double c, double scale) { return scaled_const(c * scale); }

// -------------------------------------------------------------- sampling --
SplitMix64::SplitMix64(u64 seed, u64 tag) : s(seed ^ (tag * 0xD1B54A32D192ED03ULL)) { next(); }
u64 SplitMix64::next() {
    s += 0x9E3779B97F4A7C15ULL;
    u64 z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
namespace {
inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
inline void quarter(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d) {
    a += b, d ^= a, d = rotl32(d, 16);
    c += d, b ^= c, b = rotl32(b, 12);
    a += b, d ^= a, d = rotl32(d, 8);
    c += d, b ^= c, b = rotl32(b, 7);
}
}  // namespace

void chacha20_block(const uint32_t key[8], uint32_t counter, const uint32_t nonce[3], uint32_t out[16]) {
    uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
    for (int i = 0; i < 8; ++i) s[4 + i] = key[i];
    s[12] = counter;
    s[13] = nonce[0], s[14] = nonce[1], s[15] = nonce[2];
    uint32_t x[16];
    std::memcpy(x, s, sizeof x);
    for (int r = 0; r < 10; ++r) {
        quarter(x[0], x[4], x[8], x[12]);
        quarter(x[1], x[5], x[9], x[13]);
        quarter(x[2], x[6], x[10], x[14]);
        quarter(x[3], x[7], x[11], x[15]);
        quarter(x[0], x[5], x[10], x[15]);
        quarter(x[1], x[6], x[11], x[12]);
        quarter(x[2], x[7], x[8], x[13]);
        quarter(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; ++i) out[i] = x[i] + s[i];
}
ChaCha20::ChaCha20(const uint32_t k[8], u64 tag) {
    std::memcpy(key, k, sizeof key);
    nonce[0] = (uint32_t)tag, nonce[1] = (uint32_t)(tag >> 32), nonce[2] = 0x53454846u;  // "FHES"
}
u64 ChaCha20::next() {
    if (pos >= 16) {
        if (counter == 0xffffffffu) throw std::runtime_error("ChaCha20: stream exhausted");
        chacha20_block(key, counter++, nonce, buf);
        pos = 0;
    }
    const u64 r = (u64)buf[pos] | ((u64)buf[pos + 1] << 32);
    pos += 2;
    return r;
}
Entropy Entropy::from_seed(u64 seed) {
    Entropy e;
    if (seed) {
        e.seed = seed;
        return e;
    }
    e.secure = true;
    uint32_t w[10];
    size_t got = 0;
    while (got < sizeof w) {
        const ssize_t r = getrandom(reinterpret_cast<char *>(w) + got, sizeof w - got, 0);
        if (r < 0) {
            if (errno == EINTR) continue;
            throw std::runtime_error("getrandom failed: cannot seed the key / encryption sampler");
        }
        got += (size_t)r;
    }
    std::memcpy(e.key, w, sizeof e.key);
    e.seed_a = (u64)w[8] | ((u64)w[9] << 32);
    std::memset(w, 0, sizeof w);
    return e;
}
Prng::Prng(const Entropy &e, u64 tag, bool pub)
    : use_cc(e.secure && !pub), sm(e.secure ? e.seed_a : e.seed, tag), cc(e.key, tag) {}

// ---------------------------------------------- fp64 sums of products --
// One target row of an fp64 basis conversion (kernels.hip k_moddown_rescale_fp).
// The kernel feeds source k as two exact doubles with y_k = yh 2^30 + yl + off_k,
// |yh| <= yh_max, |yl| <= yl_max, and accumulates
//   H = sum_k yh h(c'_k) + yl h(c_k),  L = cst + sum_k yh l(c'_k) + yl l(c_k),
// so sum_k y_k c_k = 2^20 H + L (mod q) with c' = 2^30 c mod q: every product
// and partial sum is an integer the FMA represents exactly while the bounds
// below stay under 2^53.  Returns the split class: 0 = whole sums fit, 1 = fit
// with one exact reduction (mod q) after source (S + 1) / 2 - 1, -1 = neither.
struct FpSrc {
    u64 yh_max, yl_max, off;
};
static int fp_conv_row(const std::vector<u64> &c, u64 q, const std::vector<FpSrc> &src, double *row, double *tq) {
    const Modulus m(q);
    const size_t S = c.size();
    auto cen = [q](u64 x) { return x > q / 2 ? (i64)x - (i64)q : (i64)x; };
    auto split = [](i64 v, i64 &h, i64 &l) {
        h = (v + (1 << 19)) >> 20;  // round to nearest: l in [-2^19, 2^19)
        l = v - h * ((i64)1 << 20);
    };
    const u64 two30 = ((u64)1 << 30) % q;
    u64 cst = 0, bh[2] = {0, 0}, bl[2] = {0, 0};
    const size_t half = (S + 1) / 2;
    for (size_t k = 0; k < S; ++k) {
        i64 hp, lp, h, l;
        split(cen(mulmod(c[k] % q, two30, m)), hp, lp);
        split(cen(c[k] % q), h, l);
        row[4 * k + 0] = (double)hp;
        row[4 * k + 1] = (double)h;
        row[4 * k + 2] = (double)lp;
        row[4 * k + 3] = (double)l;
        const int p = k < half ? 0 : 1;
        bh[p] += src[k].yh_max * (u64)std::llabs(hp) + src[k].yl_max * (u64)std::llabs(h);
        bl[p] += src[k].yh_max * (u64)std::llabs(lp) + src[k].yl_max * (u64)std::llabs(l);
        cst = (cst + mulmod(src[k].off % q, c[k] % q, m)) % q;
    }
    tq[0] = (double)cst;
    tq[1] = (double)q;
    tq[2] = 1.0 / (double)q;
    tq[3] = 0.0;
    const u64 lim = (u64)1 << 53;
    // the final reduction adds L to a remainder below q; a halfway reduction
    // leaves |H|, |L| <= q
    if (bh[0] + bh[1] < lim && cst + bl[0] + bl[1] + 2 * q < lim) return 0;
    if (bh[0] < lim && cst + bl[0] < lim && q + bh[1] < lim && 3 * q + bl[1] < lim) return 1;
    return -1;
}

// ---------------------------------------------------------- level tables --
LevelTables make_level_tables(const Params &P) {
    LevelTables T;
    const size_t nq = P.nq(), K = (size_t)P.K, alpha = (size_t)P.alpha;
    std::vector<Modulus> mods;
    for (u64 q : P.primes) mods.emplace_back(q);
    // prime maps
    const size_t Wmax = nq + K;
    T.extmap.assign((nq + 1) * Wmax, 0);
    for (size_t ell = 1; ell <= nq; ++ell) {
        for (size_t t = 0; t < ell; ++t) T.extmap[ell * Wmax + t] = (int)t;
        for (size_t k = 0; k < K; ++k) T.extmap[ell * Wmax + ell + k] = (int)(nq + k);
    }
    // ModUp
    T.modup_map_off.assign(nq + 1, 0);
    T.modup_map_cnt.assign(nq + 1, 0);
    for (size_t ell = 1; ell <= nq; ++ell) {
        const size_t W = ell + K, digits = (ell + alpha - 1) / alpha;
        T.modup_map_off[ell] = T.modup_smap.size();
        for (size_t j = 0; j < digits; ++j) {
            const size_t lo = j * alpha, hi = std::min(ell, (j + 1) * alpha);
            for (size_t t = 0; t < W; ++t) {
                if (t >= lo && t < hi) continue;
                T.modup_smap.push_back((int)(j * W + t));
                T.modup_pmap.push_back(T.extmap[ell * Wmax + t]);
            }
        }
        T.modup_map_cnt[ell] = T.modup_smap.size() - T.modup_map_off[ell];
    }
    T.modup_off.assign(nq + 1, {});
    T.modup_fp_off.assign(nq + 1, {});
    int fp_cls = -2;  // worst fp64 class over the rows (-2: none yet)
    for (size_t ell = 1; ell <= nq; ++ell) {
        const size_t W = ell + K;
        const size_t digits = (ell + alpha - 1) / alpha;
        for (size_t j = 0; j < digits; ++j) {
            const size_t lo = j * alpha, hi = std::min(ell, (j + 1) * alpha);
            T.modup_off[ell].push_back(T.modup.size());
            // layout (device): qhinv[alpha], qhinv_s[alpha], qhat[W][alpha]; rows
            // zero-padded to alpha so every digit runs the same unrolled code
            std::vector<u64> qhinv(alpha, 0), qhinv_s(alpha, 0), qhat(W * alpha, 0);
            for (size_t i = lo; i < hi; ++i) {
                u64 prod = 1;
                for (size_t s = lo; s < hi; ++s)
                    if (s != i) prod = mulmod(prod, P.primes[s] % P.primes[i], mods[i]);
                // times n^-1: the inverse NTT feeding the conversion is unscaled
                qhinv[i - lo] = mulmod(invmod(prod, mods[i]), invmod(((u64)1 << P.logN) % P.primes[i], mods[i]),
                                       mods[i]);
                qhinv_s[i - lo] = shoup(qhinv[i - lo], P.primes[i]);
            }
            for (size_t t = 0; t < W; ++t) {
                if (t >= lo && t < hi) continue;
                const size_t pt = t < ell ? t : nq + (t - ell);
                const Modulus &mt = mods[pt];
                for (size_t i = lo; i < hi; ++i) {
                    u64 prod = 1;
                    for (size_t s = lo; s < hi; ++s)
                        if (s != i) prod = mulmod(prod, P.primes[s] % mt.q, mt);
                    qhat[t * alpha + (i - lo)] = prod;
                }
            }
            T.modup.insert(T.modup.end(), qhinv.begin(), qhinv.end());
            T.modup.insert(T.modup.end(), qhinv_s.begin(), qhinv_s.end());
            T.modup.insert(T.modup.end(), qhat.begin(), qhat.end());
            // fp64 rows: source i (< 2^60) enters as yh = (y >> 30) - oh, yl =
            // (y & (2^30 - 1)) - 2^29 with oh = 2^29 for a prime >= 2^41 (q_0), else 0
            // (y < 2^41: |yh| < 2^11); padding sources have zero constants
            std::vector<FpSrc> src(hi - lo);
            for (size_t i = lo; i < hi; ++i) {
                const bool big = P.primes[i] >= ((u64)1 << 41);
                src[i - lo] = FpSrc{big ? (u64)1 << 29 : (u64)1 << 11, (u64)1 << 29,
                                    (big ? (u64)1 << 59 : 0) + ((u64)1 << 29)};
            }
            const size_t fo = T.modup_fp.size();
            T.modup_fp_off[ell].push_back(fo);
            T.modup_fp.resize(fo + W * alpha * 4 + W * 4, 0.0);
            for (size_t t = 0; t < W; ++t) {
                if (t >= lo && t < hi) continue;
                const size_t pt = t < ell ? t : nq + (t - ell);
                if (P.primes[pt] >= ((u64)1 << 41)) {  // integer targets keep the 128-bit sums (flag 1)
                    T.modup_fp[fo + W * alpha * 4 + t * 4 + 3] = 1.0;
                    continue;
                }
                // the digit's hi - lo sources (a partial last digit launches with that
                // many, so the halfway split falls where the kernel's does)
                std::vector<u64> c(qhat.begin() + t * alpha, qhat.begin() + t * alpha + (hi - lo));
                const int r = fp_conv_row(c, P.primes[pt], src, &T.modup_fp[fo + t * alpha * 4],
                                          &T.modup_fp[fo + W * alpha * 4 + t * 4]);
                fp_cls = (r < 0 || fp_cls == -1) ? -1 : std::max(fp_cls, r);
            }
        }
    }
    T.modup_fp_mid = fp_cls == -2 ? -1 : fp_cls;
    // ModDown
    T.phinv.resize(K);
    T.phinv_s.resize(K);
    T.phat.assign(nq * K, 0);  // [nq][K]: the K constants of one target are contiguous
    T.pinv.resize(nq);
    T.pinv_s.resize(nq);
    T.pinvd.resize(K);
    for (size_t k = 0; k < K; ++k) T.pinvd[k] = 1.0 / (double)P.primes[nq + k];
    T.pmod.resize(nq);
    T.pmod_s.resize(nq);
    for (size_t k = 0; k < K; ++k) {
        const Modulus &mk = mods[nq + k];
        u64 prod = 1;
        for (size_t s = 0; s < K; ++s)
            if (s != k) prod = mulmod(prod, P.primes[nq + s] % mk.q, mk);
        T.phinv[k] = mulmod(invmod(prod, mk), invmod(((u64)1 << P.logN) % mk.q, mk), mk);  // times n^-1 (as qhinv)
        T.phinv_s[k] = shoup(T.phinv[k], mk.q);
    }
    for (size_t i = 0; i < nq; ++i) {
        const Modulus &mi = mods[i];
        u64 Pm = 1;
        for (size_t k = 0; k < K; ++k) {
            u64 prod = 1;
            for (size_t s = 0; s < K; ++s)
                if (s != k) prod = mulmod(prod, P.primes[nq + s] % mi.q, mi);
            T.phat[i * K + k] = prod;
            Pm = mulmod(Pm, P.primes[nq + k] % mi.q, mi);
        }
        T.pinv[i] = invmod(Pm, mi);
        T.pinv_s[i] = shoup(T.pinv[i], mi.q);
        T.pmod[i] = Pm;
        T.pmod_s[i] = shoup(Pm, mi.q);
    }
    // fp64 ModDown + rescale rows: the K scaled special residues y_k < 2^60 enter
    // as yh = (y >> 30) - 2^29, yl = (y & (2^30 - 1)) - 2^29 (off = 2^59 + 2^29);
    // the P term pv = centred(y_last) - count (|pv| < 2^40 + K) as pv >> 30 and
    // its low 30 bits
    {
        std::vector<FpSrc> src(K + 1, FpSrc{(u64)1 << 29, (u64)1 << 29, ((u64)1 << 59) + ((u64)1 << 29)});
        src[K] = FpSrc{(u64)1 << 11, (u64)1 << 30, 0};
        T.mdfp_c.assign(nq * (K + 1) * 4, 0.0);
        T.mdfp_q.assign(nq * 4, 0.0);
        int cls = -2;  // worst class over the fp targets (-2: none yet)
        for (size_t i = 0; i < nq; ++i) {
            if (P.primes[i] >= ((u64)1 << 41)) {  // integer targets keep the 128-bit sums (flag 1)
                T.mdfp_q[i * 4 + 3] = 1.0;
                continue;
            }
            std::vector<u64> c(K + 1);
            for (size_t k = 0; k < K; ++k) c[k] = T.phat[i * K + k];
            c[K] = T.pmod[i];
            const int r = fp_conv_row(c, P.primes[i], src, &T.mdfp_c[i * (K + 1) * 4], &T.mdfp_q[i * 4]);
            cls = (r < 0 || cls == -1) ? -1 : std::max(cls, r);
        }
        T.mdfp_mid = cls == -2 ? -1 : cls;
    }
    // Rescale
    T.qlinv.assign((nq + 1) * nq, 0);
    T.qlinv_s.assign((nq + 1) * nq, 0);
    for (size_t ell = 2; ell <= nq; ++ell) {
        const u64 ql = P.primes[ell - 1];
        for (size_t i = 0; i + 1 < ell; ++i) {
            const u64 v = invmod(ql % P.primes[i], mods[i]);
            T.qlinv[ell * nq + i] = v;
            T.qlinv_s[ell * nq + i] = shoup(v, P.primes[i]);
        }
    }
    T.pqlinv.assign((nq + 1) * nq, 0);
    T.pqlinv_s.assign((nq + 1) * nq, 0);
    for (size_t ell = 2; ell <= nq; ++ell)
        for (size_t i = 0; i + 1 < ell; ++i) {
            const u64 v = mulmod(T.qlinv[ell * nq + i], T.pinv[i], mods[i]);
            T.pqlinv[ell * nq + i] = v;
            T.pqlinv_s[ell * nq + i] = shoup(v, P.primes[i]);
        }
    return T;
}

}  // namespace host
}  // namespace fhe
