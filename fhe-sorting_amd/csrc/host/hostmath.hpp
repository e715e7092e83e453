// Host-side RNS-CKKS parameter generation, precomputation, canonical-embedding
// encoder and seeded sampling for the MI355X engine.  Compiled with g++
// -ffp-contract=off so the fp64 encoder rounds deterministically (the spec in
// DESIGN.md §3 fixes every floating-point step).
#pragma once
#include <complex>
#include <cstddef>
#include <cstdint>
#include <map>
#include <vector>

namespace fhe {
namespace host {

using u64 = uint64_t;
using i64 = int64_t;
using u128 = unsigned __int128;

struct Modulus {
    u64 q = 0, mu = 0;
    int k = 0;
    Modulus() = default;
    explicit Modulus(u64 q_);
};
u64 mulmod(u64 a, u64 b, const Modulus &m);
u64 powmod(u64 a, u64 e, const Modulus &m);
u64 invmod(u64 a, const Modulus &m);
u64 shoup(u64 w, u64 q);
u64 to_mod(i64 v, u64 q);
bool is_prime(u64 n);

struct Params {
    int logN = 0;
    size_t n = 0;
    int L = 0, dnum = 3, alpha = 0, K = 0;
    int scale_bits = 40, first_bits = 60;
    std::vector<u64> primes;    // Q (L+1) then P (K)
    std::vector<double> delta;  // canonical scale per level
    size_t nq() const { return (size_t)L + 1; }
    size_t nall() const { return primes.size(); }
    size_t limbs_at(int level) const { return (size_t)(L + 1 - level); }
    int digits_at(size_t ell) const { return (int)((ell + alpha - 1) / alpha); }
};
Params make_params(int logN, int L, int scale_bits, int first_bits, int dnum);

// NTT tables for one prime: psi^{brev(k)}, psi^{-brev(k)} and Shoup companions
struct NttTable {
    u64 psi = 0;
    std::vector<u64> fwd, fwd_s, inv, inv_s;
    u64 ninv = 0, ninv_s = 0;
};
NttTable make_ntt_table(u64 q, int logN);
std::vector<uint32_t> automorphism_perm(int logN, u64 g);
u64 galois_for_rotation(int logN, long k);

// the encoder's tables, for the device encoder (engine encode_masks): ksi
// [2n + 1] interleaved (cos, sin) of 2 pi k / 2n, rot [n / 2] = 5^j mod 2n
void embedding_tables(size_t n, std::vector<double> &ksi, std::vector<uint32_t> &rot);
// canonical embedding (special FFT, fp64) -> signed integer coefficients
std::vector<i64> encode_coeffs(const std::vector<double> &v, size_t n, int slots, double scale);
std::vector<i64> encode_coeffs_complex(const std::vector<std::complex<double>> &v, size_t n, int slots,
                                       double scale);
// m0 (and m1 when q1 != 0): message limbs in coefficient form; 2 limbs => CRT lift
std::vector<double> decode_coeffs(const u64 *m0, const u64 *m1, size_t n, u64 q0, u64 q1, int slots,
                                  double scale);

// constants of the scale bookkeeping.  A scaled constant
// x = c * scale is carried as k * 2^sh: k = llround(x) while |x| <= 2^62,
// beyond that k = llround(x / 2^sh) with sh = ceil(log2 |x|) - 62 (OpenFHE's
// large-constant approximation, MAX_BITS_IN_WORD = 62), so 59- and 60-bit
// scales take constants such as g3's 25614/1024.
struct SConst {
    i64 k = 0;
    int sh = 0;
};
SConst scaled_const(double x);
SConst const_to_target(double c, double delta_target, u64 q_dropped, double scale_in);
SConst const_at_scale(double c, double scale);

// Sampling ("Sampling").  Two modes:
//  * deterministic (a nonzero context seed; tests and the CPU oracle, which
//    restates exactly these streams): SplitMix64 streams keyed by (seed, tag);
//  * secure (seed 0, the default of the client and every deserialised
//    context): the secret, every error and the encryption randomness come from
//    ChaCha20 (RFC 8439 block function) under a 256-bit key drawn from the OS
//    CSPRNG (getrandom), the stream's tag as nonce; the public uniform parts
//    (pk a, switching-key a) from SplitMix64 under an independent random seed.
struct SplitMix64 {
    u64 s;
    SplitMix64(u64 seed, u64 tag);
    u64 next();
};
// RFC 8439 §2.3 ChaCha20 block: 16 output words for (key, counter, nonce)
void chacha20_block(const uint32_t key[8], uint32_t counter, const uint32_t nonce[3], uint32_t out[16]);
struct ChaCha20 {
    uint32_t key[8], nonce[3], counter = 0, buf[16];
    int pos = 16;
    ChaCha20(const uint32_t k[8], u64 tag);
    u64 next();
};
struct Entropy {
    bool secure = false;
    u64 seed = 0;    // deterministic streams
    u64 seed_a = 0;  // secure mode: public uniform streams
    uint32_t key[8] = {};
    static Entropy from_seed(u64 seed);  // seed 0 -> secure (getrandom), else deterministic
};
// one sampling stream: `pub` marks the public uniform parts
struct Prng {
    Prng(const Entropy &e, u64 tag, bool pub = false);
    u64 next() { return use_cc ? cc.next() : sm.next(); }
    bool use_cc;
    SplitMix64 sm;
    ChaCha20 cc;
};
template <class G>
u64 sample_uniform_mod(G &g, u64 q) {
    const int bits = 64 - __builtin_clzll(q);
    for (;;) {
        const u64 r = g.next() >> (64 - bits);
        if (r < q) return r;
    }
}
template <class G>
int sample_ternary(G &g) {
    const u64 r = g.next() % 3;
    return r == 0 ? 0 : (r == 1 ? 1 : -1);
}
// centred binomial, eta = 21
template <class G>
int sample_cbd(G &g) {
    const u64 m = (1ULL << 21) - 1;
    const u64 a = g.next(), b = g.next();
    return __builtin_popcountll(a & m) - __builtin_popcountll(b & m);
}
namespace tags {
constexpr u64 secret = 1, pk_a = 2, pk_e = 3;
inline u64 swk_a(u64 kid, int j) { return 0x100000ULL + kid * 16 + 2 * (u64)j; }
inline u64 swk_e(u64 kid, int j) { return 0x100000ULL + kid * 16 + 2 * (u64)j + 1; }
inline u64 enc_v(u64 c) { return 0x80000000ULL + 3 * c; }
inline u64 enc_e0(u64 c) { return 0x80000000ULL + 3 * c + 1; }
inline u64 enc_e1(u64 c) { return 0x80000000ULL + 3 * c + 2; }
}  // namespace tags

// Precomputed key-switching / rescale constants for every level.
struct LevelTables {
    // ModUp, per ell (1..nq) and digit: [qhinv(alpha), qhinv_s(alpha), qhat(W*alpha) as [t][i]];
    // qhinv and phinv include n^-1 (their inputs come from unscaled inverse NTTs)
    std::vector<u64> modup;             // packed
    std::vector<std::vector<size_t>> modup_off;  // [ell][digit] offset into modup
    // fp64 form of the ModUp conversion (kernels.hip k_modup_fp), per ell and
    // digit: rows [W][alpha][4] of {h(c'), h(c), l(c'), l(c)} (c = qhat[t][i], zero
    // for the integer targets and the padding sources), then [W][4] {cst, q, 1/q, 0}
    // ({0, 0, 0, 1} for an integer target)
    // (the mdfp_* scheme below); modup_fp_mid as mdfp_mid over every row
    std::vector<double> modup_fp;
    std::vector<std::vector<size_t>> modup_fp_off;  // [ell][digit] offset into modup_fp
    int modup_fp_mid = -1;
    // ModDown (level independent)
    std::vector<u64> phinv, phinv_s;    // [K]
    std::vector<u64> phat;              // [nq][K]
    std::vector<u64> pinv, pinv_s;      // [nq]
    std::vector<u64> pmod, pmod_s;      // [nq]  P mod q_i
    std::vector<double> pinvd;          // [K]   1 / p_k (ModDown's centring count)
    // fp64 form of the fused ModDown + rescale conversion (kernels.hip
    // k_moddown_rescale_fp; DESIGN.md §5 "fp64 conversions"): per target i with
    // q_i < 2^41, for each source k (the K special residues, then the P term)
    // {h(c'), h(c), l(c'), l(c)} with c = phat[i][k] (pmod[i] for the P term),
    // c' = 2^30 c mod q_i, both centred and split v = h 2^20 + l, |l| <= 2^19;
    // mdfp_q[i] = {sum_k off_k c_k mod q_i, q_i, 1 / q_i, 0} ({0, 0, 0, 1}: an integer
    // target, q_i >= 2^41, which keeps the 128-bit sums).  mdfp_mid: 0 = the
    // sums fit 2^53 whole, 1 = with one reduction halfway, -1 = not usable
    std::vector<double> mdfp_c, mdfp_q;  // [nq][K+1][4], [nq][4]
    int mdfp_mid = -1;
    // fused ModDown + rescale (HMult tail): pqlinv[ell][i] = (P q_{ell-1})^{-1} mod q_i
    std::vector<u64> pqlinv, pqlinv_s;  // [nq+1][nq]
    // Rescale, per ell: qlinv[ell][i] = q_{ell-1}^{-1} mod q_i
    std::vector<u64> qlinv, qlinv_s;    // [nq+1][nq]
    // prime maps: ext[ell] = {0..ell-1, nq..nq+K-1}
    std::vector<int> extmap;            // [nq+1][nq+K]
    // ModUp forward-NTT map per ell: the non-own limbs of every digit,
    // slot j*W + t (in units of n) and its prime; concatenated over ell
    std::vector<int> modup_smap, modup_pmap;
    std::vector<size_t> modup_map_off, modup_map_cnt;  // [nq+1]
};
LevelTables make_level_tables(const Params &P);

}  // namespace host
}  // namespace fhe
