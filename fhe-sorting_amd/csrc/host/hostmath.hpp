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

// seeded sampling
struct SplitMix64 {
    u64 s;
    SplitMix64(u64 seed, u64 tag);
    u64 next();
};
u64 sample_uniform_mod(SplitMix64 &g, u64 q);
int sample_ternary(SplitMix64 &g);
int sample_cbd(SplitMix64 &g);
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
    // ModDown (level independent)
    std::vector<u64> phinv, phinv_s;    // [K]
    std::vector<u64> phat;              // [nq][K]
    std::vector<u64> pinv, pinv_s;      // [nq]
    std::vector<u64> pmod, pmod_s;      // [nq]  P mod q_i
    std::vector<double> pinvd;          // [K]   1 / p_k (ModDown's centring count)
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
