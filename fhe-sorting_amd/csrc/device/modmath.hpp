// 64-bit modular arithmetic for gfx950 (CDNA4) — pure integer VALU work.
//
// Residues are u64 < q < 2^61.  CDNA4 has no 64x64->128 multiply; hipcc
// lowers a*b (low half) to v_mul_lo_u32/v_mul_hi_u32/v_mad_u64_u32 sequences
// and __umul64hi to the matching high-half sequence.  Two reduction flavours:
//   * Shoup  (one operand is a precomputed constant w, w' = floor(w 2^64 / q)):
//            1 mulhi + 2 mullo, valid for ANY a < 2^64, result < 2q before the
//            final conditional subtraction.
//   * Barrett (both operands variable, a,b < q): mu = floor(2^(2k)/q), k = bitlen(q).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace fhe {
namespace dev {

using u64 = uint64_t;

struct Mod {
    u64 q;
    u64 mu;     // floor(2^(2k) / q)
    int k;      // bit length of q
    int pad;
    u64 r64, r64s;  // 2^64 mod q and its Shoup companion (128-bit reductions)
};

__device__ __forceinline__ u64 mulhi(u64 a, u64 b) { return __umul64hi(a, b); }

__device__ __forceinline__ u64 add_mod(u64 a, u64 b, u64 q) {
    u64 r = a + b;
    return r >= q ? r - q : r;
}
__device__ __forceinline__ u64 sub_mod(u64 a, u64 b, u64 q) { return a >= b ? a - b : a + q - b; }

__device__ __forceinline__ u64 mul_shoup(u64 a, u64 w, u64 wp, u64 q) {
    u64 hi = mulhi(a, wp);
    u64 r = a * w - hi * q;
    return r >= q ? r - q : r;
}
// lazy Shoup: result in [0, 2q)
__device__ __forceinline__ u64 mul_shoup_lazy(u64 a, u64 w, u64 wp, u64 q) {
    return a * w - mulhi(a, wp) * q;
}

__device__ __forceinline__ u64 mul_barrett(u64 a, u64 b, const Mod &m) {
    const u64 lo = a * b, hi = mulhi(a, b);
    const u64 t = (hi << (65 - m.k)) | (lo >> (m.k - 1));       // z >> (k-1)
    const u64 plo = t * m.mu, phi = mulhi(t, m.mu);
    const u64 qh = (phi << (63 - m.k)) | (plo >> (m.k + 1));     // (t*mu) >> (k+1)
    u64 r = lo - qh * m.q;
    if (r >= m.q) r -= m.q;
    if (r >= m.q) r -= m.q;
    return r;
}

// reduce an arbitrary u64 (< 2^64) modulo q (q >= 2^32 assumed by callers)
__device__ __forceinline__ u64 reduce64(u64 a, const Mod &m) {
    // Barrett with z = a < 2^64 <= q^2 since q >= 2^32
    const u64 t = (m.k - 1 >= 64) ? 0 : (a >> (m.k - 1));
    const u64 plo = t * m.mu, phi = mulhi(t, m.mu);
    const u64 qh = (phi << (63 - m.k)) | (plo >> (m.k + 1));
    u64 r = a - qh * m.q;
    if (r >= m.q) r -= m.q;
    if (r >= m.q) r -= m.q;
    return r;
}

// Lazy 128-bit accumulation for sums of products (basis conversions, linear
// sums, plaintext inner products): each term is a full 64x64 -> 128 product
// built from four 32x32 -> 64 multiplies (v_mad_u64_u32), and the sum is
// reduced once.  Residues are < 2^61, so a product is < 2^122 and up to 32
// terms fit in 128 bits.
struct Acc128 {
    u64 lo = 0, hi = 0;
};
__device__ __forceinline__ void mac128(Acc128 &acc, u64 a, u64 b) {
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const u64 p00 = (u64)a0 * b0, p01 = (u64)a0 * b1, p10 = (u64)a1 * b0, p11 = (u64)a1 * b1;
    const u64 mid = (p00 >> 32) + (uint32_t)p01 + (uint32_t)p10;
    const u64 lo = (mid << 32) | (uint32_t)p00;
    const u64 hi = p11 + (p01 >> 32) + (p10 >> 32) + (mid >> 32);
    acc.lo += lo;
    acc.hi += hi + (acc.lo < lo);
}
// (hi 2^64 + lo) mod q
__device__ __forceinline__ u64 reduce128(const Acc128 &a, const Mod &m) {
    return add_mod(reduce64(a.lo, m), mul_shoup(a.hi, m.r64, m.r64s, m.q), m.q);
}

// Basis-conversion accumulator: every prime is < 2^60 (checked at context
// creation), so operands split into 30-bit halves and the four partial sums
// a0*b0, a0*b1, a1*b0, a1*b1 (each < 2^60 per term) absorb up to 16 terms in
// 64 bits -- one v_mad_u64_u32 with accumulate per partial product, no carry
// handling until the single reduction per output.
constexpr u64 MASK30 = (1ull << 30) - 1;
struct Acc4 {
    u64 s00 = 0, s01 = 0, s10 = 0, s11 = 0;
};
struct Split30 {
    uint32_t lo, hi;
};
__device__ __forceinline__ Split30 split30(u64 b) { return Split30{(uint32_t)(b & MASK30), (uint32_t)(b >> 30)}; }
__device__ __forceinline__ void mac4(Acc4 &s, Split30 a, Split30 b) {
    s.s00 += (u64)a.lo * b.lo;
    s.s01 += (u64)a.lo * b.hi;
    s.s10 += (u64)a.hi * b.lo;
    s.s11 += (u64)a.hi * b.hi;
}
// r += s00 + (s01 + s10) 2^30 + s11 2^60  (exact, 128-bit)
__device__ __forceinline__ void fold4(Acc128 &r, const Acc4 &s) {
    const u64 mid = s.s01 + s.s10;
    const u64 mc = mid < s.s01;  // carry of the middle sum (bit 64)
    r.lo += s.s00;
    r.hi += (r.lo < s.s00);
    const u64 ml = mid << 30;
    r.lo += ml;
    r.hi += (mid >> 34) + (mc << 30) + (r.lo < ml);
    const u64 tl = s.s11 << 60;
    r.lo += tl;
    r.hi += (s.s11 >> 4) + (r.lo < tl);
}
// a sum longer than Acc4's 16 terms: after term i (0-based) of T, fold every
// full group of 16 into the exact 128-bit total (compiled out for T <= 16)
template <int T>
__device__ __forceinline__ void spill4(Acc128 &r, Acc4 &s, int i) {
    if (T > 16 && i % 16 == 15 && i + 1 < T) {
        fold4(r, s);
        s = Acc4{};
    }
}
// s00 + (s01 + s10) 2^30 + s11 2^60 mod q
__device__ __forceinline__ u64 reduce4(const Acc4 &s, const Mod &m) {
    Acc128 r;
    fold4(r, s);
    return reduce128(r, m);
}

}  // namespace dev
}  // namespace fhe
