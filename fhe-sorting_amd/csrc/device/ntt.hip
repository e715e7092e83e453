// Register-blocked negacyclic NTT for gfx950.
//
// n = 2^logN is split into a column pass over the top k1 index bits and a row
// pass over the low k2 bits (k1 = ceil(logN/2)).  Each pass is a batch of
// 2^PB-point transforms; one transform is owned by T = 2^(PB-EB) lanes that
// each hold E = 2^EB coefficients in VGPRs:
//   round 1: the E coefficients of a lane differ in the top EB index bits, so
//            EB radix-2 stages run in registers with no LDS traffic;
//   one LDS exchange (bank-conflict-free tile) re-deals the coefficients so that each lane
//   owns 2^(PB-EB)-point groups differing in the low bits;
//   round 2: the remaining PB-EB stages in registers.
// A limb therefore crosses HBM twice per transform (one read + one write per
// pass) and LDS once per pass.  Twiddles are psi^brev tables with Shoup
// companions; round-1 twiddles of the column pass are wave-uniform.
// The inverse runs the same machinery in Gentleman-Sande order (row pass first,
// low bits first) and folds n^-1 into the final store.
#include <hip/hip_ext.h>

#include <cstdlib>
#include <map>
#include <atomic>
#include <mutex>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "kernels.hpp"

namespace fhe {
namespace dev {

namespace {

constexpr int NTB = 256;  // threads per block (row passes, small rings)

// compile-time dispatch of a small runtime integer (the digit count of ntt_row_ks)
template <int Lo, int Hi, typename F>
void dispatch_int(int v, F &&f) {
    if constexpr (Lo > Hi) {
        throw std::invalid_argument("unsupported digit count " + std::to_string(v));
    } else {
        if (v == Lo) f(std::integral_constant<int, Lo>{});
        else dispatch_int<Lo + 1, Hi>(v, std::forward<F>(f));
    }
}
// Wide column passes (FHE_NTT_COL_WIDE, off by default -- measured slower,
// DESIGN.md §5 round-4 table): a 256-point column pass
// runs 64 columns per 1024-thread block, so lane = column and wave = t, the
// lane's position in its transform: every twiddle of both rounds is then
// wave-uniform (scalar loads, no VGPRs -- the 16-column blocks held up to 60
// VGPRs of per-lane round-2 twiddles), a wave's loads and stores are 512-B
// runs, and the 32-bit exchange tile (66.5 KB) leaves room for two blocks per CU.
#ifndef FHE_NTT_COL_WIDE
#define FHE_NTT_COL_WIDE 0
#endif
template <int PB, bool COLS>
constexpr int nthreads() {
    return (FHE_NTT_COL_WIDE && COLS && PB == 8) ? 1024 : NTB;
}

// LDS exchange tile.  ROWS: the lanes of one transform are adjacent, so each
// transform owns a contiguous run padded by one u64 per 16.  COLS: adjacent
// lanes are adjacent transforms, so the tile is element-major with a stride of
// NB + 1 u64 -- a 16-lane ds_write_b64 group then hits 32 distinct banks and a
// 32-lane ds_read_b64 group lands on the two bank halves (a per-transform run
// here would put all 16 transforms of a group on one bank).
template <int PB, int NB, bool COLS>
constexpr int lds_words() {
    return COLS ? (1 << PB) * (NB + 1) : NB * ((1 << PB) + (1 << PB) / 16);
}
template <int PB, int NB, bool COLS>
__device__ __forceinline__ int lds_at(int tr, int idx) {
    return COLS ? idx * (NB + 1) + tr : tr * ((1 << PB) + (1 << PB) / 16) + idx + (idx >> 4);
}

// 32-bit exchanges (FHE_NTT_LDS32, default on for the column passes): a
// non-split exchange moves the low and then the high halves of the coefficients
// through a tile of 32-bit words, half the LDS of a 64-bit tile, so twice the
// blocks fit a CU: with the 4-KB column twiddle table the inverse column pass
// (70-72 VGPRs) goes from 4 blocks (38.9 KB) to 7 (21.5 KB) per CU.  Two more
// barriers; no more registers (the low halves are dead once written).  Measured
// neutral in r4_a, before the column twiddles moved to LDS; since then 577.8 /
// 576.0 -> 572.6 / 574.7 ms, inverse column 98 -> 95 us (profiles/r4_l).
#ifndef FHE_NTT_LDS32
#define FHE_NTT_LDS32 1
#endif
// (row passes keep the 64-bit tile: with theirs at 32 bits the rescale and
// HMult-tail row passes ran 461 -> 530 and 385 -> 403 us, profiles/r4_a)
// LDS twiddles for the 256-point column passes (FHE_NTT_COL_TWL, default on): a
// column pass of prime p uses table entries 1..255 only (forward: stage s reads
// [2^s, 2^(s+1)); inverse: [2^(7-s), 2^(8-s))), the same for every block of the
// limb, so each thread stages one of them into LDS at the start and the
// per-lane twiddles (forward round 2, inverse round A, which depend on the
// lane's place t in its transform) are LDS reads instead of vector-cache loads
// the round had to wait for.
#ifndef FHE_NTT_COL_TWL
#define FHE_NTT_COL_TWL 1
#endif
// Buffer-addressed column passes (FHE_NTT_COL_BUF): a lane's E coefficients of a
// column sit 2^k2 words apart, too far for a global load's 13-bit immediate, so
// every global_load / global_store carried its own 64-bit VGPR address (32 VGPRs
// of addresses with all 16 loads in flight).  As buffer_load / buffer_store the
// limb base is one scalar resource, the lane's offset one VGPR and the per-register
// offset r T 2^k2 8 an SGPR.
#ifndef FHE_NTT_COL_BUF
#define FHE_NTT_COL_BUF 1
#endif
// Wave-uniform twiddles of the column passes (forward round 1, inverse round B)
// read through the constant address space, i.e. scalar loads into SGPRs (the
// tables never change while a kernel runs); as vector loads they held 4 VGPRs
// each.  A/B: -DFHE_NTT_COL_SCALAR=0.
#ifndef FHE_NTT_COL_SCALAR
#define FHE_NTT_COL_SCALAR 1
#endif
// FP row passes with fused epilogues: load the epilogue operands before the
// butterflies (1, as the integer passes) or in the store loop (0: fewer VGPRs)
#ifndef FHE_NTT_FP_EPI_PRE
#define FHE_NTT_FP_EPI_PRE 1
#endif
// the same for the HMult-tail / key-switch-finish rows alone (A/B: -DFHE_NTT_FP_EPI_PRE_MT=n)
#ifndef FHE_NTT_FP_EPI_PRE_MT
#define FHE_NTT_FP_EPI_PRE_MT FHE_NTT_FP_EPI_PRE
#endif
typedef const __attribute__((address_space(4))) u64 const_u64_t;
__device__ __forceinline__ ulonglong2 scalar_tw(const ulonglong2 *p, size_t i) {
    const const_u64_t *q = (const const_u64_t *)p + 2 * i;
    return make_ulonglong2(q[0], q[1]);
}
typedef const __attribute__((address_space(4))) double const_f64_t;
__device__ __forceinline__ double scalar_tw(const double *p, size_t i) { return ((const const_f64_t *)p)[i]; }
// raw buffer resource over one limb (wave-uniform base; CDNA word 3)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t limb_rsrc(const u64 *base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<u64 *>(base), 0, 0x7ffffff0, 0x00020000);
}
__device__ __forceinline__ u64 bload64(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
    return ((u64)v[1] << 32) | v[0];
}
__device__ __forceinline__ void bstore64(__amdgpu_buffer_rsrc_t r, int voff, int soff, u64 x) {
    typedef unsigned v2u __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(v2u{(unsigned)x, (unsigned)(x >> 32)}, r, voff, soff, 0);
}
template <bool COLS>
constexpr bool lds32() {
    return FHE_NTT_LDS32 != 0 && COLS;
}
// x'[j] = coefficient at tile position rpos(j), after every lane stored its x[r]
// at wpos(r)
template <int E, class WP, class RP>
__device__ __forceinline__ void exchange32(uint32_t *t32, u64 (&x)[E], WP wpos, RP rpos) {
#pragma unroll
    for (int r = 0; r < E; ++r) t32[wpos(r)] = (uint32_t)x[r];
    __syncthreads();
    uint32_t lo[E];
#pragma unroll
    for (int j = 0; j < E; ++j) lo[j] = t32[rpos(j)];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < E; ++r) t32[wpos(r)] = (uint32_t)(x[r] >> 32);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < E; ++j) x[j] = (u64)lo[j] | ((u64)t32[rpos(j)] << 32);
}

// Split exchange (column passes with G = E / T >= 2 groups per lane: the
// 512-point columns of ring 2^17).  The L1 -> L2 re-deal runs in G phases
// through a tile of 1/G the size: phase g moves the L1 registers r = G u + g
// (exactly the elements of every lane's L2 group g) and the lane reads its group
// g back into those same registers, so no second register set is needed.  L2
// group g element r therefore lives in register G r + g.  Halving the tile
// (69.6 -> 34.8 KB) doubles the blocks an LDS holds.
template <int G, int T, bool SPLIT>
__device__ constexpr int l2reg(int g, int r) {
    return SPLIT ? G * r + g : g * T + r;
}

// Lazy Shoup product a * w mod q in [0, 2q): a*w - floor(a*w'/2^64)*q taken
// mod 2^64, written as a*w + h*nq with nq = 2^64 - q so both low products
// share one multiply-accumulate chain (2 v_mad_u64_u32 + 4 v_mul_lo_u32) and
// no borrow chain is needed.
__device__ __forceinline__ u64 shoup_fold(u64 a, u64 w, u64 wp, u64 nq) {
    const u64 h = mulhi(a, wp);
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), w0 = (uint32_t)w, w1 = (uint32_t)(w >> 32);
    const uint32_t h0 = (uint32_t)h, h1 = (uint32_t)(h >> 32), n0 = (uint32_t)nq, n1 = (uint32_t)(nq >> 32);
    const u64 t = (u64)a0 * w0 + (u64)h0 * n0;
    const uint32_t cross = a0 * w1 + a1 * w0 + h0 * n1 + h1 * n0;
    return t + ((u64)cross << 32);
}
// Butterfly twiddle product with an approximate Shoup quotient: the high half
// of a * w' drops the a0*w'0 product and the carries of the two cross terms, so
// the quotient is short by 0..2 and the product lands in [0, 4q) instead of
// [0, 2q) -- 4 v_mad_u64_u32 + 2 v_mul_hi_u32 instead of 6 + 1 (and fewer
// moves): the butterfly is VALU-bound, and every prime < 2^60
// leaves room for the wider lazy ranges below (8q < 2^63).
__device__ __forceinline__ u64 mulhi_approx(u64 a, u64 b) {
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    return (u64)a1 * b1 + (((u64)a1 * b0) >> 32) + (((u64)a0 * b1) >> 32);
}
__device__ __forceinline__ u64 shoup_fold4(u64 a, u64 w, u64 wp, u64 nq) {  // [0, 4q) for any a < 2^64
    const u64 h = mulhi_approx(a, wp);
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), w0 = (uint32_t)w, w1 = (uint32_t)(w >> 32);
    const uint32_t h0 = (uint32_t)h, h1 = (uint32_t)(h >> 32), n0 = (uint32_t)nq, n1 = (uint32_t)(nq >> 32);
    const u64 t = (u64)a0 * w0 + (u64)h0 * n0;
    // (writing the + (cross << 32) as a 32-bit high-word add in inline asm cut
    // 60 VALU slots per row pass but measured 9% slower: the asm blocks the
    // scheduler's interleaving of independent butterflies)
    const uint32_t cross = a0 * w1 + a1 * w0 + h0 * n1 + h1 * n0;
    return t + ((u64)cross << 32);
}
// lazy forward CT butterfly (q4 = 4q): x, y < B q -> x, y < (B' + 4) q with
// B' = B, or B' = 8 when R (x >= 8q loses 8q; needs B <= 16).  Every prime is
// < 2^60, so values up to 16q fit in 64 bits and a pass reduces only on the
// stages fwd_reduce picks (about every other one) instead of on every stage.
template <bool R>
__device__ __forceinline__ void ct_bfly(u64 &x, u64 &y, ulonglong2 w, u64 q4, u64 nq) {
    u64 u = x;
    if (R) u = u >= 2 * q4 ? u - 2 * q4 : u;      // [0, 8q)
    const u64 v = shoup_fold4(y, w.x, w.y, nq);  // [0, 4q)
    x = u + v;
    y = u + q4 - v;
}
// Bound schedule of the forward passes (in units of q).  Column-pass inputs are
// < 8q (canonical or lazy producers); the column pass leaves values < 16q; the
// row pass starts from 16 and its last stage always reduces, so the fused
// epilogues see v < 12q.  Stage s of a pass reduces iff the bound would pass 16
// (or 12 at the row pass's last stage).
__host__ __device__ constexpr bool fwd_reduce(bool cols, int pb, int s) {
    // 512-point passes (ring 2^17 columns) reduce on every stage: with the lazy
    // schedule the compiler spilled their 32 coefficients per lane to scratch
    // (132 VGPRs + 272 B, 3x slower); 2^16-point and smaller passes do not
    if (pb >= 9) return true;
    int B = cols ? 8 : 16;
    for (int k = 0;; ++k) {
        const bool r = B + 4 > 16 || (!cols && k == pb - 1 && B + 4 > 12);
        if (k == s) return r;
        B = (r ? 8 : B) + 4;
    }
}
template <int PB>
__device__ __forceinline__ void ct_stage(bool cols, int s, u64 &x, u64 &y, ulonglong2 w, u64 q4, u64 nq) {
    if (fwd_reduce(cols, PB, s)) ct_bfly<true>(x, y, w, q4, nq);
    else ct_bfly<false>(x, y, w, q4, nq);
}
// lazy inverse GS butterfly: x, y in [0, 4q) -> x, y in [0, 4q)
__device__ __forceinline__ void gs_bfly(u64 &x, u64 &y, ulonglong2 w, u64 q4, u64 nq) {
    const u64 u = x, v = y;
    u64 s = u + v;
    x = s >= q4 ? s - q4 : s;
    y = shoup_fold4(u + q4 - v, w.x, w.y, nq);
}
// ---------------------------------------------------------------------------
// fp64 butterflies for the primes below 2^41 (the 40-bit scaling primes), run
// by separate "FP" launches over those limbs (launch_pass splits a launch by
// prime class; DESIGN.md §5 "fp64 NTT for the 40-bit limbs").  A coefficient
// is an exactly represented signed integer |v| < 2^52 held as a double; the
// twiddle product y w mod q is
//   b = fl(y w), e = y w - b (exact, one FMA), h = rint(fl(b / q)),
//   r = (b - h q) + e            (the FMA b - h q is exact: |b - h q| < 2^53)
// = y w - h q with |r| <= (1/2 + eps) q, eps = |y| 3 2^-53 (|y| <= 2^50 keeps
// eps <= 3/8).  Six fp64 operations (v_fma_f64 / v_mul_f64 / v_rndne_f64 issue
// at the half rate of v_mul_lo_u32, ~33 T lane-ops/s, against v_mad_u64_u32's
// ~23 T; profiles/r5_rates) where the integer Shoup product takes 4
// v_mad_u64_u32 + 2 v_mul_hi_u32 + 4 v_mul_lo_u32, and the butterfly sums are
// plain fp64 adds with no conditional subtractions: forward values grow by
// <= q/2 per stage, inverse sums double per stage (bounded per pass below).
// Loads and stores convert with the 2^52 trick: for an integer 0 <= x < 2^52
// the double with bits 0x433 << 52 | x is 2^52 + x.
constexpr double FP_TWO52 = 4503599627370496.0;
constexpr u64 FP_MAGIC = 0x4330000000000000ull;
constexpr int FP_QBITS = 41;  // FP launches take primes q < 2^41
__device__ __forceinline__ double dbits(u64 x) { return __longlong_as_double((long long)x); }
__device__ __forceinline__ u64 ubits(double d) { return (u64)__double_as_longlong(d); }
// u64 x < 2^52 -> the double x - off, with c = 2^52 + off (exact)
__device__ __forceinline__ double fp_in(u64 x, double c) { return dbits(x | FP_MAGIC) - c; }
// integer-valued v with 0 <= v + off < 2^52 -> the u64 v + off, with c = 2^52 + off
__device__ __forceinline__ u64 fp_out(double v, double c) { return ubits(v + c) ^ FP_MAGIC; }
__device__ __forceinline__ double fp_mulmod(double y, double w, double q, double qi) {
    const double b = y * w;
    const double e = __builtin_fma(y, w, -b);
    const double h = __builtin_rint(b * qi);
    return __builtin_fma(-h, q, b) + e;
}
// v - q rint(v / q): |result| <= (1/2 + |v| 3 2^-53) q
__device__ __forceinline__ double fp_reduce(double v, double q, double qi) {
    return __builtin_fma(-__builtin_rint(v * qi), q, v);
}
// per-launch arithmetic constants of one prime: integer (Shoup butterflies)
// and fp64 (q and its rounded reciprocal)
struct Ar {
    u64 q4, nq;
    double q, qi;
};
template <bool FP>
using TwT = typename std::conditional<FP, double, ulonglong2>::type;
__device__ __forceinline__ void ct_bfly_fp(u64 &x, u64 &y, double w, const Ar &A) {
    const double u = dbits(x), v = fp_mulmod(dbits(y), w, A.q, A.qi);
    x = ubits(u + v);
    y = ubits(u - v);
}
__device__ __forceinline__ void gs_bfly_fp(u64 &x, u64 &y, double w, const Ar &A) {
    const double u = dbits(x), v = dbits(y);
    x = ubits(u + v);
    y = ubits(fp_mulmod(u - v, w, A.q, A.qi));
}
template <bool FP, int PB>
__device__ __forceinline__ void ct_any(bool cols, int s, u64 &x, u64 &y, TwT<FP> w, const Ar &A) {
    if constexpr (FP) ct_bfly_fp(x, y, w, A);
    else if (fwd_reduce(cols, PB, s)) ct_bfly<true>(x, y, w, A.q4, A.nq);
    else ct_bfly<false>(x, y, w, A.q4, A.nq);
}
template <bool FP>
__device__ __forceinline__ void gs_any(u64 &x, u64 &y, TwT<FP> w, const Ar &A) {
    if constexpr (FP) gs_bfly_fp(x, y, w, A);
    else gs_bfly(x, y, w, A.q4, A.nq);
}
// Bounds of the FP passes (q < 2^41, so 2^50 = 512 q):
//   forward column: inputs < 8q loaded as x - 4q (|x| <= 4q); 9 stages add
//     <= 0.51 q each -> |x| < 8.6 q, stored + 9q (< 18 q);
//   forward row: loaded - 9q (|x| < 8.6 q), 8 stages -> < 12.7 q, then reduced
//     (fp_reduce) for the canonical store or the integer epilogues;
//   inverse row: inputs < 4q loaded - 2q (|x| <= 2q); a GS sum at most doubles
//     per stage -> |x| <= 2^8 2q = 512 q, twiddle inputs |u - v| <= 512 q;
//     reduced (|r| <= 0.88 q) and stored + q (< 2q, the integer pass's range);
//   inverse column: loaded - q (|x| <= 0.88 q), 9 stages -> <= 2^9 0.88 q < 2^50,
//     then times n^-1 (fp_mulmod, canonicalised) or reduced to [0, 2q) (raw).
// Every intermediate is an integer below 2^52 and every twiddle input below
// 2^50, so each operation above is exact (tests/test_fp_mulmod.py checks the
// product and reduction at these bounds against exact integer arithmetic).
constexpr double FP_FWD_COL_IN = 4.0, FP_FWD_COL_OUT = 9.0, FP_INV_ROW_IN = 2.0, FP_INV_ROW_OUT = 1.0;

__device__ __forceinline__ u64 smod64(int64_t v, const Mod &m) {  // signed integer -> [0, q)
    if (v >= 0) return reduce64((u64)v, m);
    const u64 r = reduce64((u64)0 - (u64)v, m);
    return r ? m.q - r : 0;
}
__device__ __forceinline__ u64 smod64(int64_t v, int sh, const Mod &m) {  // v * 2^sh -> [0, q)
    u64 r = smod64(v, m);
    for (int i = 0; i < sh; ++i) r = r + r >= m.q ? r + r - m.q : r + r;
    return r;
}
__device__ __forceinline__ u64 canon12(u64 x, u64 q, u64 q2) {  // [0, 12q) -> [0, q)
    x = x >= 4 * q2 ? x - 4 * q2 : x;
    x = x >= 2 * q2 ? x - 2 * q2 : x;
    x = x >= q2 ? x - q2 : x;
    return x >= q ? x - q : x;
}
__device__ __forceinline__ u64 canon8(u64 x, u64 q, u64 q2) {  // [0, 8q) -> [0, q)
    x = x >= 2 * q2 ? x - 2 * q2 : x;
    x = x >= q2 ? x - q2 : x;
    return x >= q ? x - q : x;
}

// ---------------------------------------------------------------------------
// Register-only 256-point row passes (PB = 8, 16 lanes x 16 coefficients).
//
// A coefficient's 8-bit in-row index is split into 4 lane bits and 4 register
// bits; a butterfly stage needs its bit among the register bits.  Instead of
// re-dealing the whole transform through LDS, a stage whose bit sits in a lane
// bit swaps that lane bit with a register bit whose stage is done: lanes t and
// t ^ 2^m exchange half of their registers with DPP moves (no LDS, no
// barrier).  The forward schedule needs 5 such swaps per pass, all against
// register bit 3 (slots j and j + 8), the inverse 4 (inv_swap); both end in
//   idx = lane_index(t) + 16 * r      (lane bits = index bits 0..3),
// so loads and stores are fully coalesced: the 16 lanes of a transform cover
// one 128-B line per 8-B instruction.
struct RowLayout {
    int lane[4];  // index bit held by lane bit m
    int reg[4];   // index bit held by register bit p
};
struct RowSwap {
    int m, p;  // swap lane bit m with register bit p before the stage (m < 0: none)
};
// GS inverse: stages take index bits 0, 1, ..., 7.  The inverse pass loads 16-B
// pairs (register bit 0 = index bit 0, lanes = index bits 1..4, still one 256-B
// run per transform and instruction), so stage 0 needs no swap and stages 1..4
// each bring their lane bit in for the finished register bit 0: 4 swaps, ending
// in lanes = index bits 0..3 for the coalesced 8-B stores
__device__ constexpr RowSwap inv_swap(int s) {
    return s >= 1 && s <= 4 ? RowSwap{s - 1, 0} : RowSwap{-1, 0};
}
// CT forward: stages take index bits 7, 6, ..., 0; stage 8 is the final
// fix-up swap (no butterfly) back to lane bits = index bits 0..3
__device__ constexpr RowSwap fwd_swap(int s) {
    return s < 4 ? RowSwap{-1, 0} : s < 8 ? RowSwap{7 - s, 3} : RowSwap{3, 3};
}
template <bool FWD>
__device__ constexpr RowLayout row_layout(int s) {  // layout in effect during stage s (after its swap)
    RowLayout L = FWD ? RowLayout{{0, 1, 2, 3}, {4, 5, 6, 7}} : RowLayout{{1, 2, 3, 4}, {0, 5, 6, 7}};
    for (int k = 0; k <= s; ++k) {
        const RowSwap w = FWD ? fwd_swap(k) : inv_swap(k);
        if (w.m >= 0) {
            const int t = L.lane[w.m];
            L.lane[w.m] = L.reg[w.p];
            L.reg[w.p] = t;
        }
    }
    return L;
}
__device__ __forceinline__ int lane_index(const RowLayout &L, int t) {
    int v = 0;
#pragma unroll
    for (int m = 0; m < 4; ++m) v |= ((t >> m) & 1) << L.lane[m];
    return v;
}
__device__ constexpr int reg_index(const RowLayout &L, int r) {
    int v = 0;
    for (int p = 0; p < 4; ++p) v |= ((r >> p) & 1) << L.reg[p];
    return v;
}
// value of lane t ^ 2^m within the 16-lane row (DPP, VALU only)
template <int M>
__device__ __forceinline__ uint32_t xor_lane32(uint32_t v) {
    // every source lane of these patterns lies inside the lane's own 16-lane row,
    // so no lane keeps an "old" value: mov_dpp (old undefined, bound_ctrl) needs
    // no zero-initialised destination and can fold into the consuming select
    int x = (int)v;
    if (M == 0) x = __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, true);        // quad_perm [1,0,3,2]
    else if (M == 1) x = __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, true);   // quad_perm [2,3,0,1]
    else if (M == 2) {                                                        // ^7 then ^3
        x = __builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, true);               // row_half_mirror
        x = __builtin_amdgcn_mov_dpp(x, 0x1B, 0xF, 0xF, true);                // quad_perm [3,2,1,0]
    } else x = __builtin_amdgcn_mov_dpp(x, 0x128, 0xF, 0xF, true);            // row_ror:8
    return (uint32_t)x;
}
template <int M>
__device__ __forceinline__ u64 xor_lane(u64 v) {
    return (u64)xor_lane32<M>((uint32_t)v) | ((u64)xor_lane32<M>((uint32_t)(v >> 32)) << 32);
}
// swap lane bit M with register bit P for the pair (x[j], x[j + 2^P]), bit P of j clear:
// afterwards x[j] holds the element whose (new) register bit P is 0
template <int M, int P>
__device__ __forceinline__ void swap_pair(u64 &lo, u64 &hi, int t) {
    const u64 r0 = xor_lane<M>(lo), r1 = xor_lane<M>(hi);
    const bool up = (t >> M) & 1;
    const u64 nlo = up ? r1 : lo, nhi = up ? hi : r0;
    lo = nlo;
    hi = nhi;
}
template <int P>
__device__ __forceinline__ void swap_regs(u64 *x, int t, int m) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        if (j & (1 << P)) continue;
        switch (m) {
        case 0: swap_pair<0, P>(x[j], x[j + (1 << P)], t); break;
        case 1: swap_pair<1, P>(x[j], x[j + (1 << P)], t); break;
        case 2: swap_pair<2, P>(x[j], x[j + (1 << P)], t); break;
        default: swap_pair<3, P>(x[j], x[j + (1 << P)], t); break;
        }
    }
}
// the register bit holding index bit b in layout L
__device__ constexpr int reg_of(const RowLayout &L, int b) {
    int p = -1;
    for (int k = 0; k < 4; ++k)
        if (L.reg[k] == b) p = k;
    return p;
}
// LDS offset of stage S's twiddles in a row's table (row_twiddles): forward
// stage S uses 2^S of them, inverse stage S 2^(7 - S)
template <bool FWD>
__device__ constexpr int twl_off(int S) {
    return FWD ? (1 << S) - 1 : 256 - (256 >> S);
}
// The 255 twiddle pairs of one row (every stage of a 256-point row pass) into
// LDS, by the block's first 255 threads; the caller synchronises.  Used when
// every transform of the block is the same row (16 segments per block), so
// the row's twiddles are read from HBM / L2 once per block and from LDS per
// butterfly instead of from the vector cache.
template <bool FWD, class TW>
__device__ __forceinline__ void row_twiddles(TW *twl, const TW *tw, size_t row, size_t n, int S0) {
    const int e = threadIdx.x;
    if (e >= 255) return;
    int S = 0;
    while (S < 7 && e >= twl_off<FWD>(S + 1)) ++S;
    const int j = e - twl_off<FWD>(S);
    twl[e] = FWD ? tw[((size_t)1 << (S0 + S)) + (row << S) + j] : tw[(n >> (S + 1)) + (row << (7 - S)) + j];
}
// the tables of R consecutive rows row0 .. row0 + R - 1, row r at twl + 256 r:
// a block whose 16 transforms are 16 / R segments x R rows reads each row's
// twiddles from HBM / L2 once.  Thread f < 255 copies entry f of every row (its
// stage and offset computed once; R <= 16 independent loads, then the stores).
// The row-pass kernels take the table in dynamic LDS sized for their R
// (launch_pass_one); the fused relinearisation's R <= TWL_ROWS is static.
constexpr int TWL_ROWS = 4;
template <bool FWD, class TW>
__device__ __forceinline__ void row_twiddles_multi(TW *twl, const TW *tw, size_t row0, int R, size_t n, int S0) {
    const int f = threadIdx.x;  // blockDim 256
    if (f >= 255) return;
    const size_t rows = n >> 8;
    int S = 0;
    while (S < 7 && f >= twl_off<FWD>(S + 1)) ++S;
    const int j = f - twl_off<FWD>(S);
    const size_t step = FWD ? ((size_t)1 << S) : ((size_t)1 << (7 - S));
    const TW *src = (FWD ? tw + ((size_t)1 << (S0 + S)) : tw + (n >> (S + 1))) + row0 * step + j;
    const size_t rmax = rows - 1 - row0;  // (grids cover whole rows; the clamp keeps small rings in bounds)
#pragma unroll
    for (int r0 = 0; r0 < 16; r0 += 4) {
        if (r0 >= R) break;
        TW v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = src[min((size_t)(r0 + k), rmax) * step];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (r0 + k < R && (size_t)(r0 + k) <= rmax) twl[256 * (r0 + k) + f] = v[k];
    }
}
template <bool FWD, int S, bool TWL, bool FP>
__device__ __forceinline__ void row_stage(u64 *x, int t, size_t row, const TwT<FP> *tw, size_t n, int S0,
                                          const Ar &A) {
    constexpr RowSwap w = FWD ? fwd_swap(S) : inv_swap(S);
    if (w.m >= 0) swap_regs<w.p>(x, t, w.m);
    if (S >= 8) return;  // the forward pass's final fix-up swap
    constexpr RowLayout L = row_layout<FWD>(S);
    constexpr int b = FWD ? 7 - S : S;  // index bit of this stage
    constexpr int P = reg_of(L, b);
    const int li = lane_index(L, t);
    // twiddle index = stage base + row part + (idx0 >> shift), idx0 = li | reg_index(j):
    // lane and register bits are disjoint, so the shift splits into a per-lane
    // offset and a compile-time one -> one address per stage, immediate offsets
    constexpr int SH = FWD ? 8 - S : S + 1;
    const TwT<FP> *tws = TWL ? tw + twl_off<FWD>(S) + (li >> SH)  // tw: the row's LDS table
                         : FWD ? tw + ((size_t)1 << (S0 + S)) + (row << S) + (uint32_t)(li >> SH)
                               : tw + (n >> (S + 1)) + (row << (7 - S)) + (uint32_t)(li >> SH);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        if (j & (1 << P)) continue;
        const TwT<FP> w = tws[reg_index(L, j) >> SH];
        if (FWD) ct_any<FP, 8>(false, S, x[j], x[j + (1 << P)], w, A);
        else gs_any<FP>(x[j], x[j + (1 << P)], w, A);
    }
}
template <bool FWD, bool TWL, bool FP>
__device__ __forceinline__ void row_pass_shfl(u64 *x, int t, size_t row, const TwT<FP> *tw, size_t n, int S0,
                                              const Ar &A) {
    row_stage<FWD, 0, TWL, FP>(x, t, row, tw, n, S0, A);
    row_stage<FWD, 1, TWL, FP>(x, t, row, tw, n, S0, A);
    row_stage<FWD, 2, TWL, FP>(x, t, row, tw, n, S0, A);
    row_stage<FWD, 3, TWL, FP>(x, t, row, tw, n, S0, A);
    row_stage<FWD, 4, TWL, FP>(x, t, row, tw, n, S0, A);
    row_stage<FWD, 5, TWL, FP>(x, t, row, tw, n, S0, A);
    row_stage<FWD, 6, TWL, FP>(x, t, row, tw, n, S0, A);
    row_stage<FWD, 7, TWL, FP>(x, t, row, tw, n, S0, A);
    if (FWD) row_stage<FWD, 8, TWL, FP>(x, t, row, tw, n, S0, A);
}
// in-row index of lane t's register r after a pass (both passes end in this layout)
template <bool FWD>
__device__ __forceinline__ int row_final_index(int t, int r) {
    constexpr RowLayout L = row_layout<FWD>(FWD ? 8 : 7);
    return lane_index(L, t) + reg_index(L, r);
}
// FHE_NTT_ROW_SHFL bit mask (A/B timing): 1 inverse row pass, 2 every forward row
// pass, 4 / 8 / 16 only the fused HMult-tail / rescale / key-switch-finish forward
// rows use the register-only DPP passes.  0 keeps all on the LDS-exchange passes.
// Default 15 (inverse rows, every plain forward row, HMult-tail and rescale rows):
// at two lanes the DPP HMult tail (66-175 VGPRs instead of 220) took the sort
// 590.9 / 589.2 -> 584.9 / 582.5 ms (profiles/r4_j; at three lanes it had measured
// even, profiles/r4_f), the DPP rescale rows 575.4 / 577.5 -> 572.4 / 574.6 ms
// (profiles/r4_k), the plain forward rows (ModUp; with the LDS row twiddles, so
// no per-row twiddle re-reads) 573.0 / 575.4 -> 566.6 / 568.4 ms (profiles/r4_n).
// The key-switch-finish rows were neutral and stay on the LDS passes.
int &row_shfl_enabled() {
    static int v = [] {
        const char *e = std::getenv("FHE_NTT_ROW_SHFL");
        return e ? std::atoi(e) : 15;
    }();
    return v;
}

// Fused forward modes (MODE): 0 plain; 1 column pass loads the centred lift
// of one coefficient-form limb (`last`, prime lastp) instead of `data`
// (rescale: the lifted limb is never materialised per prime); 2 row pass
// stores out = (x - NTT) * c1 (rescale finish); 3 row pass stores
// out = (x + d * c2 - NTT) * c1 (fused ModDown+rescale finish of an HMult);
// 4 row pass stores out = (x - NTT) * c1 + d (the ModDown finish of a key
// switch: x the accumulators, c1 = P^-1, d the permuted c0 added to the even
// segments, member z / 2 at (z / 2) * seg_d, or none).
// Modes 2-4 do not write `data` back.
enum { NTT_PLAIN = 0, NTT_LIFT = 1, NTT_RESCALE = 2, NTT_MULTAIL = 3, NTT_KSFINISH = 4 };

// COLS: the transform index is a column `col`, element idx sits at idx * 2^k2 + col.
// ROWS: the transform index is a row `hi`, element idx sits at hi * 2^PB + idx.
// SH (row passes with PB = 8 only): register-only stages with DPP lane swaps
// (row_pass_shfl) instead of the two LDS exchanges.
template <int PB, int EB, bool COLS, int MODE, bool SH, bool FULL, bool TWL = false, bool FP = false>
__device__ __forceinline__ void ntt_fwd_body(u64 *data, size_t seg, const int *pmap, const int *smap, int logN,
                                             const NttTables &Tb, const NttFuse &F) {
    static_assert(!SH || (!COLS && PB == 8 && EB == 4), "shuffle row pass: 16 lanes x 16 coefficients");
    constexpr int E = 1 << EB;          // coefficients per lane
    constexpr int RB = PB - EB;         // bits of round 2
    constexpr int T = 1 << RB;          // lanes per transform
    constexpr int NB = nthreads<PB, COLS>() / T;  // transforms per block
    constexpr int G = E >> RB;          // round-2 groups per lane
    constexpr int LEN = 1 << PB;
    constexpr bool SPLIT = COLS && G >= 2;
    constexpr int TPB = SPLIT ? PB - (EB - RB) : PB;  // points per exchange phase (log2)
    constexpr bool X32 = lds32<COLS>() && !SPLIT;
    __shared__ u64 tile[SH ? 1 : X32 ? (lds_words<TPB, NB, COLS>() + 1) / 2 : lds_words<TPB, NB, COLS>()];
    uint32_t *const t32 = reinterpret_cast<uint32_t *>(tile);
    constexpr bool CTW = FHE_NTT_COL_TWL && COLS && !SPLIT && PB == 8 && nthreads<PB, COLS>() == 256;
    using TW = TwT<FP>;
    __shared__ TW twc[CTW ? 256 : 1];

    const size_t n = (size_t)1 << logN;
    const int k2 = COLS ? logN - PB : 0;
    // grid: x = segment (fastest, so the blocks of one prime's row/column
    // block across all segments run back to back and share its twiddles in
    // L2), y = block within the limb, z = limb (through the launch's limb runs)
    const int limb = F.limb_of(blockIdx.z);
    const int p = pmap ? __builtin_amdgcn_readfirstlane(pmap[limb]) : limb;
    int t, tr;  // lane within its transform, transform within the block
    if (COLS) {
        tr = threadIdx.x % NB;
        // NB = 64: t is the wave index -- said so, so the twiddle addresses
        // built from it are scalar
        t = NB == 64 ? __builtin_amdgcn_readfirstlane(threadIdx.x / NB) : threadIdx.x / NB;
    } else {
        tr = threadIdx.x / T;
        t = threadIdx.x % T;
    }
    // SH: the block's transforms are one row of 2^F.lsegb segments (x 16 >> lsegb
    // rows), so the per-row twiddles are loaded once per block and shared in L1
    const int zseg = SH ? (int)blockIdx.x * (1 << F.lsegb) + (tr & ((1 << F.lsegb) - 1)) : (int)blockIdx.x;
    const size_t tid_global = SH ? (size_t)blockIdx.y * (NB >> F.lsegb) + (tr >> F.lsegb)
                                 : (size_t)blockIdx.y * NB + tr;  // column or row index
    const bool valid = FULL || (tid_global < ((size_t)1 << (logN - PB)) && (!SH || zseg < F.segs));
    u64 *a = data + (size_t)zseg * seg + (smap ? (size_t)__builtin_amdgcn_readfirstlane(smap[limb]) : (size_t)limb) * n;
    const u64 q = Tb.mods[p].q, q2 = 2 * q, q4 = 4 * q, nq = (u64)0 - q;
    const TW *tw;
    if constexpr (FP) tw = Tb.fwdd + (size_t)p * n;
    else tw = Tb.fwd2 + (size_t)p * n;
    Ar A{q4, nq, 0.0, 0.0};
    if constexpr (FP) {
        const double2 qd = Tb.qd[p];
        A.q = qd.x;
        A.qi = qd.y;
    }
    // FP: the load offset (column: inputs < 8q centred by 4q; row: the column
    // pass's store offset)
    const double fin = FP ? FP_TWO52 + (COLS ? FP_FWD_COL_IN : FP_FWD_COL_OUT) * A.q : 0.0;
    constexpr bool CBUF = FHE_NTT_COL_BUF && COLS && FULL;  // (FULL: no bounds check; COLS: zseg is blockIdx.x)
    const int S0 = COLS ? 0 : logN - PB;                      // global stage of local stage 0
    if (CTW) twc[threadIdx.x] = tw[threadIdx.x];  // read after the exchange's barrier (round 2)

    u64 x[E];
    // ---- load, layout L1: idx = t + T * r
    if (MODE == NTT_LIFT) {
        // centred lift of c mod q_last into prime p: q_last / 2 < q_p (checked at
        // context creation), so c or q_p - (q_last - c) is already reduced
        const Mod ml = Tb.mods[F.lastp];
        const u64 ql = ml.q, qh = ql >> 1;
        const u64 kl = F.scalar ? smod64(F.scalar, F.scalar_sh, ml) : 0;  // K mod q_last (scaled rescale)
        const u64 *src = F.last + (size_t)zseg * F.seg_last;
        const auto rs = limb_rsrc(src);
        const int vo = (int)((((size_t)t << k2) + tid_global) * 8);
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const int idx = t + T * r;
            u64 c = CBUF ? bload64(rs, vo, (T * r << k2) * 8)
                         : valid ? src[(size_t)idx * ((size_t)1 << k2) + tid_global] : 0;
            if (F.scalar) c = mul_barrett(c, kl, ml);
            x[r] = c > qh ? q - (ql - c) : c;
        }
    } else if constexpr (CBUF) {
        const auto rs = limb_rsrc(a);
        const int vo = (int)((((size_t)t << k2) + tid_global) * 8);
#pragma unroll
        for (int r = 0; r < E; ++r) x[r] = bload64(rs, vo, (T * r << k2) * 8);
    } else {
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const int idx = t + T * r;
            const size_t off = COLS ? (size_t)idx * ((size_t)1 << k2) + tid_global : tid_global * LEN + idx;
            x[r] = valid ? a[off] : 0;
        }
    }
    if constexpr (FP) {
#pragma unroll
        for (int r = 0; r < E; ++r) x[r] = ubits(fp_in(x[r], fin));
    }
    // fused row-pass epilogues: their operands (the rescale input / the HMult
    // accumulators and d) are loaded now, so the loads overlap the butterflies
    // instead of stalling the store loop (the tile's LDS bounds occupancy, the
    // extra VGPRs do not)
    // (FP rows: FHE_NTT_FP_EPI_PRE=0 loads them in the store loop instead -- A/B)
    constexpr bool EPI_PRE = MODE == NTT_RESCALE ? FHE_NTT_FP_EPI_PRE : FHE_NTT_FP_EPI_PRE_MT;
    constexpr bool EPI_X = !COLS && (MODE == NTT_RESCALE || MODE == NTT_MULTAIL || MODE == NTT_KSFINISH) &&
                           (!FP || EPI_PRE);
    constexpr bool EPI_D = !COLS && (MODE == NTT_MULTAIL || MODE == NTT_KSFINISH) && (!FP || EPI_PRE);
    // key-switch finish: only c0 segments (even z) take the added polynomial
    const bool has_d = MODE == NTT_KSFINISH ? (F.d != nullptr && !(zseg & 1)) : true;
    const size_t d_base = MODE == NTT_KSFINISH ? (size_t)(zseg >> 1) * F.seg_d : (size_t)zseg * F.seg_d;
    u64 ex[EPI_X ? E : 1], ed[EPI_D ? E : 1];
    if (EPI_X) {
        const size_t lo = (size_t)limb * n + tid_global * LEN;
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const int idx = SH ? row_final_index<true>(t, r) : t + T * r;  // where the pass leaves element r
            ex[r] = valid ? F.x[(size_t)zseg * F.seg_x + lo + idx] : 0;
            if (EPI_D) ed[EPI_D ? r : 0] = valid && has_d ? F.d[d_base + lo + idx] : 0;
        }
    }
    // per-limb epilogue constants (fused row-pass modes)
    const bool EPI = !COLS && (MODE == NTT_RESCALE || MODE == NTT_MULTAIL || MODE == NTT_KSFINISH);
    const Mod mp = Tb.mods[p];
    const u64 c1 = EPI ? F.c1[limb] : 0, c1s = EPI ? F.c1s[limb] : 0;
    const u64 c2 = MODE == NTT_MULTAIL ? F.c2[limb] : 0, c2s = MODE == NTT_MULTAIL ? F.c2s[limb] : 0;
    // scaled rescale: out = (K x - v) q_last^-1 = x (K q_last^-1) - v q_last^-1
    const u64 kq = (MODE == NTT_RESCALE && F.scalar) ? mul_shoup(smod64(F.scalar, F.scalar_sh, mp), c1, c1s, q) : 0;
    // row-pass store of transform value v (lazy, [0, 12q)) for element r at in-row index idx
    auto store_row = [&](int r, int idx, u64 v) {
        const size_t z = (size_t)zseg, lo = (size_t)limb * n + tid_global * LEN;
        if constexpr (FP) {
            // |v| < 12.7 q -> centred residue |r| < 0.51 q; the epilogues take r + q
            // (< 12q as they require), the plain store the canonical residue
            const double rr = fp_reduce(dbits(v), A.q, A.qi);
            if (MODE == NTT_PLAIN) {
                a[tid_global * LEN + idx] = fp_out(rr < 0.0 ? rr + A.q : rr, FP_TWO52);
                return;
            }
            v = fp_out(rr, FP_TWO52 + A.q);
        }
        // lazy epilogues: v in [0, 12q), every intermediate < 2^64 (q < 2^60), one
        // final conditional subtraction (the exact Shoup products are in [0, 2q))
        if (MODE == NTT_RESCALE) {
            const u64 xin = EPI_X ? ex[EPI_X ? r : 0] : F.x[z * F.seg_x + lo + idx];
            u64 o;
            if (F.scalar) {  // (K x - v) q_last^-1 = x kq - v c1: [0, q) + 2q - [0, 2q)
                o = mul_barrett(xin, kq, mp) + q2 - shoup_fold(v, c1, c1s, nq);
                o = o >= q2 ? o - q2 : o;
            } else {  // (x - v) q_last^-1, x + 12q - v < 13q
                o = shoup_fold(xin + 3 * q4 - v, c1, c1s, nq);
            }
            F.out[z * F.seg_out + lo + idx] = o >= q ? o - q : o;
        } else if (MODE == NTT_MULTAIL) {  // (acc + d c2 - v) c1, acc + d c2 + 12q - v < 15q
            const u64 acc = EPI_X ? ex[EPI_X ? r : 0] : F.x[z * F.seg_x + lo + idx];
            const u64 dd = EPI_D ? ed[EPI_D ? r : 0] : F.d[z * F.seg_d + lo + idx];
            const u64 tt = acc + shoup_fold(dd, c2, c2s, nq) + 3 * q4 - v;
            const u64 o = shoup_fold(tt, c1, c1s, nq);
            F.out[z * F.seg_out + lo + idx] = o >= q ? o - q : o;
        } else if (MODE == NTT_KSFINISH) {  // (acc - v) P^-1 + d, acc + 12q - v < 13q
            const u64 acc = EPI_X ? ex[EPI_X ? r : 0] : F.x[z * F.seg_x + lo + idx];
            u64 o = shoup_fold(acc + 3 * q4 - v, c1, c1s, nq);
            const u64 dv = EPI_D ? ed[EPI_D ? r : 0] : (has_d ? F.d[d_base + lo + idx] : 0);
            o = (o >= q ? o - q : o) + dv;  // d = 0 on c1 segments
            F.out[z * F.seg_out + lo + idx] = o >= q ? o - q : o;
        } else {
            a[tid_global * LEN + idx] = canon12(v, q, q2);
        }
    };
    if constexpr (SH) {
        if constexpr (TWL) {  // the block's rows blockIdx.y R .. + R - 1, R = 16 >> lsegb (dynamic LDS, R x 256)
            extern __shared__ __attribute__((aligned(16))) unsigned char row_twl_lds[];
            TW *const twl = reinterpret_cast<TW *>(row_twl_lds);
            const int R = 16 >> F.lsegb;
            const size_t row0 = (size_t)blockIdx.y * R;
            row_twiddles_multi<true>(twl, tw, row0, R, n, S0);
            __syncthreads();
            row_pass_shfl<true, true, FP>(x, t, tid_global, twl + 256 * (int)(tid_global - row0), n, S0, A);
        } else {
            row_pass_shfl<true, false, FP>(x, t, tid_global, tw, n, S0, A);
        }
        if (!valid) return;
#pragma unroll
        for (int r = 0; r < E; ++r) store_row(r, row_final_index<true>(t, r), x[r]);
        return;
    }
    // ---- round 1: local stages 0..EB-1
#pragma unroll
    for (int s = 0; s < EB; ++s) {
        const int hb = EB - 1 - s;  // pair bit in r
#pragma unroll
        for (int b = 0; b < E / 2; ++b) {  // butterfly b: r0 = b with a 0 inserted at bit hb
            const int r0 = ((b >> hb) << (hb + 1)) | (b & ((1 << hb) - 1));
            const int idx0 = t + T * r0;
            // COLS: (t + T r0) >> (PB - s) = r0 >> (EB - s) since t < T -- a
            // compile-time index into the prime's table, so the twiddle is a
            // scalar load (constant address space) instead of 4 VGPRs
            const size_t i = COLS ? ((size_t)r0 >> (EB - s)) : (tid_global << s) + (size_t)(idx0 >> (PB - s));
            const size_t wi = ((size_t)1 << (S0 + s)) + i;
            ct_any<FP, PB>(COLS, s, x[r0], x[r0 + (1 << hb)], (COLS && FHE_NTT_COL_SCALAR) ? scalar_tw(tw, wi) : tw[wi],
                           A);
        }
    }
    // round-2 twiddles (G == 1: stage s needs 2^(s-EB) of them per lane, index
    // t 2^(s-EB) + (r0 >> (PB-s))), loaded before the exchange so their latency
    // overlaps the LDS round trip and barrier instead of stalling round 2
    // (row passes only: in the column pass the extra VGPRs cost a wave of occupancy)
    constexpr bool PRE = G == 1 && !COLS;
    constexpr int NT2 = (1 << RB) - 1;
    TW tw2[PRE ? NT2 : 1];
    if (PRE) {
#pragma unroll
        for (int s = EB, o = 0; s < PB; ++s)
#pragma unroll
            for (int u = 0; u < (1 << (s - EB)); ++u, ++o) {
                const size_t i = (COLS ? 0 : (tid_global << s)) + ((size_t)t << (s - EB)) + (size_t)u;
                tw2[PRE ? o : 0] = tw[((size_t)1 << (S0 + s)) + i];
            }
    }
    // ---- exchange through LDS: L1 -> L2 (idx = (t*G + g) * 2^RB + r)
    if constexpr (SPLIT) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            if (g) __syncthreads();  // the previous phase's reads are done
#pragma unroll
            for (int u = 0; u < T; ++u) tile[lds_at<TPB, NB, COLS>(tr, u * T + t)] = x[G * u + g];
            __syncthreads();
#pragma unroll
            for (int r = 0; r < T; ++r) x[G * r + g] = tile[lds_at<TPB, NB, COLS>(tr, t * T + r)];
        }
    } else if constexpr (X32) {
        exchange32<E>(
            t32, x, [&](int r) { return lds_at<PB, NB, COLS>(tr, t + T * r); },
            [&](int j) { return lds_at<PB, NB, COLS>(tr, (t * G + j / T) * T + j % T); });
    } else {
#pragma unroll
        for (int r = 0; r < E; ++r) tile[lds_at<PB, NB, COLS>(tr, t + T * r)] = x[r];
        __syncthreads();
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int r = 0; r < T; ++r) x[g * T + r] = tile[lds_at<PB, NB, COLS>(tr, (t * G + g) * T + r)];
    }
    // ---- round 2: local stages EB..PB-1 (pair bit PB-1-s < RB)
#pragma unroll
    for (int s = EB; s < PB; ++s) {
        const int hb = PB - 1 - s;
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int r0 = 0; r0 < T; ++r0) {
                if (r0 & (1 << hb)) continue;
                const int idx0 = (t * G + g) * T + r0;
                const size_t i = (COLS ? 0 : (tid_global << s)) + (size_t)(idx0 >> (PB - s));
                const size_t wi = ((size_t)1 << (S0 + s)) + i;
                const TW w = PRE ? tw2[PRE ? ((1 << (s - EB)) - 1) + (r0 >> (PB - s)) : 0] : CTW ? twc[wi] : tw[wi];
                ct_any<FP, PB>(COLS, s, x[l2reg<G, T, SPLIT>(g, r0)], x[l2reg<G, T, SPLIT>(g, r0 + (1 << hb))], w, A);
            }
    }
    // ---- store.  COLS: layout L2 is already lane-contiguous in memory
    // (adjacent lanes = adjacent columns).  ROWS: a lane now owns T
    // consecutive coefficients, so the values go back through LDS to layout
    // L1 and every store instruction writes contiguous 128-B runs.  Each lane
    // rewrites only the tile words it read itself, so one barrier suffices.
    if constexpr (FP && COLS) {  // the row pass loads them back with the same offset
        const double fo = FP_TWO52 + FP_FWD_COL_OUT * A.q;
#pragma unroll
        for (int r = 0; r < E; ++r) x[r] = fp_out(dbits(x[r]), fo);
    }
    if constexpr (CBUF) {
        const auto rs = limb_rsrc(a);
        const int vo = (int)((((size_t)t * G * T << k2) + tid_global) * 8);
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int r = 0; r < T; ++r) bstore64(rs, vo, ((g * T + r) << k2) * 8, x[l2reg<G, T, SPLIT>(g, r)]);
    } else if (COLS) {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int r = 0; r < T; ++r) {
                const int idx = (t * G + g) * T + r;
                if (valid) a[(size_t)idx * ((size_t)1 << k2) + tid_global] = x[l2reg<G, T, SPLIT>(g, r)];
            }
    } else if constexpr (X32) {
        // each lane rewrites only tile words it read itself in the L1 -> L2
        // exchange (a permutation), so no barrier is needed before it
        exchange32<E>(
            t32, x, [&](int j) { return lds_at<PB, NB, COLS>(tr, (t * G + j / T) * T + j % T); },
            [&](int r) { return lds_at<PB, NB, COLS>(tr, t + T * r); });
#pragma unroll
        for (int r = 0; r < E; ++r)
            if (valid) store_row(r, t + T * r, x[r]);
    } else {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int r = 0; r < T; ++r)  // fused epilogues take the lazy [0, 4q) value
                tile[lds_at<PB, NB, COLS>(tr, (t * G + g) * T + r)] = x[g * T + r];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const int idx = t + T * r;
            const u64 v = tile[lds_at<PB, NB, COLS>(tr, idx)];
            if (valid) store_row(r, idx, v);
        }
    }
}

// Inverse: global GS stage sg has pair distance 2^sg, twiddle psi^-brev(m + i),
// m = n >> (sg + 1), i = j >> (sg + 1).  ROWS covers sg in [0, PB) (low bits),
// COLS covers sg in [logN - PB, logN) and multiplies by n^-1 on the way out.
// F.src (optional): read the input from there instead (out-of-place first
// pass; segment z, limb l at F.src + z * F.seg_src + l * n)
template <int PB, int EB, bool COLS, bool SH, bool FULL, bool TWL = false, bool FP = false>
__device__ __forceinline__ void ntt_inv_body(u64 *data, size_t seg, const int *pmap, const int *smap, int logN,
                                             const NttTables &Tb, const NttFuse &F) {
    static_assert(!SH || (!COLS && PB == 8 && EB == 4), "shuffle row pass: 16 lanes x 16 coefficients");
    constexpr int E = 1 << EB;
    constexpr int RB = PB - EB;
    constexpr int T = 1 << RB;
    constexpr int NB = nthreads<PB, COLS>() / T;
    constexpr int G = E >> RB;
    constexpr int LEN = 1 << PB;
    constexpr bool SPLIT = COLS && G >= 2;  // split exchange (see l2reg)
    constexpr int TPB = SPLIT ? PB - (EB - RB) : PB;
    constexpr bool X32 = lds32<COLS>() && !SPLIT;
    __shared__ u64 tile[SH ? 1 : X32 ? (lds_words<TPB, NB, COLS>() + 1) / 2 : lds_words<TPB, NB, COLS>()];
    uint32_t *const t32 = reinterpret_cast<uint32_t *>(tile);
    constexpr bool CTW = FHE_NTT_COL_TWL && COLS && !SPLIT && PB == 8 && nthreads<PB, COLS>() == 256;
    using TW = TwT<FP>;
    __shared__ TW twc[CTW ? 256 : 1];

    const size_t n = (size_t)1 << logN;
    const int k2 = COLS ? logN - PB : 0;
    // grid: x = segment (fastest, so the blocks of one prime's row/column
    // block across all segments run back to back and share its twiddles in
    // L2), y = block within the limb, z = limb (through the launch's limb runs)
    const int limb = F.limb_of(blockIdx.z);
    const int p = pmap ? __builtin_amdgcn_readfirstlane(pmap[limb]) : limb;
    int t, tr;
    if (COLS) {
        tr = threadIdx.x % NB;
        t = NB == 64 ? __builtin_amdgcn_readfirstlane(threadIdx.x / NB) : threadIdx.x / NB;
    } else {
        tr = threadIdx.x / T;
        t = threadIdx.x % T;
    }
    // SH: one row of 2^F.lsegb segments per block (shared per-row twiddles)
    const int zseg = SH ? (int)blockIdx.x * (1 << F.lsegb) + (tr & ((1 << F.lsegb) - 1)) : (int)blockIdx.x;
    const size_t tid_global = SH ? (size_t)blockIdx.y * (NB >> F.lsegb) + (tr >> F.lsegb) : (size_t)blockIdx.y * NB + tr;
    const bool valid = FULL || (tid_global < ((size_t)1 << (logN - PB)) && (!SH || zseg < F.segs));
    u64 *a = data + (size_t)zseg * seg + (smap ? (size_t)__builtin_amdgcn_readfirstlane(smap[limb]) : (size_t)limb) * n;
    const u64 q = Tb.mods[p].q, q2 = 2 * q, q4 = 4 * q, nq = (u64)0 - q;
    const TW *tw;
    if constexpr (FP) tw = Tb.invd + (size_t)p * n;
    else tw = Tb.inv2 + (size_t)p * n;
    Ar A{q4, nq, 0.0, 0.0};
    if constexpr (FP) {
        const double2 qd = Tb.qd[p];
        A.q = qd.x;
        A.qi = qd.y;
    }
    const double fin = FP ? FP_TWO52 + (COLS ? FP_INV_ROW_OUT : FP_INV_ROW_IN) * A.q : 0.0;  // FP load offset
    constexpr bool CBUF = FHE_NTT_COL_BUF && COLS && FULL;
    const int SG0 = COLS ? logN - PB : 0;  // global GS stage of local stage 0
    if (CTW) twc[threadIdx.x] = tw[threadIdx.x];  // round A reads it after the barrier below

    const u64 *ain = F.src ? F.src + (size_t)zseg * F.seg_src + (size_t)limb * n : a;
    u64 x[E];
    if constexpr (SH) {  // coalesced 16-B loads (idx = 2t + 32m + b -> x[2m + b]), register-only stages
#pragma unroll
        for (int m = 0; m < E / 2; ++m) {
            const ulonglong2 v = valid ? *reinterpret_cast<const ulonglong2 *>(ain + tid_global * LEN + 2 * t + 32 * m)
                                       : make_ulonglong2(0, 0);
            x[2 * m] = FP ? ubits(fp_in(v.x, fin)) : v.x;
            x[2 * m + 1] = FP ? ubits(fp_in(v.y, fin)) : v.y;
        }
        if constexpr (TWL) {  // the block's rows blockIdx.y R .. + R - 1, R = 16 >> lsegb (dynamic LDS, R x 256)
            extern __shared__ __attribute__((aligned(16))) unsigned char row_twl_lds[];
            TW *const twl = reinterpret_cast<TW *>(row_twl_lds);
            const int R = 16 >> F.lsegb;
            const size_t row0 = (size_t)blockIdx.y * R;
            row_twiddles_multi<false>(twl, tw, row0, R, n, 0);
            __syncthreads();
            row_pass_shfl<false, true, FP>(x, t, tid_global, twl + 256 * (int)(tid_global - row0), n, 0, A);
        } else {
            row_pass_shfl<false, false, FP>(x, t, tid_global, tw, n, 0, A);
        }
        if (!valid) return;
        const double fo = FP_TWO52 + FP_INV_ROW_OUT * A.q;
#pragma unroll
        for (int r = 0; r < E; ++r)
            a[tid_global * LEN + row_final_index<false>(t, r)] = FP ? fp_out(fp_reduce(dbits(x[r]), A.q, A.qi), fo) : x[r];
        return;
    }
    // ---- load, layout L2 (low bits within a lane group).  The ROWS pass's
    // per-lane runs of T consecutive words are read 16 B at a time (L1 serves
    // the rest of each line; routing them through LDS measured slower).
    if constexpr (CBUF) {
        const auto rs = limb_rsrc(ain);
        const int vo = (int)((((size_t)t * G * T << k2) + tid_global) * 8);
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int r = 0; r < T; ++r) x[l2reg<G, T, SPLIT>(g, r)] = bload64(rs, vo, ((g * T + r) << k2) * 8);
    } else if (COLS || (T & 1)) {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int r = 0; r < T; ++r) {
                const int idx = (t * G + g) * T + r;
                const size_t off = COLS ? (size_t)idx * ((size_t)1 << k2) + tid_global : tid_global * LEN + idx;
                x[l2reg<G, T, SPLIT>(g, r)] = valid ? ain[off] : 0;
            }
    } else {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int r = 0; r < T; r += 2) {
                const int idx = (t * G + g) * T + r;
                const ulonglong2 v = valid ? *reinterpret_cast<const ulonglong2 *>(ain + tid_global * LEN + idx)
                                           : make_ulonglong2(0, 0);
                x[g * T + r] = v.x;
                x[g * T + r + 1] = v.y;
            }
    }
    if constexpr (FP) {
#pragma unroll
        for (int r = 0; r < E; ++r) x[r] = ubits(fp_in(x[r], fin));
    }
    // ---- round A: local stages 0..RB-1 (pair bit s)
    if (CTW) __syncthreads();  // the staged twiddle table (the data loads are in flight)
#pragma unroll
    for (int s = 0; s < RB; ++s) {
        // twiddle index (row offset + idx0) >> (s + 1) with idx0 = t E + c, c < E:
        // E is a multiple of 2^(s+1), so it splits into a per-lane base and the
        // compile-time c >> (s + 1) (COLS: the column bits of idx0 << k2 vanish)
        const int sg = SG0 + s;
        const size_t lane_base = ((COLS ? 0 : tid_global * LEN) + (size_t)t * E) >> (s + 1);
        const TW *tws = (CTW ? twc : tw) + (n >> (sg + 1)) + lane_base;
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int r0 = 0; r0 < T; ++r0) {
                if (r0 & (1 << s)) continue;
                gs_any<FP>(x[l2reg<G, T, SPLIT>(g, r0)], x[l2reg<G, T, SPLIT>(g, r0 + (1 << s))],
                           tws[(g * T + r0) >> (s + 1)], A);
            }
    }
    // ---- exchange L2 -> L1 (idx = t + T * r)
    if constexpr (SPLIT) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            if (g) __syncthreads();
#pragma unroll
            for (int r = 0; r < T; ++r) tile[lds_at<TPB, NB, COLS>(tr, t * T + r)] = x[G * r + g];
            __syncthreads();
#pragma unroll
            for (int u = 0; u < T; ++u) x[G * u + g] = tile[lds_at<TPB, NB, COLS>(tr, u * T + t)];
        }
    } else if constexpr (X32) {
        exchange32<E>(
            t32, x, [&](int j) { return lds_at<PB, NB, COLS>(tr, (t * G + j / T) * T + j % T); },
            [&](int r) { return lds_at<PB, NB, COLS>(tr, t + T * r); });
    } else {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int r = 0; r < T; ++r) tile[lds_at<PB, NB, COLS>(tr, (t * G + g) * T + r)] = x[g * T + r];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < E; ++r) x[r] = tile[lds_at<PB, NB, COLS>(tr, t + T * r)];
    }
    // ---- round B: local stages RB..PB-1 (pair bit s >= RB, i.e. bit s-RB of r)
#pragma unroll
    for (int s = RB; s < PB; ++s) {
        const int hb = s - RB;
#pragma unroll
        for (int b = 0; b < E / 2; ++b) {
            const int r0 = ((b >> hb) << (hb + 1)) | (b & ((1 << hb) - 1));
            const int idx0 = t + T * r0;
            const int sg = SG0 + s;
            const size_t j = COLS ? 0 : tid_global * LEN;
            // COLS: i = idx0 >> (s + 1) with t < T <= 2^(s+1), i.e. (T r0) >> (s + 1):
            // a compile-time offset from a wave-uniform base -> scalar loads, no VGPRs
            const size_t i = COLS ? ((size_t)T * r0) >> (s + 1)
                                  : (j + (size_t)idx0) >> (sg + 1);
            const size_t wi = (n >> (sg + 1)) + i;
            gs_any<FP>(x[r0], x[r0 + (1 << hb)], (COLS && FHE_NTT_COL_SCALAR) ? scalar_tw(tw, wi) : tw[wi], A);
        }
    }
    // ---- store, layout L1 (COLS: times n^-1, or raw: reduced to [0, 2q) for
    // the conversions' 30-bit operand split; ROWS: lazy [0, 4q))
    const u64 ni = Tb.ninv[p], nis = Tb.ninv_s[p];
    const bool scale = COLS && !F.raw;
    const auto rso = limb_rsrc(a);
    const int vso = (int)((((size_t)t << k2) + tid_global) * 8);
    const double nid = FP ? fp_in(ni, FP_TWO52) : 0.0;
#pragma unroll
    for (int r = 0; r < E; ++r) {
        const int idx = t + T * r;
        const size_t off = COLS ? (size_t)idx * ((size_t)1 << k2) + tid_global : tid_global * LEN + idx;
        u64 v;
        if constexpr (FP) {
            // column: times n^-1 (|r| <= 0.7 q, canonicalised) or reduced and + q
            // ([0, 2q), the raw range); row (LDS passes): reduced + q, as the DPP rows
            const double xr = dbits(x[r]);
            if (scale) {
                const double m = fp_mulmod(xr, nid, A.q, A.qi);
                v = fp_out(m < 0.0 ? m + A.q : m, FP_TWO52);
            } else {
                v = fp_out(fp_reduce(xr, A.q, A.qi), FP_TWO52 + FP_INV_ROW_OUT * A.q);
            }
        } else {
            v = scale ? mul_shoup(x[r], ni, nis, q) : COLS ? (x[r] >= q2 ? x[r] - q2 : x[r]) : x[r];
        }
        if constexpr (CBUF)
            bstore64(rso, vso, (T * r << k2) * 8, v);
        else if (valid)
            a[off] = v;
    }
}

// FULL: the grid covers the transforms exactly (every launch on rings >= 2^11),
// so no lane needs the bounds check and the loads / stores carry no exec-mask
// branches.  (Waves-per-EU hints and "lean" epilogue variants were measured
// slower in round 2 and removed)
// minimum waves per SIMD the compiler must allow (register budget) for the
// forward column passes (A/B: -DFHE_NTT_COL_WPE=n)
#ifndef FHE_NTT_COL_WPE
#define FHE_NTT_COL_WPE 1
#endif
// FP: the fp64 butterflies (every limb of the launch has a prime < 2^FP_QBITS)
template <int PB, int EB, bool COLS, int MODE, bool FULL, bool FP>
__global__ __launch_bounds__((nthreads<PB, COLS>())) __attribute__((amdgpu_waves_per_eu(COLS ? FHE_NTT_COL_WPE : 1, 8))) void k_ntt_fwd(
    u64 *data, size_t seg, const int *pmap, const int *smap, int logN, NttTables Tb, NttFuse F) {
    ntt_fwd_body<PB, EB, COLS, MODE, false, FULL, false, FP>(data, seg, pmap, smap, logN, Tb, F);
}
template <int PB, int EB, bool COLS, bool FULL, bool FP>
__global__ __launch_bounds__((nthreads<PB, COLS>())) __attribute__((amdgpu_waves_per_eu(COLS ? FHE_NTT_COL_WPE : 1, 8))) void k_ntt_inv(
    u64 *data, size_t seg, const int *pmap, const int *smap, int logN, NttTables Tb, NttFuse F) {
    ntt_inv_body<PB, EB, COLS, false, FULL, false, FP>(data, seg, pmap, smap, logN, Tb, F);
}
// register-only row passes (PB = 8)
// minimum waves per SIMD for the register-only row passes with LDS twiddles
// (their twiddles are cheap to re-read, so a register budget need not spill)
#ifndef FHE_NTT_ROW_WPE
#define FHE_NTT_ROW_WPE 1
#endif
// minimum waves per SIMD of the FP forward rows (A/B: -DFHE_NTT_FP_ROW_WPE=n)
#ifndef FHE_NTT_FP_ROW_WPE
#define FHE_NTT_FP_ROW_WPE 1
#endif
// the FP rescale rows alone (A/B: -DFHE_NTT_FP_RESCALE_WPE=n)
#ifndef FHE_NTT_FP_RESCALE_WPE
#define FHE_NTT_FP_RESCALE_WPE FHE_NTT_FP_ROW_WPE
#endif
template <int MODE, bool FULL, bool TWL, bool FP>
__global__ __launch_bounds__(NTB) __attribute__((amdgpu_waves_per_eu(FP ? (MODE == NTT_RESCALE ? FHE_NTT_FP_RESCALE_WPE : FHE_NTT_FP_ROW_WPE) : TWL ? FHE_NTT_ROW_WPE : 1, 8))) void k_ntt_fwd_row(
    u64 *data, size_t seg, const int *pmap, const int *smap, int logN, NttTables Tb, NttFuse F) {
    ntt_fwd_body<8, 4, false, MODE, true, FULL, TWL, FP>(data, seg, pmap, smap, logN, Tb, F);
}
template <bool FULL, bool TWL, bool FP>
__global__ __launch_bounds__(NTB) __attribute__((amdgpu_waves_per_eu(TWL ? FHE_NTT_ROW_WPE : 1, 8))) void k_ntt_inv_row(
    u64 *data, size_t seg, const int *pmap, const int *smap, int logN, NttTables Tb, NttFuse F) {
    ntt_inv_body<8, 4, false, true, FULL, TWL, FP>(data, seg, pmap, smap, logN, Tb, F);
}
// ModUp's forward row pass fused with the key-switch inner product (HMult
// relinearisation; kernels.hpp ntt_row_ks).  Block: 16 transforms of one
// target limb t = 2^lmb members x 16 / 2^lmb rows (2^lmb = 16 for wide
// batches; 4 or 8 when a sharded rank holds fewer members, so no lane idles),
// one 16-lane transform each, the rows' twiddles staged in LDS.  For each digit j the lane group either loads
// the own-digit limb dntt[t] (NTT form already) or runs the row pass on
// ext[j][t] (after its column pass), then multiplies by the key rows of digit
// j and accumulates; acc[m][0][t] and acc[m][1][t] are written once.  The
// sums are the canonical residues ks_inner computes (integer limbs:
// mul_barrett + add_mod exactly as k_ks_inner_mc; FP limbs: fp_mulmod terms,
// one final reduction -- the same residue), so the words are unchanged.
#ifndef FHE_ROW_KS_WPE
#define FHE_ROW_KS_WPE 2
#endif
// D = 1 (no accumulation across digits): 4 waves per SIMD
#ifndef FHE_ROW_KS_WPE1
#define FHE_ROW_KS_WPE1 4
#endif
template <int D, bool FP, bool FULL>
__global__ __launch_bounds__(NTB) __attribute__((amdgpu_waves_per_eu(D == 1 ? FHE_ROW_KS_WPE1 : FHE_ROW_KS_WPE, 8))) void k_ntt_row_ks(u64 *acc, const u64 *ext, const u64 *dntt, const u64 *key,
                                                    int ell, int W, int nall, int alpha, int members,
                                                    const int *pmap_ext, int logN, NttTables Tb, KsStrides st,
                                                    KsFold fold, NttFuse Fz, int lmb) {
    using TW = TwT<FP>;
    __shared__ TW twl[TWL_ROWS * 256];
    const size_t n = (size_t)1 << logN;
    const int t = Fz.limb_of(blockIdx.z);
    const int pt = __builtin_amdgcn_readfirstlane(pmap_ext[t]);
    const int tr = threadIdx.x >> 4, tl = threadIdx.x & 15;
    const int R = 16 >> lmb;  // rows per block
    const int mb = ((int)blockIdx.x << lmb) + (tr & ((1 << lmb) - 1));
    const bool valid = FULL || mb < members;
    const size_t row0 = (size_t)blockIdx.y * R, row = row0 + (tr >> lmb), rb = row * 256;
    const Mod md = Tb.mods[pt];
    const u64 q = md.q, q2 = 2 * q;
    Ar A{4 * q, (u64)0 - q, 0.0, 0.0};
    const TW *tw;
    if constexpr (FP) {
        tw = Tb.fwdd + (size_t)pt * n;
        const double2 qd = Tb.qd[pt];
        A.q = qd.x;
        A.qi = qd.y;
    } else {
        tw = Tb.fwd2 + (size_t)pt * n;
    }
    const int S0 = logN - 8;
    row_twiddles_multi<true>(twl, tw, row0, R, n, S0);
    __syncthreads();
    const TW *twr = twl + 256 * (tr >> lmb);
    const size_t m = valid ? (size_t)mb : 0;
    // element r of a lane sits at in-row index row_final_index<true>(tl, r) =
    // lane part + a compile-time register part
    const int li = row_final_index<true>(tl, 0);
#define IDX(r) (li + (row_final_index<true>(0, r)))
    const bool folded = fold.d && t == ell - 1;
    const u64 *fd = fold.d + m * fold.member;
    // x = digit j's row of the target limb in NTT form (own digit: dntt itself)
    auto digit_row = [&](int j, u64(&x)[16]) {
        const int lo = j * alpha, hi = min((j + 1) * alpha, ell);
        if (t >= lo && t < hi) {  // own digit: the switched polynomial itself (NTT form)
            const u64 *src = dntt + m * st.d + (size_t)t * n + rb;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const u64 v = valid ? src[IDX(r)] : 0;
                x[r] = FP ? ubits(fp_in(v, FP_TWO52)) : v;
            }
        } else {
            const u64 *src = ext + m * st.ext + ((size_t)j * W + t) * n + rb;
            const double fin = FP ? FP_TWO52 + FP_FWD_COL_OUT * A.q : 0.0;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const u64 v = valid ? src[tl + 16 * r] : 0;
                x[r] = FP ? ubits(fp_in(v, fin)) : v;
            }
            row_pass_shfl<true, true, FP>(x, tl, row, twr, n, S0, A);
            if constexpr (!FP) {
#pragma unroll
                for (int r = 0; r < 16; ++r) x[r] = canon12(x[r], q, q2);
            }
        }
    };
    // a += x * key_j
    auto mac = [&](int j, const u64(&x)[16], u64(&a0)[16], u64(&a1)[16]) {
        const u64 *kb = key + (((size_t)j * 2 + 0) * nall + pt) * n + rb;
        const u64 *ka = key + (((size_t)j * 2 + 1) * nall + pt) * n + rb;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const u64 b = kb[IDX(r)], c = ka[IDX(r)];
            if constexpr (FP) {
                const double xv = dbits(x[r]);
                a0[r] = ubits(dbits(a0[r]) + fp_mulmod(xv, fp_in(b, FP_TWO52), A.q, A.qi));
                a1[r] = ubits(dbits(a1[r]) + fp_mulmod(xv, fp_in(c, FP_TWO52), A.q, A.qi));
            } else {
                a0[r] = add_mod(a0[r], mul_barrett(x[r], b, md), q);
                a1[r] = add_mod(a1[r], mul_barrett(x[r], c, md), q);
            }
        }
    };
    // the folded (dropped) limb's term, scaled
    auto fold_of = [&](int r, u64 &f0, u64 &f1) {
        f0 = f1 = 0;
        if (folded && valid) {
            f0 = mul_shoup(fd[rb + IDX(r)], fold.w, fold.ws, q);
            f1 = mul_shoup(fd[fold.seg + rb + IDX(r)], fold.w, fold.ws, q);
        }
    };
    u64 *o0 = acc + m * st.acc + (size_t)t * n + rb;
    u64 *o1 = acc + m * st.acc + ((size_t)W + t) * n + rb;
    // canonical store of one accumulator value
    auto fin = [&](u64 v) -> u64 {
        if constexpr (FP) {  // |a| <= (D 0.51 + 1) q: one reduction, canonical
            const double r0 = fp_reduce(dbits(v), A.q, A.qi);
            return fp_out(r0 < 0.0 ? r0 + A.q : r0, FP_TWO52);
        } else {
            return v;
        }
    };
    if constexpr (D == 1) {  // one digit: each value stored as it is made (no accumulator arrays)
        u64 x[16];
        digit_row(0, x);
        const u64 *kb = key + (size_t)pt * n + rb;
        const u64 *ka = key + ((size_t)nall + pt) * n + rb;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            u64 f0, f1, v0, v1;
            fold_of(r, f0, f1);
            const u64 b = kb[IDX(r)], c = ka[IDX(r)];
            if constexpr (FP) {
                const double xv = dbits(x[r]);
                v0 = ubits(fp_in(f0, FP_TWO52) + fp_mulmod(xv, fp_in(b, FP_TWO52), A.q, A.qi));
                v1 = ubits(fp_in(f1, FP_TWO52) + fp_mulmod(xv, fp_in(c, FP_TWO52), A.q, A.qi));
            } else {
                v0 = add_mod(f0, mul_barrett(x[r], b, md), q);
                v1 = add_mod(f1, mul_barrett(x[r], c, md), q);
            }
            if (valid) {
                o0[IDX(r)] = fin(v0);
                o1[IDX(r)] = fin(v1);
            }
        }
        return;
    }
    u64 a0[16], a1[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        u64 f0, f1;
        fold_of(r, f0, f1);
        a0[r] = FP ? ubits(fp_in(f0, FP_TWO52)) : f0;
        a1[r] = FP ? ubits(fp_in(f1, FP_TWO52)) : f1;
    }
#pragma unroll 1
    for (int j = 0; j < D; ++j) {
        u64 x[16];
        digit_row(j, x);
        mac(j, x, a0, a1);
    }
    if (!valid) return;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        o0[IDX(r)] = fin(a0[r]);
        o1[IDX(r)] = fin(a1[r]);
    }
#undef IDX
}

// FHE_NTT_TWL (A/B, default 1): the register-only row passes stage a row's
// twiddles in LDS when the block is one row of 16 segments
int &row_twl_enabled() {
    static int v = [] {
        const char *e = std::getenv("FHE_NTT_TWL");
        return e ? std::atoi(e) : 1;
    }();
    return v;
}

// FHE_NTT_TWL_ROWS (A/B, default 4): most rows per block whose twiddles are
// staged in LDS -- blocks of >= 4 segments.  Staging the 8 / 16 rows of the
// one- and two-segment blocks too (32 / 64 KB of dynamic LDS) measured slower:
// k-way 2845 ms at 4, 2883 at 8, 2978 at 16; the N=1024 sort 538.1 / 538.2 at
// 4 against 539.7 / 543.8 at 16; MEHP24 11.24 s against 11.26 s (profiles/r5_m)
int &row_twl_rows() {
    static int v = [] {
        const char *e = std::getenv("FHE_NTT_TWL_ROWS");
        return e ? std::atoi(e) : 4;
    }();
    return v;
}

// FHE_NTT_FULL (A/B timing): which passes take the exact-grid variant (bit mask:
// 1 forward column, 2 forward column + lift, 4 forward row, 8 rescale row,
// 16 HMult-tail row, 32 inverse column, 64 inverse row, 128 key-switch-finish row)
int &ntt_full_mask() {
    static int v = [] {
        const char *e = std::getenv("FHE_NTT_FULL");
        return e ? std::atoi(e) : 53 | 128;  // measured: the rescale row, inverse row and lift column passes keep the checks (more VGPRs without them)
    }();
    return v;
}
template <bool COLS, bool FWD, int MODE>
constexpr int full_bit() {
    return FWD ? (COLS ? (MODE == NTT_LIFT ? 2 : 1)
                       : MODE == NTT_RESCALE ? 8 : MODE == NTT_MULTAIL ? 16 : MODE == NTT_KSFINISH ? 128 : 4)
               : (COLS ? 32 : 64);
}

template <int PB, int EB, bool COLS, bool FWD, int MODE, bool FP>
void launch_pass_one(u64 *data, int limbs, int segs, size_t seg, const int *pmap, const int *smap, const NttTables &T,
                     const NttFuse &F, hipStream_t st) {
    constexpr int NTHR = nthreads<PB, COLS>();
    constexpr int NB = NTHR >> (PB - EB);
    constexpr bool CAN_SH = !COLS && PB == 8 && EB == 4;
    // bits: 1 inverse rows, 2 every forward row, 4 / 8 / 16 the forward HMult-tail /
    // rescale / key-switch-finish rows only
    const int mode = row_shfl_enabled();
    const int fwd_bit = MODE == NTT_MULTAIL ? 4 : MODE == NTT_RESCALE ? 8 : MODE == NTT_KSFINISH ? 16 : 0;
    const bool sh = CAN_SH && (mode & (FWD ? 2 | fwd_bit : 1)) != 0;
    const int count = 1 << (T.logN - PB);  // columns (COLS) or rows (ROWS)
    dim3 grid((unsigned)segs, (unsigned)((count + NB - 1) / NB), (unsigned)limbs);
    const bool want_full = (ntt_full_mask() & full_bit<COLS, FWD, MODE>()) != 0;
    bool full = want_full && count % NB == 0;
    NttFuse Fs = F;
    if (sh) {  // 2^lsegb segments of one row per block (lsegb <= 4: 16 transforms per block)
        Fs.lsegb = 0;
        while (Fs.lsegb < 4 && (2 << Fs.lsegb) <= segs) ++Fs.lsegb;
        Fs.segs = segs;
        const int rows_pb = NB >> Fs.lsegb;
        grid = dim3((unsigned)((segs + (1 << Fs.lsegb) - 1) >> Fs.lsegb), (unsigned)((count + rows_pb - 1) / rows_pb),
                    (unsigned)limbs);
        full = want_full && count % rows_pb == 0 && segs % (1 << Fs.lsegb) == 0;
    }
    LaunchClock *clk = launch_clock();
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const int slot = clk ? clk->events(e0, e1) : -1;
    note_launch(FWD ? (COLS ? "k_ntt_fwd(col)" : "k_ntt_fwd(row)") : (COLS ? "k_ntt_inv(col)" : "k_ntt_inv(row)"), grid,
                dim3(NTHR));
    // staged row twiddles (dynamic LDS: the block's 16 >> lsegb rows x 256 entries)
    // when a block holds at most row_twl_rows() rows
    const int rows_blk = 16 >> Fs.lsegb;
    const bool twl = sh && rows_blk <= row_twl_rows() && row_twl_enabled() != 0;
    const unsigned lds_dyn = twl ? (unsigned)(rows_blk * 256 * (FP ? sizeof(double) : sizeof(TwT<false>))) : 0u;
#define FHE_NTT_LAUNCH(K, FF) \
    hipExtLaunchKernelGGL((K), grid, dim3(NTHR), lds_dyn, st, e0, e1, 0, data, seg, pmap, smap, T.logN, T, FF)
    if (FWD && sh) {
        if (full && twl) FHE_NTT_LAUNCH((k_ntt_fwd_row<MODE, true, true, FP>), Fs);
        else if (full) FHE_NTT_LAUNCH((k_ntt_fwd_row<MODE, true, false, FP>), Fs);
        else if (twl) FHE_NTT_LAUNCH((k_ntt_fwd_row<MODE, false, true, FP>), Fs);
        else FHE_NTT_LAUNCH((k_ntt_fwd_row<MODE, false, false, FP>), Fs);
    } else if (FWD) {
        if (full) FHE_NTT_LAUNCH((k_ntt_fwd<PB, EB, COLS, MODE, true, FP>), F);
        else FHE_NTT_LAUNCH((k_ntt_fwd<PB, EB, COLS, MODE, false, FP>), F);
    } else if (sh) {
        if (full && twl) FHE_NTT_LAUNCH((k_ntt_inv_row<true, true, FP>), Fs);
        else if (full) FHE_NTT_LAUNCH((k_ntt_inv_row<true, false, FP>), Fs);
        else if (twl) FHE_NTT_LAUNCH((k_ntt_inv_row<false, true, FP>), Fs);
        else FHE_NTT_LAUNCH((k_ntt_inv_row<false, false, FP>), Fs);
    } else {
        if (full) FHE_NTT_LAUNCH((k_ntt_inv<PB, EB, COLS, true, FP>), F);
        else FHE_NTT_LAUNCH((k_ntt_inv<PB, EB, COLS, false, FP>), F);
    }
#undef FHE_NTT_LAUNCH
    if (clk) {
        // same spelling as the demangled symbol rocprofv3 prints, plus the caller tag
        // (the instantiation the branches above launched)
        const std::string fps = FP ? "true>" : "false>";
        const std::string pe = std::to_string(PB) + ", " + std::to_string(EB) + (COLS ? ", true" : ", false");
        const std::string fl = (full ? "true, " : "false, ") + fps;
        const std::string fl2 = (full ? "true, " : "false, ") + std::string(twl ? "true, " : "false, ") + fps;
        const std::string base = FWD && sh ? "k_ntt_fwd_row<" + std::to_string(MODE) + ", " + fl2
                                 : FWD     ? "k_ntt_fwd<" + pe + ", " + std::to_string(MODE) + ", " + fl
                                 : sh      ? "k_ntt_inv_row<" + fl2
                                           : "k_ntt_inv<" + pe + ", " + fl;
        static std::map<std::string, std::string> names;  // stable c_str() per (kernel, caller)
        static std::mutex mu;
        const char *ph = launch_phase();
        const std::string key = ph ? base + "@" + ph : base;
        std::lock_guard<std::mutex> lk(mu);
        auto it = names.find(key);
        if (it == names.end()) it = names.emplace(key, key).first;
        // one read + one write of every limb touched (fused epilogues: + the extra operands)
        const double extra = MODE == NTT_RESCALE ? 1.0 : MODE == NTT_MULTAIL ? 2.0 : MODE == NTT_KSFINISH ? 1.5 : 0.0;
        clk->record(slot, it->second.c_str(), (2.0 + extra) * 8.0 * (double)limbs * segs * ((size_t)1 << T.logN));
    }
}

// FHE_NTT_FP (A/B, default 1): limbs whose prime is < 2^FP_QBITS run the fp64
// butterflies in launches of their own
int &ntt_fp_enabled() {
    static int v = [] {
        const char *e = std::getenv("FHE_NTT_FP");
        return e ? std::atoi(e) : 1;
    }();
    return v;
}
// host copies of the device prime maps (ntt_register_map), by device address;
// `gen` counts (un)registrations so the per-thread lookup cache below can tell
// when its entries went stale
struct MapRegistry {
    std::mutex mu;
    std::map<const int *, std::vector<int>> maps;
    std::atomic<unsigned long> gen{0};
};
MapRegistry &map_registry() {
    static MapRegistry r;
    return r;
}
// the prime of each limb of a launch, if its map is known on the host.  Every
// pass of every transform asks this (several times per HMult), so the answers
// are cached per thread by (map, limbs) -- no lock, search or copy on a hit
// (advisor r5); the cache empties itself when a map is (un)registered.  Both
// passes of one transform (the column pass here, the fused row pass in
// ntt_row_ks) ask the same registry, so they classify every limb alike.
bool launch_primes(const int *pmap, int limbs, std::vector<int> &out) {
    out.resize(limbs);
    if (!pmap) {
        for (int z = 0; z < limbs; ++z) out[z] = z;
        return true;
    }
    MapRegistry &R = map_registry();
    struct Entry {
        const int *pmap;
        int limbs;
        bool known;
        std::vector<int> primes;
    };
    static thread_local std::vector<Entry> cache;
    static thread_local unsigned long cache_gen = ~0ul;
    const unsigned long g = R.gen.load(std::memory_order_acquire);
    if (g != cache_gen) {
        cache.clear();
        cache_gen = g;
    }
    for (const Entry &e : cache)
        if (e.pmap == pmap && e.limbs == limbs) {
            if (e.known) out = e.primes;
            return e.known;
        }
    bool known = false;
    {
        std::lock_guard<std::mutex> lk(R.mu);
        auto it = R.maps.upper_bound(pmap);
        if (it != R.maps.begin()) {
            --it;
            const size_t off = (size_t)(pmap - it->first);
            if (off + (size_t)limbs <= it->second.size()) {
                for (int z = 0; z < limbs; ++z) out[z] = it->second[off + z];
                known = true;
            }
        }
    }
    if (cache.size() >= 256) cache.clear();
    cache.push_back(Entry{pmap, limbs, known, known ? out : std::vector<int>{}});
    return known;
}
// FHE_NTT_AUX (A/B, default 0 -- measured slower: 539.1 / 540.9 ms without,
// 548.6 / 548.2 ms with, profiles/r5_j; the event fork / join costs more than the
// overlap gains): a pass split into an FP and an integer launch
// whose smaller launch covers at most AUX_MAX_LIMBS limbs (q_0 beside the 40-bit
// limbs: one limb of a 1/40 share that alone would half-fill the chip for its
// whole latency) runs the small one on an auxiliary stream, forked from and
// joined back into the caller's stream by events, so it overlaps the big one.
// Both launches touch disjoint limbs; everything after the pass waits for both.
constexpr int AUX_MAX_LIMBS = 2;
int &ntt_aux_enabled() {
    static int v = [] {
        const char *e = std::getenv("FHE_NTT_AUX");
        return e ? std::atoi(e) : 0;
    }();
    return v;
}
struct AuxStream {
    hipStream_t s = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
};
AuxStream *aux_for(hipStream_t st) {  // one per caller stream (lanes are threads with streams of their own)
    static std::mutex mu;
    static std::map<hipStream_t, AuxStream> m;
    std::lock_guard<std::mutex> lk(mu);
    auto it = m.find(st);
    if (it != m.end()) return &it->second;
    AuxStream a;
    if (hipStreamCreateWithFlags(&a.s, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&a.fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&a.join, hipEventDisableTiming) != hipSuccess)
        return nullptr;
    return &m.emplace(st, a).first->second;
}
// One launch per class (integer / FP), each over the class's limbs as at most
// two contiguous runs (NttFuse::limb_of); more runs take more launches.  A
// launch whose limb map is unknown on the host stays one integer launch.
template <int PB, int EB, bool COLS, bool FWD, int MODE>
void launch_pass(u64 *data, int limbs, int segs, size_t seg, const int *pmap, const int *smap, const NttTables &T,
                 const NttFuse &F, hipStream_t st) {
    std::vector<int> pr;
    if (!ntt_fp_enabled() || !T.fp_host || !launch_primes(pmap, limbs, pr)) {
        launch_pass_one<PB, EB, COLS, FWD, MODE, false>(data, limbs, segs, seg, pmap, smap, T, F, st);
        return;
    }
    struct Piece {
        bool fp;
        NttFuse G;
        int cnt;
    };
    std::vector<Piece> pieces;
    for (int cls = 0; cls < 2; ++cls) {
        std::vector<std::pair<int, int>> runs;  // (start, length)
        for (int z = 0; z < limbs; ++z) {
            if ((T.fp_host[pr[z]] != 0) != (cls == 1)) continue;
            if (!runs.empty() && runs.back().first + runs.back().second == z) ++runs.back().second;
            else runs.emplace_back(z, 1);
        }
        for (size_t r = 0; r < runs.size(); r += 2) {
            NttFuse G = F;
            G.zs0 = runs[r].first;
            G.zn0 = runs[r].second;
            G.zs1 = r + 1 < runs.size() ? runs[r + 1].first : 0;
            const int cnt = runs[r].second + (r + 1 < runs.size() ? runs[r + 1].second : 0);
            pieces.push_back(Piece{cls == 1, G, cnt});
        }
    }
    auto go = [&](const Piece &p, hipStream_t s) {
        if (p.fp) launch_pass_one<PB, EB, COLS, FWD, MODE, true>(data, p.cnt, segs, seg, pmap, smap, T, p.G, s);
        else launch_pass_one<PB, EB, COLS, FWD, MODE, false>(data, p.cnt, segs, seg, pmap, smap, T, p.G, s);
    };
    AuxStream *aux = nullptr;
    // (not under the live clock: it books each launch's own span, so the
    // roofline sort keeps one kernel at a time)
    if (pieces.size() == 2 && ntt_aux_enabled() && !launch_clock() &&
        std::min(pieces[0].cnt, pieces[1].cnt) <= AUX_MAX_LIMBS)
        aux = aux_for(st);
    if (!aux) {
        for (auto &p : pieces) go(p, st);
        return;
    }
    const int small = pieces[0].cnt <= pieces[1].cnt ? 0 : 1;
    (void)hipEventRecord(aux->fork, st);
    (void)hipStreamWaitEvent(aux->s, aux->fork, 0);
    go(pieces[small], aux->s);
    (void)hipEventRecord(aux->join, aux->s);
    go(pieces[1 - small], st);
    (void)hipStreamWaitEvent(st, aux->join, 0);
}

// pass bits -> (PB, EB): EB = ceil(PB / 2)
template <bool COLS, bool FWD, int MODE>
void dispatch(int PB, u64 *data, int limbs, int segs, size_t seg, const int *pmap, const int *smap,
              const NttTables &T, const NttFuse &F, hipStream_t st) {
    switch (PB) {
    case 2: launch_pass<2, 1, COLS, FWD, MODE>(data, limbs, segs, seg, pmap, smap, T, F, st); break;
    case 3: launch_pass<3, 2, COLS, FWD, MODE>(data, limbs, segs, seg, pmap, smap, T, F, st); break;
    case 4: launch_pass<4, 2, COLS, FWD, MODE>(data, limbs, segs, seg, pmap, smap, T, F, st); break;
    case 5: launch_pass<5, 3, COLS, FWD, MODE>(data, limbs, segs, seg, pmap, smap, T, F, st); break;
    case 6: launch_pass<6, 3, COLS, FWD, MODE>(data, limbs, segs, seg, pmap, smap, T, F, st); break;
    case 7: launch_pass<7, 4, COLS, FWD, MODE>(data, limbs, segs, seg, pmap, smap, T, F, st); break;
    case 8: launch_pass<8, 4, COLS, FWD, MODE>(data, limbs, segs, seg, pmap, smap, T, F, st); break;
    case 9: launch_pass<9, 5, COLS, FWD, MODE>(data, limbs, segs, seg, pmap, smap, T, F, st); break;
    default: break;
    }
}

}  // namespace

void ntt_register_map(const int *dev, const int *host, size_t count) {
    MapRegistry &R = map_registry();
    std::lock_guard<std::mutex> lk(R.mu);
    R.maps[dev].assign(host, host + count);
    R.gen.fetch_add(1, std::memory_order_release);
}
void ntt_unregister_map(const int *dev) {
    MapRegistry &R = map_registry();
    std::lock_guard<std::mutex> lk(R.mu);
    R.maps.erase(dev);
    R.gen.fetch_add(1, std::memory_order_release);
}
bool ntt_fp_prime(u64 q) { return (q >> FP_QBITS) == 0; }

LaunchClock *&launch_clock() {
    static LaunchClock *clk = nullptr;
    return clk;
}
const char *&launch_phase() {
    static thread_local const char *ph = nullptr;
    return ph;
}
const char *&algo_phase() {
    static thread_local const char *ph = nullptr;
    return ph;
}
const char *intern_name(const std::string &s) {
    static std::map<std::string, std::string> names;
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    auto it = names.find(s);
    if (it == names.end()) it = names.emplace(s, s).first;
    return it->second.c_str();
}

void ntt_forward(u64 *data, int limbs, int segs, size_t seg, const int *pmap, const NttTables &T, hipStream_t st) {
    if (limbs <= 0 || segs <= 0) return;
    const int k1 = (T.logN + 1) / 2, k2 = T.logN - k1;
    const NttFuse F;
    dispatch<true, true, NTT_PLAIN>(k1, data, limbs, segs, seg, pmap, nullptr, T, F, st);
    dispatch<false, true, NTT_PLAIN>(k2, data, limbs, segs, seg, pmap, nullptr, T, F, st);
}

void ntt_inverse(u64 *data, int limbs, int segs, size_t seg, const int *pmap, const NttTables &T, hipStream_t st,
                 bool raw) {
    if (limbs <= 0 || segs <= 0) return;
    const int k1 = (T.logN + 1) / 2, k2 = T.logN - k1;
    NttFuse F;
    F.raw = raw;
    dispatch<false, false, NTT_PLAIN>(k2, data, limbs, segs, seg, pmap, nullptr, T, F, st);
    dispatch<true, false, NTT_PLAIN>(k1, data, limbs, segs, seg, pmap, nullptr, T, F, st);
}

void ntt_inverse_from(u64 *dst, const u64 *src, size_t seg_src, int limbs, int segs, size_t seg, const int *pmap,
                      const NttTables &T, hipStream_t st, bool raw) {
    if (limbs <= 0 || segs <= 0) return;
    const int k1 = (T.logN + 1) / 2, k2 = T.logN - k1;
    NttFuse F;
    F.src = src;
    F.seg_src = seg_src;
    dispatch<false, false, NTT_PLAIN>(k2, dst, limbs, segs, seg, pmap, nullptr, T, F, st);
    NttFuse G;
    G.raw = raw;
    dispatch<true, false, NTT_PLAIN>(k1, dst, limbs, segs, seg, pmap, nullptr, T, G, st);
}

void ntt_row_pass(u64 *data, int limbs, int segs, size_t seg, const int *pmap, const NttTables &T, hipStream_t st,
                  bool forward) {  // one row pass alone (kernel timing)
    if (limbs <= 0 || segs <= 0) return;
    const int k2 = T.logN - (T.logN + 1) / 2;
    const NttFuse F;
    if (forward)
        dispatch<false, true, NTT_PLAIN>(k2, data, limbs, segs, seg, pmap, nullptr, T, F, st);
    else
        dispatch<false, false, NTT_PLAIN>(k2, data, limbs, segs, seg, pmap, nullptr, T, F, st);
}

void ntt_forward_mapped(u64 *data, int count, int segs, size_t seg, const int *smap, const int *pmap,
                        const NttTables &T, hipStream_t st) {
    if (count <= 0 || segs <= 0) return;
    const int k1 = (T.logN + 1) / 2, k2 = T.logN - k1;
    const NttFuse F;
    dispatch<true, true, NTT_PLAIN>(k1, data, count, segs, seg, pmap, smap, T, F, st);
    dispatch<false, true, NTT_PLAIN>(k2, data, count, segs, seg, pmap, smap, T, F, st);
}

void ntt_forward_rescale(u64 *tmp, int limbs, int segs, const NttFuse &F, const NttTables &T, hipStream_t st) {
    if (limbs <= 0 || segs <= 0) return;
    const int k1 = (T.logN + 1) / 2, k2 = T.logN - k1;
    const size_t seg = (size_t)limbs << T.logN;
    dispatch<true, true, NTT_LIFT>(k1, tmp, limbs, segs, seg, nullptr, nullptr, T, F, st);
    dispatch<false, true, NTT_RESCALE>(k2, tmp, limbs, segs, seg, nullptr, nullptr, T, F, st);
}

void ntt_forward_multail(u64 *corr, int limbs, int segs, const NttFuse &F, const NttTables &T, hipStream_t st) {
    if (limbs <= 0 || segs <= 0) return;
    const int k1 = (T.logN + 1) / 2, k2 = T.logN - k1;
    const size_t seg = (size_t)limbs << T.logN;
    dispatch<true, true, NTT_PLAIN>(k1, corr, limbs, segs, seg, nullptr, nullptr, T, F, st);
    dispatch<false, true, NTT_MULTAIL>(k2, corr, limbs, segs, seg, nullptr, nullptr, T, F, st);
}

void ntt_forward_ksfinish(u64 *conv, int limbs, int segs, const NttFuse &F, const NttTables &T, hipStream_t st) {
    if (limbs <= 0 || segs <= 0) return;
    const int k1 = (T.logN + 1) / 2, k2 = T.logN - k1;
    const size_t seg = (size_t)limbs << T.logN;
    dispatch<true, true, NTT_PLAIN>(k1, conv, limbs, segs, seg, nullptr, nullptr, T, F, st);
    dispatch<false, true, NTT_KSFINISH>(k2, conv, limbs, segs, seg, nullptr, nullptr, T, F, st);
}

void ntt_forward_mapped_cols(u64 *data, int count, int segs, size_t seg, const int *smap, const int *pmap,
                             const NttTables &T, hipStream_t st) {
    if (count <= 0 || segs <= 0) return;
    const int k1 = (T.logN + 1) / 2;
    const NttFuse F;
    dispatch<true, true, NTT_PLAIN>(k1, data, count, segs, seg, pmap, smap, T, F, st);
}

void ntt_forward_mapped_rows(u64 *data, int count, int segs, size_t seg, const int *smap, const int *pmap,
                             const NttTables &T, hipStream_t st) {
    if (count <= 0 || segs <= 0) return;
    const int k2 = T.logN - (T.logN + 1) / 2;
    const NttFuse F;
    dispatch<false, true, NTT_PLAIN>(k2, data, count, segs, seg, pmap, smap, T, F, st);
}

std::vector<std::pair<int, int>> ntt_class_runs(const int *pmap, int count, bool fp, const NttTables &T) {
    std::vector<int> pr;
    const bool known = launch_primes(pmap, count, pr);
    std::vector<std::pair<int, int>> runs;
    for (int z = 0; z < count; ++z) {
        const bool f = ntt_fp_enabled() && T.fp_host && known && T.fp_host[pr[z]] != 0;
        if (f != fp) continue;
        if (!runs.empty() && runs.back().first + runs.back().second == z) ++runs.back().second;
        else runs.emplace_back(z, 1);
    }
    return runs;
}

void ntt_row_ks(u64 *acc, const u64 *ext, const u64 *dntt, const u64 *key, int ell, int K, int nall, int alpha,
                int digits, const int *pmap_ext, int members, KsStrides str, KsFold fold, const NttTables &T,
                hipStream_t st, bool fp_only) {
    const int W = ell + K;
    if (T.logN != 16 && T.logN != 17) throw std::invalid_argument("ntt_row_ks: the row pass is 256 points (rings 2^16, 2^17)");
    if (digits < 1 || digits > 8) throw std::invalid_argument("ntt_row_ks: 1..8 digits");
    if (members < 1) return;
    std::vector<int> pr;
    const bool known = launch_primes(pmap_ext, W, pr);
    (void)pr;
    // the column pass (launch_pass) classed the limbs through the ModUp map; the
    // row pass here must class them the same way, so the map must be known
    if (!known && ntt_fp_enabled() && T.fp_host) throw std::invalid_argument("ntt_row_ks: unregistered prime map");
    // 2^lmb members per block (16 / 2^lmb rows): the largest power of two <= members, 4..16
    int lmb = 4;
    while (lmb > 2 && (1 << lmb) > members) --lmb;
    const bool full = members % (1 << lmb) == 0;
    const dim3 blk(NTB);
    for (int cls = fp_only ? 1 : 0; cls < 2; ++cls) {
        const std::vector<std::pair<int, int>> runs = ntt_class_runs(pmap_ext, W, cls == 1, T);
        for (size_t r = 0; r < runs.size(); r += 2) {
            NttFuse Fz;
            Fz.zs0 = runs[r].first;
            Fz.zn0 = runs[r].second;
            Fz.zs1 = r + 1 < runs.size() ? runs[r + 1].first : 0;
            const int cnt = runs[r].second + (r + 1 < runs.size() ? runs[r + 1].second : 0);
            const dim3 grid((unsigned)((members + (1 << lmb) - 1) >> lmb), (unsigned)((1u << (T.logN - 8)) >> (4 - lmb)),
                            (unsigned)cnt);
            // ext rows (digits - 1 or digits per target) + own-digit rows + 2 accumulators per member; keys once
            const double bytes = 8.0 * ((double)members * (digits + 2.0) + 2.0 * digits) * cnt * ((size_t)1 << T.logN);
            dispatch_int<1, 8>(digits, [&](auto c) {
                constexpr int DD = decltype(c)::value;
                auto go = [&](auto fpc, auto fullc) {
                    constexpr bool FPV = decltype(fpc)::value, FU = decltype(fullc)::value;
                    launch_clocked(inst_name<DD, FPV, FU>("k_ntt_row_ks"), bytes, k_ntt_row_ks<DD, FPV, FU>, grid, blk,
                                   st, acc, ext, dntt, key, ell, W, nall, alpha, members, pmap_ext, T.logN, T, str,
                                   fold, Fz, lmb);
                };
                if (cls && full) go(std::true_type{}, std::true_type{});
                else if (cls) go(std::true_type{}, std::false_type{});
                else if (full) go(std::false_type{}, std::true_type{});
                else go(std::false_type{}, std::false_type{});
            });
        }
    }
}

}  // namespace dev
}  // namespace fhe
