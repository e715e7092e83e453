// gfx950 kernels for the RNS-CKKS ciphertext-op engine.
//
// 64-bit integer modular arithmetic on the VALU, except the sums of products
// that can run as an integer GEMM on the i8 matrix cores (k_*_mfma, see
// "RNS sums of products on MFMA" below and DESIGN.md §5).  Design notes:
//   * the NTT lives in ntt.hip (register-blocked, two passes per transform).
//   * element-wise kernels move 16 B per lane (ulonglong2) and are launched
//     3-D: x = coefficient blocks, y = limb (prime), z = polynomial segment.
//   * basis conversions (ModUp / ModDown) hold the source residues of one
//     coefficient in registers and emit a chunk of target limbs per thread;
//     every constant multiply is a Shoup multiply with a precomputed
//     companion.
#include <fcntl.h>
#include <signal.h>
#include <sys/syscall.h>
#include <ucontext.h>
#include <unistd.h>

#include <atomic>
#include <cstdlib>
#include <mutex>
#include "kernels.hpp"

#include <cstdlib>
#include <stdexcept>
#include <utility>
#include <type_traits>
#include <string>

namespace fhe {
namespace dev {

namespace {

constexpr int NT = 256;     // threads per block
// Basis conversions give each thread one coefficient and a chunk of target
// limbs: all of them (the per-coefficient prologue -- loading and scaling the
// source residues -- then runs once) unless the launch is too narrow to fill the
// chip (a single ciphertext at ring 2^16: n / NT x digits = 768 blocks, 3 waves
// per SIMD, each looping over ~40 targets), then the targets are chunked so the
// grid has >= 3072 blocks (12 per CU), >= 4 targets per chunk.  The outputs are
// independent, so the words do not depend on the chunking.
inline int conv_chunk(int logN, int targets, int zdim) {
    static const int force = [] {
        const char *e = std::getenv("FHE_CONV_CHUNK");  // A/B: a fixed chunk (0 = adaptive)
        return e ? std::atoi(e) : 0;
    }();
    if (targets < 1) return 1;
    if (force > 0) return force;
    const size_t base = (((size_t)1 << logN) + NT - 1) / NT * (size_t)std::max(zdim, 1);
    if (targets <= 4 || base >= 3072) return targets;
    const int chunks = (int)((3072 + base - 1) / base);
    return std::max(4, (targets + chunks - 1) / chunks);
}

// compile-time dispatch of a small runtime integer (digit size, special-prime count)
template <int Lo, int Hi, typename F>
void dispatch_int(int v, F &&f) {
    if constexpr (Lo > Hi) {
        throw std::invalid_argument("unsupported basis size " + std::to_string(v));
    } else {
        if (v == Lo)
            f(std::integral_constant<int, Lo>{});
        else
            dispatch_int<Lo + 1, Hi>(v, std::forward<F>(f));
    }
}

// i8-MFMA sums of products; FHE_MFMA is a mask of the kernels that use them
// (1: PS linear sums, 2: ModUp, 4: ModDown+rescale; 0 = the VALU kernels --
// the words are the same either way; fhe_set_mfma_sums sets it at run time)
enum { MF_LIN = 1, MF_MODUP = 2, MF_MODDOWN = 4 };
constexpr int MFMA_DEFAULT = MF_LIN;  // measured: linear sums gain on MFMA, the conversions do not
std::atomic<int> g_mfma_mask{-1};  // -1: not yet read from FHE_MFMA
inline int mfma_mask() {
    int m = g_mfma_mask.load(std::memory_order_relaxed);
    if (m < 0) {
        const char *e = std::getenv("FHE_MFMA");
        m = e ? std::atoi(e) & 7 : MFMA_DEFAULT;
        g_mfma_mask.store(m, std::memory_order_relaxed);
    }
    return m;
}
inline bool use_mfma_sums(int which) { return (mfma_mask() & which) != 0; }

__device__ __forceinline__ int lane_id() { return threadIdx.x; }

// --------------------------------------------------------- element-wise ----
// grid: x = n / (2 NT), y = limb, z = segment; 2 coefficients per lane.
// Segment z of out / a / b starts at z * S.o / S.a / S.b (u64 units), so one
// launch covers both polynomials of every member of a ciphertext batch, reads
// a wider (undropped) input in place, or broadcasts a plaintext (S.b = 0).
#define EW_PROLOGUE                                                           \
    const size_t n = (size_t)1 << logN;                                       \
    const int l = blockIdx.y;                                                 \
    const size_t ln = (size_t)l * n;                                          \
    const size_t k = ((size_t)blockIdx.x * NT + threadIdx.x) * 2;             \
    if (k >= n) return;                                                       \
    const size_t oo = (size_t)blockIdx.z * S.o + ln + k;                      \
    const size_t oa = (size_t)blockIdx.z * S.a + ln + k;                      \
    const size_t ob = (size_t)blockIdx.z * S.b + ln + k;                      \
    (void)ob;                                                                 \
    const u64 q = mods[l].q;

__device__ __forceinline__ ulonglong2 ld2(const u64 *p) { return *reinterpret_cast<const ulonglong2 *>(p); }
__device__ __forceinline__ void st2(u64 *p, ulonglong2 v) { *reinterpret_cast<ulonglong2 *>(p) = v; }

__global__ __launch_bounds__(NT) void k_add(u64 *out, const u64 *a, const u64 *b, Seg S, const Mod *mods, int logN) {
    EW_PROLOGUE
    const ulonglong2 x = ld2(a + oa), y = ld2(b + ob);
    st2(out + oo, make_ulonglong2(add_mod(x.x, y.x, q), add_mod(x.y, y.y, q)));
}
__global__ __launch_bounds__(NT) void k_sub(u64 *out, const u64 *a, const u64 *b, Seg S, const Mod *mods, int logN) {
    EW_PROLOGUE
    const ulonglong2 x = ld2(a + oa), y = ld2(b + ob);
    st2(out + oo, make_ulonglong2(sub_mod(x.x, y.x, q), sub_mod(x.y, y.y, q)));
}
__global__ __launch_bounds__(NT) void k_neg(u64 *out, const u64 *a, Seg S, const Mod *mods, int logN) {
    EW_PROLOGUE
    const ulonglong2 x = ld2(a + oa);
    st2(out + oo, make_ulonglong2(sub_mod(0, x.x, q), sub_mod(0, x.y, q)));
}
__device__ __forceinline__ u64 smod(int64_t v, const Mod &m) {
    if (v >= 0) return reduce64((u64)v, m);
    const u64 r = reduce64((u64)0 - (u64)v, m);
    return r ? m.q - r : 0;
}
// (v * 2^sh) mod q: a constant too large for 62 bits is carried as a rounded
// mantissa and a power of two (host::SConst)
__device__ __forceinline__ u64 smod(int64_t v, int sh, const Mod &m) {
    u64 r = smod(v, m);
    for (int i = 0; i < sh; ++i) r = add_mod(r, r, m.q);
    return r;
}
__global__ __launch_bounds__(NT) void k_mul_scalar(u64 *out, const u64 *a, int64_t K, int sh, Seg S,
                                                   const Mod *mods, int logN) {
    EW_PROLOGUE
    const Mod m = mods[l];
    const u64 w = smod(K, sh, m);
    (void)q;
    const ulonglong2 x = ld2(a + oa);
    st2(out + oo, make_ulonglong2(mul_barrett(x.x, w, m), mul_barrett(x.y, w, m)));
}
// out[l] += a[l] * W.w[l] (per-limb constants < q_l): key generation's P * s'
// term over the primes of one digit in one launch
__global__ __launch_bounds__(NT) void k_add_scaled(u64 *out, const u64 *a, LimbConsts W, Seg S, const Mod *mods,
                                                   int logN) {
    EW_PROLOGUE
    const Mod m = mods[l];
    const u64 w = W.w[l];
    const ulonglong2 x = ld2(a + oa), o = ld2(out + oo);
    st2(out + oo, make_ulonglong2(add_mod(o.x, mul_barrett(x.x, w, m), q), add_mod(o.y, mul_barrett(x.y, w, m), q)));
}
__global__ __launch_bounds__(NT) void k_add_scalar(u64 *out, const u64 *a, int64_t K, int sh, Seg S,
                                                   const Mod *mods, int logN) {
    EW_PROLOGUE
    const u64 w = smod(K, sh, mods[l]);
    const ulonglong2 x = ld2(a + oa);
    st2(out + oo, make_ulonglong2(add_mod(x.x, w, q), add_mod(x.y, w, q)));
}
// out = a with the c0 of every member changed (one pass over both polys, no
// separate copy): segment z = 2 member + poly, ln = limbs n.  mode 0: c0 + K 2^sh;
// 1: c0 + p; 2: c0 - p; 3: p - c0 and c1 negated (p - a)
__global__ __launch_bounds__(NT) void k_c0_op(u64 *out, const u64 *a, const u64 *p, int64_t K, int sh, int mode,
                                              size_t ln_seg, const Mod *mods, int logN) {
    const size_t n = (size_t)1 << logN;
    const int l = blockIdx.y;
    const size_t k = ((size_t)blockIdx.x * NT + threadIdx.x) * 2;
    if (k >= n) return;
    const int z = blockIdx.z;
    const size_t o = (size_t)z * ln_seg + (size_t)l * n + k;
    const u64 q = mods[l].q;
    ulonglong2 x = ld2(a + o);
    if (!(z & 1)) {
        if (mode == 0) {
            const u64 w = smod(K, sh, mods[l]);
            x = make_ulonglong2(add_mod(x.x, w, q), add_mod(x.y, w, q));
        } else {
            const ulonglong2 y = ld2(p + (size_t)l * n + k);
            x = mode == 1 ? make_ulonglong2(add_mod(x.x, y.x, q), add_mod(x.y, y.y, q))
              : mode == 2 ? make_ulonglong2(sub_mod(x.x, y.x, q), sub_mod(x.y, y.y, q))
                          : make_ulonglong2(sub_mod(y.x, x.x, q), sub_mod(y.y, x.y, q));
        }
    } else if (mode == 3) {
        x = make_ulonglong2(sub_mod(0, x.x, q), sub_mod(0, x.y, q));
    }
    st2(out + o, x);
}
__global__ __launch_bounds__(NT) void k_mul_plain(u64 *out, const u64 *a, const u64 *p, Seg S, const Mod *mods,
                                                  int logN) {
    EW_PROLOGUE
    const Mod m = mods[l];
    (void)q;
    const ulonglong2 x = ld2(a + oa), y = ld2(p + ob);
    st2(out + oo, make_ulonglong2(mul_barrett(x.x, y.x, m), mul_barrett(x.y, y.y, m)));
}
// member z: a, b [2][limbs][n] at z * sa / z * sb (sb = 0 broadcasts b);
// d01 [members][2][limbs][n], d2 [members][limbs][n]
// a2 (optional, member stride sa2): a + a2 is the left operand (the PS node's
// T_{k 2^j} + c(u), formed on load instead of in a separate pass)
__global__ __launch_bounds__(NT) void k_tensor(u64 *d01, u64 *d2, const u64 *a, const u64 *b, size_t ln_all,
                                               size_t sa, size_t sb, const u64 *a2, size_t sa2, const Mod *mods,
                                               int logN) {
    const size_t n = (size_t)1 << logN;
    const int l = blockIdx.y;
    const size_t k = ((size_t)blockIdx.x * NT + threadIdx.x) * 2;
    if (k >= n) return;
    const Mod m = mods[l];
    const size_t z = blockIdx.z, o = (size_t)l * n + k;
    const u64 *A = a + z * sa, *Bp = b + z * sb;
    ulonglong2 a0 = ld2(A + o), a1 = ld2(A + ln_all + o);
    if (a2) {
        const u64 *A2 = a2 + z * sa2;
        const ulonglong2 c0 = ld2(A2 + o), c1 = ld2(A2 + ln_all + o);
        a0 = make_ulonglong2(add_mod(a0.x, c0.x, m.q), add_mod(a0.y, c0.y, m.q));
        a1 = make_ulonglong2(add_mod(a1.x, c1.x, m.q), add_mod(a1.y, c1.y, m.q));
    }
    const ulonglong2 b0 = ld2(Bp + o), b1 = ld2(Bp + ln_all + o);
    ulonglong2 e0, e1, e2;
    e0.x = mul_barrett(a0.x, b0.x, m);
    e0.y = mul_barrett(a0.y, b0.y, m);
    e1.x = add_mod(mul_barrett(a0.x, b1.x, m), mul_barrett(a1.x, b0.x, m), m.q);
    e1.y = add_mod(mul_barrett(a0.y, b1.y, m), mul_barrett(a1.y, b0.y, m), m.q);
    e2.x = mul_barrett(a1.x, b1.x, m);
    e2.y = mul_barrett(a1.y, b1.y, m);
    st2(d01 + z * 2 * ln_all + o, e0);
    st2(d01 + z * 2 * ln_all + ln_all + o, e1);
    st2(d2 + z * ln_all + o, e2);
}
// k_tensor with mul_add's summands folded into (d0, d1) (round 5): d_p of member z
// += sum_i (K_i 2^sh_i mod q_l) x_i[2 z + p] -- the same lazy 128-bit sum and one
// reduction as k_linear_sum accumulating into d01 after the tensor, so the words
// are unchanged, without that pass's re-read and re-write of d01 (4 of its
// 2 (M + 2) limb-units per member).  M <= TL_MAX summands of one limb count.
constexpr int TL_MAX = 4;
struct TensorLin {
    const u64 *x[TL_MAX];
    int64_t K[TL_MAX];
    uint8_t sh[TL_MAX];
    size_t xseg;  // segment stride of the summands (segment 2 member + poly)
};
template <int M>
__global__ __launch_bounds__(NT) void k_tensor_lin(u64 *d01, u64 *d2, const u64 *a, const u64 *b, size_t ln_all,
                                                   size_t sa, size_t sb, const u64 *a2, size_t sa2, TensorLin L,
                                                   const Mod *mods, int logN) {
    __shared__ u64 w[TL_MAX];
    const size_t n = (size_t)1 << logN;
    const int l = blockIdx.y;
    const Mod m = mods[l];
    if ((int)threadIdx.x < M) w[threadIdx.x] = smod(L.K[threadIdx.x], L.sh[threadIdx.x], m);
    __syncthreads();
    const size_t k = ((size_t)blockIdx.x * NT + threadIdx.x) * 2;
    if (k >= n) return;
    const size_t z = blockIdx.z, o = (size_t)l * n + k;
    const u64 *A = a + z * sa, *Bp = b + z * sb;
    ulonglong2 a0 = ld2(A + o), a1 = ld2(A + ln_all + o);
    if (a2) {
        const u64 *A2 = a2 + z * sa2;
        const ulonglong2 c0 = ld2(A2 + o), c1 = ld2(A2 + ln_all + o);
        a0 = make_ulonglong2(add_mod(a0.x, c0.x, m.q), add_mod(a0.y, c0.y, m.q));
        a1 = make_ulonglong2(add_mod(a1.x, c1.x, m.q), add_mod(a1.y, c1.y, m.q));
    }
    const ulonglong2 b0 = ld2(Bp + o), b1 = ld2(Bp + ln_all + o);
    ulonglong2 xs[2][M];  // the summands' loads issued with the operands'
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int i = 0; i < M; ++i) xs[p][i] = ld2(L.x[i] + (2 * z + p) * L.xseg + o);
    Acc128 r[2][2];
    r[0][0].lo = mul_barrett(a0.x, b0.x, m);
    r[0][1].lo = mul_barrett(a0.y, b0.y, m);
    r[1][0].lo = add_mod(mul_barrett(a0.x, b1.x, m), mul_barrett(a1.x, b0.x, m), m.q);
    r[1][1].lo = add_mod(mul_barrett(a0.y, b1.y, m), mul_barrett(a1.y, b0.y, m), m.q);
    ulonglong2 e2;
    e2.x = mul_barrett(a1.x, b1.x, m);
    e2.y = mul_barrett(a1.y, b1.y, m);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
        for (int i = 0; i < M; ++i) {
            mac128(r[p][0], xs[p][i].x, w[i]);
            mac128(r[p][1], xs[p][i].y, w[i]);
        }
        st2(d01 + z * 2 * ln_all + p * ln_all + o, make_ulonglong2(reduce128(r[p][0], m), reduce128(r[p][1], m)));
    }
    st2(d2 + z * ln_all + o, e2);
}
// out [2][limbs][n] = sum over members of in [members][2][limbs][n]
__global__ __launch_bounds__(NT) void k_sum_members(u64 *out, const u64 *in, int members, size_t ln_all,
                                                    const Mod *mods, int logN) {
    const size_t n = (size_t)1 << logN;
    const int l = blockIdx.y;
    const size_t k = ((size_t)blockIdx.x * NT + threadIdx.x) * 2;
    if (k >= n) return;
    const u64 q = mods[l].q;
    const size_t o = (size_t)blockIdx.z * ln_all + (size_t)l * n + k;
    u64 r0 = 0, r1 = 0;
    for (int m = 0; m < members; ++m) {
        const ulonglong2 x = ld2(in + (size_t)m * 2 * ln_all + o);
        r0 = add_mod(r0, x.x, q);
        r1 = add_mod(r1, x.y, q);
    }
    st2(out + o, make_ulonglong2(r0, r1));
}
constexpr int LIN_MAX = 32;
struct LinArgs {
    const u64 *x[LIN_MAX];
    int64_t K[LIN_MAX];
    uint8_t sh[LIN_MAX];  // K[i] * 2^sh[i]
    int m, accumulate;
    size_t xseg;
};
// out = sum_i (K_i mod q_l) x_i: the block's limb constants are reduced once
// into LDS, the sum is accumulated lazily in 128 bits and reduced once.
__global__ __launch_bounds__(NT) void k_linear_sum(u64 *out, LinArgs A, size_t seg, const Mod *mods, int logN) {
    __shared__ u64 w[LIN_MAX];
    const size_t n = (size_t)1 << logN;
    const int l = blockIdx.y;
    const Mod md = mods[l];
    if ((int)threadIdx.x < A.m) w[threadIdx.x] = smod(A.K[threadIdx.x], A.sh[threadIdx.x], md);
    __syncthreads();
    const size_t off = (size_t)blockIdx.z * seg + (size_t)l * n;
    const size_t k = ((size_t)blockIdx.x * NT + threadIdx.x) * 2;
    if (k >= n) return;
    Acc128 r0, r1;
    if (A.accumulate) {
        const ulonglong2 o = ld2(out + off + k);
        r0.lo = o.x;
        r1.lo = o.y;
    }
    const size_t xo = (size_t)blockIdx.z * A.xseg + (size_t)l * n + k;
    for (int i = 0; i < A.m; ++i) {
        const ulonglong2 x = ld2(A.x[i] + xo);
        mac128(r0, x.x, w[i]);
        mac128(r1, x.y, w[i]);
    }
    st2(out + off + k, make_ulonglong2(reduce128(r0, md), reduce128(r1, md)));
}
// Several linear sums over one input set in one pass: out_g = sum_i (K[g][i]
// mod q_l) x_i for g < G.  Each input coefficient is read once for all G
// outputs (the Paterson-Stockmeyer leaves all combine the same baby steps).
// Inputs may have different limb counts (segment stride xseg[i]); constants
// are reduced once per block into LDS; lazy 128-bit accumulation.
constexpr int MLS_G = 10, MLS_M = 32;  // arguments: 3.5 KB of the 4 KB kernel-argument limit
struct MultiLinArgs {
    u64 *out[MLS_G];
    const u64 *x[MLS_M];
    size_t xseg[MLS_M];
    int64_t K[MLS_G * MLS_M];  // [g][i]
    uint8_t sh[MLS_G * MLS_M];  // K[t] * 2^sh[t]
    int m, G, accumulate;
};
// One coefficient per lane, G outputs.  Every residue and constant is < 2^60,
// so both split into 30-bit halves and a term costs four v_mad_u64_u32 with
// accumulate (mac4, no carries); 16 terms fit the four 64-bit partial sums, so
// each chunk of 16 baby steps folds into a 128-bit running sum per output,
// reduced once at the end (a reduction per chunk measured 3.7% slower,
// profiles/r2_l).  The constants are split once per block into LDS
// (wave-uniform broadcast reads).
template <int G>
__global__ __launch_bounds__(NT) void k_linear_sum_multi(MultiLinArgs A, size_t seg, const Mod *mods, int logN) {
    __shared__ Split30 w[G * MLS_M];
    const size_t n = (size_t)1 << logN;
    const int l = blockIdx.y;
    const Mod md = mods[l];
    for (int t = threadIdx.x; t < G * MLS_M; t += NT) w[t] = split30((t % MLS_M) < A.m ? smod(A.K[t], A.sh[t], md) : 0);
    __syncthreads();
    const size_t k = (size_t)blockIdx.x * NT + threadIdx.x;
    if (k >= n) return;
    const size_t ln = (size_t)l * n + k, oo = (size_t)blockIdx.z * seg + ln;
    Acc128 run[G];
#pragma unroll
    for (int g = 0; g < G; ++g) run[g].lo = A.accumulate ? A.out[g][oo] : 0;
    for (int base = 0; base < A.m; base += 16) {
        const int end = min(A.m, base + 16);
        Acc4 s[G];
        // issue the chunk's loads up front (memory-level parallelism), then MAC
        u64 xv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) xv[u] = base + u < end ? A.x[base + u][(size_t)blockIdx.z * A.xseg[base + u] + ln] : 0;
        // fully unrolled (a `break` here kept the loop rolled: xv[] indexed at
        // run time and one exposed LDS round trip per baby step); the guard is
        // wave-uniform
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            if (base + u < end) {
                const Split30 x = split30(xv[u]);
#pragma unroll
                for (int g = 0; g < G; ++g) mac4(s[g], x, w[g * MLS_M + base + u]);
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) fold4(run[g], s[g]);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) A.out[g][oo] = reduce128(run[g], md);
}

// ------------------------------------------------ RNS sums of products on MFMA ----
// A sum of products out_t = sum_i c_{t,i} y_i mod q with word-sized residues is
// a GEMM over the integers followed by one reduction per output, so it runs on
// the i8 matrix cores (v_mfma_i32_16x16x64_i8):
//   * y (< 2^60) is split into 8 bytes u_a; bytes 0..6 are XORed with 0x80,
//     which makes them the signed bytes u_a - 128 (byte 7 < 16 stays as it is):
//     sum_a s_a 256^a = y - C0, C0 = 0x0080808080808080;
//   * c (< 2^60) is written in balanced base-256 digits e_0..e_7 in [-128, 128);
//   * the K index runs over (source i, byte a) and the M index over (output t,
//     shift s = a + c'), with A[(t, s), (i, a)] = e_{s-a}(c_{t,i}), so row s of
//     output t accumulates sum_{i, a} s_{i,a} e_{s-a} exactly in int32 (at most
//     256 terms of magnitude <= 2^14 per row);
//   * out_t = sum_s v_s 256^s + C0 sum_i c_{t,i}: sixteen int32 rows combined
//     into a signed 128-bit value (|value| < 32 * 2^120) and reduced once.
// Rows are ordered so that one lane holds all sixteen shifts of one output: a
// 16x16 tile kk of a group of four outputs has row 4 g + r = (output g, shift
// 4 kk + r), and the C/D layout (col = lane & 15, row = 4 (lane >> 4) + reg)
// puts output g = lane >> 4, shifts 4 kk .. 4 kk + 3 into lane `lane`'s four
// accumulator registers of tile kk.  A and B take their k index from the same
// (lane >> 4, byte) pair, so the sum is over matching (i, a) whatever order the
// hardware gives the 64 k slots.  The words equal the VALU sums' (one exact
// integer sum, one canonical reduction).
typedef int v4i __attribute__((ext_vector_type(4)));
constexpr u64 XMASK = 0x0080808080808080ull;  // bytes 0..6 -> signed (u - 128); also C0

// balanced base-256 digits of c < 2^60 as bytes (digit d in byte d)
__device__ __forceinline__ u64 balanced_digits(u64 c) {
    u64 e = 0;
    int64_t v = (int64_t)c;
#pragma unroll
    for (int d = 0; d < 8; ++d) {
        int dig = (int)(v & 255);
        if (dig >= 128) dig -= 256;
        v = (v - dig) >> 8;
        e |= (u64)(uint8_t)(int8_t)dig << (8 * d);
    }
    return e;
}
// the 8 A bytes of row shift s for one source: byte a = e_{s-a} (0 outside 0..7)
__device__ __forceinline__ u64 shift_window(u64 e, int s) {
    const u64 r = __builtin_bswap64(e);  // byte p = e_{7-p}
    if (s <= 7) return r >> (8 * (7 - s));
    return s == 15 ? 0 : r << (8 * (s - 7));
}
// sum_{kk, r} v[kk][r] 256^(4 kk + r) + 2^126, reduced mod q.  |v| < 2^22, so
// v0 + 256 v1 fits an int32 and each four-row group L_kk an int64 (< 2^47); the
// signed 128-bit sum (|sum| < 2^125) is biased by 2^126 so the reduction sees
// a non-negative value -- the caller's per-output constant takes 2^126 off again.
__device__ __forceinline__ u64 combine_rows(const v4i (&v)[4], const Mod &m) {
    int64_t L[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
        const int32_t p = v[kk][0] + (v[kk][1] << 8), q = v[kk][2] + (v[kk][3] << 8);
        L[kk] = (int64_t)p + ((int64_t)q << 16);
    }
    Acc128 a;
    a.lo = (u64)L[0] + ((u64)L[1] << 32);
    const u64 c = a.lo < (u64)L[0];
    a.hi = (u64)(L[0] >> 63) + (u64)(L[1] >> 32) + c + (u64)L[2] + ((u64)L[3] << 32) + (1ull << 62);
    return reduce128(a, m);
}
// combine_rows plus a (< 2q), canonical, with one two-term Shoup step for the
// 128-bit value lo + 2^64 hi: lo * 1 - floor(lo w1s / 2^64) q and hi r64 -
// floor(hi r64s / 2^64) q are each in [0, 2q) (w1s = floor(2^64 / q)), so
// r = lo + hi r64 - (both quotients) q + a lies in [0, 6q) (< 2^64: q < 2^61)
// and three conditional subtractions finish it.  Same residue as
// add_mod(combine_rows(v), a) (round 5: about half its instructions).
__device__ __forceinline__ u64 combine_rows_add(const v4i (&v)[4], const Mod &m, u64 w1s, u64 a) {
    int64_t L[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
        const int32_t p = v[kk][0] + (v[kk][1] << 8), q = v[kk][2] + (v[kk][3] << 8);
        L[kk] = (int64_t)p + ((int64_t)q << 16);
    }
    const u64 lo = (u64)L[0] + ((u64)L[1] << 32);
    const u64 c = lo < (u64)L[0];
    const u64 hi = (u64)(L[0] >> 63) + (u64)(L[1] >> 32) + c + (u64)L[2] + ((u64)L[3] << 32) + (1ull << 62);
    u64 r = lo + hi * m.r64 - (mulhi(lo, w1s) + mulhi(hi, m.r64s)) * m.q + a;
    const u64 q2 = 2 * m.q, q4 = 4 * m.q;
    r = r >= q4 ? r - q4 : r;
    r = r >= q2 ? r - q2 : r;
    return r >= m.q ? r - m.q : r;
}
// floor(2^64 / q) from the Barrett constant floor(2^2k / q) (k >= 32)
__device__ __forceinline__ u64 shoup_one(const Mod &m) { return m.mu >> (2 * m.k - 64); }
// the per-output constant C0 * sum_i c_i - 2^126 mod q
__device__ __forceinline__ u64 sums_constant(u64 csum, const Mod &m) {
    const u64 b126 = mul_shoup(reduce64(1ull << 62, m), m.r64, m.r64s, m.q);
    return sub_mod(mul_barrett(csum, reduce64(XMASK, m), m), b126, m.q);
}

// A fragments in LDS: [group][kk][ks][lane] x 16 B; one wave reads 1 KB contiguous.
// Window (output t, source i, shift s) -> its 8 bytes in that image.
template <int KS>
__device__ __forceinline__ int afrag_offset(int t, int i, int s) {
    const int grp = t >> 2, row = 4 * (t & 3) + (s & 3), lane = 16 * ((i & 7) >> 1) + row;
    return ((((grp * 4 + (s >> 2)) * KS + (i >> 3)) * 64 + lane) * 16 + 8 * (i & 1)) >> 3;  // u64 units
}

// One group of four outputs for four column tiles: acc[c][kk] = tile kk of
// column tile c, from the group's A image in LDS ([kk][ks][lane] x 16 B).
template <int KS, int NC = 4>
__device__ __forceinline__ void mfma_group(const u64 *img, const v4i (&bf)[NC][KS], v4i (&acc)[NC][4], int lane) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) acc[c][kk] = v4i{0, 0, 0, 0};
    // the A fragments of row block kk + 1 are read while row block kk multiplies
    v4i af[2][KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) af[0][ks] = *reinterpret_cast<const v4i *>(&img[(ks * 64 + lane) * 2]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
        if (kk < 3) {
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
                af[(kk + 1) & 1][ks] = *reinterpret_cast<const v4i *>(&img[(((kk + 1) * KS + ks) * 64 + lane) * 2]);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this block's products
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
            for (int c = 0; c < NC; ++c)
                acc[c][kk] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[kk & 1][ks], bf[c][ks], acc[c][kk], 0, 0, 0);
    }
}
// a pointer read back from LDS is generic (flat loads, which also wait on LDS
// traffic); the sources are global memory
typedef __attribute__((address_space(1))) const u64 gu64;
__device__ __forceinline__ gu64 *to_global(const u64 *p) { return (gu64 *)p; }
__device__ __forceinline__ v4i bytes_of(u64 y0, u64 y1) {
    return v4i{(int)(uint32_t)y0, (int)(uint32_t)(y0 >> 32), (int)(uint32_t)y1, (int)(uint32_t)(y1 >> 32)};
}

// k-slot order (hi x, hi y, lo x, lo y) of k_leaf_sums_mfma's fragments
__device__ __forceinline__ v4i bytes_hilo(u64 y0, u64 y1) {
    return v4i{(int)(uint32_t)(y0 >> 32), (int)(uint32_t)(y1 >> 32), (int)(uint32_t)y0, (int)(uint32_t)y1};
}
typedef int v16i __attribute__((ext_vector_type(16)));

// Coefficients per block of the leaf sums: wide launches take 4096 (round 3:
// 2238-2245 us against 2303-2305 us at 1024 per launch, profiles/r3_mfma); narrow
// ones (one ciphertext: the bootstrap's series) halve it until the grid has
// >= 2048 blocks, down to 256.
constexpr int LS_CH_MAX = 4096;
// Paterson-Stockmeyer leaf sums in one pass (round 4): up to 16 outputs x 64
// baby steps per launch, so the degree-6510 doubled sinc's 52 baby steps and a
// level's leaves are read once (round 3: passes of 10 leaves x 32 steps, the
// second pass re-reading and re-writing its outputs).  The constants come from
// a device table ([G][m] K and shift, cached by the engine per series and level)
// instead of the 4-KB argument block.  The A fragments are no longer an LDS image
// of every 16-shift window (G m 128 B: 114 KB at 16 x 56): a lane reads the two
// byte-reversed digit words of its (output, source pair) -- 16 B from a G m 8-B
// LDS table -- and shifts its window out of them per row block (two 64-bit
// shifts), so the LDS holds 16 KB and never bounds occupancy.  Each wave owns two
// 16-coefficient column tiles; every source's B fragment stays in registers
// across the output groups.  Same exact sums and reductions as
// round 3's LDS-image kernel and k_linear_sum_multi (word-identical).
struct LeafArgs {
    u64 *out[LEAF_G];
    const u64 *x[LEAF_M];
    uint32_t xseg[LEAF_M];  // segment strides in words (limbs * n < 2^32)
    const int64_t *K;       // device [G][m]
    const uint8_t *sh;      // device [G][m]
    int m, G, accumulate;
    int six;  // k_leaf_sums_fold: the FP primes' six-digit rows (FHE_LEAF_SIX)
};
#ifndef FHE_LF_NC  // 16-coefficient column tiles per wave sharing one set of windows (A/B: -DFHE_LF_NC=4)
#define FHE_LF_NC 2
#endif
constexpr int LF_NC = FHE_LF_NC, LF_NT = 256;
#ifndef FHE_LF_WPE  // waves per SIMD asked of the compiler (A/B: -DFHE_LF_WPE=4)
#define FHE_LF_WPE 3
#endif
template <int KS, int NG>
__global__ __launch_bounds__(LF_NT) __attribute__((amdgpu_waves_per_eu(FHE_LF_WPE, 8))) void k_leaf_sums_mfma(LeafArgs A, size_t seg, const Mod *mods, int logN,
                                                          int chunk) {
    __shared__ u64 etab[4 * NG][8 * KS];  // byte-reversed balanced digits of each constant
    __shared__ u64 corr[4 * NG];
    __shared__ const u64 *xptr[8 * KS];
    __shared__ size_t xoff[8 * KS];
    __shared__ u64 *optr[4 * NG];
    const size_t n = (size_t)1 << logN;
    const int l = blockIdx.y;
    const Mod md = mods[l];
    const int tid = threadIdx.x;
    const int ngr = (A.G + 3) >> 2;  // groups of four outputs in this launch (<= NG)
    for (int p = tid; p < 4 * ngr * 8 * KS; p += LF_NT) {
        const int t = p / (8 * KS), i = p % (8 * KS);
        const u64 c = (t < A.G && i < A.m) ? smod(A.K[t * A.m + i], A.sh[t * A.m + i], md) : 0;
        etab[t][i] = __builtin_bswap64(balanced_digits(c));
    }
    if (tid < 8 * KS) {  // padding sources read source 0 (their constants are zero)
        const int i = tid < A.m ? tid : 0;
        xptr[tid] = A.x[i];
        xoff[tid] = (size_t)blockIdx.z * A.xseg[i] + (size_t)l * n;
    }
    __syncthreads();
    if (tid < 4 * ngr) {
        optr[tid] = tid < A.G ? A.out[tid] : nullptr;
        u64 s = 0;
        if (tid < A.G)
            for (int i = 0; i < A.m; ++i) s = add_mod(s, smod(A.K[tid * A.m + i], A.sh[tid * A.m + i], md), md.q);
        corr[tid] = sums_constant(s, md);
    }
    __syncthreads();
    const int lane = tid & 63, wave = tid >> 6, col = lane & 15, lg = lane >> 4;
    const int ta = (lane & 15) >> 2, rr = lane & 3;  // A row: output ta of the group, shift 4 kk + rr
    const uint32_t ab = 3 - rr;                            // window byte offset (see the products below)
    const u64 w1s = shoup_one(md);
    const size_t oo_l = (size_t)blockIdx.z * seg + (size_t)l * n;
    for (size_t nb = (size_t)blockIdx.x * chunk + wave * 16 * LF_NC; nb < (size_t)(blockIdx.x + 1) * chunk && nb < n;
         nb += LF_NT / 4 * LF_NC) {
        // B fragments: sources 8 ks + 2 lg, +1 of coefficient nb + 16 c + col
        v4i bf[LF_NC][KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int i0 = 8 * ks + 2 * lg;
            const gu64 *p0 = to_global(xptr[i0]) + xoff[i0] + nb + col;
            const gu64 *p1 = to_global(xptr[i0 + 1]) + xoff[i0 + 1] + nb + col;
#pragma unroll
            for (int c = 0; c < LF_NC; ++c) bf[c][ks] = bytes_hilo(p0[16 * c] ^ XMASK, p1[16 * c] ^ XMASK);
        }
#pragma unroll 1
        for (int grp = 0; grp < ngr; ++grp) {
            const int t = 4 * grp + lg;
            u64 *o = optr[t < A.G ? t : 0] + oo_l + nb + col;
            v4i acc[LF_NC][4];
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const ulonglong2 e = *reinterpret_cast<const ulonglong2 *>(&etab[4 * grp + ta][8 * ks + 2 * lg]);
                // shift_window(e, s), s = 4 kk + rr, is bytes 15 - s .. 22 - s of the
                // 24-byte string 0^8 e 0^8: its dwords are byte-aligned extracts at
                // offset 3 - rr, and the four row blocks share three of them per source
                // ((lo, hi) = kk 0: (P, 0), 1: (Q, P), 2: (R, Q), 3: (0, R)).  With the
                // k slots of a lane in the order (hi x, hi y, lo x, lo y) -- bf the same
                // -- the fragment of row block kk is dwords 2 kk .. 2 kk + 3 of
                // 0 0 Px Py Qx Qy Rx Ry 0 0, so the four share registers
                const uint32_t x0 = (uint32_t)e.x, x1 = (uint32_t)(e.x >> 32);
                const uint32_t y0 = (uint32_t)e.y, y1 = (uint32_t)(e.y >> 32);
                const v16i sq = {0, 0, (int)__builtin_amdgcn_alignbyte(0u, x1, ab), (int)__builtin_amdgcn_alignbyte(0u, y1, ab),
                                 (int)__builtin_amdgcn_alignbyte(x1, x0, ab), (int)__builtin_amdgcn_alignbyte(y1, y0, ab),
                                 (int)__builtin_amdgcn_alignbyte(x0, 0u, ab), (int)__builtin_amdgcn_alignbyte(y0, 0u, ab),
                                 0, 0, 0, 0, 0, 0, 0, 0};
                const v4i af[4] = {__builtin_shufflevector(sq, sq, 0, 1, 2, 3), __builtin_shufflevector(sq, sq, 2, 3, 4, 5),
                                   __builtin_shufflevector(sq, sq, 4, 5, 6, 7), __builtin_shufflevector(sq, sq, 6, 7, 8, 9)};
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
#pragma unroll
                    for (int c = 0; c < LF_NC; ++c)  // (first step: zero accumulator operand, an inline constant)
                        acc[c][kk] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[kk], bf[c][ks],
                                                                          ks ? acc[c][kk] : v4i{0, 0, 0, 0}, 0, 0, 0);
                }
                // one source step's windows at a time (hoisting every step's
                // fragments ahead spilled the one-group instantiations)
                __builtin_amdgcn_sched_barrier(0);
            }
            if (t < A.G) {
                // (accumulating launches read the running sums only now: loaded
                // before the products they held 4 VGPRs across the MFMA loop)
                u64 prev[LF_NC] = {};
                if (A.accumulate) {
#pragma unroll
                    for (int c = 0; c < LF_NC; ++c) prev[c] = o[16 * c];
                }
                const u64 cr = corr[t];
#pragma unroll
                for (int c = 0; c < LF_NC; ++c) o[16 * c] = combine_rows_add(acc[c], md, w1s, cr + prev[c]);
            }
        }
    }
}

// Folded-constant leaf sums (round 5, FHE_LEAF_FOLD): the byte shifts move into
// the constants.  With d_{t,i,a} = 256^a c_{t,i} mod q and y_i = sum_a u_{i,a} 256^a,
//   out_t = sum_{i,a} u_{i,a} d_{t,i,a}  (mod q),
// and d = sum_b e_b(d) 256^b in balanced digits, so the M index runs over
// (output, digit b < 8) -- two 16-row blocks per group of four outputs instead of
// four, half the MFMAs -- and the A fragment of (t, b) over k = (i, a) is the byte
// string e_b(d_{t,i,0..7}): a table lookup, no windows.  The block builds the table
// once ([group][row block][source step][lane] x 16 B, 14 KB per group at 56 sources)
// and keeps it in LDS; every wave streams four 16-coefficient column tiles per
// step with its B fragments in registers, so an A fragment read serves four MFMAs.
// Rows: |v_b| < 448 * 2^14, so V = L0 + 2^32 L1 (L = four rows, < 2^47) -- one
// 128-bit fold (combine_rows_add's two-term Shoup step, bias 2^126) per output.
// Byte 0..6 of y are read as signed (u - 128), so out = V + 128 sum_{i, a<7} d.
// Same residues as k_leaf_sums_mfma (exact integer sums, canonical results).
constexpr int LFF_NT = 512, LFF_NC = 4;
// FHE_LEAF_SIX (A/B, default 1): the FP-class primes' six-digit row layout below
inline bool leaf_six_enabled_host() {
    static const bool v = [] {
        const char *e = std::getenv("FHE_LEAF_SIX");
        return !e || std::atoi(e) != 0;
    }();
    return v;
}
typedef int v8i __attribute__((ext_vector_type(8)));
__device__ __forceinline__ u64 fold_rows2(const v4i &r0, const v4i &r1, const Mod &m, u64 w1s, u64 a) {
    const int32_t p0 = r0[0] + (r0[1] << 8), q0 = r0[2] + (r0[3] << 8);
    const int32_t p1 = r1[0] + (r1[1] << 8), q1 = r1[2] + (r1[3] << 8);
    const int64_t L0 = (int64_t)p0 + ((int64_t)q0 << 16), L1 = (int64_t)p1 + ((int64_t)q1 << 16);
    const u64 lo = (u64)L0 + ((u64)L1 << 32);
    const u64 c = lo < (u64)L0;
    const u64 hi = (u64)(L0 >> 63) + (u64)(L1 >> 32) + c + (1ull << 62);
    u64 r = lo + hi * m.r64 - (mulhi(lo, w1s) + mulhi(hi, m.r64s)) * m.q + a;
    const u64 q2 = 2 * m.q, q4 = 4 * m.q;
    r = r >= q4 ? r - q4 : r;
    r = r >= q2 ? r - q2 : r;
    return r >= m.q ? r - m.q : r;
}
// fold_rows2 for a prime q < 2^41 in fp64 (exact): 2^32 mod q = 2^32, so with
// L0, L1 exact doubles (|L| < 2^47) b = L1 2^32 is exact, h = rint(b / q) is
// within one of the true quotient and r1 = fma(-h, q, b) = b - h q exactly
// (|r1| < 1.5 q); t = r1 + L0 + a is an exact integer below 2^49, and one more
// rint / fma leaves (-q/2, q/2].  The same canonical residue as fold_rows2 (whose
// 2^126 bias the caller's constant a does not carry here).
constexpr u64 FOLD_FP_QMAX = 1ull << 41;
__device__ __forceinline__ u64 fold_rows2_fp(const v4i &r0, const v4i &r1, double q, double qi, u64 a) {
    const int32_t p0 = r0[0] + (r0[1] << 8), q0 = r0[2] + (r0[3] << 8);
    const int32_t p1 = r1[0] + (r1[1] << 8), q1 = r1[2] + (r1[3] << 8);
    const double L0 = (double)p0 + (double)q0 * 65536.0, L1 = (double)p1 + (double)q1 * 65536.0;  // exact
    const double b = L1 * 4294967296.0;
    const double h = __builtin_rint(b * qi);
    const double t = __builtin_fma(-h, q, b) + L0 + (double)a;
    const double h2 = __builtin_rint(t * qi);
    double r = __builtin_fma(-h2, q, t);
    r = r < 0.0 ? r + q : r;
    return (u64)__double_as_longlong(r + 4503599627370496.0) ^ 0x4330000000000000ull;  // r in [0, q) < 2^52
}
// fp64 conversion outputs of NTG (1, 2 or 4) targets for the NT coefficients of a
// block (NT / 64 per lane), from the sources' (yh, yl) pairs in LDS (ys[s][x]):
//   H = sum_s yh h(c'_s) + yl h(c_s),  L = cst + sum_s yh l(c'_s) + yl l(c_s),
//   out = 2^20 H + L mod q  (two rint / fma reductions; MID: one exact reduction
// of H and L halfway).  Sources outermost: a source's 4 NTG constants are scalar
// loads that serve 4 NTG (NT / 64) FMAs per lane, and one ds_read_b128 of a
// coefficient's (yh, yl) serves 4 NTG of them, so neither the scalar cache nor the
// LDS bounds the FMAs.  Canonical residues.
struct FpTargets {
    const double *c[4];   // rows [S][4]
    const double *tq[4];  // {cst, q, 1 / q, flag}
    u64 *o[4];            // the block's first output coefficient of each target
};
// (YS: double2, or int2 -- the sources' (yh, yl) as int32 in half the LDS, converted
// on the read, FHE_MDFP_I32)
__device__ __forceinline__ double2 fp_src(const double2 &v) { return v; }
__device__ __forceinline__ double2 fp_src(const int2 &v) { return make_double2((double)v.x, (double)v.y); }
template <int S, int MID, int NTG, typename YS>
__device__ __forceinline__ void fp_targets(const YS (*ys)[NT], int lane, const FpTargets &F) {
    constexpr int G = NT / 64;
    double H[NTG][G], L[NTG][G], q[NTG], qi[NTG];
#pragma unroll
    for (int t = 0; t < NTG; ++t) {
        q[t] = F.tq[t][1];
        qi[t] = F.tq[t][2];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            H[t][g] = 0.0;
            L[t][g] = F.tq[t][0];
        }
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
        double c[NTG][4];
#pragma unroll
        for (int t = 0; t < NTG; ++t)
#pragma unroll
            for (int e = 0; e < 4; ++e) c[t][e] = F.c[t][4 * s + e];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const double2 y = fp_src(ys[s][64 * g + lane]);
#pragma unroll
            for (int t = 0; t < NTG; ++t) {
                H[t][g] = __builtin_fma(y.x, c[t][0], H[t][g]);
                H[t][g] = __builtin_fma(y.y, c[t][1], H[t][g]);
                L[t][g] = __builtin_fma(y.x, c[t][2], L[t][g]);
                L[t][g] = __builtin_fma(y.y, c[t][3], L[t][g]);
                if (MID && s == (S + 1) / 2 - 1) {
                    H[t][g] = __builtin_fma(-__builtin_rint(H[t][g] * qi[t]), q[t], H[t][g]);
                    L[t][g] = __builtin_fma(-__builtin_rint(L[t][g] * qi[t]), q[t], L[t][g]);
                }
            }
        }
    }
#pragma unroll
    for (int t = 0; t < NTG; ++t)
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const double b = H[t][g] * 1048576.0;  // 2^20 H, exact
            const double tt = __builtin_fma(-__builtin_rint(b * qi[t]), q[t], b) + L[t][g];
            double r = __builtin_fma(-__builtin_rint(tt * qi[t]), q[t], tt);
            r = r < 0.0 ? r + q[t] : r;
            F.o[t][64 * g + lane] = (u64)__double_as_longlong(r + 4503599627370496.0) ^ 0x4330000000000000ull;
        }
}
template <int KS, int NG>
__global__ __launch_bounds__(LFF_NT) __attribute__((amdgpu_waves_per_eu(2, 8))) void k_leaf_sums_fold(
    LeafArgs A, size_t seg, const Mod *mods, int logN, int chunk) {
    __shared__ v4i afr[NG * 2 * KS * 64];       // A fragments, 1 KB per (group, row block, step)
    __shared__ u64 psum[4 * NG][8 * KS];         // sum_{a<7} d_{t,i,a} mod q per (t, i)
    __shared__ u64 corr[4 * NG], cfp[4 * NG];
    __shared__ const u64 *xptr[8 * KS];
    __shared__ size_t xoff[8 * KS];
    __shared__ u64 *optr[4 * NG];
    const size_t n = (size_t)1 << logN;
    const int l = blockIdx.y;
    const Mod md = mods[l];
    const int tid = threadIdx.x;
    const int ngr = (A.G + 3) >> 2;
    // a prime below 2^41 (FP class; uniform: one prime per block) has d < 2^41, so
    // its balanced digits 6 and 7 are zero: with NG >= 2 a pair of groups then takes
    // three row blocks instead of four -- each group's digits 0-3, and one block of
    // both groups' digits 4-5 (row 4 ta + 2 g + b - 4) -- a quarter fewer MFMAs
    const bool fpq = md.q < FOLD_FP_QMAX;
    const bool six = NG >= 2 && KS <= 7 && fpq && A.six;  // (KS = 8: the third accumulator spills)
    const int ngt = six ? (ngr + 1) & ~1 : ngr;  // table groups (whole pairs)
    {
        u64 *const img = reinterpret_cast<u64 *>(afr);
        for (int p = tid; p < 4 * ngt * 8 * KS; p += LFF_NT) {
            const int t = p / (8 * KS), i = p % (8 * KS);
            u64 d = (t < A.G && i < A.m) ? smod(A.K[t * A.m + i], A.sh[t * A.m + i], md) : 0;
            u64 dig[8], s7 = 0;
#pragma unroll
            for (int a = 0; a < 8; ++a) {
                dig[a] = balanced_digits(d);  // byte b = e_b(d_{t,i,a})
                if (a < 7) s7 = add_mod(s7, d, md.q);
                d = mul_barrett(d, 256, md);  // (q > 256)
            }
            psum[t][i] = s7;
            const int grp = t >> 2, ta = t & 3, ks = i >> 3, lgi = (i & 7) >> 1, half = i & 1;
            if (six) {
                const int pr = grp >> 1, g = grp & 1;
#pragma unroll
                for (int b = 0; b < 6; ++b) {
                    u64 e = 0;
#pragma unroll
                    for (int a = 0; a < 8; ++a) e |= ((dig[a] >> (8 * b)) & 255) << (8 * a);
                    const int blk = b < 4 ? 3 * pr + g : 3 * pr + 2;
                    const int row = b < 4 ? 4 * ta + b : 4 * ta + 2 * g + (b - 4);
                    img[2 * ((blk * KS + ks) * 64 + 16 * lgi + row) + half] = e;
                }
                continue;
            }
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                u64 e = 0;
#pragma unroll
                for (int a = 0; a < 8; ++a) e |= ((dig[a] >> (8 * b)) & 255) << (8 * a);
                const int lane = 16 * lgi + 4 * ta + (b & 3);
                img[2 * (((grp * 2 + (b >> 2)) * KS + ks) * 64 + lane) + half] = e;
            }
        }
    }
    if (tid < 8 * KS) {  // padding sources read source 0 (their constants are zero)
        const int i = tid < A.m ? tid : 0;
        xptr[tid] = A.x[i];
        xoff[tid] = (size_t)blockIdx.z * A.xseg[i] + (size_t)l * n;
    }
    __syncthreads();
    if (tid < 4 * ngr) {
        optr[tid] = tid < A.G ? A.out[tid] : nullptr;
        u64 s = 0;
        for (int i = 0; i < A.m; ++i) s = add_mod(s, psum[tid][i], md.q);
        // + 128 sum d (the signed bytes) - 2^126 (fold_rows2's bias)
        const u64 b126 = mul_shoup(reduce64(1ull << 62, md), md.r64, md.r64s, md.q);
        corr[tid] = sub_mod(mul_barrett(s, 128, md), b126, md.q);
        cfp[tid] = mul_barrett(s, 128, md);  // (the fp64 epilogue has no bias)
    }
    __syncthreads();
    const int lane = tid & 63, wave = tid >> 6, col = lane & 15, lg = lane >> 4;
    const u64 w1s = shoup_one(md);
    const double qd = (double)md.q, qid = 1.0 / qd;
    const size_t oo_l = (size_t)blockIdx.z * seg + (size_t)l * n;
    for (size_t nb = (size_t)blockIdx.x * chunk + wave * 16 * LFF_NC; nb < (size_t)(blockIdx.x + 1) * chunk && nb < n;
         nb += LFF_NT / 4 * LFF_NC) {
        v4i bf[LFF_NC][KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int i0 = 8 * ks + 2 * lg;
            const gu64 *p0 = to_global(xptr[i0]) + xoff[i0] + nb + col;
            const gu64 *p1 = to_global(xptr[i0 + 1]) + xoff[i0 + 1] + nb + col;
#pragma unroll
            for (int c = 0; c < LFF_NC; ++c) bf[c][ks] = bytes_of(p0[16 * c] ^ XMASK, p1[16 * c] ^ XMASK);
        }
        if constexpr (NG >= 2 && KS <= 7) {
            if (six) {
#pragma unroll 1
                for (int pr = 0; pr < ngt >> 1; ++pr) {
                    v4i acc[LFF_NC][3];
                    const v4i *ag = afr + (size_t)pr * 3 * KS * 64 + lane;
#pragma unroll
                    for (int ks = 0; ks < KS; ++ks) {
                        const v4i a0 = ag[ks * 64], a1 = ag[(KS + ks) * 64], a2 = ag[(2 * KS + ks) * 64];
#pragma unroll
                        for (int c = 0; c < LFF_NC; ++c) {
                            acc[c][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, bf[c][ks], ks ? acc[c][0] : v4i{0, 0, 0, 0}, 0, 0, 0);
                            acc[c][1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, bf[c][ks], ks ? acc[c][1] : v4i{0, 0, 0, 0}, 0, 0, 0);
                            acc[c][2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a2, bf[c][ks], ks ? acc[c][2] : v4i{0, 0, 0, 0}, 0, 0, 0);
                        }
                    }
#pragma unroll
                    for (int g = 0; g < 2; ++g) {
                        const int t = 8 * pr + 4 * g + lg;
                        if (t < A.G) {
                            u64 *o = optr[t] + oo_l + nb + col;
                            const u64 cr = cfp[t];
#pragma unroll
                            for (int c = 0; c < LFF_NC; ++c)
                                o[16 * c] = fold_rows2_fp(acc[c][g], v4i{acc[c][2][2 * g], acc[c][2][2 * g + 1], 0, 0}, qd, qid, cr);
                        }
                    }
                }
                continue;
            }
        }
#pragma unroll 1
        for (int grp = 0; grp < ngr; ++grp) {
            const int t = 4 * grp + lg;
            v4i acc[LFF_NC][2];
            const v4i *ag = afr + (size_t)grp * 2 * KS * 64 + lane;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const v4i a0 = ag[ks * 64], a1 = ag[(KS + ks) * 64];
#pragma unroll
                for (int c = 0; c < LFF_NC; ++c) {
                    acc[c][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, bf[c][ks], ks ? acc[c][0] : v4i{0, 0, 0, 0}, 0, 0, 0);
                    acc[c][1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, bf[c][ks], ks ? acc[c][1] : v4i{0, 0, 0, 0}, 0, 0, 0);
                }
            }
            if (t < A.G) {
                u64 *o = optr[t] + oo_l + nb + col;
                if (fpq) {
                    const u64 cr = cfp[t];
#pragma unroll
                    for (int c = 0; c < LFF_NC; ++c) o[16 * c] = fold_rows2_fp(acc[c][0], acc[c][1], qd, qid, cr);
                } else {
                    const u64 cr = corr[t];
#pragma unroll
                    for (int c = 0; c < LFF_NC; ++c) o[16 * c] = fold_rows2(acc[c][0], acc[c][1], md, w1s, cr);  // (never accumulating)
                }
            }
        }
    }
}

// out[m][c] = sum_i ct_i[m][c] * pt_i  (accumulate: + out), lazy 128-bit.
// Segment z = 2m + c; ct_i member m at m * cmember (0 = broadcast), its c1 at
// + cpoly; plaintexts are shared by all members.
struct PlainSumArgs {
    const u64 *ct[LIN_MAX];
    const u64 *pt[LIN_MAX];
    int m, accumulate;
    size_t cmember, cpoly;
    int xcd, segs, cblocks;  // XCD-grouped flat grid (k_mul_plain_sum)
};
// grid: x = segment (fastest: the segments that read one plaintext block run
// back to back while it is still cached: 449 -> 393 us per launch; the L2 fetch
// bytes stay 1.32x the algorithmic ones, r4_final6), y = coefficient block,
// z = limb.  XCD (round 5, A.xcd): the workgroup dispatcher deals consecutive
// blocks round-robin over the 8 XCDs, so the segments of one plaintext block
// landed on 8 L2s and each fetched it; with A.xcd the launch is a flat grid of
// S x T blocks (T = coefficient blocks x limbs, a multiple of 8) whose linear
// id b runs tile 8 (b / 8 / S) + b % 8, segment (b / 8) % S: every segment of a
// tile runs on the same XCD, back to back.
__global__ __launch_bounds__(NT) void k_mul_plain_sum(u64 *out, PlainSumArgs A, size_t seg, const Mod *mods,
                                                      int logN) {
    const size_t n = (size_t)1 << logN;
    int l, z, cb;
    if (A.xcd) {
        const unsigned b = blockIdx.x, j = b >> 3;
        const unsigned tile = 8 * (j / (unsigned)A.segs) + (b & 7);
        z = (int)(j % (unsigned)A.segs);
        cb = (int)(tile % (unsigned)A.cblocks);
        l = (int)(tile / (unsigned)A.cblocks);
    } else {
        l = blockIdx.z;
        z = blockIdx.x;
        cb = blockIdx.y;
    }
    const size_t k = ((size_t)cb * NT + threadIdx.x) * 2;
    if (k >= n) return;
    const Mod md = mods[l];
    const size_t ln = (size_t)l * n + k;
    const size_t co = (size_t)(z >> 1) * A.cmember + (size_t)(z & 1) * A.cpoly + ln;
    u64 *o = out + (size_t)z * seg + ln;
    Acc128 r0, r1;
    if (A.accumulate) {
        const ulonglong2 v = ld2(o);
        r0.lo = v.x;
        r1.lo = v.y;
    }
    // four terms' loads issued before their products (the one-at-a-time loop
    // waited out every load: 0.74 of the wave cycles in s_waitcnt, r4_final3);
    // exact 128-bit sums, so the grouping does not change the words
    int i = 0;
    for (; i + 4 <= A.m; i += 4) {
        ulonglong2 x[4], p[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            x[u] = ld2(A.ct[i + u] + co);
            p[u] = ld2(A.pt[i + u] + ln);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            mac128(r0, x[u].x, p[u].x);
            mac128(r1, x[u].y, p[u].y);
        }
    }
    for (; i < A.m; ++i) {
        const ulonglong2 x = ld2(A.ct[i] + co), p = ld2(A.pt[i] + ln);
        mac128(r0, x.x, p.x);
        mac128(r1, x.y, p.y);
    }
    st2(o, make_ulonglong2(reduce128(r0, md), reduce128(r1, md)));
}

// grid: x = n / NT, y = limb, z = segment
__global__ __launch_bounds__(NT) void k_permute(u64 *out, const u64 *in, const uint32_t *perm, Seg S, int logN) {
    const size_t n = (size_t)1 << logN;
    const size_t ln = (size_t)blockIdx.y * n;
    const size_t k = (size_t)blockIdx.x * NT + threadIdx.x;
    if (k >= n) return;
    out[(size_t)blockIdx.z * S.o + ln + k] = in[(size_t)blockIdx.z * S.a + ln + perm[k]];
}
__global__ __launch_bounds__(NT) void k_signed_to_rns(u64 *out, const int64_t *coef, const int *pmap,
                                                      const Mod *mods, int logN, size_t os, size_t cs) {
    const size_t n = (size_t)1 << logN;
    const int l = blockIdx.y;
    const size_t k = (size_t)blockIdx.x * NT + threadIdx.x;
    if (k >= n) return;
    out += blockIdx.z * os;  // member z (batched device encodes)
    coef += blockIdx.z * cs;
    const Mod m = mods[pmap ? pmap[l] : l];
    const int64_t v = coef[k];
    u64 r;
    if (v >= 0) {
        r = reduce64((u64)v, m);
    } else {
        r = reduce64((u64)(-v), m);
        r = r ? m.q - r : 0;
    }
    out[(size_t)l * n + k] = r;
}
// ModRaise: out[z][l][k] = centred(in[z][k] mod q_src) mod q_l  (in: coefficient form,
// values in [0, 2 q_src); the centred lift of x > q_src / 2 is x - q_src)
__global__ __launch_bounds__(NT) void k_lift_centered(u64 *out, const u64 *in, size_t seg_in, size_t seg_out,
                                                      int src, const Mod *mods, int logN) {
    const size_t n = (size_t)1 << logN;
    const int l = blockIdx.y;
    const size_t k = (size_t)blockIdx.x * NT + threadIdx.x;
    if (k >= n) return;
    const u64 qs = mods[src].q;
    u64 x = in[(size_t)blockIdx.z * seg_in + k];
    if (x >= qs) x -= qs;
    const Mod m = mods[l];
    u64 r;
    if (x > qs / 2) {
        r = reduce64(qs - x, m);
        r = r ? m.q - r : 0;
    } else {
        r = reduce64(x, m);
    }
    out[(size_t)blockIdx.z * seg_out + (size_t)l * n + k] = r;
}
__global__ __launch_bounds__(NT) void k_reduce(u64 *x, Seg S, const Mod *mods, int logN) {
    EW_PROLOGUE
    const Mod m = mods[l];
    (void)q;
    (void)oa;
    ulonglong2 v = ld2(x + oo);
    v.x = reduce64(v.x, m);
    v.y = reduce64(v.y, m);
    st2(x + oo, v);
}

// ------------------------------------------------------------ keyswitch ----
struct ModUpArgs {
    const u64 *qhinv[8], *qhinv_s[8], *qhat[8];  // per digit; qhat [W][qstride] (zero-padded rows)
    int lo[8], hi[8];
    int digits, qstride;
    size_t coef_stride, ext_stride;
    // fp64 rows per digit (host::LevelTables modup_fp): [W][qstride][4], then [W][4]
    const double *fpc[8], *fpq[8];
};

// grid: x = n / NT, y = target chunks of tch (conv_chunk), z = member * digits + digit.
// coef: member m at m * A.coef_stride ([ell][n], coefficient form);
// ext: member m at m * A.ext_stride ([digits][W][n]).  AT = alpha (digit
// size): the source loop is straight-line; a shorter last digit reads a
// clamped limb times a zero constant.
template <int AT>
// tbeg: the first target (0, or ell: the special-prime targets only, beside a
// k_modup_fp launch that takes the Q targets)
__global__ __launch_bounds__(NT) void k_modup_convert(u64 *__restrict__ ext, const u64 *__restrict__ coef, int W, int ell, ModUpArgs A,
                                                      const int *pmap_ext, const Mod *mods, int logN, int tch,
                                                      int tbeg) {
    const size_t n = (size_t)1 << logN;
    const size_t k = (size_t)blockIdx.x * NT + threadIdx.x;
    if (k >= n) return;
    const int j = (int)(blockIdx.z % (unsigned)A.digits);
    const size_t mb = blockIdx.z / (unsigned)A.digits;
    coef += mb * A.coef_stride;
    ext += mb * A.ext_stride;
    const int lo = A.lo[j], hi = A.hi[j];
    const int t0 = tbeg + blockIdx.y * tch;
    Split30 y[AT];
#pragma unroll
    for (int i = 0; i < AT; ++i) {
        const int src = min(lo + i, ell - 1);
        y[i] = split30(mul_shoup(coef[(size_t)src * n + k], A.qhinv[j][i], A.qhinv_s[j][i], mods[src].q));
    }
    const u64 *qh = A.qhat[j];
    for (int t = t0; t < t0 + tch && t < W; ++t) {
        if (t >= lo && t < hi) continue;
        const Mod mt = mods[pmap_ext[t]];
        Acc4 acc;  // lazy: one reduction per output
        Acc128 r;
#pragma unroll
        for (int i = 0; i < AT; ++i) {
            mac4(acc, y[i], split30(qh[(size_t)t * A.qstride + i]));
            spill4<AT>(r, acc, i);
        }
        fold4(r, acc);
        ext[((size_t)j * W + t) * n + k] = reduce128(r, mt);
    }
}

// The same in exact fp64 for the targets below 2^41 (round 6; the scheme of
// k_moddown_rescale_fp, whose fp_target it shares): source i enters as
// yh = (y >> 30) - oh_i, yl = (y & (2^30 - 1)) - 2^29 with oh = 2^29 for a prime
// >= 2^41 (q_0) and 0 for the 40-bit primes (|yh| < 2^11), so a target costs
// 4 AT fp64 FMAs against two accumulators plus the two-step reduction; the
// integer targets (the special primes, q_0; flag tq[3]) rebuild y from (yh, yl)
// and keep the 128-bit sums.  Block: 256 coefficients; the scaled sources are
// computed once into LDS, then wave w takes targets w, w + 4, ... with the
// constants scalar-loaded once per wave (4 coefficients per lane).  Same
// canonical residues.  grid: x = n / 256, y = target chunks, z = member * digits + digit.
template <int AT, int MID>
// qonly: the Q targets (t < ell) only; the special primes run in k_modup_convert
// (tbeg = ell) beside it
__global__ __launch_bounds__(NT) void k_modup_fp(u64 *__restrict__ ext, const u64 *__restrict__ coef, int W, int ell, ModUpArgs A,
                                                 const int *pmap_ext, const Mod *mods, int logN, int tch, int qonly) {
    __shared__ int2 ys[AT][NT];  // (yh, yl) as int32 (|yh|, |yl| <= 2^29)
    const size_t n = (size_t)1 << logN;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const size_t k0 = (size_t)blockIdx.x * NT;  // (n is a multiple of NT)
    const int j = (int)(blockIdx.z % (unsigned)A.digits);
    const size_t mb = blockIdx.z / (unsigned)A.digits;
    coef += mb * A.coef_stride;
    ext += mb * A.ext_stride;
    const int lo = A.lo[j], hi = A.hi[j];
#pragma unroll
    for (int i = 0; i < AT; ++i) {
        const int src = min(lo + i, ell - 1);
        const u64 qs = mods[src].q;
        const int oh = qs >= FOLD_FP_QMAX ? (1 << 29) : 0;
        const u64 yv = mul_shoup(coef[(size_t)src * n + k0 + tid], A.qhinv[j][i], A.qhinv_s[j][i], qs);
        ys[i][tid] = make_int2((int)(uint32_t)(yv >> 30) - oh, (int)((uint32_t)yv & (uint32_t)MASK30) - (1 << 29));
    }
    __syncthreads();
    const u64 *qh = A.qhat[j];
    const double *fc = A.fpc[j], *fq = A.fpq[j];
    u64 *eo = ext + (size_t)j * W * n + k0;
    // an integer target (the special primes, q_0): the 128-bit sums over y rebuilt from (yh, yl)
    auto int_target = [&](int t) {
        const Mod mt = mods[pmap_ext[t]];
#pragma unroll 1
        for (int g = 0; g < NT / 64; ++g) {
            const int x = 64 * g + lane;
            Acc4 acc;
            Acc128 r;
#pragma unroll
            for (int i = 0; i < AT; ++i) {
                const int oh = mods[min(lo + i, ell - 1)].q >= FOLD_FP_QMAX ? (1 << 29) : 0;
                const int2 y = ys[i][x];
                const u64 yv = ((u64)(y.x + oh) << 30) + (u64)(y.y + (1 << 29));
                mac4(acc, split30(yv), split30(qh[(size_t)t * A.qstride + i]));
                spill4<AT>(r, acc, i);
            }
            fold4(r, acc);
            eo[(size_t)t * n + x] = reduce128(r, mt);
        }
    };
    // this block's targets, own digit skipped (tau -> t); wave w: pairs w, w + 4, ...
    const int na = hi - lo, T = (qonly ? ell : W) - na;
    const int tau0 = blockIdx.y * tch, tau1 = min(tau0 + tch, T);
    for (int ta = tau0 + 2 * wave; ta < tau1; ta += 2 * (NT / 64)) {
        const bool hasb = ta + 1 < tau1;
        const int t0 = ta < lo ? ta : ta + na, t1 = ta + 1 < lo ? ta + 1 : ta + 1 + na;
        const bool int0 = fq[(size_t)t0 * 4 + 3] != 0.0, int1 = hasb && fq[(size_t)t1 * 4 + 3] != 0.0;
        if (hasb && !int0 && !int1) {
            const FpTargets F{{fc + (size_t)t0 * A.qstride * 4, fc + (size_t)t1 * A.qstride * 4},
                              {fq + (size_t)t0 * 4, fq + (size_t)t1 * 4},
                              {eo + (size_t)t0 * n, eo + (size_t)t1 * n}};
            fp_targets<AT, MID, 2, int2>(ys, lane, F);
            continue;
        }
        for (int u = 0; u <= (hasb ? 1 : 0); ++u) {
            const int t = u ? t1 : t0;
            if (fq[(size_t)t * 4 + 3] != 0.0) {
                int_target(t);
            } else {
                const FpTargets F{{fc + (size_t)t * A.qstride * 4, nullptr}, {fq + (size_t)t * 4, nullptr},
                                  {eo + (size_t)t * n, nullptr}};
                fp_targets<AT, MID, 1, int2>(ys, lane, F);
            }
        }
    }
}

// ModUp basis conversion on MFMA (the sums of products above with c_{t,i} =
// qhat[t][i], y_i = [x_i qhinv_i]_{q_i}); same arguments and outputs as
// k_modup_convert.  Block: 256 coefficients (4 waves x 4 column tiles), groups
// of four targets [blockIdx.y * gpc, +gpc) of the digit's T = W - alpha_j
// targets (target index tau skips the digit's own limbs).  Each group's A
// image is built in LDS (double-buffered: one barrier per group).
// grid: x = n / 256, y = group chunks, z = member * digits + digit.
template <int KS>
__global__ __launch_bounds__(NT) void k_modup_mfma(u64 *__restrict__ ext, const u64 *__restrict__ coef, int W, int ell,
                                                   ModUpArgs A, const int *pmap_ext, const Mod *mods, int logN,
                                                   int gpc) {
    __shared__ u64 img[2][4 * KS * 64 * 2];
    __shared__ Mod tm[2][4];
    __shared__ u64 corr[2][4];
    const size_t n = (size_t)1 << logN;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, col = lane & 15, lg = lane >> 4;
    const int j = (int)(blockIdx.z % (unsigned)A.digits);
    const size_t mb = blockIdx.z / (unsigned)A.digits;
    coef += mb * A.coef_stride;
    ext += mb * A.ext_stride;
    const int lo = A.lo[j], hi = A.hi[j], na = hi - lo, T = W - na;
    const int g0 = blockIdx.y * gpc, g1 = min((T + 3) / 4, g0 + gpc);
    const size_t nb = (size_t)blockIdx.x * 256 + wave * 64;
    // B fragments: scaled source residues of sources 8 ks + 2 lg, +1
    v4i bf[4][KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        u64 y[2][4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            // padding sources (i >= na) read the digit's last limb: zero constants
            const int i = min(8 * ks + 2 * lg + h, na - 1);
            const u64 w = A.qhinv[j][i], wp = A.qhinv_s[j][i], q = mods[lo + i].q;
            const u64 *src = coef + (size_t)(lo + i) * n + nb + col;
#pragma unroll
            for (int c = 0; c < 4; ++c) y[h][c] = mul_shoup(src[16 * c], w, wp, q) ^ XMASK;
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) bf[c][ks] = bytes_of(y[0][c], y[1][c]);
    }
    const u64 *qh = A.qhat[j];
    for (int grp = g0; grp < g1; ++grp) {
        const int b = grp & 1;
        // A windows of the group's 4 x 8 KS constants
        for (int p = tid; p < 4 * 8 * KS; p += NT) {
            const int tl = p / (8 * KS), i = p % (8 * KS), tau = 4 * grp + tl;
            const int t = tau < lo ? tau : tau + na;
            const u64 c = (tau < T && i < na) ? qh[(size_t)t * A.qstride + i] : 0;
            const u64 e = balanced_digits(c);
#pragma unroll
            for (int s = 0; s < 16; ++s) img[b][afrag_offset<KS>(tl, i, s)] = shift_window(e, s);
        }
        if (tid < 4) {
            const int tau = 4 * grp + tid, t = tau < lo ? tau : tau + na;
            if (tau < T) {
                const Mod mt = mods[pmap_ext[t]];
                u64 s = 0;
                for (int i = 0; i < na; ++i) s = add_mod(s, qh[(size_t)t * A.qstride + i], mt.q);
                tm[b][tid] = mt;
                corr[b][tid] = sums_constant(s, mt);
            }
        }
        __syncthreads();
        v4i acc[4][4];
        mfma_group<KS>(img[b], bf, acc, lane);
        const int tau = 4 * grp + lg;
        if (tau < T) {
            const int t = tau < lo ? tau : tau + na;
            const Mod mt = tm[b][lg];
            const u64 cr = corr[b][lg];
            u64 *o = ext + ((size_t)j * W + t) * n + nb + col;
#pragma unroll
            for (int c = 0; c < 4; ++c) o[16 * c] = add_mod(combine_rows(acc[c], mt), cr, mt.q);
        }
    }
}

// ModUp basis conversion with folded constants (round 5, FHE_MODUP_FOLD; the
// leaf sums' k_leaf_sums_fold scheme): with d_{t,i,a} = 256^a qhat[t][i] mod q_t,
// ext_t = sum_{i,a} u_{i,a} d_{t,i,a} over the bytes u of y_i = [x_i qhinv_i]_{q_i},
// so the rows are (target, balanced digit b of d) and the A fragments are a table
// built once per block in LDS (targets [blockIdx.y * gpc groups of four, + gpc)),
// while the B fragments (the scaled source residues of four 16-coefficient tiles
// per wave) stay in registers across every target group.  One 128-bit fold per
// output with the target's own modulus.  Same residues as k_modup_convert.
// grid: x = n / chunk, y = target-group chunks, z = member * digits + digit.
constexpr int MUF_NT = 512;
// target groups per block: the LDS table holds 2 KS KB per group (<= ~110 KB)
__host__ __device__ constexpr int muf_gpc(int ks) { return ks <= 3 ? 16 : 48 / ks; }
template <int KS>
__global__ __launch_bounds__(MUF_NT) __attribute__((amdgpu_waves_per_eu(2, 8))) void k_modup_fold(
    u64 *__restrict__ ext, const u64 *__restrict__ coef, int W, int ell, ModUpArgs A, const int *pmap_ext,
    const Mod *mods, int logN, int gpc, int chunk) {
    constexpr int GPC = muf_gpc(KS);
    __shared__ v4i afr[GPC * 2 * KS * 64];
    __shared__ u64 psum[4 * GPC][8 * KS];
    __shared__ Mod tm[4 * GPC];
    __shared__ double tqi[4 * GPC];  // 1 / q_t (the fp64 epilogue)
    __shared__ u64 corr[4 * GPC], cfp[4 * GPC];
    const size_t n = (size_t)1 << logN;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, col = lane & 15, lg = lane >> 4;
    const int j = (int)(blockIdx.z % (unsigned)A.digits);
    const size_t mb = blockIdx.z / (unsigned)A.digits;
    coef += mb * A.coef_stride;
    ext += mb * A.ext_stride;
    const int lo = A.lo[j], hi = A.hi[j], na = hi - lo, T = W - na;
    const int g0 = blockIdx.y * gpc, ng = min((T + 3) / 4 - g0, gpc);  // this block's groups
    const u64 *qh = A.qhat[j];
    {
        u64 *const img = reinterpret_cast<u64 *>(afr);
        for (int p = tid; p < 4 * ng * 8 * KS; p += MUF_NT) {
            const int tl = p / (8 * KS), i = p % (8 * KS), tau = 4 * g0 + tl;
            const int t = tau < lo ? tau : tau + na;
            u64 d = 0;
            Mod mt{};
            if (tau < T) {
                mt = mods[pmap_ext[t]];
                if (i < na) d = qh[(size_t)t * A.qstride + i];
            }
            u64 dig[8], s7 = 0;
#pragma unroll
            for (int a = 0; a < 8; ++a) {
                dig[a] = balanced_digits(d);
                if (tau < T) {
                    if (a < 7) s7 = add_mod(s7, d, mt.q);
                    d = mul_barrett(d, 256, mt);
                }
            }
            psum[tl][i] = s7;
            const int grp = tl >> 2, ta = tl & 3, ks = i >> 3, lgi = (i & 7) >> 1, half = i & 1;
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                u64 e = 0;
#pragma unroll
                for (int a = 0; a < 8; ++a) e |= ((dig[a] >> (8 * b)) & 255) << (8 * a);
                img[2 * (((grp * 2 + (b >> 2)) * KS + ks) * 64 + 16 * lgi + 4 * ta + (b & 3)) + half] = e;
            }
        }
    }
    __syncthreads();
    if (tid < 4 * ng) {
        const int tau = 4 * g0 + tid;
        if (tau < T) {
            const Mod mt = mods[pmap_ext[tau < lo ? tau : tau + na]];
            u64 s = 0;
            for (int i = 0; i < na; ++i) s = add_mod(s, psum[tid][i], mt.q);
            const u64 b126 = mul_shoup(reduce64(1ull << 62, mt), mt.r64, mt.r64s, mt.q);
            tm[tid] = mt;
            tqi[tid] = 1.0 / (double)mt.q;
            corr[tid] = sub_mod(mul_barrett(s, 128, mt), b126, mt.q);
            cfp[tid] = mul_barrett(s, 128, mt);
        }
    }
    __syncthreads();
    for (size_t nb = (size_t)blockIdx.x * chunk + wave * 64; nb < (size_t)(blockIdx.x + 1) * chunk && nb < n;
         nb += MUF_NT) {
        // B fragments: scaled source residues of sources 8 ks + 2 lg, +1
        v4i bf[4][KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            u64 y[2][4];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                // padding sources (i >= na) read the digit's last limb: zero constants
                const int i = min(8 * ks + 2 * lg + h, na - 1);
                const u64 w = A.qhinv[j][i], wp = A.qhinv_s[j][i], q = mods[lo + i].q;
                const u64 *src = coef + (size_t)(lo + i) * n + nb + col;
#pragma unroll
                for (int c = 0; c < 4; ++c) y[h][c] = mul_shoup(src[16 * c], w, wp, q) ^ XMASK;
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) bf[c][ks] = bytes_of(y[0][c], y[1][c]);
        }
#pragma unroll 1
        for (int grp = 0; grp < ng; ++grp) {
            v4i acc[4][2];
            const v4i *ag = afr + (size_t)grp * 2 * KS * 64 + lane;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const v4i a0 = ag[ks * 64], a1 = ag[(KS + ks) * 64];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    acc[c][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, bf[c][ks], ks ? acc[c][0] : v4i{0, 0, 0, 0}, 0, 0, 0);
                    acc[c][1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, bf[c][ks], ks ? acc[c][1] : v4i{0, 0, 0, 0}, 0, 0, 0);
                }
            }
            const int tl = 4 * grp + lg, tau = 4 * g0 + tl;
            if (tau < T) {
                const int t = tau < lo ? tau : tau + na;
                const Mod mt = tm[tl];
                u64 *o = ext + ((size_t)j * W + t) * n + nb + col;
                if (mt.q < FOLD_FP_QMAX) {
                    const double qd = (double)mt.q, qid = tqi[tl];
                    const u64 cr = cfp[tl];
#pragma unroll
                    for (int c = 0; c < 4; ++c) o[16 * c] = fold_rows2_fp(acc[c][0], acc[c][1], qd, qid, cr);
                } else {
                    const u64 w1s = shoup_one(mt), cr = corr[tl];
#pragma unroll
                    for (int c = 0; c < 4; ++c) o[16 * c] = fold_rows2(acc[c][0], acc[c][1], mt, w1s, cr);
                }
            }
        }
    }
}

// Member m: acc at m * st.acc
// ([2][W][n]), ext at m * st.ext, the switched polynomial (NTT) at m * st.d.
// fold (HMult tail, may be null): on limb t = ell-1 the accumulators start at
// P * (d0, d1)[ell-1] of the member, so the fused ModDown+rescale sees
// x = d P + acc there.
template <int D>  // D = digits: the 3 D loads of a thread are all issued before the first product
__global__ __launch_bounds__(NT) void k_ks_inner(u64 *acc, const u64 *ext, const u64 *dntt, const u64 *key,
                                                 int ell, int W, int nall, int alpha,
                                                 const uint32_t *perm, const int *pmap_ext, const Mod *mods,
                                                 int logN, KsStrides st, KsFold fold) {
    // grid: x = member (fastest: the blocks reading one key block for all
    // members run back to back and share it in L2), y = coefficient block, z = target.
    // (An XCD-aware swizzle keeping those runs on one L2 measured 12% slower.)
    const size_t n = (size_t)1 << logN;
    const size_t k = (size_t)blockIdx.y * NT + threadIdx.x;
    if (k >= n) return;
    const int t = st.target_of(blockIdx.z);
    const size_t mb = blockIdx.x;
    acc += mb * st.acc;
    ext += mb * st.ext;
    dntt += mb * st.d;
    const int pt = pmap_ext[t];
    const Mod m = mods[pt];
    const size_t kk = perm ? perm[k] : k;
    u64 x[D], kb[D], ka[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        const int lo = j * alpha, hi = min((j + 1) * alpha, ell);
        x[j] = (t >= lo && t < hi) ? dntt[(size_t)t * n + kk] : ext[((size_t)j * W + t) * n + kk];
        kb[j] = key[(((size_t)j * 2 + 0) * nall + pt) * n + k];
        ka[j] = key[(((size_t)j * 2 + 1) * nall + pt) * n + k];
    }
    u64 a0 = 0, a1 = 0;
    if (fold.d && t == ell - 1) {
        const u64 *fd = fold.d + mb * fold.member;
        a0 = mul_shoup(fd[k], fold.w, fold.ws, m.q);
        a1 = mul_shoup(fd[fold.seg + k], fold.w, fold.ws, m.q);
    }
#pragma unroll
    for (int j = 0; j < D; ++j) {
        a0 = add_mod(a0, mul_barrett(x[j], kb[j], m), m.q);
        a1 = add_mod(a1, mul_barrett(x[j], ka[j], m), m.q);
    }
    acc[(size_t)t * n + k] = a0;
    acc[((size_t)W + t) * n + k] = a1;
}

// Member-blocked variant: a thread owns one (coefficient, target) and MC
// members; the 2D key words it needs are loaded once into registers and reused
// for every member (no reliance on L2 for key reuse), and the D x-words of all
// its members are loaded before the products.  grid: x = coefficient block,
// y = target, z = member group.
template <int D, int MC>
__global__ __launch_bounds__(NT) void k_ks_inner_mc(u64 *acc, const u64 *ext, const u64 *dntt, const u64 *key,
                                                    int ell, int W, int nall, int alpha, int members,
                                                    const uint32_t *perm, const int *pmap_ext, const Mod *mods,
                                                    int logN, KsStrides st, KsFold fold) {
    const size_t n = (size_t)1 << logN;
    const size_t k = (size_t)blockIdx.x * NT + threadIdx.x;
    if (k >= n) return;
    const int t = st.target_of(blockIdx.y);
    const int m0 = blockIdx.z * MC;
    const int pt = pmap_ext[t];
    const Mod m = mods[pt];
    const size_t kk = perm ? perm[k] : k;
    u64 kb[D], ka[D], x[MC][D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        kb[j] = key[(((size_t)j * 2 + 0) * nall + pt) * n + k];
        ka[j] = key[(((size_t)j * 2 + 1) * nall + pt) * n + k];
    }
#pragma unroll
    for (int u = 0; u < MC; ++u) {
        const size_t mb = (size_t)(m0 + u);
        if (m0 + u >= members) break;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const int lo = j * alpha, hi = min((j + 1) * alpha, ell);
            x[u][j] = (t >= lo && t < hi) ? dntt[mb * st.d + (size_t)t * n + kk]
                                          : ext[mb * st.ext + ((size_t)j * W + t) * n + kk];
        }
    }
#pragma unroll
    for (int u = 0; u < MC; ++u) {
        const size_t mb = (size_t)(m0 + u);
        if (m0 + u >= members) break;
        u64 a0 = 0, a1 = 0;
        if (fold.d && t == ell - 1) {
            const u64 *fd = fold.d + mb * fold.member;
            a0 = mul_shoup(fd[k], fold.w, fold.ws, m.q);
            a1 = mul_shoup(fd[fold.seg + k], fold.w, fold.ws, m.q);
        }
#pragma unroll
        for (int j = 0; j < D; ++j) {
            a0 = add_mod(a0, mul_barrett(x[u][j], kb[j], m), m.q);
            a1 = add_mod(a1, mul_barrett(x[u][j], ka[j], m), m.q);
        }
        u64 *ac = acc + mb * st.acc;
        ac[(size_t)t * n + k] = a0;
        ac[((size_t)W + t) * n + k] = a1;
    }
}

// Multi-key variant (hoisted rotations by several amounts / per-member
// rotations): grid x = member (fastest), y = coefficient block, z = target.
template <int D>
__global__ __launch_bounds__(NT) void k_ks_inner_mk(u64 *acc, const u64 *ext, const u64 *dntt, KsKeys KK, int ell,
                                                    int W, int nall, int alpha, const int *pmap_ext, const Mod *mods,
                                                    int logN, KsStrides st) {
    const size_t n = (size_t)1 << logN;
    const size_t k = (size_t)blockIdx.y * NT + threadIdx.x;
    if (k >= n) return;
    const int t = blockIdx.z;
    const size_t mb = blockIdx.x;
    acc += mb * st.acc;
    ext += mb * st.ext;
    dntt += mb * st.d;
    const u64 *key = KK.key[mb];
    const uint32_t *perm = KK.perm[mb];
    const int pt = pmap_ext[t];
    const Mod m = mods[pt];
    const size_t kk = perm ? perm[k] : k;
    u64 x[D], kb[D], ka[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        const int lo = j * alpha, hi = min((j + 1) * alpha, ell);
        x[j] = (t >= lo && t < hi) ? dntt[(size_t)t * n + kk] : ext[((size_t)j * W + t) * n + kk];
        kb[j] = key[(((size_t)j * 2 + 0) * nall + pt) * n + k];
        ka[j] = key[(((size_t)j * 2 + 1) * nall + pt) * n + k];
    }
    u64 a0 = 0, a1 = 0;
#pragma unroll
    for (int j = 0; j < D; ++j) {
        a0 = add_mod(a0, mul_barrett(x[j], kb[j], m), m.q);
        a1 = add_mod(a1, mul_barrett(x[j], ka[j], m), m.q);
    }
    acc[(size_t)t * n + k] = a0;
    acc[((size_t)W + t) * n + k] = a1;
}
// Summed multi-key variant (the giant steps of a bootstrap's linear transform):
// acc (+)= sum_m <ext_m o perm_m, key_m> over the count members, one
// accumulator pair.  grid: x = coefficient block, y = target.
template <int D>
__global__ __launch_bounds__(NT) void k_ks_inner_mk_sum(u64 *acc, const u64 *ext, const u64 *dntt, KsKeys KK,
                                                        int count, int accumulate, int ell, int W, int nall,
                                                        int alpha, const int *pmap_ext, const Mod *mods, int logN,
                                                        KsStrides st) {
    const size_t n = (size_t)1 << logN;
    const size_t k = (size_t)blockIdx.x * NT + threadIdx.x;
    if (k >= n) return;
    const int t = blockIdx.y;
    const int pt = pmap_ext[t];
    const Mod m = mods[pt];
    u64 a0 = accumulate ? acc[(size_t)t * n + k] : 0, a1 = accumulate ? acc[((size_t)W + t) * n + k] : 0;
    for (int mb = 0; mb < count; ++mb) {
        const u64 *key = KK.key[mb];
        const uint32_t *perm = KK.perm[mb];
        const size_t kk = perm ? perm[k] : k;
        u64 x[D], kb[D], ka[D];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const int lo = j * alpha, hi = min((j + 1) * alpha, ell);
            x[j] = (t >= lo && t < hi) ? dntt[(size_t)mb * st.d + (size_t)t * n + kk]
                                       : ext[(size_t)mb * st.ext + ((size_t)j * W + t) * n + kk];
            kb[j] = key[(((size_t)j * 2 + 0) * nall + pt) * n + k];
            ka[j] = key[(((size_t)j * 2 + 1) * nall + pt) * n + k];
        }
#pragma unroll
        for (int j = 0; j < D; ++j) {
            a0 = add_mod(a0, mul_barrett(x[j], kb[j], m), m.q);
            a1 = add_mod(a1, mul_barrett(x[j], ka[j], m), m.q);
        }
    }
    acc[(size_t)t * n + k] = a0;
    acc[((size_t)W + t) * n + k] = a1;
}
// grid: x = coefficient block, y = target t < W (the prime of t: pmap_ext[t])
template <int D>
__global__ __launch_bounds__(NT) void k_lt_inner(u64 *out, const u64 *ext, const u64 *c, LtArgs A, int accumulate,
                                                 int ell, int W, int nall, int alpha, const int *pmap_ext,
                                                 const u64 *pmodq, const u64 *pmodq_s, const Mod *mods, int logN) {
    const size_t n = (size_t)1 << logN;
    const size_t k = (size_t)blockIdx.x * NT + threadIdx.x;
    if (k >= n) return;
    const int t = blockIdx.y;
    const int pt = pmap_ext[t];
    const Mod m = mods[pt];
    const bool ql = t < ell;  // a Q limb: P sigma(c0) enters; on the P limbs P = 0
    const u64 Pt = ql ? pmodq[t] : 0, Pts = ql ? pmodq_s[t] : 0;
    const u64 *c0 = c + (size_t)t * n, *c1 = c + ((size_t)ell + t) * n;
    u64 a0 = accumulate ? out[(size_t)t * n + k] : 0, a1 = accumulate ? out[((size_t)W + t) * n + k] : 0;
    for (int b = 0; b < A.nb; ++b) {
        const u64 w = A.pt[b][(size_t)t * n + k];
        u64 b0 = 0, b1 = 0;
        if (!A.key[b]) {
            if (ql) {
                b0 = mul_shoup(c0[k], Pt, Pts, m.q);
                b1 = mul_shoup(c1[k], Pt, Pts, m.q);
            }
        } else {
            const u64 *key = A.key[b];
            const size_t kk = A.perm[b][k];
            u64 x[D], kb[D], ka[D];
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const int lo = j * alpha, hi = min((j + 1) * alpha, ell);
                x[j] = (t >= lo && t < hi) ? c1[kk] : ext[((size_t)j * W + t) * n + kk];
                kb[j] = key[(((size_t)j * 2 + 0) * nall + pt) * n + k];
                ka[j] = key[(((size_t)j * 2 + 1) * nall + pt) * n + k];
            }
#pragma unroll
            for (int j = 0; j < D; ++j) {
                b0 = add_mod(b0, mul_barrett(x[j], kb[j], m), m.q);
                b1 = add_mod(b1, mul_barrett(x[j], ka[j], m), m.q);
            }
            if (ql) b0 = add_mod(b0, mul_shoup(c0[kk], Pt, Pts, m.q), m.q);
        }
        a0 = add_mod(a0, mul_barrett(b0, w, m), m.q);
        a1 = add_mod(a1, mul_barrett(b1, w, m), m.q);
    }
    out[(size_t)t * n + k] = a0;
    out[((size_t)W + t) * n + k] = a1;
}
// out (+)= sum_m in_m o perm_m over `count` members (input m at m * S.a).
// grid: x = n / NT, y = limb
__global__ __launch_bounds__(NT) void k_permute_sum(u64 *out, const u64 *in, KsKeys KK, int count, int accumulate,
                                                    Seg S, const Mod *mods, int logN) {
    const size_t n = (size_t)1 << logN;
    const size_t ln = (size_t)blockIdx.y * n;
    const size_t k = (size_t)blockIdx.x * NT + threadIdx.x;
    if (k >= n) return;
    const u64 q = mods[blockIdx.y].q;
    u64 r = accumulate ? out[ln + k] : 0;
    for (int mb = 0; mb < count; ++mb) r = add_mod(r, in[(size_t)mb * S.a + ln + KK.perm[mb][k]], q);
    out[ln + k] = r;
}
// grid: x = n / NT, y = limb, z = member
__global__ __launch_bounds__(NT) void k_permute_mk(u64 *out, const u64 *in, KsKeys KK, Seg S, int logN) {
    const size_t n = (size_t)1 << logN;
    const size_t ln = (size_t)blockIdx.y * n;
    const size_t k = (size_t)blockIdx.x * NT + threadIdx.x;
    if (k >= n) return;
    const uint32_t *perm = KK.perm[blockIdx.z];
    out[(size_t)blockIdx.z * S.o + ln + k] = in[(size_t)blockIdx.z * S.a + ln + perm[k]];
}

// grid: x = n / NT, y = ceil(ell / tch), z = segment.  KT = K special primes;
// phat [nq][KT] (the constants of one target contiguous: one scalar burst)
// Exact centred conversion: y_k = [x P_k^-1]_{p_k}, x mod P = sum_k y_k P_k -
// v P with v = round(sum_k y_k / p_k) (fp64, fixed order; oracle: moddown), so
// ModDown rounds x / P to nearest instead of flooring with a 0..K overshoot --
// that overshoot is a biased error which, multiplied by s, concentrates in a
// few slots (numeric specification).
template <int KT>
__device__ __forceinline__ u64 centre_count(const u64 (&y)[KT], const double *pinvd) {
    double t = 0.0;
#pragma unroll
    for (int kk = 0; kk < KT; ++kk) t = t + (double)y[kk] * pinvd[kk];
    return (u64)(t + 0.5);
}
template <int KT>
__global__ __launch_bounds__(NT) void k_moddown_convert(u64 *__restrict__ conv, const u64 *__restrict__ pc, int ell, int nq, size_t seg_in,
                                                        size_t seg_out, const u64 *phinv, const u64 *phinv_s,
                                                        const u64 *phat, const u64 *pmod, const double *pinvd,
                                                        const Mod *mods, int logN, int tch) {
    const size_t n = (size_t)1 << logN;
    const size_t k = (size_t)blockIdx.x * NT + threadIdx.x;
    if (k >= n) return;
    const u64 *src = pc + (size_t)blockIdx.z * seg_in;
    u64 *dst = conv + (size_t)blockIdx.z * seg_out;
    u64 y[KT];
    Split30 v[KT];
#pragma unroll
    for (int i = 0; i < KT; ++i) {
        y[i] = mul_shoup(src[(size_t)i * n + k], phinv[i], phinv_s[i], mods[nq + i].q);
        v[i] = split30(y[i]);
    }
    const Split30 cnt = split30(centre_count<KT>(y, pinvd));
    const int i0 = blockIdx.y * tch;
    for (int i = i0; i < i0 + tch && i < ell; ++i) {
        Acc4 acc;
        Acc128 r;
#pragma unroll
        for (int kk = 0; kk < KT; ++kk) {
            mac4(acc, v[kk], split30(phat[(size_t)i * KT + kk]));
            spill4<KT + 1>(r, acc, kk);
        }
        mac4(acc, cnt, split30(mods[i].q - pmod[i]));  // - v P
        fold4(r, acc);
        dst[(size_t)i * n + k] = reduce128(r, mods[i]);
    }
}

// grid: x = n / (2 NT), y = limb i < ell, z = segment.  `add` (rotation: the
// permuted c0) is added to the even segments (c0 of each member), member
// s / 2 at (s / 2) * seg_add.
__global__ __launch_bounds__(NT) void k_moddown_finish(u64 *out, const u64 *acc, const u64 *conv, const u64 *add,
                                                       size_t seg_out, size_t seg_acc, size_t seg_add,
                                                       const u64 *pinv, const u64 *pinv_s, const Mod *mods,
                                                       int logN) {
    const size_t n = (size_t)1 << logN;
    const int l = blockIdx.y, s = blockIdx.z;
    const size_t k = ((size_t)blockIdx.x * NT + threadIdx.x) * 2;
    if (k >= n) return;
    const u64 q = mods[l].q, w = pinv[l], wp = pinv_s[l];
    const size_t lo = (size_t)l * n + k;
    const ulonglong2 x = ld2(acc + (size_t)s * seg_acc + lo);
    const ulonglong2 c = ld2(conv + (size_t)s * seg_out + lo);
    ulonglong2 r;
    r.x = mul_shoup(sub_mod(x.x, c.x, q), w, wp, q);
    r.y = mul_shoup(sub_mod(x.y, c.y, q), w, wp, q);
    if (add && !(s & 1)) {
        const ulonglong2 d = ld2(add + (size_t)(s >> 1) * seg_add + lo);
        r.x = add_mod(r.x, d.x, q);
        r.y = add_mod(r.y, d.y, q);
    }
    st2(out + (size_t)s * seg_out + lo, r);
}

// ------------------------------------------- fused ModDown + rescale ----
// HMult tail.  acc [2][W][n]: limbs < ell-1 NTT form; limb ell-1 (= x_last =
// d_last P + acc_last) and the K special limbs already inverse-transformed.
// corr_i = Conv_{P->q_i}(acc_P) + P * [y_last]_centred  for i < ell-1, where
// y_last = (x_last - Conv_{P->q_last}(acc_P)) * P^-1 mod q_last is the last
// limb of the ModDown output.  grid: x = n / NT, y = ceil((ell-1) / tch), z = seg
template <int KT>
__global__ __launch_bounds__(NT) void k_moddown_rescale_convert(u64 *__restrict__ corr, const u64 *__restrict__ acc, int ell, int nq,
                                                                size_t seg_acc, size_t seg_corr, const u64 *phinv,
                                                                const u64 *phinv_s, const u64 *phat, const u64 *pinv,
                                                                const u64 *pinv_s, const u64 *pmod, const double *pinvd,
                                                                const u64 *ninv, const u64 *ninv_s, const Mod *mods,
                                                                int logN, int tch) {
    const size_t n = (size_t)1 << logN;
    const size_t k = (size_t)blockIdx.x * NT + threadIdx.x;
    if (k >= n) return;
    const int last = ell - 1;
    const u64 *src = acc + (size_t)blockIdx.z * seg_acc + (size_t)last * n;
    u64 *dst = corr + (size_t)blockIdx.z * seg_corr;
    u64 yk[KT];
    Split30 v[KT];
#pragma unroll
    for (int i = 0; i < KT; ++i) {
        yk[i] = mul_shoup(src[(size_t)(1 + i) * n + k], phinv[i], phinv_s[i], mods[nq + i].q);
        v[i] = split30(yk[i]);
    }
    const u64 cntv = centre_count<KT>(yk, pinvd);  // exact centred Conv (k_moddown_convert)
    const Split30 cnt = split30(cntv);
    const Mod ml = mods[last];
    const u64 ql = ml.q;
    Acc4 cacc;
    Acc128 cr;
#pragma unroll
    for (int kk = 0; kk < KT; ++kk) {
        mac4(cacc, v[kk], split30(phat[(size_t)last * KT + kk]));
        spill4<KT + 1>(cr, cacc, kk);
    }
    mac4(cacc, cnt, split30(ql - pmod[last]));
    fold4(cr, cacc);
    const u64 cl = reduce128(cr, ml);
    // the limbs arrive from an unscaled inverse NTT (n x, in [0, 2q)): phinv
    // carries n^-1 for the special limbs, x_last takes it here
    const u64 xl = mul_shoup(src[k], ninv[last], ninv_s[last], ql);
    const u64 y = mul_shoup(sub_mod(xl, cl, ql), pinv[last], pinv_s[last], ql);
    const bool neg = y > (ql >> 1);
    const int i0 = blockIdx.y * tch;
    for (int i = i0; i < i0 + tch && i < last; ++i) {
        const Mod mi = mods[i];
        // centred lift of y: q_last / 2 < q_i (checked at context creation)
        const u64 lift = neg ? mi.q - (ql - y) : y;
        // P (lift - v): one term, K + 1 in all
        const u64 lv = lift >= cntv ? lift - cntv : lift + mi.q - cntv;
        Acc4 a4;
        Acc128 r;
        mac4(a4, split30(lv), split30(pmod[i]));
#pragma unroll
        for (int kk = 0; kk < KT; ++kk) {
            mac4(a4, v[kk], split30(phat[(size_t)i * KT + kk]));
            spill4<KT + 1>(r, a4, kk + 1);
        }
        fold4(r, a4);
        dst[(size_t)i * n + k] = reduce128(r, mi);
    }
}

// The same in exact fp64 for the targets q_i < 2^41 (round 6; the integer
// targets -- q_0 -- keep the 128-bit sums above).  Each source enters as two
// exact doubles, y_k = yh 2^30 + yl + off_k with |yh|, |yl| <= 2^29 (the K
// scaled special residues; off = 2^59 + 2^29) or yh = pv >> 30, yl its low 30
// bits (the P term pv = centred(y) - count, |pv| < 2^40 + K), and one target is
//   H = sum_k yh h(c'_k) + yl h(c_k),  L = cst + sum_k yh l(c'_k) + yl l(c_k)
// (c' = 2^30 c mod q_i centred, split at 2^20 with |l| <= 2^19: every product
// is below 2^49 and the host checks that every partial sum stays below 2^53,
// hostmath.cpp fp_conv_row), so each term is one exact FMA and
// corr_i = 2^20 H + L mod q_i takes two rint / fma reductions: 4 (K+1) fp64
// FMAs + 8 fp64 operations per output where the 128-bit form issues 4 (K+1)
// v_mad_u64_u32 + its fold and reduce128.  MID: one exact reduction of H and L
// halfway.  Same canonical residues as k_moddown_rescale_convert.
// the per-coefficient part: sources of coefficient k as (yh, yl) doubles
template <int KT>
__device__ __forceinline__ void md_sources(const u64 *src, size_t k, size_t n, int nq, int last, const u64 *phinv,
                                           const u64 *phinv_s, const u64 *phat, const u64 *pinv, const u64 *pinv_s,
                                           const u64 *pmod, const double *pinvd, const u64 *ninv, const u64 *ninv_s,
                                           const Mod *mods, double (&yh)[KT + 1], double (&yl)[KT + 1]) {
    u64 yk[KT];
#pragma unroll
    for (int i = 0; i < KT; ++i) {
        yk[i] = mul_shoup(src[(size_t)(1 + i) * n + k], phinv[i], phinv_s[i], mods[nq + i].q);
        yh[i] = (double)((int)(uint32_t)(yk[i] >> 30) - (1 << 29));
        yl[i] = (double)((int)((uint32_t)yk[i] & (uint32_t)MASK30) - (1 << 29));
    }
    const u64 cntv = centre_count<KT>(yk, pinvd);
    const Mod ml = mods[last];
    const u64 ql = ml.q;
    Acc4 cacc;
    Acc128 cr;
#pragma unroll
    for (int kk = 0; kk < KT; ++kk) {
        mac4(cacc, split30(yk[kk]), split30(phat[(size_t)last * KT + kk]));
        spill4<KT + 1>(cr, cacc, kk);
    }
    mac4(cacc, split30(cntv), split30(ql - pmod[last]));
    fold4(cr, cacc);
    const u64 cl = reduce128(cr, ml);
    const u64 xl = mul_shoup(src[k], ninv[last], ninv_s[last], ql);
    const u64 y = mul_shoup(sub_mod(xl, cl, ql), pinv[last], pinv_s[last], ql);
    const int64_t pv = (y > (ql >> 1) ? (int64_t)y - (int64_t)ql : (int64_t)y) - (int64_t)cntv;
    const int64_t ph = pv >> 30;
    yh[KT] = (double)ph;
    yl[KT] = (double)(int)(pv - ph * ((int64_t)1 << 30));
}
// Block: 256 coefficients.  Phase 1: thread x computes coefficient x's sources
// (md_sources, once per coefficient) into LDS ([K+1][256] (yh, yl) pairs: int32 by
// default, I32 = 0 doubles; |yh|, |yl| <= 2^30, exact either way).  Phase 2:
// wave w takes the targets i0 + w, i0 + w + 4, ...; a target's constants are
// scalar-loaded once per wave and serve its 256 coefficients (4 per lane, read
// back from LDS with conflict-free ds_read_b64), so the scalar traffic per FMA is
// a quarter of a thread-per-coefficient loop's and the table never has to stay in
// the scalar cache.  grid: x = n / 256, y = target chunks of tch, z = segment.
template <int KT, int MID, int TPI, int I32>
__global__ __launch_bounds__(NT) void k_moddown_rescale_fp(u64 *__restrict__ corr, const u64 *__restrict__ acc, int ell, int nq,
                                                           size_t seg_acc, size_t seg_corr, const u64 *phinv,
                                                           const u64 *phinv_s, const u64 *phat, const u64 *pinv,
                                                           const u64 *pinv_s, const u64 *pmod, const double *pinvd,
                                                           const u64 *ninv, const u64 *ninv_s, const Mod *mods,
                                                           const double *__restrict__ fpc, const double *__restrict__ fpq,
                                                           int logN, int tch) {
    using YS = std::conditional_t<I32 != 0, int2, double2>;
    __shared__ YS ys[KT + 1][NT];
    const size_t n = (size_t)1 << logN;
    // (readfirstlane: the compiler then knows the wave index, so each target's
    // constants go through scalar loads)
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const size_t k0 = (size_t)blockIdx.x * NT;  // (n is a multiple of NT)
    const int last = ell - 1;
    const u64 *src = acc + (size_t)blockIdx.z * seg_acc + (size_t)last * n;
    u64 *dst = corr + (size_t)blockIdx.z * seg_corr + k0;
    {
        double yh[KT + 1], yl[KT + 1];
        md_sources<KT>(src, k0 + tid, n, nq, last, phinv, phinv_s, phat, pinv, pinv_s, pmod, pinvd, ninv, ninv_s, mods,
                       yh, yl);
#pragma unroll
        for (int s = 0; s <= KT; ++s) {
            if constexpr (I32)
                ys[s][tid] = make_int2((int)yh[s], (int)yl[s]);
            else
                ys[s][tid] = make_double2(yh[s], yl[s]);
        }
    }
    __syncthreads();
    // an integer target (host flag: q_i >= 2^41): the 128-bit sums over y rebuilt from (yh, yl)
    auto int_target = [&](int i) {
        const Mod mi = mods[i];
#pragma unroll 1
        for (int g = 0; g < NT / 64; ++g) {
            const int x = 64 * g + lane;
            const double2 yp = fp_src(ys[KT][x]);
            const int64_t pv = (int64_t)yp.x * ((int64_t)1 << 30) + (int64_t)yp.y;
            const u64 lv = pv < 0 ? mi.q - (u64)(-pv) : (u64)pv;  // |pv| < 2^41 <= q_i
            Acc4 a4;
            Acc128 r;
            mac4(a4, split30(lv), split30(pmod[i]));
#pragma unroll
            for (int kk = 0; kk < KT; ++kk) {
                const double2 y = fp_src(ys[kk][x]);
                const u64 yv = ((u64)((int)y.x + (1 << 29)) << 30) + (u64)((int)y.y + (1 << 29));
                mac4(a4, split30(yv), split30(phat[(size_t)i * KT + kk]));
                spill4<KT + 1>(r, a4, kk + 1);
            }
            fold4(r, a4);
            dst[(size_t)i * n + x] = reduce128(r, mi);
        }
    };
    // wave w: target groups w, w + 4, ... of TPI targets of this block's chunk; a
    // group holding q_0 (the one integer target of a 40-bit context) or cut short
    // by the chunk's end runs as integer targets, pairs and singles
    const int i0 = blockIdx.y * tch, i1 = min(i0 + tch, last);
    auto is_int = [&](int i) { return fpq[(size_t)i * 4 + 3] != 0.0; };
    auto fpt = [&](int i, int u, FpTargets &F) {
        F.c[u] = fpc + (size_t)i * (KT + 1) * 4;
        F.tq[u] = fpq + (size_t)i * 4;
        F.o[u] = dst + (size_t)i * n;
    };
    for (int ia = i0 + TPI * wave; ia < i1; ia += TPI * (NT / 64)) {
        const int cnt = min(TPI, i1 - ia);
        bool anyint = false;
        for (int u = 0; u < cnt; ++u) anyint |= is_int(ia + u);
        if (cnt == TPI && !anyint) {
            FpTargets F{};
            for (int u = 0; u < TPI; ++u) fpt(ia + u, u, F);
            fp_targets<KT + 1, MID, TPI, YS>(ys, lane, F);
            continue;
        }
        for (int i = ia; i < ia + cnt;) {
            if (is_int(i)) {
                int_target(i);
                ++i;
            } else if (i + 1 < ia + cnt && !is_int(i + 1)) {
                FpTargets F{};
                fpt(i, 0, F);
                fpt(i + 1, 1, F);
                fp_targets<KT + 1, MID, 2, YS>(ys, lane, F);
                i += 2;
            } else {
                FpTargets F{};
                fpt(i, 0, F);
                fp_targets<KT + 1, MID, 1, YS>(ys, lane, F);
                ++i;
            }
        }
    }
}

// The same on MFMA: the K-source conversion of the special limbs to the ell-1
// remaining Q limbs runs as the i8 sums of products (c_{i,k} = phat[i][k]); the
// per-coefficient part (scaled special residues, the centred count, the last
// limb's conversion and y) is computed once per coefficient by the lane that
// owns it and handed to the lanes of its column by __shfl; the P (lift - v)
// term is one Shoup product in the epilogue.  Same words as the VALU kernel.
// grid: x = n / 256, y = group chunks of the ell-1 targets, z = segment.
template <int KS, int KT>
__global__ __launch_bounds__(NT) void k_moddown_rescale_mfma(u64 *__restrict__ corr_out, const u64 *__restrict__ acc,
                                                             int ell, int nq, size_t seg_acc, size_t seg_corr,
                                                             const u64 *phinv, const u64 *phinv_s, const u64 *phat,
                                                             const u64 *pinv, const u64 *pinv_s, const u64 *pmod,
                                                             const u64 *pmod_s, const double *pinvd, const u64 *ninv,
                                                             const u64 *ninv_s, const Mod *mods, int logN, int gpc) {
    __shared__ u64 img[2][4 * KS * 64 * 2];
    __shared__ Mod tm[2][4];
    __shared__ u64 cadd[2][4], pm[2][4], pms[2][4];
    const size_t n = (size_t)1 << logN;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, col = lane & 15, lg = lane >> 4;
    const int last = ell - 1, T = last;
    const u64 *src = acc + (size_t)blockIdx.z * seg_acc + (size_t)last * n;
    u64 *dst = corr_out + (size_t)blockIdx.z * seg_corr;
    const size_t nb = (size_t)blockIdx.x * 256 + wave * 64;
    // per-coefficient part, coefficient nb + lane
    u64 y, cntv;
    {
        const size_t k = nb + lane;
        u64 yk[KT];
        Split30 v[KT];
#pragma unroll
        for (int i = 0; i < KT; ++i) {
            yk[i] = mul_shoup(src[(size_t)(1 + i) * n + k], phinv[i], phinv_s[i], mods[nq + i].q);
            v[i] = split30(yk[i]);
        }
        cntv = centre_count<KT>(yk, pinvd);
        const Mod ml = mods[last];
        const u64 ql = ml.q;
        Acc4 cacc;
        Acc128 cr;
#pragma unroll
        for (int kk = 0; kk < KT; ++kk) {
            mac4(cacc, v[kk], split30(phat[(size_t)last * KT + kk]));
            spill4<KT + 1>(cr, cacc, kk);
        }
        mac4(cacc, split30(cntv), split30(ql - pmod[last]));
        fold4(cr, cacc);
        const u64 cl = reduce128(cr, ml);
        const u64 xl = mul_shoup(src[k], ninv[last], ninv_s[last], ql);
        y = mul_shoup(sub_mod(xl, cl, ql), pinv[last], pinv_s[last], ql);
    }
    const u64 ql = mods[last].q;
    u64 yc[4], cc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        yc[c] = __shfl(y, 16 * c + col);
        cc[c] = __shfl(cntv, 16 * c + col);
    }
    // B fragments: scaled special residues, sources 8 ks + 2 lg, +1
    v4i bf[4][KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        u64 yy[2][4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int i = min(8 * ks + 2 * lg + h, KT - 1);  // padding: zero constants
            const u64 w = phinv[i], wp = phinv_s[i], q = mods[nq + i].q;
            const u64 *sp = src + (size_t)(1 + i) * n + nb + col;
#pragma unroll
            for (int c = 0; c < 4; ++c) yy[h][c] = mul_shoup(sp[16 * c], w, wp, q) ^ XMASK;
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) bf[c][ks] = bytes_of(yy[0][c], yy[1][c]);
    }
    const int g0 = blockIdx.y * gpc, g1 = min((T + 3) / 4, g0 + gpc);
    for (int grp = g0; grp < g1; ++grp) {
        const int b = grp & 1;
        for (int p = tid; p < 4 * 8 * KS; p += NT) {
            const int tl = p / (8 * KS), i = p % (8 * KS), t = 4 * grp + tl;
            const u64 c = (t < T && i < KT) ? phat[(size_t)t * KT + i] : 0;
            const u64 e = balanced_digits(c);
#pragma unroll
            for (int s = 0; s < 16; ++s) img[b][afrag_offset<KS>(tl, i, s)] = shift_window(e, s);
        }
        if (tid < 4) {
            const int t = 4 * grp + tid;
            if (t < T) {
                const Mod mt = mods[t];
                u64 sum = 0;
                for (int i = 0; i < KT; ++i) sum = add_mod(sum, phat[(size_t)t * KT + i], mt.q);
                tm[b][tid] = mt;
                cadd[b][tid] = sums_constant(sum, mt);
                pm[b][tid] = pmod[t];
                pms[b][tid] = pmod_s[t];
            }
        }
        __syncthreads();
        v4i a4[4][4];
        mfma_group<KS>(img[b], bf, a4, lane);
        const int t = 4 * grp + lg;
        if (t < T) {
            const Mod mt = tm[b][lg];
            const u64 ca = cadd[b][lg], w = pm[b][lg], wp = pms[b][lg];
            u64 *o = dst + (size_t)t * n + nb + col;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                // centred lift of y: q_last / 2 < q_t (checked at context creation)
                const u64 lift = yc[c] > (ql >> 1) ? mt.q - (ql - yc[c]) : yc[c];
                const u64 lv = lift >= cc[c] ? lift - cc[c] : lift + mt.q - cc[c];
                const u64 conv = add_mod(combine_rows(a4[c], mt), ca, mt.q);
                o[16 * c] = add_mod(conv, mul_shoup(lv, w, wp, mt.q), mt.q);
            }
        }
    }
}
// Fused ModDown + rescale conversion with folded constants (round 5,
// FHE_MODDOWN_FOLD; the k_modup_fold scheme).  Sources: the K scaled special
// residues with constants phat[t][i], and one more, the signed P-term
// lv = centred(y) - count (+ 2^61 so it is a positive value below 2^62) with
// constant pmod[t] -- so the whole output is one sum of products:
//   corr_t = sum_i yk_i phat[t][i] + lv pmod[t]  (mod q_t),
// the same residue as k_moddown_rescale_convert.  The per-coefficient part (yk,
// the centred count, the last limb's conversion, y) is computed by the lane
// that owns the coefficient and handed to its column's lanes by __shfl.
// grid: x = n / chunk, y = target-group chunks, z = segment.
constexpr int MDF_NT = 512;
template <int KS, int KT>
__global__ __launch_bounds__(MDF_NT) __attribute__((amdgpu_waves_per_eu(2, 8))) void k_moddown_rescale_fold(
    u64 *__restrict__ corr_out, const u64 *__restrict__ acc, int ell, int nq, size_t seg_acc, size_t seg_corr,
    const u64 *phinv, const u64 *phinv_s, const u64 *phat, const u64 *pinv, const u64 *pinv_s, const u64 *pmod,
    const double *pinvd, const u64 *ninv, const u64 *ninv_s, const Mod *mods, int logN, int gpc, int chunk) {
    static_assert(8 * KS >= KT + 1, "K special sources + the P term");
    constexpr int GPC = muf_gpc(KS);
    __shared__ v4i afr[GPC * 2 * KS * 64];
    __shared__ u64 psum[4 * GPC][8 * KS];
    __shared__ Mod tm[4 * GPC];
    __shared__ double tqi[4 * GPC];  // 1 / q_t (the fp64 epilogue)
    __shared__ u64 corr[4 * GPC], cfp[4 * GPC];
    const size_t n = (size_t)1 << logN;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, col = lane & 15, lg = lane >> 4;
    const int last = ell - 1, T = last;
    const u64 *src = acc + (size_t)blockIdx.z * seg_acc + (size_t)last * n;
    u64 *dst = corr_out + (size_t)blockIdx.z * seg_corr;
    const int g0 = blockIdx.y * gpc, ng = min((T + 3) / 4 - g0, gpc);
    {
        u64 *const img = reinterpret_cast<u64 *>(afr);
        for (int p = tid; p < 4 * ng * 8 * KS; p += MDF_NT) {
            const int tl = p / (8 * KS), i = p % (8 * KS), t = 4 * g0 + tl;
            u64 d = 0;
            Mod mt{};
            if (t < T) {
                mt = mods[t];
                d = i < KT ? phat[(size_t)t * KT + i] : i == KT ? pmod[t] : 0;
            }
            u64 dig[8], s7 = 0;
#pragma unroll
            for (int a = 0; a < 8; ++a) {
                dig[a] = balanced_digits(d);
                if (t < T) {
                    if (a < 7) s7 = add_mod(s7, d, mt.q);
                    d = mul_barrett(d, 256, mt);
                }
            }
            psum[tl][i] = s7;
            const int grp = tl >> 2, ta = tl & 3, ks = i >> 3, lgi = (i & 7) >> 1, half = i & 1;
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                u64 e = 0;
#pragma unroll
                for (int a = 0; a < 8; ++a) e |= ((dig[a] >> (8 * b)) & 255) << (8 * a);
                img[2 * (((grp * 2 + (b >> 2)) * KS + ks) * 64 + 16 * lgi + 4 * ta + (b & 3)) + half] = e;
            }
        }
    }
    __syncthreads();
    if (tid < 4 * ng) {
        const int t = 4 * g0 + tid;
        if (t < T) {
            const Mod mt = mods[t];
            u64 s = 0;
            for (int i = 0; i <= KT; ++i) s = add_mod(s, psum[tid][i], mt.q);
            // + 128 sum d (signed bytes) - 2^61 pmod (the P term's offset) - 2^126 (bias)
            const u64 b126 = mul_shoup(reduce64(1ull << 62, mt), mt.r64, mt.r64s, mt.q);
            const u64 off = mul_barrett(reduce64(1ull << 61, mt), pmod[t], mt);
            tm[tid] = mt;
            tqi[tid] = 1.0 / (double)mt.q;
            corr[tid] = sub_mod(sub_mod(mul_barrett(s, 128, mt), b126, mt.q), off, mt.q);
            cfp[tid] = sub_mod(mul_barrett(s, 128, mt), off, mt.q);
        }
    }
    __syncthreads();
    const Mod ml = mods[last];
    const u64 ql = ml.q;
    for (size_t nb = (size_t)blockIdx.x * chunk + wave * 64; nb < (size_t)(blockIdx.x + 1) * chunk && nb < n;
         nb += MDF_NT) {
        // per-coefficient part, coefficient nb + lane: the P term's source value
        u64 pv;
        {
            const size_t k = nb + lane;
            u64 yk[KT];
            Split30 v[KT];
#pragma unroll
            for (int i = 0; i < KT; ++i) {
                yk[i] = mul_shoup(src[(size_t)(1 + i) * n + k], phinv[i], phinv_s[i], mods[nq + i].q);
                v[i] = split30(yk[i]);
            }
            const u64 cntv = centre_count<KT>(yk, pinvd);
            Acc4 cacc;
            Acc128 cr;
#pragma unroll
            for (int kk = 0; kk < KT; ++kk) {
                mac4(cacc, v[kk], split30(phat[(size_t)last * KT + kk]));
                spill4<KT + 1>(cr, cacc, kk);
            }
            mac4(cacc, split30(cntv), split30(ql - pmod[last]));
            fold4(cr, cacc);
            const u64 cl = reduce128(cr, ml);
            const u64 xl = mul_shoup(src[k], ninv[last], ninv_s[last], ql);
            const u64 y = mul_shoup(sub_mod(xl, cl, ql), pinv[last], pinv_s[last], ql);
            // centred y - count, offset by 2^61: |centred y| <= q_last / 2 < 2^60,
            // count < K, so 0 < pv < 2^62 (its top byte < 64, a positive signed byte)
            const int64_t yc = y > (ql >> 1) ? (int64_t)y - (int64_t)ql : (int64_t)y;
            pv = (u64)(yc - (int64_t)cntv + (int64_t)(1ull << 61));
        }
        u64 pvc[4];  // the P term of column tile c, coefficient nb + 16 c + col
#pragma unroll
        for (int c = 0; c < 4; ++c) pvc[c] = __shfl(pv, 16 * c + col);
        // B fragments: the scaled special residues (sources i < KT) and the P term (i = KT)
        v4i bf[4][KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            u64 yy[2][4];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int i = 8 * ks + 2 * lg + h;
                if (i < KT) {
                    const u64 w = phinv[i], wp = phinv_s[i], q = mods[nq + i].q;
                    const u64 *sp = src + (size_t)(1 + i) * n + nb + col;
#pragma unroll
                    for (int c = 0; c < 4; ++c) yy[h][c] = mul_shoup(sp[16 * c], w, wp, q) ^ XMASK;
                } else {
#pragma unroll
                    for (int c = 0; c < 4; ++c) yy[h][c] = (i == KT ? pvc[c] : 0) ^ XMASK;
                }
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) bf[c][ks] = bytes_of(yy[0][c], yy[1][c]);
        }
#pragma unroll 1
        for (int grp = 0; grp < ng; ++grp) {
            v4i a4[4][2];
            const v4i *ag = afr + (size_t)grp * 2 * KS * 64 + lane;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const v4i a0 = ag[ks * 64], a1 = ag[(KS + ks) * 64];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    a4[c][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, bf[c][ks], ks ? a4[c][0] : v4i{0, 0, 0, 0}, 0, 0, 0);
                    a4[c][1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, bf[c][ks], ks ? a4[c][1] : v4i{0, 0, 0, 0}, 0, 0, 0);
                }
            }
            const int tl = 4 * grp + lg, t = 4 * g0 + tl;
            if (t < T) {
                const Mod mt = tm[tl];
                u64 *o = dst + (size_t)t * n + nb + col;
                if (mt.q < FOLD_FP_QMAX) {
                    const double qd = (double)mt.q, qid = tqi[tl];
                    const u64 cr = cfp[tl];
#pragma unroll
                    for (int c = 0; c < 4; ++c) o[16 * c] = fold_rows2_fp(a4[c][0], a4[c][1], qd, qid, cr);
                } else {
                    const u64 w1s = shoup_one(mt), cr = corr[tl];
#pragma unroll
                    for (int c = 0; c < 4; ++c) o[16 * c] = fold_rows2(a4[c][0], a4[c][1], mt, w1s, cr);
                }
            }
        }
    }
}
inline dim3 ew_grid(int logN, int limbs, int segs) {
    const size_t n = (size_t)1 << logN;
    return dim3((unsigned)((n / 2 + NT - 1) / NT), (unsigned)limbs, (unsigned)segs);
}
inline dim3 pt_grid(int logN, int y, int z) {
    const size_t n = (size_t)1 << logN;
    return dim3((unsigned)((n + NT - 1) / NT), (unsigned)y, (unsigned)z);
}
}  // namespace

int set_mfma_sums(int mask) {
    const int prev = mfma_mask();
    if (mask >= 0) g_mfma_mask.store(mask & 7, std::memory_order_relaxed);
    return prev;
}

// ============================================================ wrappers =====
void ew_add(u64 *out, const u64 *a, const u64 *b, int limbs, int segs, Seg S, const Mod *mods, int logN,
            hipStream_t st) {
    if (limbs <= 0 || segs <= 0) return;
    const double B = 8.0 * 3 * limbs * segs * ((size_t)1 << logN);
    launch_clocked("k_add", B, k_add, ew_grid(logN, limbs, segs), dim3(NT), st, out, a, b, S, mods, logN);
}
void ew_sub(u64 *out, const u64 *a, const u64 *b, int limbs, int segs, Seg S, const Mod *mods, int logN,
            hipStream_t st) {
    if (limbs <= 0 || segs <= 0) return;
    hipLaunchKernelGGL(k_sub, ew_grid(logN, limbs, segs), dim3(NT), 0, st, out, a, b, S, mods, logN);
}
void ew_neg(u64 *out, const u64 *a, int limbs, int segs, Seg S, const Mod *mods, int logN, hipStream_t st) {
    if (limbs <= 0 || segs <= 0) return;
    hipLaunchKernelGGL(k_neg, ew_grid(logN, limbs, segs), dim3(NT), 0, st, out, a, S, mods, logN);
}
void ew_mul_scalar(u64 *out, const u64 *a, int64_t K, int limbs, int segs, Seg S, const Mod *mods, int logN,
                   hipStream_t st, int sh) {
    if (limbs <= 0 || segs <= 0) return;
    const double B = 8.0 * 2 * limbs * segs * ((size_t)1 << logN);
    launch_clocked("k_mul_scalar", B, k_mul_scalar, ew_grid(logN, limbs, segs), dim3(NT), st, out, a, K, sh, S, mods,
                   logN);
}
void ew_add_scaled(u64 *out, const u64 *a, const LimbConsts &W, int limbs, Seg S, const Mod *mods, int logN,
                   hipStream_t st) {
    if (limbs <= 0) return;
    if (limbs > LIMB_CONSTS_MAX) throw std::invalid_argument("ew_add_scaled: too many limbs");
    const double B = 8.0 * 3 * limbs * ((size_t)1 << logN);
    launch_clocked("k_add_scaled", B, k_add_scaled, ew_grid(logN, limbs, 1), dim3(NT), st, out, a, W, S, mods, logN);
}
void ew_add_scalar(u64 *out, const u64 *a, int64_t K, int limbs, int segs, Seg S, const Mod *mods, int logN,
                   hipStream_t st, int sh) {
    if (limbs <= 0 || segs <= 0) return;
    hipLaunchKernelGGL(k_add_scalar, ew_grid(logN, limbs, segs), dim3(NT), 0, st, out, a, K, sh, S, mods, logN);
}
void ew_c0_op(u64 *out, const u64 *a, const u64 *p, int64_t K, int sh, int mode, int limbs, int members,
              const Mod *mods, int logN, hipStream_t st) {
    if (limbs <= 0 || members <= 0) return;
    hipLaunchKernelGGL(k_c0_op, ew_grid(logN, limbs, 2 * members), dim3(NT), 0, st, out, a, p, K, sh, mode,
                       (size_t)limbs << logN, mods, logN);
}
void ew_mul_plain(u64 *out, const u64 *a, const u64 *p, int limbs, int segs, Seg S, const Mod *mods, int logN,
                  hipStream_t st) {
    if (limbs <= 0 || segs <= 0) return;
    hipLaunchKernelGGL(k_mul_plain, ew_grid(logN, limbs, segs), dim3(NT), 0, st, out, a, p, S, mods, logN);
}
void ew_tensor(u64 *d01, u64 *d2, const u64 *a, const u64 *b, int limbs, int members, size_t sa, size_t sb,
               const Mod *mods, int logN, hipStream_t st, const u64 *a2, size_t sa2) {
    if (limbs <= 0 || members <= 0) return;
    const size_t ln_all = (size_t)limbs << logN;
    const double B = 8.0 * (5.0 * members + 2.0 * (sb ? members : 1) + (a2 ? 2.0 * members : 0.0)) * ln_all;
    launch_clocked("k_tensor", B, k_tensor, ew_grid(logN, limbs, members), dim3(NT), st, d01, d2, a, b, ln_all, sa, sb,
                   a2, sa2, mods, logN);
}
bool ew_tensor_lin(u64 *d01, u64 *d2, const u64 *a, const u64 *b, int limbs, int members, size_t sa, size_t sb,
                   const u64 *const *xs, const int64_t *K, const uint8_t *sh, int m, size_t xseg, const Mod *mods,
                   int logN, hipStream_t st, const u64 *a2, size_t sa2) {
    if (m < 1 || m > TL_MAX || limbs <= 0 || members <= 0) return false;
    const size_t ln_all = (size_t)limbs << logN;
    TensorLin L{};
    for (int i = 0; i < m; ++i) {
        L.x[i] = xs[i];
        L.K[i] = K[i];
        L.sh[i] = sh ? sh[i] : 0;
    }
    L.xseg = xseg;
    const double B = 8.0 * (5.0 * members + 2.0 * (sb ? members : 1) + (a2 ? 2.0 * members : 0.0) + 2.0 * m * members) *
                     ln_all;
    dispatch_int<1, TL_MAX>(m, [&](auto mm) {
        constexpr int MM = decltype(mm)::value;
        launch_clocked(inst_name<MM>("k_tensor_lin"), B, k_tensor_lin<MM>, ew_grid(logN, limbs, members), dim3(NT), st,
                       d01, d2, a, b, ln_all, sa, sb, a2, sa2, L, mods, logN);
    });
    return true;
}
void ew_sum_members(u64 *out, const u64 *in, int members, int limbs, const Mod *mods, int logN, hipStream_t st) {
    if (limbs <= 0 || members <= 0) return;
    const size_t ln_all = (size_t)limbs << logN;
    hipLaunchKernelGGL(k_sum_members, ew_grid(logN, limbs, 2), dim3(NT), 0, st, out, in, members, ln_all, mods, logN);
}
void ew_linear_sum(u64 *out, const u64 *const *xs, const int64_t *K, int m, int limbs, int segs, size_t seg,
                   size_t xseg, const Mod *mods, int logN, hipStream_t st, bool accumulate, const uint8_t *sh) {
    if (limbs <= 0) return;
    for (int base = 0; base < m || (m == 0 && base == 0); base += LIN_MAX) {
        LinArgs A{};
        A.m = std::min(LIN_MAX, m - base);
        A.accumulate = base > 0 || accumulate;
        A.xseg = xseg;
        for (int i = 0; i < A.m; ++i) {
            A.x[i] = xs[base + i];
            A.K[i] = K[base + i];
            A.sh[i] = sh ? sh[base + i] : 0;
        }
        const double B = 8.0 * (A.m + A.accumulate + 1) * limbs * segs * ((size_t)1 << logN);
        launch_clocked("k_linear_sum", B, k_linear_sum, ew_grid(logN, limbs, segs), dim3(NT), st, out, A, seg, mods,
                       logN);
        if (m == 0) break;
    }
}
// FHE_LEAF_FOLD (A/B, default 1): the folded-constant leaf-sum kernel
// (k_leaf_sums_fold) for rings >= 2^10; 0 keeps the window kernel.  Measured with
// 32-leaf passes: leaf launch 8428 -> 6881 us, sort 531.5 / 531.5 -> 523.2 / 523.1
// ms (profiles/r5_p)
int leaf_fold_enabled() {
    static const int v = [] {
        const char *e = std::getenv("FHE_LEAF_FOLD");
        return e ? std::atoi(e) : 1;
    }();
    return v;
}
bool linear_sums_on_mfma(int logN) { return use_mfma_sums(MF_LIN) && logN >= 8; }
void ew_linear_sum_multi(u64 *const *outs, int G, const u64 *const *xs, const size_t *xseg, const int64_t *K, int m,
                         int limbs, int segs, size_t seg, const Mod *mods, int logN, hipStream_t st,
                         const uint8_t *sh, const int64_t *dK, const uint8_t *dsh) {
    if (limbs <= 0 || segs <= 0 || G <= 0 || m <= 0) return;
    if (G > LEAF_G) throw std::invalid_argument("ew_linear_sum_multi: at most LEAF_G outputs per call");
    const size_t n = (size_t)1 << logN;
    if (linear_sums_on_mfma(logN) && dK && dsh && m <= LEAF_M) {
        // one pass: every series the sorts evaluate has k <= 52 baby steps (more
        // than 64 inputs take the VALU passes below)
        {
            LeafArgs A{};
            A.m = m;
            A.G = G;
            A.accumulate = 0;
            for (int g = 0; g < G; ++g) A.out[g] = outs[g];
            A.six = leaf_six_enabled_host();
            for (int i = 0; i < A.m; ++i) {
                A.x[i] = xs[i];
                A.xseg[i] = (uint32_t)xseg[i];
            }
            A.K = dK;
            A.sh = dsh;
            const double B = 8.0 * (A.m + (double)G * (1 + A.accumulate)) * limbs * segs * (double)n;
            size_t ch = std::min<size_t>(LS_CH_MAX, n);
            while (ch > 256 && (n / ch) * (size_t)limbs * (size_t)segs < 2048) ch /= 2;
            const dim3 grid((unsigned)((n + ch - 1) / ch), (unsigned)limbs, (unsigned)segs);
            // NG: the LDS table's groups of four outputs, the launch's rounded up to 1, 2, 4, 8
            const int ngc = (G + 3) / 4 <= 1 ? 1 : (G + 3) / 4 <= 2 ? 2 : (G + 3) / 4 <= 4 ? 3 : 4;
            if (leaf_fold_enabled() && n >= 2 * (size_t)LFF_NT) {
                size_t chf = std::min<size_t>(LS_CH_MAX, n);
                while (chf > 2 * (size_t)LFF_NT && (n / chf) * (size_t)limbs * (size_t)segs < 1024) chf /= 2;
                const dim3 gridf((unsigned)((n + chf - 1) / chf), (unsigned)limbs, (unsigned)segs);
                dispatch_int<1, 8>((A.m + 7) / 8, [&](auto ks) {
                    dispatch_int<1, 4>(ngc, [&](auto ng) {
                        constexpr int KS = decltype(ks)::value, NG = 1 << (decltype(ng)::value - 1);
                        launch_clocked(inst_name<KS, NG>("k_leaf_sums_fold"), B, k_leaf_sums_fold<KS, NG>, gridf,
                                       dim3(LFF_NT), st, A, seg, mods, logN, (int)chf);
                    });
                });
                return;
            }
            dispatch_int<1, 8>((A.m + 7) / 8, [&](auto ks) {
                dispatch_int<1, 4>(ngc, [&](auto ng) {
                    constexpr int KS = decltype(ks)::value, NG = 1 << (decltype(ng)::value - 1);
                    launch_clocked(inst_name<KS, NG>("k_leaf_sums_mfma"), B, k_leaf_sums_mfma<KS, NG>, grid, dim3(LF_NT),
                                   st, A, seg, mods, logN, (int)ch);
                });
            });
        }
        return;
    }
    // VALU: passes of <= 10 outputs x 32 inputs
    for (int g0 = 0; g0 < G; g0 += MLS_G) {
        const int Gp = std::min(MLS_G, G - g0);
        for (int base = 0; base < m; base += MLS_M) {
            MultiLinArgs A{};
            A.m = std::min(MLS_M, m - base);
            A.G = Gp;
            A.accumulate = base > 0;
            for (int g = 0; g < Gp; ++g) A.out[g] = outs[g0 + g];
            for (int i = 0; i < A.m; ++i) {
                A.x[i] = xs[base + i];
                A.xseg[i] = xseg[base + i];
                for (int g = 0; g < Gp; ++g) {
                    A.K[g * MLS_M + i] = K[(size_t)(g0 + g) * m + base + i];
                    A.sh[g * MLS_M + i] = sh ? sh[(size_t)(g0 + g) * m + base + i] : 0;
                }
            }
            const double B = 8.0 * (A.m + (double)Gp * (1 + A.accumulate)) * limbs * segs * (double)n;
            const dim3 grid = pt_grid(logN, limbs, segs);
            switch (Gp) {
#define MLS_CASE(g)                                                                                               \
    case g:                                                                                                       \
        launch_clocked(inst_name<g>("k_linear_sum_multi"), B, k_linear_sum_multi<g>, grid, dim3(NT), st, A, seg, mods, \
                       logN);                                                                                     \
        break;
                MLS_CASE(1) MLS_CASE(2) MLS_CASE(3) MLS_CASE(4) MLS_CASE(5) MLS_CASE(6) MLS_CASE(7) MLS_CASE(8) MLS_CASE(9)
                    MLS_CASE(10)
#undef MLS_CASE
            }
        }
    }
}
void ew_mul_plain_sum(u64 *out, const u64 *const *cts, const u64 *const *pts, int m, int limbs, int members,
                      size_t cmember, size_t cpoly, const Mod *mods, int logN, hipStream_t st) {
    if (limbs <= 0 || members <= 0 || m <= 0) return;
    const size_t seg = (size_t)limbs << logN;
    for (int base = 0; base < m; base += LIN_MAX) {
        PlainSumArgs A{};
        A.m = std::min(LIN_MAX, m - base);
        A.accumulate = base > 0;
        A.cmember = cmember;
        A.cpoly = cpoly;
        for (int i = 0; i < A.m; ++i) {
            A.ct[i] = cts[base + i];
            A.pt[i] = pts[base + i];
        }
        const double B = 8.0 * ((double)A.m * (cmember ? 2 * members : 2) + A.m + 2.0 * members * (1 + A.accumulate)) *
                         limbs * ((size_t)1 << logN);
        const dim3 g0 = ew_grid(logN, limbs, 2 * members);
        // FHE_PS_XCD (A/B, default 1): XCD-grouped flat grid when the tiles divide by 8
        static const int xcd_env = [] {
            const char *e = std::getenv("FHE_PS_XCD");
            return e ? std::atoi(e) : 1;
        }();
        const unsigned tiles = g0.x * g0.y;
        if (xcd_env && tiles % 8 == 0 && (size_t)tiles * g0.z < (1ull << 31)) {
            A.xcd = 1;
            A.segs = (int)g0.z;
            A.cblocks = (int)g0.x;
            launch_clocked("k_mul_plain_sum", B, k_mul_plain_sum, dim3(tiles * g0.z), dim3(NT), st, out, A, seg, mods,
                           logN);
        } else {
            launch_clocked("k_mul_plain_sum", B, k_mul_plain_sum, dim3(g0.z, g0.x, g0.y), dim3(NT), st, out, A, seg,
                           mods, logN);
        }
    }
}
void ew_permute(u64 *out, const u64 *in, const uint32_t *perm, int limbs, int segs, Seg S, int logN,
                hipStream_t st) {
    if (limbs <= 0 || segs <= 0) return;
    note_launch("k_permute", pt_grid(logN, limbs, segs), dim3(NT));
    hipLaunchKernelGGL(k_permute, pt_grid(logN, limbs, segs), dim3(NT), 0, st, out, in, perm, S, logN);
}
void ew_signed_to_rns(u64 *out, const int64_t *coef, int limbs, const int *pmap, const Mod *mods, int logN,
                      hipStream_t st, int members, size_t out_stride, size_t coef_stride) {
    if (limbs <= 0 || members <= 0) return;
    hipLaunchKernelGGL(k_signed_to_rns, pt_grid(logN, limbs, members), dim3(NT), 0, st, out, coef, pmap, mods, logN,
                       out_stride, coef_stride);
}
void ew_lift_centered(u64 *out, const u64 *in, int src, int limbs, int segs, size_t seg_in, size_t seg_out,
                      const Mod *mods, int logN, hipStream_t st) {
    if (limbs <= 0 || segs <= 0) return;
    hipLaunchKernelGGL(k_lift_centered, pt_grid(logN, limbs, segs), dim3(NT), 0, st, out, in, seg_in, seg_out, src,
                       mods, logN);
}
// empty one-wave kernels delimiting a profiled region in a rocprofv3 kernel
// trace or PMC pass (scripts/pmc_meta.py region filter); write nothing
__global__ void k_region_begin() {}
__global__ void k_region_end() {}
void region_marker(bool begin, hipStream_t st) {
    if (begin)
        hipLaunchKernelGGL(k_region_begin, dim3(1), dim3(64), 0, st);
    else
        hipLaunchKernelGGL(k_region_end, dim3(1), dim3(64), 0, st);
}
void ew_reduce(u64 *x, int limbs, int segs, size_t seg, const Mod *mods, int logN, hipStream_t st) {
    if (limbs <= 0 || segs <= 0) return;
    hipLaunchKernelGGL(k_reduce, ew_grid(logN, limbs, segs), dim3(NT), 0, st, x, Seg{seg, seg, 0}, mods, logN);
}

// FHE_MODUP_FOLD (A/B): the folded-constant MFMA ModUp conversion (k_modup_fold):
// 0 off, 1 always, N >= 2 launches of >= N (member, digit) pairs; default -1:
// digits of more than 16 sources (MEHP24's alpha = 22: 11.08 -> 10.80 s; at the
// N=1024 sort's alpha = 14 it ties the VALU kernel, 154.6 vs 158.2 us avg;
// profiles/r5_s, r5_u)
int modup_fold_enabled() {
    static const int v = [] {
        const char *e = std::getenv("FHE_MODUP_FOLD");
        return e ? std::atoi(e) : -1;
    }();
    return v;
}
// FHE_MODUP_FP (A/B): 0 = the 128-bit kernel only, N >= 1 = the fp64 kernel for
// digits of at least N sources (default 0: measured slower, profiles/r6_c)
int modup_fp_min_sources() {
    static const int v = [] {
        const char *e = std::getenv("FHE_MODUP_FP");
        return e ? std::atoi(e) : 0;
    }();
    return v;
}
void modup_convert(u64 *ext, const u64 *coef, int ell, int K, int alpha, int digits, int members,
                   size_t coef_stride, size_t ext_stride, const int *pmap_ext, const u64 *tabs,
                   const size_t *tab_off, const Mod *mods, int logN, hipStream_t st, const double *fptab,
                   const size_t *fp_off, int fpmid) {
    const int W = ell + K;
    ModUpArgs A{};
    for (int j = 0; j < digits; ++j) {
        const u64 *base = tabs + tab_off[j];
        A.qhinv[j] = base;
        A.qhinv_s[j] = base + alpha;
        A.qhat[j] = base + 2 * alpha;
        A.lo[j] = j * alpha;
        A.hi[j] = std::min((j + 1) * alpha, ell);
        if (fptab && fp_off) {
            A.fpc[j] = fptab + fp_off[j];
            A.fpq[j] = fptab + fp_off[j] + (size_t)W * alpha * 4;
        }
    }
    const bool fp0 = fptab && fp_off && fpmid >= 0 && modup_fp_min_sources() > 0 && ((size_t)1 << logN) % NT == 0;
    A.digits = digits;
    A.qstride = alpha;
    A.coef_stride = coef_stride;
    A.ext_stride = ext_stride;
    // a partial last digit (ell % alpha sources) runs in its own launch with a
    // straight-line source loop of its true length, instead of alpha terms of
    // which most multiply a zero constant (at the PS levels, ell ~ 17-25 with
    // alpha 14, that was up to 4x the MACs of that digit)
    const int last = ell - (digits - 1) * alpha;
    const int full = last == alpha ? digits : digits - 1;
    const size_t n = (size_t)1 << logN;
    auto launch = [&](int nd, int at, const ModUpArgs &Ar, u64 *ext0) {
        const double B = 8.0 * members * (double)((size_t)nd * W) * (double)n;  // sources in + targets out
        const bool fp = fp0 && at >= modup_fp_min_sources();
        const int mf = modup_fold_enabled();
        const bool fold = mf < 0 ? at > 16 : mf == 1 || (mf >= 2 && nd * members >= mf);
        if (fold && n >= (size_t)MUF_NT && at <= 32) {  // (KS <= 4: no spills)
            // every target group of a digit in one block when they fit the LDS table
            // (muf_gpc groups of four), else chunks over grid.y; coefficient chunks
            // of up to 4096 per block, smaller while the grid has < 2048 blocks
            const int ngt = (W - at + 3) / 4;
            dispatch_int<1, 4>((at + 7) / 8, [&](auto c) {
                constexpr int KS = decltype(c)::value;
                const int chunks = (ngt + muf_gpc(KS) - 1) / muf_gpc(KS), gpc = (ngt + chunks - 1) / chunks;
                size_t ch = std::min<size_t>(4096, n);
                while (ch > (size_t)MUF_NT && (n / ch) * (size_t)chunks * (size_t)(nd * members) < 2048) ch /= 2;
                launch_clocked(inst_name<KS>("k_modup_fold"), B, k_modup_fold<KS>,
                               dim3((unsigned)(n / ch), (unsigned)chunks, (unsigned)(nd * members)), dim3(MUF_NT), st,
                               ext0, coef, W, ell, Ar, pmap_ext, mods, logN, gpc, (int)ch);
            });
            return;
        }
        if (use_mfma_sums(MF_MODUP) && n >= 256) {
            // groups of four targets, chunked over grid.y when the launch is narrow
            const int ngt = (W - at + 3) / 4;
            const size_t base = n / 256 * (size_t)(nd * members);
            const int chunks = base >= 2048 ? 1 : std::min(ngt, (int)((2048 + base - 1) / base));
            const int gpc = (ngt + chunks - 1) / chunks;
            dispatch_int<1, 3>((at + 7) / 8, [&](auto c) {
                constexpr int KS = decltype(c)::value;
                launch_clocked(inst_name<KS>("k_modup_mfma"), B, k_modup_mfma<KS>,
                               dim3((unsigned)(n / 256), (unsigned)((ngt + gpc - 1) / gpc), (unsigned)(nd * members)),
                               dim3(NT), st, ext0, coef, W, ell, Ar, pmap_ext, mods, logN, gpc);
            });
            return;
        }
        dispatch_int<1, 24>(at, [&](auto c) {
            constexpr int AT = decltype(c)::value;
            if (!fp) {
                const int tch = conv_chunk(logN, W, nd * members);
                launch_clocked(inst_name<AT>("k_modup_convert"), B, k_modup_convert<AT>,
                               pt_grid(logN, (W + tch - 1) / tch, nd * members), dim3(NT), st, ext0, coef, W, ell, Ar,
                               pmap_ext, mods, logN, tch, 0);
                return;
            }
            // the fp64 kernel takes the Q targets (q_0 through its integer path), the
            // 128-bit kernel the K special primes beside it (each reads the sources)
            const int Tq = ell - at, Kt = W - ell;
            const double Bq = 8.0 * members * (double)nd * (at + Tq) * (double)n;
            const double Bk = 8.0 * members * (double)nd * (at + Kt) * (double)n;
            const int tq = conv_chunk(logN, Tq, nd * members);
            const dim3 gq = pt_grid(logN, (Tq + tq - 1) / tq, nd * members);
            if (Tq > 0) {
                if (fpmid == 0)
                    launch_clocked(inst_name<AT, 0>("k_modup_fp"), Bq, k_modup_fp<AT, 0>, gq, dim3(NT), st, ext0, coef, W,
                                   ell, Ar, pmap_ext, mods, logN, tq, 1);
                else
                    launch_clocked(inst_name<AT, 1>("k_modup_fp"), Bq, k_modup_fp<AT, 1>, gq, dim3(NT), st, ext0, coef, W,
                                   ell, Ar, pmap_ext, mods, logN, tq, 1);
            }
            const int tk = conv_chunk(logN, Kt, nd * members);
            launch_clocked(inst_name<AT>("k_modup_convert"), Bk, k_modup_convert<AT>,
                           pt_grid(logN, (Kt + tk - 1) / tk, nd * members), dim3(NT), st, ext0, coef, W, ell, Ar,
                           pmap_ext, mods, logN, tk, ell);
        });
    };
    if (full > 0) {
        ModUpArgs Af = A;
        Af.digits = full;
        launch(full, alpha, Af, ext);
    }
    if (full < digits) {
        const int j = digits - 1;
        ModUpArgs Al = A;
        Al.digits = 1;
        Al.qhinv[0] = A.qhinv[j];
        Al.qhinv_s[0] = A.qhinv_s[j];
        Al.qhat[0] = A.qhat[j];
        Al.lo[0] = A.lo[j];
        Al.hi[0] = A.hi[j];
        Al.fpc[0] = A.fpc[j];
        Al.fpq[0] = A.fpq[j];
        launch(1, last, Al, ext + (size_t)j * W * n);
    }
}
void ks_inner(u64 *acc, const u64 *ext, const u64 *dntt, const u64 *key, int ell, int K, int nq, int nall,
              int alpha, int digits, const uint32_t *perm, const int *pmap_ext, const Mod *mods, int logN,
              hipStream_t st, int members, KsStrides str, KsFold fold, int tcount) {
    (void)nq;
    const int W = ell + K;
    const int TW = tcount < 0 ? W : tcount;  // targets of this launch
    if (TW == 0) return;
    // ext (+ own digit) and 2 accumulators per member; the key once
    const double B = 8.0 * ((double)members * (digits * TW + 2.0 * TW) + 2.0 * digits * TW) * ((size_t)1 << logN);
    // member groups of MC (FHE_KS_MC=4 for A/B): the key words stay in registers
    // for the MC members of a thread; 8 reads the key half as often as 4
    // (MEHP24 12.74 -> 12.69 s, DirectSort 690.8 -> 689.0 ms, profiles/r3_h)
    static const int mc_env = [] {
        const char *e = std::getenv("FHE_KS_MC");
        return e && std::atoi(e) == 4 ? 4 : 8;
    }();
    if (members >= 4) {
        dispatch_int<1, 8>(digits, [&](auto c) {
            constexpr int D = decltype(c)::value;
            auto go = [&](auto mcc) {
                constexpr int MC = decltype(mcc)::value;
                const dim3 grid((unsigned)((((size_t)1 << logN) + NT - 1) / NT), (unsigned)TW,
                                (unsigned)((members + MC - 1) / MC));
                launch_clocked(inst_name<D, MC>("k_ks_inner_mc"), B, k_ks_inner_mc<D, MC>, grid, dim3(NT), st, acc, ext, dntt, key, ell, W,
                               nall, alpha, members, perm, pmap_ext, mods, logN, str, fold);
            };
            // 8 members x 5+ digits would spill the x words to scratch
            if constexpr (D <= 4) {
                if (mc_env == 8 && members >= 8)
                    go(std::integral_constant<int, 8>{});
                else
                    go(std::integral_constant<int, 4>{});
            } else {
                go(std::integral_constant<int, 4>{});
            }
        });
        return;
    }
    const dim3 grid((unsigned)members, (unsigned)((((size_t)1 << logN) + NT - 1) / NT), (unsigned)TW);
    dispatch_int<1, 8>(digits, [&](auto c) {
        constexpr int D = decltype(c)::value;
        launch_clocked(inst_name<D>("k_ks_inner"), B, k_ks_inner<D>, grid, dim3(NT), st, acc, ext, dntt, key, ell, W, nall, alpha,
                       perm, pmap_ext, mods, logN, str, fold);
    });
}
void ks_inner_multikey(u64 *acc, const u64 *ext, const u64 *dntt, const KsKeys &keys, int count, int ell, int K,
                       int nall, int alpha, int digits, const int *pmap_ext, const Mod *mods, int logN,
                       hipStream_t st, KsStrides str) {
    if (count <= 0) return;
    if (count > KS_MAXKEYS) throw std::invalid_argument("ks_inner_multikey: too many keys");
    const int W = ell + K;
    // ext (shared or per member), the accumulators and every member's key
    const double shared = str.ext ? 0.0 : 1.0;
    const double B = 8.0 * ((shared + (1 - shared) * count) * digits * W + count * (2.0 * W + 2.0 * digits * W)) *
                     ((size_t)1 << logN);
    const dim3 grid((unsigned)count, (unsigned)((((size_t)1 << logN) + NT - 1) / NT), (unsigned)W);
    dispatch_int<1, 8>(digits, [&](auto c) {
        constexpr int D = decltype(c)::value;
        launch_clocked(inst_name<D>("k_ks_inner_mk"), B, k_ks_inner_mk<D>, grid, dim3(NT), st, acc, ext, dntt, keys, ell, W, nall,
                       alpha, pmap_ext, mods, logN, str);
    });
}
void ks_inner_multikey_sum(u64 *acc, const u64 *ext, const u64 *dntt, const KsKeys &keys, int count, bool accumulate,
                           int ell, int K, int nall, int alpha, int digits, const int *pmap_ext, const Mod *mods,
                           int logN, hipStream_t st, KsStrides str) {
    if (count <= 0) return;
    if (count > KS_MAXKEYS) throw std::invalid_argument("ks_inner_multikey_sum: too many keys");
    const int W = ell + K;
    // every member's ext and key, one accumulator pair (read when accumulating)
    const double B = 8.0 * (count * 3.0 * digits * W + 2.0 * W * (1 + accumulate)) * ((size_t)1 << logN);
    const dim3 grid((unsigned)((((size_t)1 << logN) + NT - 1) / NT), (unsigned)W);
    dispatch_int<1, 8>(digits, [&](auto c) {
        constexpr int D = decltype(c)::value;
        launch_clocked(inst_name<D>("k_ks_inner_mk_sum"), B, k_ks_inner_mk_sum<D>, grid, dim3(NT), st, acc, ext, dntt, keys, count,
                       (int)accumulate, ell, W, nall, alpha, pmap_ext, mods, logN, str);
    });
}
void lt_inner(u64 *out, const u64 *ext, const u64 *c, const LtArgs &A, bool accumulate, int ell, int K, int nall,
              int alpha, int digits, const int *pmap_ext, const u64 *pmodq, const u64 *pmodq_s, const Mod *mods,
              int logN, hipStream_t st) {
    if (A.nb <= 0) return;
    if (A.nb > LT_MAXB) throw std::invalid_argument("lt_inner: too many babies per launch");
    const int W = ell + K;
    int keyed = 0;
    for (int b = 0; b < A.nb; ++b) keyed += A.key[b] != nullptr;
    // per keyed baby: its key and the gathered ext digits; per baby a plaintext;
    // the ciphertext once, the accumulator pair out (and in)
    const double B = 8.0 * ((double)keyed * 3.0 * digits * W + (double)A.nb * W + 2.0 * ell + 2.0 * W * (1 + accumulate)) *
                     ((size_t)1 << logN);
    const dim3 grid((unsigned)((((size_t)1 << logN) + NT - 1) / NT), (unsigned)W);
    dispatch_int<1, 8>(digits, [&](auto dc) {
        constexpr int D = decltype(dc)::value;
        launch_clocked(inst_name<D>("k_lt_inner"), B, k_lt_inner<D>, grid, dim3(NT), st, out, ext, c, A, (int)accumulate, ell, W,
                       nall, alpha, pmap_ext, pmodq, pmodq_s, mods, logN);
    });
}
void ew_permute_sum(u64 *out, const u64 *in, const KsKeys &keys, int limbs, int count, bool accumulate, size_t in_stride,
                    const Mod *mods, int logN, hipStream_t st) {
    if (limbs <= 0 || count <= 0) return;
    if (count > KS_MAXKEYS) throw std::invalid_argument("ew_permute_sum: too many keys");
    hipLaunchKernelGGL(k_permute_sum, pt_grid(logN, limbs, 1), dim3(NT), 0, st, out, in, keys, count, (int)accumulate,
                       Seg{0, in_stride, 0}, mods, logN);
}
void ew_permute_multi(u64 *out, const u64 *in, const KsKeys &keys, int limbs, int count, Seg S, int logN,
                      hipStream_t st) {
    if (limbs <= 0 || count <= 0) return;
    if (count > KS_MAXKEYS) throw std::invalid_argument("ew_permute_multi: too many keys");
    hipLaunchKernelGGL(k_permute_mk, pt_grid(logN, limbs, count), dim3(NT), 0, st, out, in, keys, S, logN);
}
// FHE_MODDOWN_FOLD (A/B, default 0): the folded-constant MFMA ModDown+rescale
// conversion -- measured slower at K = 10 (346 vs 276 us, the N=1024 sort
// 522.8 -> 528.7 ms) and no gain at MEHP24's K = 16 (profiles/r5_t, r5_u)
int moddown_fold_enabled() {
    static const int v = [] {
        const char *e = std::getenv("FHE_MODDOWN_FOLD");
        return e ? std::atoi(e) : 0;
    }();
    return v;
}
// FHE_MDFP_I32 (default 1; 0: A/B): the fp64 ModDown kernel's sources as int32
// (yh, yl) pairs in LDS -- half the LDS of double pairs, 56 / 83 VGPRs and 7 / 4
// waves per SIMD at K = 10 / 16 against 91 / 136 and 3 / 2 (MEHP24 -3.2%,
// profiles/r6_ab/mdfp_i32_ab.jsonl)
int mdfp_i32() {
    static const int v = [] {
        const char *e = std::getenv("FHE_MDFP_I32");
        return e ? std::atoi(e) : 1;
    }();
    return v;
}
// FHE_CONV_TPI (A/B, 2 or 4): targets per work item of the fp64 ModDown kernel
int conv_tpi() {
    static const int v = [] {
        const char *e = std::getenv("FHE_CONV_TPI");
        return e && std::atoi(e) == 4 ? 4 : 2;
    }();
    return v;
}
// FHE_MODDOWN_FP (A/B): 0 = the 128-bit kernel only, N >= 1 = the fp64 kernel for
// conversions of at least N targets (default 1, every conversion whose bounds
// hold: with the int32 sources the fp64 kernel wins at every size down to 6
// targets, profiles/r6_ab/mdfp_min_ab.jsonl; with double sources it lost below 16)
int moddown_fp_min_targets() {
    static const int v = [] {
        const char *e = std::getenv("FHE_MODDOWN_FP");
        return e ? std::atoi(e) : 1;
    }();
    return v;
}
void moddown_rescale_convert(u64 *corr, const u64 *acc, int ell, int K, int nq, size_t seg_acc, size_t seg_corr,
                             int segs, const u64 *phinv, const u64 *phinv_s, const u64 *phat, const u64 *pinv,
                             const u64 *pinv_s, const u64 *pmod, const double *pinvd, const u64 *ninv,
                             const u64 *ninv_s, const Mod *mods, int logN, hipStream_t st, const u64 *pmod_s,
                             const double *fpc, const double *fpq, int fpmid) {
    if (ell <= 1) return;
    const double B = 8.0 * segs * (double)(K + 1 + ell - 1) * ((size_t)1 << logN);
    const size_t n = (size_t)1 << logN;
    // FHE_MODDOWN_FOLD = 1: always; N >= 2: launches of >= N segments
    const int mdf = moddown_fold_enabled();
    if (mdf && (mdf == 1 || segs >= mdf) && n >= (size_t)MDF_NT && K + 1 <= 32) {
        const int ngt = (ell - 1 + 3) / 4;
        dispatch_int<1, 16>(K, [&](auto c) {
            constexpr int KT = decltype(c)::value, KS = (KT + 1 + 7) / 8;
            const int chunks = (ngt + muf_gpc(KS) - 1) / muf_gpc(KS), gpc = (ngt + chunks - 1) / chunks;
            size_t ch = std::min<size_t>(4096, n);
            while (ch > (size_t)MDF_NT && (n / ch) * (size_t)chunks * (size_t)segs < 2048) ch /= 2;
            launch_clocked(inst_name<KS, KT>("k_moddown_rescale_fold"), B, k_moddown_rescale_fold<KS, KT>,
                           dim3((unsigned)(n / ch), (unsigned)chunks, (unsigned)segs), dim3(MDF_NT), st, corr, acc, ell,
                           nq, seg_acc, seg_corr, phinv, phinv_s, phat, pinv, pinv_s, pmod, pinvd, ninv, ninv_s, mods,
                           logN, gpc, (int)ch);
        });
        return;
    }
    if (use_mfma_sums(MF_MODDOWN) && n >= 256 && pmod_s) {
        const int ngt = (ell - 1 + 3) / 4;
        const size_t base = n / 256 * (size_t)segs;
        const int chunks = base >= 2048 ? 1 : std::min(ngt, (int)((2048 + base - 1) / base));
        const int gpc = (ngt + chunks - 1) / chunks;
        dispatch_int<1, 16>(K, [&](auto c) {
            constexpr int KT = decltype(c)::value, KS = (KT + 7) / 8;
            launch_clocked(inst_name<KS, KT>("k_moddown_rescale_mfma"), B, k_moddown_rescale_mfma<KS, KT>,
                           dim3((unsigned)(n / 256), (unsigned)((ngt + gpc - 1) / gpc), (unsigned)segs), dim3(NT), st,
                           corr, acc, ell, nq, seg_acc, seg_corr, phinv, phinv_s, phat, pinv, pinv_s, pmod, pmod_s,
                           pinvd, ninv, ninv_s, mods, logN, gpc);
        });
        return;
    }
    if (fpc && fpq && fpmid >= 0 && (moddown_fp_min_targets() > 0 && ell - 1 >= moddown_fp_min_targets()) && n % NT == 0) {
        dispatch_int<1, 16>(K, [&](auto c) {
            constexpr int KT = decltype(c)::value;
            const int tch = conv_chunk(logN, ell - 1, segs);
            const dim3 g((unsigned)(n / NT), (unsigned)((ell - 1 + tch - 1) / tch), (unsigned)segs);
            auto go = [&](auto mid, auto tpi) {
                constexpr int MI = decltype(mid)::value, TP = decltype(tpi)::value;
                if (mdfp_i32())
                    launch_clocked(inst_name<KT, MI, TP, 1>("k_moddown_rescale_fp"), B, k_moddown_rescale_fp<KT, MI, TP, 1>, g,
                                   dim3(NT), st, corr, acc, ell, nq, seg_acc, seg_corr, phinv, phinv_s, phat, pinv, pinv_s,
                                   pmod, pinvd, ninv, ninv_s, mods, fpc, fpq, logN, tch);
                else
                    launch_clocked(inst_name<KT, MI, TP, 0>("k_moddown_rescale_fp"), B, k_moddown_rescale_fp<KT, MI, TP, 0>, g,
                                   dim3(NT), st, corr, acc, ell, nq, seg_acc, seg_corr, phinv, phinv_s, phat, pinv, pinv_s,
                                   pmod, pinvd, ninv, ninv_s, mods, fpc, fpq, logN, tch);
            };
            using I0 = std::integral_constant<int, 0>;
            using I1 = std::integral_constant<int, 1>;
            using I2 = std::integral_constant<int, 2>;
            using I4 = std::integral_constant<int, 4>;
            if (conv_tpi() == 4)
                fpmid == 0 ? go(I0{}, I4{}) : go(I1{}, I4{});
            else
                fpmid == 0 ? go(I0{}, I2{}) : go(I1{}, I2{});
        });
        return;
    }
    dispatch_int<1, 16>(K, [&](auto c) {
        constexpr int KT = decltype(c)::value;
        const int tch = conv_chunk(logN, ell - 1, segs);
        launch_clocked(inst_name<KT>("k_moddown_rescale_convert"), B, k_moddown_rescale_convert<KT>,
                       pt_grid(logN, (ell - 1 + tch - 1) / tch, segs), dim3(NT), st, corr, acc, ell, nq, seg_acc,
                       seg_corr, phinv, phinv_s, phat, pinv, pinv_s, pmod, pinvd, ninv, ninv_s, mods, logN, tch);
    });
}
void moddown_convert(u64 *conv, const u64 *pc, int ell, int K, int nq, size_t seg_in, size_t seg_out, int segs,
                     const u64 *phinv, const u64 *phinv_s, const u64 *phat, const u64 *pmod, const double *pinvd,
                     const Mod *mods, int logN, hipStream_t st) {
    const double B = 8.0 * segs * (double)(K + ell) * ((size_t)1 << logN);
    dispatch_int<1, 16>(K, [&](auto c) {
        constexpr int KT = decltype(c)::value;
        const int tch = conv_chunk(logN, ell, segs);
        launch_clocked(inst_name<KT>("k_moddown_convert"), B, k_moddown_convert<KT>, pt_grid(logN, (ell + tch - 1) / tch, segs),
                       dim3(NT), st, conv, pc, ell, nq, seg_in, seg_out, phinv, phinv_s, phat, pmod, pinvd, mods,
                       logN, tch);
    });
}
void moddown_finish(u64 *out, const u64 *acc, const u64 *conv, const u64 *add, int ell, int segs, size_t seg_out,
                    size_t seg_acc, size_t seg_add, const u64 *pinv, const u64 *pinv_s, const Mod *mods, int logN,
                    hipStream_t st) {
    const double B = 8.0 * (3.0 * segs + (add ? segs / 2 : 0)) * ell * ((size_t)1 << logN);
    launch_clocked("k_moddown_finish", B, k_moddown_finish, ew_grid(logN, ell, segs), dim3(NT), st, out, acc, conv, add,
                   seg_out, seg_acc, seg_add, pinv, pinv_s, mods, logN);
}

// ------------------------------------------------------- fault diagnostics --
namespace {
struct LaunchNote {
    std::atomic<unsigned long long> count{0};
    const char *volatile name = nullptr;
    volatile unsigned g[3] = {0, 0, 0}, b[3] = {0, 0, 0};
};
LaunchNote g_note;
struct sigaction g_prev_segv, g_prev_bus;

// async-signal-safe output helpers
void out_str(const char *s) {
    size_t n = 0;
    while (s[n]) ++n;
    ssize_t r = ::write(2, s, n);
    (void)r;
}
void out_hex(unsigned long long v) {
    char b[19] = "0x";
    for (int i = 0; i < 16; ++i) b[2 + i] = "0123456789abcdef"[(v >> (60 - 4 * i)) & 15];
    b[18] = 0;
    out_str(b);
}
void out_dec(unsigned long long v) {
    char b[24];
    int i = 23;
    b[i] = 0;
    do {
        b[--i] = (char)('0' + v % 10);
        v /= 10;
    } while (v && i > 0);
    out_str(b + i);
}
unsigned long long parse_hex(const char *&p) {
    unsigned long long v = 0;
    for (;; ++p) {
        const char c = *p;
        if (c >= '0' && c <= '9') v = v * 16 + (unsigned)(c - '0');
        else if (c >= 'a' && c <= 'f') v = v * 16 + (unsigned)(c - 'a' + 10);
        else break;
    }
    return v;
}
// print the /proc/self/maps lines whose range holds one of the addresses
void out_maps(unsigned long long a, unsigned long long b) {
    const int fd = ::open("/proc/self/maps", O_RDONLY);
    if (fd < 0) return;
    static char buf[1 << 16];
    static char line[1024];
    size_t ll = 0;
    for (;;) {
        const ssize_t r = ::read(fd, buf, sizeof buf);
        if (r <= 0) break;
        for (ssize_t i = 0; i < r; ++i) {
            const char c = buf[i];
            if (ll + 1 < sizeof line) line[ll++] = c;
            if (c != '\n') continue;
            line[ll] = 0;
            const char *p = line;
            const unsigned long long lo = parse_hex(p);
            if (*p == '-') ++p;
            const unsigned long long hi = parse_hex(p);
            if ((a >= lo && a < hi) || (b >= lo && b < hi) || (b >= hi && b - hi < (1ull << 21)) ||
                (b < lo && lo - b < (1ull << 21))) {
                out_str("  maps: ");
                out_str(line);
            }
            ll = 0;
        }
    }
    ::close(fd);
}
void on_fault(int sig, siginfo_t *si, void *ucv) {
    const auto *uc = static_cast<ucontext_t *>(ucv);
    const unsigned long long pc = uc ? (unsigned long long)uc->uc_mcontext.gregs[REG_RIP] : 0;
    const unsigned long long addr = (unsigned long long)si->si_addr;
    out_str(sig == SIGBUS ? "\n[fhe fault report] SIGBUS" : "\n[fhe fault report] SIGSEGV");
    out_str(" si_code ");
    out_dec((unsigned long long)(si->si_code < 0 ? -si->si_code : si->si_code));
    out_str(si->si_code <= 0 ? " (sent by a process)" : "");
    out_str(" pc ");
    out_hex(pc);
    out_str(" addr ");
    out_hex(addr);
    out_str(" tid ");
    out_dec((unsigned long long)::syscall(SYS_gettid));
    out_str(" pid ");
    out_dec((unsigned long long)::getpid());
    out_str("\n  launches noted: ");
    out_dec(g_note.count.load());
    out_str(", last: ");
    out_str(g_note.name ? g_note.name : "(none)");
    out_str(" grid ");
    out_dec(g_note.g[0]), out_str("x"), out_dec(g_note.g[1]), out_str("x"), out_dec(g_note.g[2]);
    out_str(" block ");
    out_dec(g_note.b[0]);
    out_str("\n");
    out_maps(pc, addr);
    // chain: the previous handler runs when the faulting instruction re-executes
    // (or now, for a signal another thread or process sent)
    sigaction(sig, sig == SIGBUS ? &g_prev_bus : &g_prev_segv, nullptr);
    if (si->si_code <= 0) raise(sig);
}
}  // namespace

bool fault_report_enabled() {
    static const bool on = std::getenv("FHE_FAULT_REPORT") != nullptr;
    return on;
}
void note_launch_slow(const char *name, dim3 grid, dim3 block) {
    g_note.count++;
    g_note.name = name;
    g_note.g[0] = grid.x, g_note.g[1] = grid.y, g_note.g[2] = grid.z;
    g_note.b[0] = block.x, g_note.b[1] = block.y, g_note.b[2] = block.z;
}
void install_fault_report() {
    if (!fault_report_enabled()) return;
    static std::once_flag once;
    std::call_once(once, [] {
        struct sigaction sa {};
        sa.sa_sigaction = on_fault;
        sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
        sigemptyset(&sa.sa_mask);
        sigaction(SIGSEGV, &sa, &g_prev_segv);
        sigaction(SIGBUS, &sa, &g_prev_bus);
        out_str("[fhe fault report] handler installed\n");
    });
}

}  // namespace dev
}  // namespace fhe
