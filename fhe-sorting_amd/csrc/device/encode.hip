// CKKS encoding on the device (round 4): the special inverse FFT of the host
// encoder (host::encode_coeffs, hostmath.cpp special_ifft) restated operation
// for operation in fp64, so the rounded coefficients -- and the plaintexts
// after the RNS split and the NTT -- are word-identical to the host's.
//
//  * stage len (S, S/2, ..., 2), butterfly (i, j < len/2):
//        u = v[i+j] + v[i+j+h];  w = (v[i+j] - v[i+j+h]) * tw_len[j]
//    with complex products written as (ac - bd, ad + bc), compiled with
//    -ffp-contract=off like the host (no fused multiply-adds), and the twiddle
//    tw_len[j] = ksi[(4 len - (rot[j] & (4 len - 1))) * M / (4 len)] read from
//    the host's own ksi / rot tables (uploaded once), never recomputed;
//  * then the bit reversal, / S, * scale and round-half-away-from-zero
//    (std::llround) into the coefficients i * gap (real) and i * gap + n/2
//    (imaginary), every other coefficient 0.
// Stages with len > 4096 run as global passes (one thread per butterfly); the
// last twelve run in one launch per 4096-slot run held in LDS (64 KB).
//
// The sort's public masks are generated on the device too (kernel k_mask_slots:
// mask_vector(k) rotated by r, checking_vector(k), src/sort_algo.h:206-233,
// 272-286), so a batch of masks needs no host-to-device copy of slot values.
#include <hip/hip_runtime.h>

#include "kernels.hpp"

namespace fhe {
namespace dev {

namespace {

constexpr int ENC_L = 4096;  // slots per LDS run (64 KB of double2)
constexpr int ENC_NT = 1024;

__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {  // (ac - bd, ad + bc), two rounded products each
    const double ac = a.x * b.x, bd = a.y * b.y, ad = a.x * b.y, bc = a.y * b.x;
    return make_double2(ac - bd, ad + bc);
}
__device__ __forceinline__ double2 twiddle(const double2 *ksi, const uint32_t *rot, int M, int len, int j) {
    const int lq = len << 2, gap = M / lq;
    return ksi[(size_t)(lq - (int)(rot[j] & (uint32_t)(lq - 1))) * gap];
}

// one stage over every member: B x S/2 butterflies
__global__ __launch_bounds__(256) void k_ifft_stage(double2 *v, int S, int len, const double2 *ksi, const uint32_t *rot,
                                                    int M, size_t total) {
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= total) return;
    const int half = S >> 1, h = len >> 1;
    const size_t b = t / half;
    const int p = (int)(t % half);
    const int i = (p / h) * len, j = p % h;
    double2 *z = v + b * (size_t)S;
    const double2 a = z[i + j], c = z[i + j + h];
    z[i + j] = cadd(a, c);
    z[i + j + h] = cmul(csub(a, c), twiddle(ksi, rot, M, len, j));
}

// stages len0, len0/2, ..., 2 on runs of L = min(S, 4096) slots in LDS; grid
// x = runs per member, y = member
__global__ __launch_bounds__(ENC_NT) void k_ifft_lds(double2 *v, int S, int len0, const double2 *ksi,
                                                     const uint32_t *rot, int M) {
    __shared__ double2 z[ENC_L];
    const int L = S < ENC_L ? S : ENC_L;
    double2 *g = v + (size_t)blockIdx.y * S + (size_t)blockIdx.x * L;
    for (int e = threadIdx.x; e < L; e += ENC_NT) z[e] = g[e];
    __syncthreads();
    for (int len = len0; len >= 2; len >>= 1) {
        const int h = len >> 1;
        for (int p = threadIdx.x; p < (L >> 1); p += ENC_NT) {
            const int i = (p / h) * len, j = p % h;
            const double2 a = z[i + j], c = z[i + j + h];
            z[i + j] = cadd(a, c);
            z[i + j + h] = cmul(csub(a, c), twiddle(ksi, rot, M, len, j));
        }
        __syncthreads();
    }
    for (int e = threadIdx.x; e < L; e += ENC_NT) g[e] = z[e];
}

__device__ __forceinline__ int brev_bits(int x, int bits) { return (int)(__brev((uint32_t)x) >> (32 - bits)); }

// coefficients of member b: bit reversal, / S, * scale[b], round; grid x covers n
__global__ __launch_bounds__(256) void k_ifft_finish(const double2 *v, int64_t *coef, int S, int logS, int n,
                                                     const double *scale, unsigned *overflow) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    const size_t b = blockIdx.y;
    const int gap = n / (2 * S), half = n >> 1;
    const int kk = k < half ? k : k - half;
    int64_t out = 0;
    if (kk % gap == 0) {
        const int i = kk / gap;
        const double2 z = v[b * (size_t)S + brev_bits(i, logS)];
        const double x = (k < half ? z.x / (double)S : z.y / (double)S) * scale[b];
        if (!(fabs(x) < 9.2e18)) atomicOr(overflow, 1u);
        out = (int64_t)round(x);  // ties away from zero, as std::llround
    }
    coef[b * (size_t)n + k] = out;
}

// sort masks: kind 0 = mask_vector(k) rotated left by r: slot i is 1 iff
// (i + r) mod S lies in [k N, (k + 1) N); kind 1 = checking_vector(k): slot i
// holds (k + i / N) mod N
__global__ __launch_bounds__(256) void k_mask_slots(double2 *v, int S, int N, const int *spec, size_t total) {
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= total) return;
    const size_t b = t / S;
    const int i = (int)(t % S);
    const int kind = spec[3 * b], k = spec[3 * b + 1], r = spec[3 * b + 2];
    double val;
    if (kind == 0) {
        const long long src = (((long long)i + r) % S + S) % S;
        val = (src >= (long long)k * N && src < (long long)(k + 1) * N) ? 1.0 : 0.0;
    } else {
        val = (double)((k + i / N) % N);
    }
    v[t] = make_double2(val, 0.0);
}

}  // namespace

void encode_ifft(double2 *v, int64_t *coef, int B, int S, int n, const double2 *ksi, const uint32_t *rot,
                 const double *scale, unsigned *overflow, hipStream_t st) {
    if (B <= 0) return;
    const int M = 2 * n;
    int logS = 0;
    while ((1 << logS) < S) ++logS;
    const int L = S < ENC_L ? S : ENC_L;
    for (int len = S; len > L; len >>= 1) {
        const size_t total = (size_t)B * (S / 2);
        hipLaunchKernelGGL(k_ifft_stage, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, v, S, len, ksi, rot, M,
                           total);
    }
    if (L >= 2)
        hipLaunchKernelGGL(k_ifft_lds, dim3((unsigned)(S / L), (unsigned)B), dim3(ENC_NT), 0, st, v, S, L, ksi, rot, M);
    hipLaunchKernelGGL(k_ifft_finish, dim3((unsigned)((n + 255) / 256), (unsigned)B), dim3(256), 0, st, v, coef, S, logS,
                       n, scale, overflow);
}

void mask_slots(double2 *v, int B, int S, int N, const int *spec, hipStream_t st) {
    const size_t total = (size_t)B * S;
    if (!total) return;
    hipLaunchKernelGGL(k_mask_slots, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, v, S, N, spec, total);
}

}  // namespace dev
}  // namespace fhe
