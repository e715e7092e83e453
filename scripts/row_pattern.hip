// Access-pattern probe (round 5): how much of the HBM roof does the NTT row
// pass's memory pattern allow with no arithmetic at all?  A [segs][limbs][n]
// u64 array (n = 2^16) is read and written back (+1) with
//   flat   : one wave streams 16 x 512-B runs (the best case);
//   seg16  : the DPP row pass's block shape: 16 transforms = one row of 16
//            segments (the TWL layout), lane t of a transform holds idx t + 16 r;
//   row16  : 16 consecutive rows of ONE segment per block (32 KB contiguous);
//   seg16x3: seg16 plus two more read streams (the HMult-tail epilogue's
//            accumulator and d operands) -> 3 reads + 1 write per element.
// Round 6 (verdict r5 item 3): the guide's float4-copy shape as well --
//   copy16_gs<U>: out-of-place 16-B copy, grid-stride loop, U loads in flight
//                 per thread before the dependent stores (grids of 2..16 blocks
//                 per CU), and its in-place twin (read + write of one buffer);
// every pattern is timed over 100 launches (was 10).
// Build: hipcc --offload-arch=gfx950 -O3 row_pattern.hip -o row_pattern
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint64_t u64;
constexpr int LOGN = 16, N = 1 << LOGN;

__global__ __launch_bounds__(256) void k_flat(u64 *a, size_t total) {
    const size_t base = ((size_t)blockIdx.x * 16) * 256 + threadIdx.x;
    u64 x[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) x[r] = a[base + r * 256];
#pragma unroll
    for (int r = 0; r < 16; ++r) a[base + r * 256] = x[r] + 1;
}
// 16-B per lane per instruction, in place / out of place; `nt`: nontemporal
typedef unsigned long long v2u __attribute__((ext_vector_type(2)));
template <bool NT>
__global__ __launch_bounds__(256) void k_flat16(u64 *a, const u64 *src) {
    const size_t base = ((size_t)blockIdx.x * 16) * 512 + 2 * threadIdx.x;
    v2u x[16];  // 256 lanes x 16 B x 16 = the block's 8192 words
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const v2u *p = reinterpret_cast<const v2u *>(src + base + r * 512);
        x[r] = NT ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        v2u *p = reinterpret_cast<v2u *>(a + base + r * 512);
        v2u v = x[r];
        v.x += 1;
        if (NT) __builtin_nontemporal_store(v, p);
        else *p = v;
    }
}
__global__ __launch_bounds__(256) void k_flat8_oop(u64 *a, const u64 *src) {
    const size_t base = ((size_t)blockIdx.x * 16) * 256 + threadIdx.x;
    u64 x[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) x[r] = src[base + r * 256];
#pragma unroll
    for (int r = 0; r < 16; ++r) a[base + r * 256] = x[r] + 1;
}
// grid (segs / 16, 256 rows, limbs)
__global__ __launch_bounds__(256) void k_seg16(u64 *a, size_t seg) {
    const int tr = threadIdx.x >> 4, t = threadIdx.x & 15;
    u64 *p = a + (size_t)(blockIdx.x * 16 + tr) * seg + (size_t)blockIdx.z * N + (size_t)blockIdx.y * 256;
    u64 x[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) x[r] = p[t + 16 * r];
#pragma unroll
    for (int r = 0; r < 16; ++r) p[t + 16 * r] = x[r] + 1;
}
// grid (segs, 16 row groups, limbs)
__global__ __launch_bounds__(256) void k_row16(u64 *a, size_t seg) {
    const int tr = threadIdx.x >> 4, t = threadIdx.x & 15;
    u64 *p = a + (size_t)blockIdx.x * seg + (size_t)blockIdx.z * N + (size_t)(blockIdx.y * 16 + tr) * 256;
    u64 x[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) x[r] = p[t + 16 * r];
#pragma unroll
    for (int r = 0; r < 16; ++r) p[t + 16 * r] = x[r] + 1;
}
// seg16 with two extra read streams b, c (same layout)
__global__ __launch_bounds__(256) void k_seg16x3(u64 *a, const u64 *b, const u64 *c, size_t seg) {
    const int tr = threadIdx.x >> 4, t = threadIdx.x & 15;
    const size_t off = (size_t)(blockIdx.x * 16 + tr) * seg + (size_t)blockIdx.z * N + (size_t)blockIdx.y * 256;
    u64 x[16], y[16], z[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) x[r] = a[off + t + 16 * r];
#pragma unroll
    for (int r = 0; r < 16; ++r) y[r] = b[off + t + 16 * r];
#pragma unroll
    for (int r = 0; r < 16; ++r) z[r] = c[off + t + 16 * r];
#pragma unroll
    for (int r = 0; r < 16; ++r) a[off + t + 16 * r] = x[r] + y[r] + z[r];
}
__global__ __launch_bounds__(256) void k_row16x3(u64 *a, const u64 *b, const u64 *c, size_t seg) {
    const int tr = threadIdx.x >> 4, t = threadIdx.x & 15;
    const size_t off = (size_t)blockIdx.x * seg + (size_t)blockIdx.z * N + (size_t)(blockIdx.y * 16 + tr) * 256;
    u64 x[16], y[16], z[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) x[r] = a[off + t + 16 * r];
#pragma unroll
    for (int r = 0; r < 16; ++r) y[r] = b[off + t + 16 * r];
#pragma unroll
    for (int r = 0; r < 16; ++r) z[r] = c[off + t + 16 * r];
#pragma unroll
    for (int r = 0; r < 16; ++r) a[off + t + 16 * r] = x[r] + y[r] + z[r];
}

// grid-stride 16-B copy: each thread issues U loads, then U stores, per trip
template <int U>
__global__ __launch_bounds__(256) void k_copy16_gs(v2u *dst, const v2u *src, size_t n16) {
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < n16; base += stride) {
        v2u x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * 256;
            x[u] = i < n16 ? src[i] : v2u{0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * 256;
            if (i < n16) {
                v2u v = x[u];
                v.x += 1;
                dst[i] = v;
            }
        }
    }
}

template <typename F>
void run(const char *name, F launch, double bytes) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    launch();
    (void)hipEventRecord(e0);
    const int it = 100;
    for (int i = 0; i < it; ++i) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= it;
    printf("{\"pattern\": \"%s\", \"us\": %.1f, \"TBps\": %.3f, \"frac\": %.3f}\n", name, ms * 1e3, bytes / ms / 1e9,
           bytes / ms / 1e9 / 8.0);
    fflush(stdout);
}

int main() {
    const int segs = 64, limbs = 38;
    const size_t seg = (size_t)limbs * N, total = (size_t)segs * seg;
    u64 *a, *b, *c;
    if (hipMalloc(&a, total * 8) || hipMalloc(&b, total * 8) || hipMalloc(&c, total * 8)) return 1;
    (void)hipMemset(a, 0, total * 8);
    (void)hipMemset(b, 0, total * 8);
    (void)hipMemset(c, 0, total * 8);
    const double B2 = 2.0 * total * 8, B4 = 4.0 * total * 8;
    run("flat", [&] { k_flat<<<dim3((unsigned)(total / 4096)), 256>>>(a, total); }, B2);
    run("flat8_oop", [&] { k_flat8_oop<<<dim3((unsigned)(total / 4096)), 256>>>(a, b); }, B2);
    run("flat16", [&] { k_flat16<false><<<dim3((unsigned)(total / 8192)), 256>>>(a, a); }, B2);
    run("flat16_oop", [&] { k_flat16<false><<<dim3((unsigned)(total / 8192)), 256>>>(a, b); }, B2);
    run("flat16_nt", [&] { k_flat16<true><<<dim3((unsigned)(total / 8192)), 256>>>(a, a); }, B2);
    run("flat16_oop_nt", [&] { k_flat16<true><<<dim3((unsigned)(total / 8192)), 256>>>(a, b); }, B2);
    run("seg16", [&] { k_seg16<<<dim3(segs / 16, 256, limbs), 256>>>(a, seg); }, B2);
    run("row16", [&] { k_row16<<<dim3(segs, 16, limbs), 256>>>(a, seg); }, B2);
    run("seg16x3", [&] { k_seg16x3<<<dim3(segs / 16, 256, limbs), 256>>>(a, b, c, seg); }, B4);
    run("row16x3", [&] { k_row16x3<<<dim3(segs, 16, limbs), 256>>>(a, b, c, seg); }, B4);
    const size_t n16 = total / 2;
    char nm[64];
    for (int bpc : {2, 4, 8, 16}) {
        const unsigned g = 256u * bpc;
        snprintf(nm, sizeof nm, "copy16_gs4_b%d", bpc);
        run(nm, [&] { k_copy16_gs<4><<<g, 256>>>((v2u *)a, (const v2u *)b, n16); }, B2);
        snprintf(nm, sizeof nm, "copy16_gs8_b%d", bpc);
        run(nm, [&] { k_copy16_gs<8><<<g, 256>>>((v2u *)a, (const v2u *)b, n16); }, B2);
        snprintf(nm, sizeof nm, "inplace16_gs8_b%d", bpc);
        run(nm, [&] { k_copy16_gs<8><<<g, 256>>>((v2u *)a, (const v2u *)a, n16); }, B2);
    }
    return 0;
}
