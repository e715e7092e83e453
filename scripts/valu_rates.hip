// Issue-rate probe for the VALU instructions the modular arithmetic uses
// (v_mad_u64_u32, v_mul_lo_u32, v_mul_hi_u32, v_fma_f64, v_add_co_u32) on
// gfx950.  Each thread runs 8 independent dependency chains so the result is
// throughput, not latency.  Build: hipcc --offload-arch=gfx950 -O3 valu_rates.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITERS = 4096;
constexpr int CH = 8;

__global__ void k_mad64(uint64_t *out, uint32_t s) {
    uint64_t a[CH];
    for (int c = 0; c < CH; ++c) a[c] = threadIdx.x + c;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) a[c] = (uint64_t)(uint32_t)a[c] * (s + c) + (a[c] >> 32);
    uint64_t r = 0;
    for (int c = 0; c < CH; ++c) r ^= a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_mullo(uint64_t *out, uint32_t s) {
    uint32_t a[CH];
    for (int c = 0; c < CH; ++c) a[c] = threadIdx.x + c;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) a[c] = a[c] * (s + c);
    uint32_t r = 0;
    for (int c = 0; c < CH; ++c) r ^= a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_mulhi(uint64_t *out, uint32_t s) {
    uint32_t a[CH];
    for (int c = 0; c < CH; ++c) a[c] = threadIdx.x + c + 12345;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) a[c] = __umulhi(a[c], s + c) ^ (s + i);
    uint32_t r = 0;
    for (int c = 0; c < CH; ++c) r ^= a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_fma64(uint64_t *out, double s) {
    double a[CH];
    for (int c = 0; c < CH; ++c) a[c] = threadIdx.x + c;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) a[c] = __fma_rn(a[c], s, 0.5);
    double r = 0;
    for (int c = 0; c < CH; ++c) r += a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)r;
}
__global__ void k_add32(uint64_t *out, uint32_t s) {
    uint32_t a[CH];
    for (int c = 0; c < CH; ++c) a[c] = threadIdx.x + c;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) a[c] = (a[c] + s) ^ c;
    uint32_t r = 0;
    for (int c = 0; c < CH; ++c) r ^= a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <typename F>
void run(const char *name, F launch, double ops_per_thread_iter) {
    const int blocks = 256 * 16, threads = 256;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    launch(blocks, threads);
    hipEventRecord(e0);
    launch(blocks, threads);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double ops = (double)blocks * threads * ITERS * CH * ops_per_thread_iter;
    printf("{\"op\": \"%s\", \"ms\": %.3f, \"Glane_ops_per_s\": %.1f}\n", name, ms, ops / ms / 1e6);
}

int main() {
    uint64_t *out;
    hipMalloc(&out, sizeof(uint64_t) * 256 * 16 * 256);
    run("v_mad_u64_u32", [&](int b, int t) { k_mad64<<<b, t>>>(out, 7u); }, 1);
    run("v_mul_lo_u32", [&](int b, int t) { k_mullo<<<b, t>>>(out, 7u); }, 1);
    run("v_mul_hi_u32(+xor)", [&](int b, int t) { k_mulhi<<<b, t>>>(out, 7u); }, 2);
    run("v_fma_f64", [&](int b, int t) { k_fma64<<<b, t>>>(out, 0.999); }, 1);
    run("v_add_u32(+xor)", [&](int b, int t) { k_add32<<<b, t>>>(out, 7u); }, 2);
    hipFree(out);
    return 0;
}
