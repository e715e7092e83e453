// Issue-rate probe, part 3 (round 5): the fp64 and 24-bit multiply forms a
// 40-bit-prime butterfly could use on gfx950 (v_fma_f64, v_mul_f64,
// v_add_f64, v_floor_f64, v_cvt_f64_u32, v_cvt_u32_f64, v_mul_u32_u24,
// v_mul_hi_u32_u24, v_mad_u32_u24).  Each thread
// runs 8 independent chains of one inline-asm instruction, so the figure is
// throughput (lane-ops/s), not latency.
// Build: hipcc --offload-arch=gfx950 -O3 valu_rates3.hip -o valu_rates3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITERS = 2048;

#define BODYT(T, INSN)                                                                   \
    T a0 = (T)threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7; \
    const T k = (T)s;                                                                    \
    for (int i = 0; i < ITERS; ++i) {                                                    \
        asm volatile(INSN : "+v"(a0) : "v"(k)); asm volatile(INSN : "+v"(a1) : "v"(k));  \
        asm volatile(INSN : "+v"(a2) : "v"(k)); asm volatile(INSN : "+v"(a3) : "v"(k));  \
        asm volatile(INSN : "+v"(a4) : "v"(k)); asm volatile(INSN : "+v"(a5) : "v"(k));  \
        asm volatile(INSN : "+v"(a6) : "v"(k)); asm volatile(INSN : "+v"(a7) : "v"(k));  \
    }                                                                                    \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);

__global__ void k_fma_f64(uint64_t *out, uint64_t s) { BODYT(double, "v_fma_f64 %0, %0, %1, %1") }
__global__ void k_mul_f64(uint64_t *out, uint64_t s) { BODYT(double, "v_mul_f64 %0, %0, %1") }
__global__ void k_add_f64(uint64_t *out, uint64_t s) { BODYT(double, "v_add_f64 %0, %0, %1") }
__global__ void k_floor_f64(uint64_t *out, uint64_t s) { BODYT(double, "v_floor_f64 %0, %0") }
__global__ void k_rndne_f64(uint64_t *out, uint64_t s) { BODYT(double, "v_rndne_f64 %0, %0") }
__global__ void k_fma_f32(uint64_t *out, uint64_t s) { BODYT(float, "v_fma_f32 %0, %0, %1, %1") }
__global__ void k_pk_fma_f32(uint64_t *out, uint64_t s) { BODYT(double, "v_pk_fma_f32 %0, %0, %1, %1") }
__global__ void k_mul_u24(uint64_t *out, uint64_t s) { BODYT(uint32_t, "v_mul_u32_u24 %0, %0, %1") }
__global__ void k_mulhi_u24(uint64_t *out, uint64_t s) { BODYT(uint32_t, "v_mul_hi_u32_u24 %0, %0, %1") }
__global__ void k_mad_u24(uint64_t *out, uint64_t s) { BODYT(uint32_t, "v_mad_u32_u24 %0, %0, %1, %0") }
// conversions: the destination is overwritten from a fixed source (independent ops)
#define BODYC(TD, TS, INSN)                                                              \
    TD a0 = (TD)threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7; \
    const TS k = (TS)s;                                                                  \
    for (int i = 0; i < ITERS; ++i) {                                                    \
        asm volatile(INSN : "+v"(a0) : "v"(k)); asm volatile(INSN : "+v"(a1) : "v"(k));  \
        asm volatile(INSN : "+v"(a2) : "v"(k)); asm volatile(INSN : "+v"(a3) : "v"(k));  \
        asm volatile(INSN : "+v"(a4) : "v"(k)); asm volatile(INSN : "+v"(a5) : "v"(k));  \
        asm volatile(INSN : "+v"(a6) : "v"(k)); asm volatile(INSN : "+v"(a7) : "v"(k));  \
    }                                                                                    \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
__global__ void k_cvt_f64_u32(uint64_t *out, uint64_t s) { BODYC(double, uint32_t, "v_cvt_f64_u32 %0, %1") }
__global__ void k_cvt_u32_f64(uint64_t *out, uint64_t s) { BODYC(uint32_t, double, "v_cvt_u32_f64 %0, %1") }

template <typename F>
void run(const char *name, F launch, double ops_per_insn_slot) {
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
    const double ops = (double)blocks * threads * ITERS * 8 * ops_per_insn_slot;
    printf("{\"op\": \"%s\", \"ms\": %.3f, \"Glane_ops_per_s\": %.1f}\n", name, ms, ops / ms / 1e6);
}

int main() {
    uint64_t *out;
    hipMalloc(&out, sizeof(uint64_t) * 256 * 16 * 256);
#define R(name, k, ops) run(name, [&](int b, int t) { k<<<b, t>>>(out, 7u); }, ops)
    R("v_fma_f64", k_fma_f64, 1);
    R("v_mul_f64", k_mul_f64, 1);
    R("v_add_f64", k_add_f64, 1);
    R("v_floor_f64", k_floor_f64, 1);
    R("v_rndne_f64", k_rndne_f64, 1);
    R("v_fma_f32", k_fma_f32, 1);
    R("v_pk_fma_f32 (2 lanes-ops each)", k_pk_fma_f32, 2);
    R("v_mul_u32_u24", k_mul_u24, 1);
    R("v_mul_hi_u32_u24", k_mulhi_u24, 1);
    R("v_mad_u32_u24", k_mad_u24, 1);
    R("v_cvt_f64_u32", k_cvt_f64_u32, 1);
    R("v_cvt_u32_f64", k_cvt_u32_f64, 1);
    hipFree(out);
    return 0;
}
