// Issue-rate probe, part 2: the 64-bit integer VALU forms the NTT butterfly
// uses on gfx950 (v_lshl_add_u64, v_lshrrev_b64, v_add_co/v_addc_co pairs,
// v_cndmask_b32, v_and_b32, v_mov_b32, v_mad_u64_u32, v_mul_lo/hi_u32).  Each
// thread runs 8 independent chains of one inline-asm instruction, so the
// figure is throughput (lane-ops/s), not latency.
// Build: hipcc --offload-arch=gfx950 -O3 valu_rates2.hip -o valu_rates2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITERS = 2048;

#define BODY64(INSN)                                                                     \
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7; \
    const uint64_t k = s;                                                                \
    for (int i = 0; i < ITERS; ++i) {                                                    \
        asm volatile(INSN : "+v"(a0) : "v"(k)); asm volatile(INSN : "+v"(a1) : "v"(k));  \
        asm volatile(INSN : "+v"(a2) : "v"(k)); asm volatile(INSN : "+v"(a3) : "v"(k));  \
        asm volatile(INSN : "+v"(a4) : "v"(k)); asm volatile(INSN : "+v"(a5) : "v"(k));  \
        asm volatile(INSN : "+v"(a6) : "v"(k)); asm volatile(INSN : "+v"(a7) : "v"(k));  \
    }                                                                                    \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;

#define BODY32(INSN)                                                                     \
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7; \
    const uint32_t k = (uint32_t)s;                                                      \
    for (int i = 0; i < ITERS; ++i) {                                                    \
        asm volatile(INSN : "+v"(a0) : "v"(k)); asm volatile(INSN : "+v"(a1) : "v"(k));  \
        asm volatile(INSN : "+v"(a2) : "v"(k)); asm volatile(INSN : "+v"(a3) : "v"(k));  \
        asm volatile(INSN : "+v"(a4) : "v"(k)); asm volatile(INSN : "+v"(a5) : "v"(k));  \
        asm volatile(INSN : "+v"(a6) : "v"(k)); asm volatile(INSN : "+v"(a7) : "v"(k));  \
    }                                                                                    \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;

__global__ void k_lshl_add_u64(uint64_t *out, uint64_t s) { BODY64("v_lshl_add_u64 %0, %0, 1, %1") }
__global__ void k_lshr_b64(uint64_t *out, uint64_t s) { BODY64("v_lshrrev_b64 %0, 3, %0") }
__global__ void k_mov_b64(uint64_t *out, uint64_t s) { BODY64("v_mov_b64 %0, %1") }
__global__ void k_add_co_pair(uint64_t *out, uint64_t s) { // 2 insns
    BODY32("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %0, vcc, 0, %0, vcc")
}
__global__ void k_and32(uint64_t *out, uint64_t s) { BODY32("v_and_b32 %0, %0, %1") }
__global__ void k_add32(uint64_t *out, uint64_t s) { BODY32("v_add_u32 %0, %0, %1") }
__global__ void k_mov32(uint64_t *out, uint64_t s) { BODY32("v_mov_b32 %0, %1") }
__global__ void k_mullo32(uint64_t *out, uint64_t s) { BODY32("v_mul_lo_u32 %0, %0, %1") }
__global__ void k_mulhi32(uint64_t *out, uint64_t s) { BODY32("v_mul_hi_u32 %0, %0, %1") }
__global__ void k_add3(uint64_t *out, uint64_t s) { BODY32("v_add3_u32 %0, %0, %1, %0") }
__global__ void k_ashr32(uint64_t *out, uint64_t s) { BODY32("v_ashrrev_i32 %0, 31, %0") }
__global__ void k_cndmask(uint64_t *out, uint64_t s) {
    BODY32("v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc")
}

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
    R("v_add_u32", k_add32, 1);
    R("v_mov_b32", k_mov32, 1);
    R("v_and_b32", k_and32, 1);
    R("v_add3_u32", k_add3, 1);
    R("v_ashrrev_i32", k_ashr32, 1);
    R("v_lshl_add_u64", k_lshl_add_u64, 1);
    R("v_lshrrev_b64", k_lshr_b64, 1);
    R("v_mov_b64", k_mov_b64, 1);
    R("v_add_co+v_addc_co (pair)", k_add_co_pair, 1);
    R("v_cmp+v_cndmask (pair)", k_cndmask, 1);
    R("v_mul_lo_u32", k_mullo32, 1);
    R("v_mul_hi_u32", k_mulhi32, 1);
    hipFree(out);
    return 0;
}
