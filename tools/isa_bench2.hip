// isa_bench2.hip -- issue cost of short instruction SEQUENCES on gfx950 (diagnostic only).
// 8 independent chains per wave, W workgroups of 256 threads per CU; the host converts the kernel's
// wall time into cycles per sequence per SIMD with the clock measured in the kernel
// (s_memtime / s_memrealtime at 100 MHz).
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CH8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ __launch_bounds__(256) void seq_kernel(unsigned long long* out, int iters, unsigned seed) {
    uint32_t a[8], b[8], c[8];
#pragma unroll
    for (int k = 0; k < 8; k++) { a[k] = threadIdx.x * (k + 3) + seed; b[k] = a[k] ^ 0x1234u; c[k] = a[k] + 77u; }
    const uint32_t c1 = seed | 3u, c2 = (seed >> 3) | 5u;
    asm volatile("v_cmp_gt_u32 vcc, %0, %1" : : "v"(a[0]), "v"(c1) : "vcc");
    asm volatile("v_cmp_gt_u32 s[8:9], %0, %1" : : "v"(a[1]), "v"(c1) : "s8", "s9");
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
#define OPK(k)                                                                                                 \
    if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[k]) : "v"(c1));                        \
    if constexpr (OP == 1) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[k]) : "v"(c1));               \
    if constexpr (OP == 2) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[k]) : "v"(c1) : "vcc"); \
    if constexpr (OP == 3) asm volatile("v_cmp_gt_u32 s[8:9], %0, %1\n v_cndmask_b32_e64 %0, %0, %1, s[8:9]" : "+v"(a[k]) : "v"(c1) : "s8", "s9"); \
    if constexpr (OP == 4) asm volatile("v_sub_co_u32 %0, vcc, %0, %3\n v_cndmask_b32 %1, %1, %2, vcc\n v_cndmask_b32 %2, %2, %0, vcc" \
                                        : "+v"(a[k]), "+v"(b[k]), "+v"(c[k]) : "v"(c1) : "vcc");                  \
    if constexpr (OP == 5) asm volatile("v_sub_co_u32 %0, s[8:9], %0, %3\n v_cndmask_b32_e64 %1, %1, %2, s[8:9]\n v_cndmask_b32_e64 %2, %2, %0, s[8:9]" \
                                        : "+v"(a[k]), "+v"(b[k]), "+v"(c[k]) : "v"(c1) : "s8", "s9");            \
    if constexpr (OP == 6) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(a[k]));                              \
    if constexpr (OP == 7) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(a[k]));                              \
    if constexpr (OP == 8) asm volatile("v_max_u32 %0, %0, %1" : "+v"(a[k]) : "v"(c1));                       \
    if constexpr (OP == 9) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[k]) : "v"(c1));                       \
    if constexpr (OP == 10) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a[k]) : "v"(c1));                      \
    if constexpr (OP == 11) asm volatile("v_or_b32 %0, %0, %1" : "+v"(a[k]) : "v"(c1));                       \
    if constexpr (OP == 12) asm volatile("v_alignbit_b32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(c1), "v"(c2));     \
    if constexpr (OP == 13) asm volatile("v_bfe_u32 %0, %0, 23, 8" : "+v"(a[k]));                             \
    if constexpr (OP == 14) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(a[k]) : "v"(c1));                   \
    if constexpr (OP == 15) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(a[k]) : "v"(c1));                   \
    if constexpr (OP == 16) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[k]) : "v"(c1));                      \
    if constexpr (OP == 17) asm volatile("v_max_f32 %0, %0, %1" : "+v"(a[k]) : "v"(c1));                      \
    if constexpr (OP == 18) asm volatile("v_sub_u32 %0, %0, %1\n v_add_u32 %1, %1, %0" : "+v"(a[k]), "+v"(b[k])); \
    if constexpr (OP == 19) asm volatile("v_cmp_gt_u32 vcc, %0, %1" : : "v"(a[k]), "v"(c1) : "vcc");          \
    if constexpr (OP == 20) asm volatile("v_addc_co_u32 %0, vcc, 0, %0, vcc" : "+v"(a[k]) : : "vcc");         \
    if constexpr (OP == 21) asm volatile("v_and_b32 %0, 31, %0\n v_add_u32 %1, %1, %0\n v_xor_b32 %2, %2, %1" : "+v"(a[k]), "+v"(b[k]), "+v"(c[k]));
            CH8(OPK)
#undef OPK
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) r ^= a[k] ^ b[k] ^ c[k];
    if (blockIdx.x == 0 && threadIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; }
    if (r == 0x12345678u) out[2] = r;
}

#define OPS(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) \
    X(17) X(18) X(19) X(20) X(21)

extern "C" int seq_run(int op, int grid, int iters, unsigned long long* dout, float* ms) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 2; rep++) {
        (void)hipEventRecord(e0, 0);
        switch (op) {
#define CASE(o) case o: hipLaunchKernelGGL(seq_kernel<o>, dim3(grid), dim3(256), 0, 0, dout, iters, 7u); break;
            OPS(CASE)
#undef CASE
            default: return -2;
        }
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
    }
    (void)hipEventElapsedTime(ms, e0, e1);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
