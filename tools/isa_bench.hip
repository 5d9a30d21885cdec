// isa_bench.hip -- per-instruction VALU issue cost on gfx950 (diagnostic only, not part of the library).
// Every kernel runs 8 independent chains of ONE instruction (inline asm, so the opcode is exactly the
// one named), W waves per SIMD (W workgroups of 256 threads per CU), and records s_memtime around
// the loop per wave.  cycles per wave-instruction per SIMD = elapsed / (W * instructions per wave).
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CH8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ __launch_bounds__(256) void isa_kernel(unsigned long long* out, int iters, unsigned seed) {
    uint32_t a[8];
    uint64_t d[8];
#pragma unroll
    for (int k = 0; k < 8; k++) { a[k] = threadIdx.x * (k + 3) + seed; d[k] = ((uint64_t)a[k] << 32) | (a[k] ^ 0x5555u); }
    const uint32_t c1 = seed | 3u, c2 = (seed >> 3) | 5u;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
#define OPK(k)                                                                                           \
    if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[k]) : "v"(c1));                  \
    if constexpr (OP == 1) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[k]) : "v"(c1));                  \
    if constexpr (OP == 2) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(a[k]) : "v"(c1));              \
    if constexpr (OP == 3) asm volatile("v_alignbit_b32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(c1), "v"(c2)); \
    if constexpr (OP == 4) asm volatile("v_bfe_u32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(c1), "v"(c2));      \
    if constexpr (OP == 5) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[k]) : "v"(c1));         \
    if constexpr (OP == 6) asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(c1), "v"(c2));     \
    if constexpr (OP == 7) asm volatile("v_lshl_or_b32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(c1), "v"(c2));  \
    if constexpr (OP == 8) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(c1), "v"(c2));   \
    if constexpr (OP == 9) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(c1), "v"(c2));     \
    if constexpr (OP == 10) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(c1), "v"(c2));    \
    if constexpr (OP == 11) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[k]) : "v"(c1));                 \
    if constexpr (OP == 12) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(c1), "v"(c2));     \
    if constexpr (OP == 13) asm volatile("v_min3_f32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(c1), "v"(c2));    \
    if constexpr (OP == 14) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(d[k]) : "v"(d[(k + 1) & 7]));  \
    if constexpr (OP == 15) asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(d[k]) : "v"(c1));             \
    if constexpr (OP == 16) asm volatile("v_sub_co_u32 %0, vcc, %0, %1" : "+v"(a[k]) : "v"(c1) : "vcc");   \
    if constexpr (OP == 17) asm volatile("v_cmp_gt_u32 vcc, %0, %1" : : "v"(a[k]), "v"(c1) : "vcc");    \
    if constexpr (OP == 18) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[k]) : "v"(c1));              \
    if constexpr (OP == 19) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a[k]) : "v"(c1), "v"(c2)); \
    if constexpr (OP == 20) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(a[k]) : "v"(c1));            \
    if constexpr (OP == 21) asm volatile("v_ffbh_u32 %0, %0" : "+v"(a[k]));                               \
    if constexpr (OP == 22) asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a[k])); \
    if constexpr (OP == 23) asm volatile("v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a[k])); \
    if constexpr (OP == 24) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[k]) : "v"(c1));              \
    if constexpr (OP == 25) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(a[k]) : "v"(c1));             \
    if constexpr (OP == 26) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a[k]) : "v"(c1));                 \
    if constexpr (OP == 27) asm volatile("v_cmp_lt_f32 vcc, %0, %1" : : "v"(a[k]), "v"(c1) : "vcc");    \
    if constexpr (OP == 28) asm volatile("v_add_lshl_u32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(c1), "v"(c2)); \
    if constexpr (OP == 29) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(d[k]) : "v"(d[(k + 1) & 7]));  \
    if constexpr (OP == 30) asm volatile("v_max_u32 %0, %0, %1" : "+v"(a[k]) : "v"(c1));                 \
    if constexpr (OP == 31) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[k]) : "v"(c1));                 \
    if constexpr (OP == 32) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[8:9]" : "+v"(a[k]) : "v"(c1) : "s8", "s9"); \
    if constexpr (OP == 33) asm volatile("v_mov_b32 %0, %1" : "=v"(a[k]) : "v"(a[(k + 1) & 7]));
            CH8(OPK)
#undef OPK
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) r ^= a[k] ^ (uint32_t)d[k] ^ (uint32_t)(d[k] >> 32);
    if ((threadIdx.x & 63) == 0) out[(blockIdx.x * 4 + (threadIdx.x >> 6)) * 2] = t1 - t0;
    if (r == 0x12345678u) out[1] = r;
}

// LDS: dependent-chain latency of ds_read_b32 (one chain per lane, addresses from the data) and the
// throughput of ds_or_b32 (LDS atomic OR) / ds_read_b32 with 8 independent streams
template <int OP>
__global__ __launch_bounds__(256) void lds_kernel(unsigned long long* out, int iters, unsigned seed) {
    __shared__ uint32_t L[8192];
    for (int i = threadIdx.x; i < 8192; i += 256) L[i] = (i * 33 + seed) & 8191;
    __syncthreads();
    uint32_t a[8];
#pragma unroll
    for (int k = 0; k < 8; k++) a[k] = (threadIdx.x * 33 + k * 1031) & 8191;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            if constexpr (OP == 0) {                 // one dependent chain
                a[0] = L[a[0]];
            } else if constexpr (OP == 1) {          // 8 independent chains
#pragma unroll
                for (int k = 0; k < 8; k++) a[k] = L[a[k]];
            } else {                                 // ds_or, 8 per step
#pragma unroll
                for (int k = 0; k < 8; k++) { atomicOr(&L[(a[k] + u * 64) & 8191], a[k]); a[k] += 0x41; }
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) r ^= a[k];
    if ((threadIdx.x & 63) == 0) out[(blockIdx.x * 4 + (threadIdx.x >> 6)) * 2] = t1 - t0;
    if (r == 0x12345678u) out[1] = r + L[r & 8191];
}

#define OPS(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) \
    X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30) X(31) X(32) X(33)

extern "C" int isa_run(int op, int lds, int grid, int iters, unsigned long long* dout, float* ms) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    if (lds) {
        if (op == 0) hipLaunchKernelGGL(lds_kernel<0>, dim3(grid), dim3(256), 0, 0, dout, iters, 7u);
        if (op == 1) hipLaunchKernelGGL(lds_kernel<1>, dim3(grid), dim3(256), 0, 0, dout, iters, 7u);
        if (op == 2) hipLaunchKernelGGL(lds_kernel<2>, dim3(grid), dim3(256), 0, 0, dout, iters, 7u);
    } else {
        switch (op) {
#define CASE(o) case o: hipLaunchKernelGGL(isa_kernel<o>, dim3(grid), dim3(256), 0, 0, dout, iters, 7u); break;
            OPS(CASE)
#undef CASE
            default: return -2;
        }
    }
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(ms, e0, e1);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
