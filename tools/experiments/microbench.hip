// microbench.hip -- calibration kernels for MI355X (diagnostic only, not part of the library):
// streaming read / copy bandwidth at several grid shapes and the shader clock under load.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void rd_kernel(const float4* __restrict__ x, long long n4, float* out) {
    float4 acc = make_float4(0, 0, 0, 0);
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
        const float4 v = x[i];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    if (acc.x + acc.y + acc.z + acc.w == 12345.0f) out[0] = 1.0f;
}

__global__ void rd16_kernel(const float4* __restrict__ x, long long n4, float* out) {   // 16 float4 per lane in flight
    float4 acc = make_float4(0, 0, 0, 0);
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i + 15 * stride < n4; i += 16 * stride) {
        float4 v[16];
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = x[i + k * stride];
#pragma unroll
        for (int k = 0; k < 16; k++) { acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w; }
    }
    if (acc.x + acc.y + acc.z + acc.w == 12345.0f) out[0] = 1.0f;
}

__global__ void cp_kernel(const float4* __restrict__ x, float4* __restrict__ y, long long n4) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x)
        y[i] = x[i];
}

__global__ void clk_kernel(unsigned long long* out, int iters) {
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    float a = threadIdx.x, b = 1.0001f;
    for (int i = 0; i < iters; i++) { a = a * b + 0.5f; b = b * 0.99999f + 0.00001f; }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) { out[0] = c1 - c0; out[1] = r1 - r0; }
    if (a == 12345.0f) out[2] = 1;
}

// VALU issue rate: 8 independent chains of 32-bit integer ops (add / xor / bfe / select / alignbit)
__global__ void valu_kernel(unsigned* out, int iters) {
    unsigned a[8];
#pragma unroll
    for (int k = 0; k < 8; k++) a[k] = threadIdx.x * (k + 3);
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            unsigned v = a[k];
            v = v + 0x9E3779B9u;
            v = v ^ (v >> 7);
            v = __builtin_amdgcn_alignbit(v, a[(k + 1) & 7], 5u);
            v = (v & 1u) ? v + 3u : v ^ 0x55u;
            a[k] = v;
        }
    }
    unsigned r = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) r ^= a[k];
    if (r == 0x12345678u) out[0] = r;
}

extern "C" int mb_run(int which, const void* x, void* y, long long nbytes, int grid, int block, int iters, float* ms,
                      unsigned long long* clk) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const long long n4 = nbytes / 16;
    for (int rep = 0; rep < 2; rep++) {
        (void)hipEventRecord(e0, 0);
        for (int i = 0; i < iters; i++) {
            if (which == 0) hipLaunchKernelGGL(rd_kernel, dim3(grid), dim3(block), 0, 0, (const float4*)x, n4, (float*)y);
            if (which == 1) hipLaunchKernelGGL(rd16_kernel, dim3(grid), dim3(block), 0, 0, (const float4*)x, n4, (float*)y);
            if (which == 2) hipLaunchKernelGGL(cp_kernel, dim3(grid), dim3(block), 0, 0, (const float4*)x, (float4*)y, n4);
            if (which == 4) hipLaunchKernelGGL(valu_kernel, dim3(grid), dim3(block), 0, 0, (unsigned*)y, (int)nbytes);
            if (which == 3) hipLaunchKernelGGL(clk_kernel, dim3(grid), dim3(block), 0, 0, (unsigned long long*)y, (int)nbytes);
        }
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
    }
    (void)hipEventElapsedTime(ms, e0, e1);
    *ms /= iters;
    if (which == 3) (void)hipMemcpy(clk, y, 16, hipMemcpyDeviceToHost);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
