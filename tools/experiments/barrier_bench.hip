// Diagnostic (not a test): the cost of a workgroup barrier and of an LDS round trip in a lone workgroup on an
// otherwise idle MI355X, and the clock it runs at (s_memtime / s_memrealtime).  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void bar_kernel(unsigned long long* out, int iters, int mode) {
    __shared__ int sh[1024];
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), t0 = __builtin_amdgcn_s_memtime();
    int acc = threadIdx.x;
    for (int i = 0; i < iters; i++) {
        if (mode == 0) {
            __syncthreads();
        } else if (mode == 1) {                             // barrier + LDS write/read exchange
            sh[threadIdx.x] = acc;
            __syncthreads();
            acc += sh[(threadIdx.x + 64) & (blockDim.x - 1)];
        } else if (mode == 2) {                             // __syncthreads_or
            acc += __syncthreads_or(acc & 1);
        } else {                                            // dependent VALU chain, no barrier
            acc = acc * 3 + 1;
        }
    }
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime(), t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = r1 - r0; out[1] = t1 - t0; out[2] = (unsigned)acc; }
}
int main() {
    unsigned long long* d;
    hipMalloc(&d, 64);
    unsigned long long h[3];
    const int iters = 20000;
    for (int mode = 0; mode < 4; mode++)
        for (int nt : {64, 256, 1024}) {
            for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(bar_kernel, dim3(1), dim3(nt), 0, 0, d, iters, mode);
            hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
            const double us = h[0] / 100.0, clk = (double)h[1] / (h[0] / 100.0) / 1e3;
            printf("mode %d (%s) threads %4d: %.3f us per iteration, %.0f cycles, clock %.2f GHz\n", mode,
                   mode == 0 ? "barrier" : mode == 1 ? "barrier+LDS" : mode == 2 ? "syncthreads_or" : "VALU chain",
                   nt, us / iters, (double)h[1] / iters, clk);
        }
    return 0;
}
