// FETCH_SIZE calibration for the codec's read patterns (MI355X_MICROARCH.md, HBM section: "other access
// widths are uncalibrated: calibrate on a known byte count in your own access pattern").  Each kernel reads
// every byte of a 1 GiB buffer (4x the Infinity Cache) exactly once, in one pattern:
//   wide    16 B per lane, consecutive lanes consecutive (the guide's calibrated case: FETCH = bytes / 2)
//   parse   parse3_kernel's staging: a lane owns a contiguous region and reads it one 128-byte line at a
//           time as two 64-byte halves of four 16-byte buffer loads; lanes' regions 640 B apart
//   decode  decode3_kernel's chunk loads: lane l reads 48 B from 32 l (its 32-byte chunk + 16 bytes of the
//           next one; the unique bytes are 32 per lane)
//   x       the encoder's tile loads (load_tile_x): 16 B per lane, a 4096-float tile per workgroup
// Run under `rocprofv3 --pmc FETCH_SIZE` (one counter pass); tools/fetch_calib.py turns the per-dispatch
// FETCH_SIZE into bytes-per-counted-byte factors for tools/pmc_to_json.py.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, long long bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

__global__ void k_wide(const uint4* __restrict__ a, long long n16, unsigned* sink) {
    unsigned acc = 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (long long)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// parse: lane region of LINES 128-byte lines; 64 lanes per wave, one wave per workgroup
template <int LINES>
__global__ __launch_bounds__(64) void k_parse(const unsigned char* __restrict__ a, long long nbytes, unsigned* sink) {
    const long long region = 128ll * LINES;
    const long long lanes = nbytes / region;
    unsigned acc = 0;
    for (long long l = (long long)blockIdx.x * 64 + threadIdx.x; l - threadIdx.x < lanes; l += (long long)gridDim.x * 64) {
        const bool act = l < lanes;
        const long long base = act ? l * region : 0;
        const long long lo = base & ~((1ll << 30) - 1);            // 1 GiB windows of the buffer resource
        const __amdgpu_buffer_rsrc_t rs = rsrc(a + lo, 1ll << 30);
        const int off = (int)(base - lo);
#pragma unroll
        for (int L = 0; L < LINES; L++) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                u32x4 v[4];
#pragma unroll
                for (int q = 0; q < 4; q++) v[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, act ? off + 128 * L + 64 * h + 16 * q : -64, 0, 0);
#pragma unroll
                for (int q = 0; q < 4; q++) acc ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
            }
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// decode: lane = 32-byte chunk; 48 bytes from its start (3 x 16 B), 256 threads per workgroup
__global__ __launch_bounds__(256) void k_decode(const unsigned char* __restrict__ a, long long nbytes, unsigned* sink) {
    const long long nch = nbytes / 32;
    unsigned acc = 0;
    const __amdgpu_buffer_rsrc_t rs = rsrc(a, nbytes);
    for (long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x; c < nch; c += (long long)gridDim.x * blockDim.x) {
#pragma unroll
        for (int q = 0; q < 3; q++) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(32 * c + 16 * q), 0, 0);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// x: one 4096-float tile per workgroup of 256 threads, 16 B per lane per load (4 loads per thread)
__global__ __launch_bounds__(256) void k_x(const float* __restrict__ x, long long n, unsigned* sink) {
    unsigned acc = 0;
    for (long long t = blockIdx.x; t * 4096 < n; t += gridDim.x) {
        const __amdgpu_buffer_rsrc_t rs = rsrc(x + t * 4096, 16384);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * (threadIdx.x + 256 * j), 0, 0);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    const long long B = 1ll << 30;
    unsigned char* a;
    unsigned* sink;
    CK(hipMalloc(&a, B + 4096));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 0x5A, B + 4096));
    CK(hipDeviceSynchronize());
    const int grid = 256 * 8;
    for (int rep = 0; rep < 2; rep++) {          // (the second round is the one to read; the first warms up)
        hipLaunchKernelGGL(k_wide, dim3(grid), dim3(256), 0, 0, (const uint4*)a, B / 16, sink);
        hipLaunchKernelGGL(k_parse<5>, dim3(B / 640 / 64 + 1), dim3(64), 0, 0, a, B, sink);
        hipLaunchKernelGGL(k_decode, dim3(grid), dim3(256), 0, 0, a, B, sink);
        hipLaunchKernelGGL(k_x, dim3(B / 16384), dim3(256), 0, 0, (const float*)a, B / 4, sink);
        CK(hipDeviceSynchronize());
    }
    // the bytes each kernel reads (every byte once; parse: whole 640-byte regions only)
    printf("{\"bytes\": {\"k_wide\": %lld, \"k_parse\": %lld, \"k_decode\": %lld, \"k_x\": %lld}}\n", B,
           (B / 640) * 640, B, B);
    CK(hipFree(a));
    CK(hipFree(sink));
    return 0;
}
