// walk_bench3.hip -- latency hiding of the token walk (diagnostic only, not the library).
// One-wave workgroups (64 lanes, 8.5 KB of LDS each) so that occupancy can reach 8 waves per SIMD;
// every lane runs ILP independent walks interleaved over the staged 1024-bit chunk rows.
#include "../data-compression_amd/csrc/dc_device.h"

using namespace dc;
constexpr int CW = 32;

template <int ILP, int REPS>
__global__ __launch_bounds__(64) void walk3_kernel(const uint32_t* __restrict__ s, long long nwords, Params P,
                                                   unsigned long long* __restrict__ out) {
    __shared__ uint32_t L[64 * (CW + 1) + 16];
    __shared__ uint8_t tlen[512];
    build_lut_len<7>(tlen, P, threadIdx.x, 64);
    const int lane = threadIdx.x;
    const long long w0 = ((long long)blockIdx.x * 64 * CW) % (nwords - 64 * CW - 64);
    for (int i = lane; i < 64 * CW + 4; i += 64) {
        const uint32_t v = __builtin_bswap32(s[w0 + i]);
        L[i + i / CW] = v;
    }
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned n = 0;
    for (int rep = 0; rep < REPS; rep++) {
        uint32_t a[ILP], b[ILP], c[ILP], addr[ILP], sh[ILP];
        int pos[ILP];
#pragma unroll
        for (int k = 0; k < ILP; k++) {
            const int ch = (lane + 13 * k) & 63;            // another lane's chunk for chain k
            const int g = ch * CW;
            a[k] = 0u; b[k] = L[g + g / CW]; c[k] = L[g + 1 + (g + 1) / CW];
            addr[k] = (uint32_t)(g + 2 + (g + 2) / CW) * 4u;
            sh[k] = 0u; pos[k] = 0;
        }
        bool any = true;
        while (any) {
            any = false;
#pragma unroll
            for (int k = 0; k < ILP; k++) {
                const bool on = pos[k] < 1024 - 32;         // stay inside the row (+1 pad word)
                const uint32_t nx = *(const uint32_t*)((const char*)L + addr[k]);
                const uint32_t tk = __builtin_amdgcn_alignbit(a[k], b[k], sh[k]);
                const int len = on ? (int)tlen[tk >> 23] : 0;
                uint32_t d;
                const bool adv = __builtin_usub_overflow(sh[k], (uint32_t)len, &d);
                sh[k] = d & 31u;
                pos[k] += len;
                a[k] = adv ? b[k] : a[k];
                b[k] = adv ? c[k] : b[k];
                c[k] = adv ? nx : c[k];
                addr[k] += adv ? 4u : 0u;
                n += on ? 1u : 0u;
                any |= on;
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned long long tot = n;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) tot += __shfl_xor(tot, d, 64);
    if (lane == 0) { atomicAdd(out, tot); atomicAdd(out + 1, t1 - t0); atomicAdd(out + 2, 1ull); }
}

static Params mk(int B, int type, uint32_t mask17) {
    Params p{};
    p.ct = 7; p.B = B; p.type = type; p.mask17 = mask17 & 0x1FFFFu;
    int m = B + (int)((p.mask17 >> 8) & 0xFF) - 127;
    p.mm = m > 23 ? 23 : (m < 0 ? 0 : m);
    p.mm0 = p.mm > 8 ? p.mm - 8 : 0;
    p.rawadd = B - 118;
    p.hm = ((1u << type) - 1u) << (31 - type);
    p.fsh = 30 - type;
    p.lm0 = type + 2 + p.mm0; p.dlm = p.mm - p.mm0;
    return p;
}

extern "C" int walk3_run(int ilp, int grid, const void* s, long long nbytes, int B, int type, unsigned mask17, void* dout,
                         float* ms) {
    const Params P = mk(B, type, mask17);
    const long long nwords = nbytes / 4;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 2; rep++) {
        (void)hipMemset(dout, 0, 32);
        (void)hipEventRecord(e0, 0);
        if (ilp == 1) hipLaunchKernelGGL((walk3_kernel<1, 32>), dim3(grid), dim3(64), 0, 0, (const uint32_t*)s, nwords, P, (unsigned long long*)dout);
        if (ilp == 2) hipLaunchKernelGGL((walk3_kernel<2, 16>), dim3(grid), dim3(64), 0, 0, (const uint32_t*)s, nwords, P, (unsigned long long*)dout);
        if (ilp == 4) hipLaunchKernelGGL((walk3_kernel<4, 8>), dim3(grid), dim3(64), 0, 0, (const uint32_t*)s, nwords, P, (unsigned long long*)dout);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
    }
    (void)hipEventElapsedTime(ms, e0, e1);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
