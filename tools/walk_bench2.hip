// walk_bench2.hip -- the token walk alone, out of LDS (diagnostic only, not the library).
// Each workgroup stages one tile of a real CT7 stream once, then walks every lane's 1024-bit chunk
// REPS times (count only).  Layouts: PAD = chunk rows padded to 33 words (the library's layout);
// TRN = per wave transposed, word w of lane l at [w][l] (every ds_read_b32 of a wave is on 32
// distinct banks whatever the lanes' offsets).  Length by the LDS table or by ALU.
#include "../data-compression_amd/csrc/dc_device.h"
#include <stdio.h>

using namespace dc;
constexpr int CW = 32;                 // words per chunk (1024 bits)

template <int LAY>
__device__ __forceinline__ uint32_t laddr(int lane_base, int c, int w) {   // byte address of chunk-word w of lane c
    if constexpr (LAY == 0) { const int g = c * CW + w; return (uint32_t)(g + (g >> 5)) * 4u; }
    else return (uint32_t)(lane_base + (w * 64 + (c & 63))) * 4u;
}

template <int LAY, int ALU, int REPS>
__global__ __launch_bounds__(256) void walk2_kernel(const uint32_t* __restrict__ s, long long nwords, Params P,
                                                    unsigned long long* __restrict__ out) {
    constexpr int TW = 256 * CW;
    __shared__ uint32_t L[TW + TW / 32 + 64 * 8 * 4];
    __shared__ uint8_t tlen[512];
    build_lut_len<7>(tlen, P, threadIdx.x, 256);
    const int c = threadIdx.x, lane = c & 63, wv = c >> 6;
    const int lane_base = wv * (CW + 4) * 64;           // TRN: a wave's 64 chunks + 4 words of slack per lane
    // stage this workgroup's tile: lane c's own chunk words 0..CW+3 (the walk may read 3 words past its end)
    const long long w0 = (long long)blockIdx.x * TW;
    for (int w = 0; w < CW + 4; w++) {
        const long long g = w0 + (long long)c * CW + w;
        const uint32_t v = g < nwords ? __builtin_bswap32(s[g]) : 0u;
        *(uint32_t*)((char*)L + laddr<LAY>(lane_base, c, w)) = v;
    }
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned n = 0;
    for (int rep = 0; rep < REPS; rep++) {
        // reader (dc::Rd convention): sh = unread bits of a; sh = 0 -> the window starts at b
        uint32_t a = 0u;
        uint32_t b = *(uint32_t*)((char*)L + laddr<LAY>(lane_base, c, 0));
        uint32_t cc = *(uint32_t*)((char*)L + laddr<LAY>(lane_base, c, 1));
        uint32_t addr = laddr<LAY>(lane_base, c, 2);
        constexpr uint32_t DADDR = LAY == 0 ? 4u : 256u;
        uint32_t sh = 0;
        int pos = 0;
        while (pos < 1024) {
            const uint32_t nx = *(uint32_t*)((char*)L + addr);
            const uint32_t tk = __builtin_amdgcn_alignbit(a, b, sh);
            int len;
            if constexpr (ALU) len = token_len_bf<7>(tk, P);
            else len = tlen[tk >> 23];
            uint32_t d;
            const bool adv = __builtin_usub_overflow(sh, (uint32_t)len, &d);
            sh = d & 31u;
            pos += len;
            a = adv ? b : a;
            b = adv ? cc : b;
            cc = adv ? nx : cc;
            addr += adv ? DADDR : 0u;
            n++;
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

extern "C" int walk2_run(int v, int grid, const void* s, long long nbytes, int B, int type, unsigned mask17, void* dout,
                         float* ms) {
    const Params P = mk(B, type, mask17);
    const long long nwords = nbytes / 4;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 2; rep++) {
        (void)hipMemset(dout, 0, 32);
        (void)hipEventRecord(e0, 0);
        if (v == 0) hipLaunchKernelGGL((walk2_kernel<0, 0, 16>), dim3(grid), dim3(256), 0, 0, (const uint32_t*)s, nwords, P, (unsigned long long*)dout);
        if (v == 1) hipLaunchKernelGGL((walk2_kernel<1, 0, 16>), dim3(grid), dim3(256), 0, 0, (const uint32_t*)s, nwords, P, (unsigned long long*)dout);
        if (v == 2) hipLaunchKernelGGL((walk2_kernel<0, 1, 16>), dim3(grid), dim3(256), 0, 0, (const uint32_t*)s, nwords, P, (unsigned long long*)dout);
        if (v == 3) hipLaunchKernelGGL((walk2_kernel<1, 1, 16>), dim3(grid), dim3(256), 0, 0, (const uint32_t*)s, nwords, P, (unsigned long long*)dout);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
    }
    (void)hipEventElapsedTime(ms, e0, e1);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
