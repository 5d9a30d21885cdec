// walk_bench.hip -- token-walk throughput on a real CT7 stream (diagnostic only, not the library).
// Every lane walks one CB-bit chunk of the stream from the chunk's first bit (count only, or count +
// value pattern), out of LDS rows padded by one word.  Variants: length by LDS table or by ALU, one or
// two interleaved chains per lane, plain or software-pipelined reader.  Prints tokens/us per variant.
#include "../data-compression_amd/csrc/dc_device.h"
#include <stdio.h>

using namespace dc;

template <int CW>
__device__ __forceinline__ int pidx(int w) { return (int)((unsigned)w + (unsigned)w / CW); }   // one pad word per row

template <int CW>
struct WR {                                   // Rd with a generic padded row
    uint32_t a, b, c, nx;
    int s, w3, pos;
    __device__ __forceinline__ void init(const uint32_t* L, int p) {
        const int wi = (p - 1) >> 5;
        s = 32 * (wi + 1) - p;
        a = L[pidx<CW>(max(wi, 0))]; b = L[pidx<CW>(wi + 1)]; c = L[pidx<CW>(wi + 2)];
        w3 = wi + 3;
        pos = p;
    }
    __device__ __forceinline__ void fetch(const uint32_t* L) { nx = L[pidx<CW>(w3)]; }
    __device__ __forceinline__ uint32_t peek() const { return __builtin_amdgcn_alignbit(a, b, (uint32_t)s); }
    __device__ __forceinline__ void step(int len) {
        uint32_t d;
        const bool adv = __builtin_usub_overflow((uint32_t)s, (uint32_t)len, &d);
        s = (int)(d & 31u);
        pos += len;
        a = adv ? b : a;
        b = adv ? c : b;
        c = adv ? nx : c;
        w3 += adv ? 1 : 0;
    }
};

// MODE: 0 LUT length, count only; 1 ALU length, count only; 2 LUT length + pattern (kv table);
//       3 ALU length + ALU pattern (token_pattern_bf)
template <int CB, int MODE, int ILP>
__global__ __launch_bounds__(256) void walk_kernel(const uint32_t* __restrict__ s, long long nwords, long long nbits,
                                                   Params P, unsigned long long* __restrict__ out) {
    constexpr int CW = CB / 32;
    constexpr int TW = 256 * ILP * CW;                 // words per tile
    __shared__ uint32_t L[TW + TW / CW + 16];
    __shared__ TokLut T;
    build_lut<7>(T, P, threadIdx.x, 256);
    uint8_t* tl = reinterpret_cast<uint8_t*>(T.kv);   // reuse: 512 one-byte lengths (kv rebuilt below if needed)
    __shared__ uint8_t tlen[512];
    build_lut_len<7>(tlen, P, threadIdx.x, 256);
    (void)tl;
    const long long ntiles = (nwords + TW - 1) / TW;
    unsigned long long tot = 0, acc = 0;
    for (long long t = blockIdx.x; t < ntiles; t += gridDim.x) {
        __syncthreads();
        const long long w0 = t * TW;
        constexpr int NQ = (TW + 8 + 1023) / 1024;
        uint4 vq[NQ];
#pragma unroll
        for (int q = 0; q < NQ; q++) {                 // every load in flight before the first LDS write
            const int i = threadIdx.x * 4 + q * 1024;
            vq[q] = (w0 + i + 4 <= nwords && i < TW + 8) ? *reinterpret_cast<const uint4*>(s + w0 + i) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            const int i = threadIdx.x * 4 + q * 1024;
            if (i < TW + 8) {
                L[pidx<CW>(i)] = __builtin_bswap32(vq[q].x); L[pidx<CW>(i + 1)] = __builtin_bswap32(vq[q].y);
                L[pidx<CW>(i + 2)] = __builtin_bswap32(vq[q].z); L[pidx<CW>(i + 3)] = __builtin_bswap32(vq[q].w);
            }
        }
        __syncthreads();
        const long long tb = w0 * 32;
        WR<CW> r[ILP];
        int end[ILP];
#pragma unroll
        for (int k = 0; k < ILP; k++) {
            const int c = threadIdx.x + 256 * k;
            const int cs = c * CB;
            end[k] = (int)min((long long)cs + CB, max(nbits - tb, 0ll));
            r[k].init(L, cs);
        }
        unsigned n = 0;
        while (true) {
            bool any = false;
#pragma unroll
            for (int k = 0; k < ILP; k++) any |= r[k].pos < end[k];
            if (!any) break;
#pragma unroll
            for (int k = 0; k < ILP; k++) {
                const bool on = r[k].pos < end[k];
                r[k].fetch(L);
                const uint32_t tk = r[k].peek();
                int len;
                if constexpr (MODE == 0 || MODE == 2) len = tlen[tk >> 23];
                else len = token_len_bf<7>(tk, P);
                if constexpr (MODE == 2) {
                    const uint32_t meta = T.meta[tk >> 23];
                    acc ^= lut_pattern(T, tk, meta);
                }
                if constexpr (MODE == 3) {
                    int code;
                    acc ^= token_pattern_bf<7>(tk, len, P, &code) + code;
                }
                r[k].step(on ? len : 0);
                n += on ? 1 : 0;
            }
        }
        tot += n;
    }
    tot += (acc == 0x123456789ull) ? 1 : 0;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) tot += __shfl_xor(tot, d, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, tot);          // one atomic per wave
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
    p.rs = type + 2;
    p.s0 = 17 - p.rs; p.s1 = 9 - p.rs;
    p.lm0 = type + 2 + p.mm0; p.dlm = p.mm - p.mm0;
    const int tl0 = p.mm0, tl1 = p.mm;
    p.c0 = (p.mask17 << 15) | (tl0 < 15 ? 1u << (14 - tl0) : 0u);
    p.k0 = tl0 > 0 ? (((1u << tl0) - 1u) << (15 - tl0)) : 0u;
    p.c1 = ((p.mask17 >> 8) << 23) | (tl1 < 23 ? 1u << (22 - tl1) : 0u);
    p.k1 = tl1 > 0 ? (((1u << tl1) - 1u) << (23 - tl1)) : 0u;
    return p;
}

#define VARIANTS(X) X(512, 0, 1) X(1024, 0, 1) X(2048, 0, 1) X(1024, 1, 1) X(2048, 1, 1) X(1024, 0, 2) \
    X(1024, 1, 2) X(1024, 2, 1) X(1024, 3, 1) X(512, 0, 2) X(512, 1, 2) X(512, 1, 1)

extern "C" int walk_run(int v, int grid, const void* s, long long nbytes, int B, int type, unsigned mask17, void* dout,
                        float* ms) {
    const Params P = mk(B, type, mask17);
    const long long nwords = nbytes / 4, nbits = nbytes * 8;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 2; rep++) {
        (void)hipMemset(dout, 0, 8);
        (void)hipEventRecord(e0, 0);
        int k = 0;
#define RUN(CB, MODE, ILP)                                                                                        \
        if (k++ == v) {                                                                                           \
            constexpr int TW = 256 * ILP * (CB / 32);                                                             \
            const long long nt = (nwords + TW - 1) / TW;                                                          \
            const int g = grid > 0 ? grid : (int)nt;                                                              \
            hipLaunchKernelGGL((walk_kernel<CB, MODE, ILP>), dim3(g), dim3(256), 0, 0, (const uint32_t*)s, nwords, \
                               nbits, P, (unsigned long long*)dout);                                               \
        }
        VARIANTS(RUN)
#undef RUN
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
    }
    (void)hipEventElapsedTime(ms, e0, e1);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
