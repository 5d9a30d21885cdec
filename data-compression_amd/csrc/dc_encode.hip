// dc_encode.hip -- bit-wise encoder for gfx950 (CT 5/6/7/11).
//
// Replaces the per-element serial loop of myCompress_bitwise (impl/dataCompression.c:3310-3444),
// myCompress_bitwise_np (:2645-2654), myCompress_bitwise_mask (:2030-2141) and
// myCompress_bitwise_op (:577-696), whose cost is one add_bit_to_bytes call (+ realloc) per output
// bit (:5456-5489).
//
// The encoder history is the ORIGINAL input (:2095-2097), so every token is a pure function of
// x[i-3..i].  Three launches, no inter-workgroup waiting:
//   encode_count_kernel : per tile of ENC_TILE floats, the total token bit length
//   encode_scan_kernel  : exclusive scan of the tile lengths -> every tile's global bit offset G
//   encode_write_kernel : tokens again, ORed MSB-first into a zeroed LDS bit buffer at offset
//                         G mod 32 + their prefix (one 64-bit shift, two ds_or each), then the tile
//                         writes every 32-bit word whose first bit lies in [G, G+T) as byte-swapped
//                         dwords, completing its last word with the first <= 31 bits of the
//                         following elements (recomputed locally, <= 11 tokens).
// The write kernel walks the tiles in reverse so the input the count kernel read last is still in
// the 256 MiB Infinity Cache when it is read again.
#include "dc_device.h"
#include <algorithm>
#include <stdlib.h>

namespace dc {

constexpr int ENC_TILE = 4096;                  // floats per tile (one offset per tile)
constexpr int ENC_TPB = 256;                    // write kernel: 4 waves per tile
constexpr int ENC_K = ENC_TILE / ENC_TPB;       // 16 consecutive floats per lane
constexpr int ENC_Q = ENC_TILE / 4 / ENC_TPB;   // coalesced float4 loads per lane
#ifndef DC_CNT_Q
#define DC_CNT_Q 4
#endif
#ifndef DC_WR_NT
#define DC_WR_NT 0
#endif
#ifndef DC_CNT_NT
#define DC_CNT_NT 1                     // the count pass streams x past the caches: measured count 85 -> 57 us
#endif
constexpr int CNT_Q = DC_CNT_Q;                 // count kernel: one wave per tile part, CNT_Q float4 per lane
constexpr int CNT_SUB = 256 * CNT_Q;            // floats per count wave
constexpr int CNT_PARTS = ENC_TILE / CNT_SUB;   // count parts per tile (tbits entries)
constexpr int ENC_LDS_WORDS = ENC_TILE + 48;    // 32 bits/elem max + offset + head slack
constexpr int STG_WORDS = ENC_TILE + ENC_TILE / 16 + 8;   // staged floats, one pad word per 16

__device__ __forceinline__ void lds_place(uint32_t* s, uint32_t off, uint32_t val, int len) {
    const uint32_t w = off >> 5, b = off & 31u;
    const int end = (int)b + len;                                  // 1..63
    if (end <= 32) {
        atomicOr(&s[w], val << (32 - end));
    } else {
        atomicOr(&s[w], val >> (end - 32));
        atomicOr(&s[w + 1], val << (64 - end));
    }
}

__device__ __forceinline__ float halo_x(const float* __restrict__ x, long long idx0, long long e) {
    // element e - (its history) when it precedes the array: unused by make_token (predict = false)
    return (idx0 + e >= 0 && e >= -3) ? x[e] : 0.0f;
}

// lane i gets v of lane i-1, lane 0 gets first (DPP wave_shr:1, a GFX9-family wavefront shift)
__device__ __forceinline__ float wave_shr1(float v, float first) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(first), __float_as_int(v), 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ float lane63(float v) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63)); }

// lengths of the CNT_Q float4s of one count part, every element predicted (history h1..h3 for
// lane 0's first element)
template <int CT>
__device__ __forceinline__ void count_tokens(const float4* f, float h1, float h2, float h3, const Params& P,
                                             uint32_t& sum, bool& neg1) {
#pragma unroll
    for (int q = 0; q < CNT_Q; q++) {
        const float b1 = wave_shr1(f[q].w, h1), b2 = wave_shr1(f[q].z, h2), b3 = wave_shr1(f[q].y, h3);
        h1 = lane63(f[q].w); h2 = lane63(f[q].z); h3 = lane63(f[q].y);
        const float xs[7] = {b3, b2, b1, f[q].x, f[q].y, f[q].z, f[q].w};
#pragma unroll
        for (int r = 0; r < 4; r++) {
            sum += (uint32_t)token_len_enc<CT>(xs[3 + r], xs[2 + r], xs[1 + r], xs[r], true, P);
            neg1 |= xs[3 + r] == -1.0f;
        }
    }
}

// count kernel: one wave per tile part; lane i holds float4 number i + 64q (q < CNT_Q), so every
// load instruction reads 1 KiB contiguous.  The history of a float4 is the previous float4: lane
// i-1's (same q) or, for lane 0, lane 63's of q-1.  One code path for every part: elements past n
// are loaded as 0.0f (a 3-bit zero token each, subtracted afterwards) and the <= 3 elements before
// global index 3 (no prediction, impl/dataCompression.c:1146) are corrected by lane 0.
// one count part's floats (whole float4s; past n -> 0.0f) and its three history floats
__device__ __forceinline__ void load_part(const float* __restrict__ x, long long n, long long idx0, long long tb,
                                          int lane, float4* f, float* hist) {
    const float4* p4 = reinterpret_cast<const float4*>(x + tb);
    if (tb + CNT_SUB <= n) {
#pragma unroll
        for (int q = 0; q < CNT_Q; q++) {
#if DC_CNT_NT
            typedef float f4v __attribute__((ext_vector_type(4)));
            const f4v w = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p4 + lane + 64 * q));
            f[q] = make_float4(w.x, w.y, w.z, w.w);
#else
            f[q] = p4[lane + 64 * q];
#endif
        }
    } else {                                                         // whole float4s only
        const int rem = (int)(n - tb);
#pragma unroll
        for (int q = 0; q < CNT_Q; q++) f[q] = 4 * (lane + 64 * q) + 4 <= rem ? p4[lane + 64 * q] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 1; k <= 3; k++) hist[k - 1] = halo_x(x, idx0, tb - k);   // wave-uniform (scalar) loads
}

// bit count of one tile part from its loaded floats; lane 0 corrects the padding and head elements
template <int CT>
__device__ __forceinline__ void count_part(const float* __restrict__ x, long long n, long long idx0, const Params& P,
                                           long long h, const float4* f, const float* hist, int lane,
                                           uint32_t* psum, unsigned* __restrict__ err) {
    const long long tb = h * CNT_SUB;
    uint32_t sum = 0;
    bool neg1 = false;
    count_tokens<CT>(f, hist[0], hist[1], hist[2], P, sum, neg1);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) sum += __shfl_xor(sum, d, 64);
    if (lane == 0) {
        int vend = CNT_SUB;                                          // elements the vector pass saw
        if (tb + CNT_SUB > n) {                                      // the 0.0f padding's tokens
            const int rem = (int)max(n - tb, 0ll);                   // 0: a part past the end
            vend = rem & ~3;
            sum -= (uint32_t)token_len_enc<CT>(0.0f, 0.0f, 0.0f, 0.0f, true, P) * (uint32_t)(CNT_SUB - vend);
            for (int j = vend; j < rem; j++) {                       // the straddling float4
                const long long e = tb + j;
                const float v = x[e];
                neg1 |= v == -1.0f;
                sum += (uint32_t)token_len_enc<CT>(v, halo_x(x, idx0, e - 1), halo_x(x, idx0, e - 2),
                                                   halo_x(x, idx0, e - 3), idx0 + e >= 3, P);
            }
        }
        if (CT != 6) {                                               // unpredicted head elements
            for (int j = 0; j < 3 && j < vend && idx0 + tb + j < 3; j++) {
                const long long e = tb + j;
                const float v = x[e], b1 = halo_x(x, idx0, e - 1), b2 = halo_x(x, idx0, e - 2),
                            b3 = halo_x(x, idx0, e - 3);
                sum += (uint32_t)(token_len_enc<CT>(v, b1, b2, b3, false, P) - token_len_enc<CT>(v, b1, b2, b3, true, P));
            }
        }
    }
    if (CT != 6 && __any(neg1) && lane == 0) atomicOr(err, 1u);    // -1.0f is the reference's sentinel
    if (lane == 0) *psum = sum;                                      // tile-part bit count
}

// one workgroup per tile (its four waves = the tile's four parts); tcnt[tile] = the tile's bits
template <int CT>
__global__ __launch_bounds__(256) void encode_count_kernel(const float* __restrict__ x, long long n, long long idx0,
                                                           Params P, uint32_t* __restrict__ tcnt, long long ntiles,
                                                           unsigned* __restrict__ err) {
    static_assert(CNT_PARTS == 4, "one workgroup of four waves per tile");
    __shared__ uint32_t wsum[4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const long long h = (long long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(wid);
    float4 f[CNT_Q];
    float hist[3];
    load_part(x, n, idx0, h * CNT_SUB, lane, f, hist);
    count_part<CT>(x, n, idx0, P, h, f, hist, lane, wsum + wid, err);
    __syncthreads();
    if (threadIdx.x == 0) tcnt[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    (void)ntiles;
}

// exclusive scan of the tile bit counts (one workgroup): coalesced, all-at-once loads of SCAN_T
// counts per thread into LDS (one pad word per 16), then each thread scans SCAN_T consecutive tiles;
// toff[t] = tile t's global bit offset
constexpr int SCAN_T = 16;
constexpr int SCAN_CH = 1024 * SCAN_T;
__global__ __launch_bounds__(1024) void encode_scan_kernel(const uint32_t* __restrict__ tcnt, uint64_t* __restrict__ toff,
                                                           long long ntiles, int start_bit,
                                                           unsigned long long* __restrict__ total_bits) {
    __shared__ uint32_t cnt[SCAN_CH + SCAN_CH / 16];           // also the u64 offsets of half the tiles
    __shared__ unsigned long long wtot[1024 / 64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    unsigned long long carry = (unsigned long long)start_bit;
    for (long long c0 = 0; c0 < ntiles; c0 += SCAN_CH) {
        uint32_t v[SCAN_T];
#pragma unroll
        for (int k = 0; k < SCAN_T; k++) {
            const long long t = c0 + k * 1024 + tid;
            v[k] = t < ntiles ? tcnt[t] : 0u;
        }
#pragma unroll
        for (int k = 0; k < SCAN_T; k++) {
            const int i = k * 1024 + tid;
            cnt[i + (i >> 4)] = v[k];
        }
        __syncthreads();
        uint32_t c[SCAN_T];
        unsigned long long sum = 0;
#pragma unroll
        for (int i = 0; i < SCAN_T; i++) {
            c[i] = cnt[tid * (SCAN_T + 1) + i];
            sum += c[i];
        }
        unsigned long long inc = sum;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long u = __shfl_up(inc, d, 64);
            if (lane >= d) inc += u;
        }
        if (lane == 63) wtot[wid] = inc;
        __syncthreads();
        unsigned long long wpre = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < 1024 / 64; w++) {
            const unsigned long long u = wtot[w];
            wpre += w < wid ? u : 0ull;
            tot += u;
        }
        unsigned long long run = carry + wpre + inc - sum;
        // offsets leave through LDS so the global stores are coalesced: half the tiles per pass
        unsigned long long* o = reinterpret_cast<unsigned long long*>(cnt);
        const int m = (int)min((long long)SCAN_CH, ntiles - c0);
#pragma unroll
        for (int half = 0; half < 2; half++) {
            __syncthreads();                                         // cnt (then o) is free
            if ((tid >> 9) == half) {
                const int b = (tid & 511) * (SCAN_T + 1);
#pragma unroll
                for (int i = 0; i < SCAN_T; i++) {
                    o[b + i] = run;
                    run += c[i];
                }
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < SCAN_CH / 2 / 1024; k++) {
                const int j = k * 1024 + tid;                        // tile within the half
                const int jj = half * (SCAN_CH / 2) + j;
                if (jj < m) toff[c0 + jj] = o[(j >> 4) * (SCAN_T + 1) + (j & 15)];
            }
        }
        carry += tot;
        __syncthreads();                                             // cnt / wtot are rewritten
    }
    if (tid == 0) *total_bits = carry;
}

// a tile's floats as coalesced float4s: thread tid holds float4 number tid + ENC_TPB*q
__device__ __forceinline__ void load_tile4(const float* __restrict__ x, long long n, long long tbase, int tid, float4* f) {
    if (tbase + ENC_TILE <= n) {
        const float4* p4 = reinterpret_cast<const float4*>(x + tbase);
#pragma unroll
        for (int q = 0; q < ENC_Q; q++) {
#if DC_WR_NT
            typedef float f4v __attribute__((ext_vector_type(4)));
            const f4v w = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p4 + tid + ENC_TPB * q));
            f[q] = make_float4(w.x, w.y, w.z, w.w);
#else
            f[q] = p4[tid + ENC_TPB * q];
#endif
        }
    } else {
#pragma unroll
        for (int q = 0; q < ENC_Q; q++) {
            const long long e = tbase + 4 * (tid + ENC_TPB * q);
            f[q].x = e < n ? x[e] : 0.0f; f[q].y = e + 1 < n ? x[e + 1] : 0.0f;
            f[q].z = e + 2 < n ? x[e + 2] : 0.0f; f[q].w = e + 3 < n ? x[e + 3] : 0.0f;
        }
    }
}

template <int CT>
__global__ __launch_bounds__(ENC_TPB) void encode_write_kernel(
    const float* __restrict__ x, long long n, long long idx0, Params P, uint32_t* __restrict__ out,
    const uint64_t* __restrict__ toff, unsigned ntiles, unsigned long long* __restrict__ dbg) {
    __shared__ uint32_t s_bits[STG_WORDS > ENC_LDS_WORDS ? STG_WORDS : ENC_LDS_WORDS];   // staging, then bits
    __shared__ uint32_t s_wsum[ENC_TPB / 64];
    __shared__ uint32_t s_head_val[12];
    __shared__ int s_head_len[12];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (unsigned k = blockIdx.x; k < ntiles; k += gridDim.x) {
    const unsigned tile = ntiles - 1 - k;
#define ESTAMP(ph) do { if (dbg && tid == 0 && tile < 8192) dbg[tile * 8 + (ph)] = __builtin_amdgcn_s_memrealtime(); } while (0)
    ESTAMP(0);
    const long long tbase = (long long)tile * ENC_TILE;
    const long long base = tbase + (long long)tid * ENC_K;
    const unsigned long long G = toff[tile];
    const bool full = tbase + ENC_TILE <= n && idx0 + tbase >= 3;
    // the first elements of the next tile (for the head tokens) are loaded now, used after the tokens
    float h0 = 0.0f, h1 = 0.0f, h2 = 0.0f, h3 = 0.0f;
    const bool hin = wid == 1 && lane < 11 && tbase + ENC_TILE + lane < n;
    if (hin) {
        const long long e = tbase + ENC_TILE + lane;
        h0 = x[e]; h1 = x[e - 1]; h2 = x[e - 2]; h3 = x[e - 3];
    }
    // ---- coalesced float4 loads -> LDS (one pad word per 16 floats), then 16 consecutive per lane
    {
        float4 f[ENC_Q];
        load_tile4(x, n, tbase, tid, f);
#pragma unroll
        for (int q = 0; q < ENC_Q; q++) {
            const int e = 4 * (tid + ENC_TPB * q);
            float* d = reinterpret_cast<float*>(s_bits) + 8 + e + (e >> 4);
            d[0] = f[q].x; d[1] = f[q].y; d[2] = f[q].z; d[3] = f[q].w;
        }
        if (tid < 3) reinterpret_cast<float*>(s_bits)[5 + tid] = halo_x(x, idx0, tbase - 3 + tid);
    }
    __syncthreads();
    float v[ENC_K + 4];
#pragma unroll
    for (int j = 1; j < ENC_K + 4; j++) {
        const int e = tid * ENC_K + j - 4;                           // tile-relative element (>= -3)
        v[j] = reinterpret_cast<const float*>(s_bits)[e < 0 ? 8 + e : 8 + e + (e >> 4)];
    }
    __syncthreads();
    for (int i = tid; i < ENC_LDS_WORDS; i += ENC_TPB) s_bits[i] = 0u;

    // ---- tokens
    uint32_t tv[ENC_K];
    uint32_t tlp[ENC_K / 4];                                         // token lengths, 4 per register
#pragma unroll
    for (int q = 0; q < ENC_K / 4; q++) tlp[q] = 0u;
    uint32_t mysum = 0;
    if (full) {
#pragma unroll
        for (int j = 0; j < ENC_K; j++) {
            int len;
            make_token_bf<CT>(v[4 + j], v[3 + j], v[2 + j], v[1 + j], true, P, tv[j], len);
            tlp[j >> 2] |= (uint32_t)len << (8 * (j & 3));
            mysum += (uint32_t)len;
        }
    } else {
#pragma unroll
        for (int j = 0; j < ENC_K; j++) {
            int len;
            make_token_bf<CT>(v[4 + j], v[3 + j], v[2 + j], v[1 + j], idx0 + base + j >= 3, P, tv[j], len);
            len = base + j < n ? len : 0;
            tv[j] = len ? tv[j] : 0u;
            tlp[j >> 2] |= (uint32_t)len << (8 * (j & 3));
            mysum += (uint32_t)len;
        }
    }
    ESTAMP(1);

    // ---- workgroup exclusive scan of bit lengths
    uint32_t inc = mysum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(inc, d, 64);
        if (lane >= d) inc += t;
    }
    if (lane == 63) s_wsum[wid] = inc;

    // ---- head: first <= 31 bits of the elements after this tile (completes our last word)
    if (wid == 1 && lane < 12) {
        uint32_t hv = 0u; int hl = 0;
        if (lane < 11 && hin) make_token<CT>(h0, h1, h2, h3, idx0 + tbase + ENC_TILE + lane >= 3, P, hv, hl);
        s_head_val[lane] = hv;
        s_head_len[lane] = hl;
    }
    __syncthreads();
    uint32_t wpre = 0, T = 0;
#pragma unroll
    for (int w = 0; w < ENC_TPB / 64; w++) {
        if (w < wid) wpre += s_wsum[w];
        T += s_wsum[w];
    }
    const uint32_t boff = (uint32_t)(G & 31ull);
    const long long wb = (long long)(G >> 5);
    ESTAMP(2);

    // ---- MSB-first packing: the LDS bit buffer is zeroed, so every token is ORed in at its bit
    // offset (measured faster than lane-local word assembly with divergent stores)
    {
        uint32_t off = boff + wpre + inc - mysum;
#pragma unroll
        for (int j = 0; j < ENC_K; j++) {
            const int len = (int)((tlp[j >> 2] >> (8 * (j & 3))) & 0xFFu);
            const uint64_t v = (uint64_t)tv[j] << ((64 - (int)(off & 31u) - len) & 63);   // len 0: tv = 0
            uint32_t* d = s_bits + (off >> 5);
            atomicOr(d, (uint32_t)(v >> 32));
            atomicOr(d + 1, (uint32_t)v);
            off += (uint32_t)len;
        }
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t ho = boff + T;
        for (int j = 0; j < 11 && s_head_len[j]; j++) {
            if (ho - boff - T >= 32u) break;
            lds_place(s_bits, ho, s_head_val[j], s_head_len[j]);
            ho += (uint32_t)s_head_len[j];
        }
    }
    __syncthreads();
    ESTAMP(3);

    // ---- write owned words: first bit in [G, G+T) (tile 0 also owns the start_bit prefix word)
    const unsigned long long Gend = G + T;
    long long w0 = (long long)((G + 31) >> 5);
    if (tile == 0) w0 = 0;
    const long long w1 = (long long)((Gend + 31) >> 5);
    for (long long w = w0 + tid; w < w1; w += ENC_TPB) out[w] = __builtin_bswap32(s_bits[w - wb]);
    ESTAMP(4);
    ESTAMP(5);
    __syncthreads();                                                 // s_bits is restaged next tile
    }
}

// ------------------------------------------------------------------------------------------------
// Single-pass encoder: encode_write_kernel's tile work with the tile offset from a decoupled
// look-back instead of the count + scan launches.  A tile publishes its bit count as soon as its
// workgroup scan is done (flag status 1), packs its tokens into LDS at a tile-relative offset (bit 0
// of buffer word 1; word 0 stays zero), and only then looks back: wave 0 reads the flags of the 64
// preceding tiles at once, adds the counts up to the nearest inclusive prefix (status 2) and moves
// 64 tiles further back if there is none.  Tiles are claimed in increasing order from an atomic
// counter, so every predecessor is running or done (no deadlock).  The tile publishes its inclusive
// prefix, then stores its owned words shifted into place with v_alignbit (G mod 32).
// flags[t] = status << 62 | (epoch mod 2^22) << 40 | value (40 bits)
__device__ __forceinline__ uint64_t eflag(uint64_t st, uint32_t epoch, unsigned long long v) {
    return (st << 62) | ((uint64_t)(epoch & 0x3FFFFFu) << 40) | (v & 0xFFFFFFFFFFull);
}

constexpr int FBUF = (STG_WORDS > ENC_LDS_WORDS ? STG_WORDS : ENC_LDS_WORDS) + 1;

// tile work up to the packed bits: stage, tokens, workgroup scan, head tokens, publish the count
// (flag status 1, tile 0: inclusive), pack at the tile-relative offset into buf (buf[0] = 0).
// Returns the tile's bit count T.
template <int CT>
__device__ __forceinline__ uint32_t fused_compute(const float* __restrict__ x, long long n, long long idx0, const Params& P,
                                                  uint64_t* __restrict__ flags, uint32_t epoch, int start_bit,
                                                  unsigned tile, uint32_t* buf, uint32_t* s_wsum, uint32_t* s_head_val,
                                                  int* s_head_len, bool& neg1) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const long long tbase = (long long)tile * ENC_TILE;
    const long long base = tbase + (long long)tid * ENC_K;
    const bool full = tbase + ENC_TILE <= n && idx0 + tbase >= 3;
    float h0 = 0.0f, h1 = 0.0f, h2 = 0.0f, h3 = 0.0f;
    const bool hin = wid == 1 && lane < 11 && tbase + ENC_TILE + lane < n;
    if (hin) {
        const long long e = tbase + ENC_TILE + lane;
        h0 = x[e]; h1 = x[e - 1]; h2 = x[e - 2]; h3 = x[e - 3];
    }
    {
        float4 f[ENC_Q];
        load_tile4(x, n, tbase, tid, f);
#pragma unroll
        for (int q = 0; q < ENC_Q; q++) {
            const int e = 4 * (tid + ENC_TPB * q);
            float* d = reinterpret_cast<float*>(buf) + 8 + e + (e >> 4);
            d[0] = f[q].x; d[1] = f[q].y; d[2] = f[q].z; d[3] = f[q].w;
        }
        if (tid < 3) reinterpret_cast<float*>(buf)[5 + tid] = halo_x(x, idx0, tbase - 3 + tid);
    }
    __syncthreads();
    float v[ENC_K + 4];
#pragma unroll
    for (int j = 1; j < ENC_K + 4; j++) {
        const int e = tid * ENC_K + j - 4;
        v[j] = reinterpret_cast<const float*>(buf)[e < 0 ? 8 + e : 8 + e + (e >> 4)];
    }
    __syncthreads();
    for (int i = tid; i < FBUF; i += ENC_TPB) buf[i] = 0u;

    uint32_t tv[ENC_K];
    uint32_t tlp[ENC_K / 4];
#pragma unroll
    for (int q = 0; q < ENC_K / 4; q++) tlp[q] = 0u;
    uint32_t mysum = 0;
    if (full) {
#pragma unroll
        for (int j = 0; j < ENC_K; j++) {
            int len;
            make_token_bf<CT>(v[4 + j], v[3 + j], v[2 + j], v[1 + j], true, P, tv[j], len);
            tlp[j >> 2] |= (uint32_t)len << (8 * (j & 3));
            mysum += (uint32_t)len;
            neg1 |= v[4 + j] == -1.0f;
        }
    } else {
#pragma unroll
        for (int j = 0; j < ENC_K; j++) {
            int len;
            make_token_bf<CT>(v[4 + j], v[3 + j], v[2 + j], v[1 + j], idx0 + base + j >= 3, P, tv[j], len);
            len = base + j < n ? len : 0;
            tv[j] = len ? tv[j] : 0u;
            tlp[j >> 2] |= (uint32_t)len << (8 * (j & 3));
            mysum += (uint32_t)len;
            neg1 |= base + j < n && v[4 + j] == -1.0f;
        }
    }
    uint32_t inc = mysum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(inc, d, 64);
        if (lane >= d) inc += t;
    }
    if (lane == 63) s_wsum[wid] = inc;
    if (wid == 1 && lane < 12) {
        uint32_t hv = 0u; int hl = 0;
        if (lane < 11 && hin) make_token<CT>(h0, h1, h2, h3, idx0 + tbase + ENC_TILE + lane >= 3, P, hv, hl);
        s_head_val[lane] = hv;
        s_head_len[lane] = hl;
    }
    __syncthreads();
    uint32_t wpre = 0, T = 0;
#pragma unroll
    for (int w = 0; w < ENC_TPB / 64; w++) {
        if (w < wid) wpre += s_wsum[w];
        T += s_wsum[w];
    }
    if (tid == 0)                                                    // publish the count early
        st_relaxed(&flags[tile], tile == 0 ? eflag(2, epoch, (unsigned long long)start_bit + T) : eflag(1, epoch, T));
    uint32_t* bb = buf + 1;                                          // tile bit 0 = MSB of buf[1]
    {
        uint32_t off = wpre + inc - mysum;
#pragma unroll
        for (int j = 0; j < ENC_K; j++) {
            const int len = (int)((tlp[j >> 2] >> (8 * (j & 3))) & 0xFFu);
            const uint64_t vv = (uint64_t)tv[j] << ((64 - (int)(off & 31u) - len) & 63);
            uint32_t* d = bb + (off >> 5);
            atomicOr(d, (uint32_t)(vv >> 32));
            atomicOr(d + 1, (uint32_t)vv);
            off += (uint32_t)len;
        }
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t ho = T;
        for (int j = 0; j < 11 && s_head_len[j]; j++) {
            if (ho - T >= 32u) break;
            lds_place(bb, ho, s_head_val[j], s_head_len[j]);
            ho += (uint32_t)s_head_len[j];
        }
    }
    __syncthreads();
    return T;
}

// look-back for the tile's exclusive prefix G (wave 0), publish the inclusive prefix, store the owned
// words of buf shifted into place
__device__ __forceinline__ void fused_finish(uint32_t* __restrict__ out, uint64_t* __restrict__ flags, uint32_t epoch,
                                             int start_bit, unsigned tile, unsigned ntiles, uint32_t T, const uint32_t* buf,
                                             unsigned long long* __restrict__ total_bits, unsigned* __restrict__ err,
                                             unsigned long long* s_G) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (wid == 0) {
        unsigned long long G = (unsigned long long)start_bit;
        if (tile > 0) {
            unsigned long long acc = 0;
            long long k = (long long)tile - 1;
            unsigned spins = 0;
            while (true) {
                const long long q = k - lane;
                const uint64_t fv = q >= 0 ? ld_relaxed(&flags[q]) : eflag(2, epoch, 0);
                const bool mine = ((fv >> 40) & 0x3FFFFFu) == (epoch & 0x3FFFFFu);
                const int stt = mine ? (int)(fv >> 62) : 0;
                const unsigned long long incl = __ballot(stt == 2);
                const int fi = incl ? __ffsll((long long)incl) - 1 : 64;
                const unsigned long long need = fi == 64 ? ~0ull : ((2ull << fi) - 1ull);
                if (__ballot(stt == 0) & need) {                     // a predecessor has not published yet
                    if (++spins > (1u << 22)) { if (lane == 0) atomicOr(err, 4u); break; }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                unsigned long long val = (lane <= fi) ? (fv & 0xFFFFFFFFFFull) : 0ull;
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) val += __shfl_xor(val, d, 64);
                acc += val;
                if (fi < 64) break;
                k -= 64;
            }
            G = acc;
        }
        if (lane == 0) {
            *s_G = G;
            if (tile > 0) st_relaxed(&flags[tile], eflag(2, epoch, G + T));
            if (tile == ntiles - 1) *total_bits = G + T;
        }
    }
    __syncthreads();
    const unsigned long long G = *s_G;
    const int sh = (int)(G & 31ull);
    const long long wb = (long long)(G >> 5);
    long long w0 = (long long)((G + 31) >> 5);
    if (tile == 0) w0 = 0;
    const long long w1 = (long long)((G + T + 31) >> 5);
    for (long long w = w0 + tid; w < w1; w += ENC_TPB) {
        const long long i = w - wb;
        const uint32_t val = sh ? __builtin_amdgcn_alignbit(buf[i], buf[i + 1], (uint32_t)sh) : buf[i + 1];
        out[w] = __builtin_bswap32(val);
    }
}

// Tiles are software-pipelined: the workgroup computes and packs tile t+1 into its second buffer
// before it looks back for tile t, so the look-back latency overlaps the next tile's work.
template <int CT>
__global__ __launch_bounds__(ENC_TPB) void encode_fused_kernel(
    const float* __restrict__ x, long long n, long long idx0, Params P, uint32_t* __restrict__ out,
    uint64_t* __restrict__ flags, unsigned* __restrict__ ctr, uint32_t epoch, int start_bit, unsigned ntiles,
    unsigned long long* __restrict__ total_bits, unsigned* __restrict__ err) {
    __shared__ uint32_t s_buf[2][FBUF];
    __shared__ uint32_t s_wsum[ENC_TPB / 64];
    __shared__ uint32_t s_head_val[12];
    __shared__ int s_head_len[12];
    __shared__ unsigned s_tile;
    __shared__ unsigned long long s_G;
    const int tid = threadIdx.x, lane = tid & 63;
    bool neg1 = false;
    if (tid == 0) s_tile = atomicAdd(&ctr[0], 1u);
    __syncthreads();
    unsigned cur = s_tile;
    int cb = 0;
    uint32_t Tcur = 0;
    if (cur < ntiles) Tcur = fused_compute<CT>(x, n, idx0, P, flags, epoch, start_bit, cur, s_buf[0], s_wsum, s_head_val,
                                               s_head_len, neg1);
    while (cur < ntiles) {
        __syncthreads();
        if (tid == 0) s_tile = atomicAdd(&ctr[0], 1u);
        __syncthreads();
        const unsigned nxt = s_tile;
        uint32_t Tn = 0;
        if (nxt < ntiles) Tn = fused_compute<CT>(x, n, idx0, P, flags, epoch, start_bit, nxt, s_buf[cb ^ 1], s_wsum,
                                                 s_head_val, s_head_len, neg1);
        fused_finish(out, flags, epoch, start_bit, cur, ntiles, Tcur, s_buf[cb], total_bits, err, &s_G);
        cur = nxt;
        Tcur = Tn;
        cb ^= 1;
    }
    if (CT != 6 && __any(neg1) && lane == 0) atomicOr(err, 1u);      // -1.0f is the reference's sentinel
    if (tid == 0) {
        __threadfence();
        if (atomicAdd(&ctr[1], 1u) == gridDim.x - 1) { atomicExch(&ctr[0], 0u); atomicExch(&ctr[1], 0u); }
    }
}

// ------------------------------------------------------------------------------------------------
#define DC_ENC_DISPATCH(KER, ...)                                                                  \
    switch (P->ct) {                                                                               \
        case 5: hipLaunchKernelGGL(KER<5>, __VA_ARGS__); break;                                    \
        case 6: hipLaunchKernelGGL(KER<6>, __VA_ARGS__); break;                                    \
        case 7: hipLaunchKernelGGL(KER<7>, __VA_ARGS__); break;                                    \
        case 11: hipLaunchKernelGGL(KER<11>, __VA_ARGS__); break;                                  \
        default: return -2;                                                                        \
    }

// write kernel grid: one workgroup per tile (measured best: write 165 -> 159 us against a resident-count
// persistent grid, 2048 and 4096 in between); DC_WRITE_GRID overrides it for sweeps
static unsigned write_grid() {
    static unsigned g = [] {
        const char* e = getenv("DC_WRITE_GRID");
        return (e && atoi(e) > 0) ? (unsigned)atoi(e) : (1u << 30);
    }();
    return g;
}

static unsigned fused_grid(int ct) {
    static unsigned cache[12];
    const int ci = (ct > 0 && ct < 12) ? ct : 0;
    if (cache[ci]) return cache[ci];
    int dev = 0, ncu = 256, per = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const void* f = ct == 5 ? (const void*)encode_fused_kernel<5> : ct == 6 ? (const void*)encode_fused_kernel<6>
                  : ct == 7 ? (const void*)encode_fused_kernel<7> : (const void*)encode_fused_kernel<11>;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, f, ENC_TPB, 0) != hipSuccess || per < 1) per = 1;
    cache[ci] = (unsigned)(per * ncu);
    return cache[ci];
}

extern "C" int dc_launch_encode(const float* x, long long n, long long idx0, const Params* P,
                                uint32_t* out, uint64_t* desc, unsigned* tile_ctr, uint32_t epoch,
                                int start_bit, unsigned long long* total_bits, unsigned* err,
                                unsigned long long* dbg, hipStream_t stream) {
    if (n <= 0) return 0;
    const unsigned ntiles = (unsigned)((n + ENC_TILE - 1) / ENC_TILE);
    // single pass (decoupled look-back, software-pipelined tiles): measured 284 us against 257 us for
    // count + scan + write at 2^26 U10 (the write kernel re-reads its tiles from the Infinity Cache
    // and hides their latency across 65536 count workgroups); kept as an option, DC_ENC_FUSED=1
    static int fused = -1;
    if (fused < 0) fused = getenv("DC_ENC_FUSED") ? 1 : 0;
    if (fused && !dbg) {
        const unsigned gf = std::min<unsigned>(ntiles, fused_grid(P->ct));
        dc_mark_phase(0, stream);
        dc_mark_phase(1, stream);
        dc_mark_phase(2, stream);
        DC_ENC_DISPATCH(encode_fused_kernel, dim3(gf), dim3(ENC_TPB), 0, stream, x, n, idx0, *P, out, desc, tile_ctr,
                        epoch, start_bit, ntiles, total_bits, err);
        dc_mark_phase(3, stream);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    uint32_t* tbits = reinterpret_cast<uint32_t*>(desc + ntiles);     // tile counts; desc: dc_encode_desc_words(n)
    dc_mark_phase(0, stream);
    // count: one workgroup per tile (a persistent count grid with prefetch measured slower)
    const unsigned gc = ntiles;                                    // count: one workgroup per tile
    const unsigned gw = std::min<unsigned>(ntiles, write_grid());
    DC_ENC_DISPATCH(encode_count_kernel, dim3(gc), dim3(256), 0, stream, x, n, idx0, *P, tbits,
                    (long long)ntiles, err);
    dc_mark_phase(1, stream);
    hipLaunchKernelGGL(encode_scan_kernel, dim3(1), dim3(1024), 0, stream, tbits, desc, (long long)ntiles, start_bit,
                       total_bits);
    dc_mark_phase(2, stream);
    DC_ENC_DISPATCH(encode_write_kernel, dim3(gw), dim3(ENC_TPB), 0, stream, x, n, idx0, *P, out, desc, ntiles,
                    dbg);
    dc_mark_phase(3, stream);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// count + scan only: total bits (start_bit + stream bits) of an encode, nothing written
extern "C" int dc_launch_encode_bits(const float* x, long long n, long long idx0, const Params* P, uint64_t* desc,
                                     unsigned long long* total_bits, unsigned* err, hipStream_t stream) {
    if (n <= 0) return 0;
    const unsigned ntiles = (unsigned)((n + ENC_TILE - 1) / ENC_TILE);
    uint32_t* tbits = reinterpret_cast<uint32_t*>(desc + ntiles);
    const unsigned gc = ntiles;
    DC_ENC_DISPATCH(encode_count_kernel, dim3(gc), dim3(256), 0, stream, x, n, idx0, *P, tbits, (long long)ntiles, err);
    hipLaunchKernelGGL(encode_scan_kernel, dim3(1), dim3(1024), 0, stream, tbits, desc, (long long)ntiles, 0, total_bits);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" long long dc_encode_tile_count(long long n) { return (n + ENC_TILE - 1) / ENC_TILE; }

// u64 words of the encode descriptor buffer: tile offsets + 32-bit tile-part counts
extern "C" long long dc_encode_desc_words(long long n) {
    const long long nt = dc_encode_tile_count(n);
    return nt + (nt + 1) / 2;
}

}  // namespace dc
