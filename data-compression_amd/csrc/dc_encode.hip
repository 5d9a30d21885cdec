// dc_encode.hip -- bit-wise encoder for gfx950 (CT 5/6/7/11).
//
// Replaces the per-element serial loop of myCompress_bitwise (impl/dataCompression.c:3310-3444),
// myCompress_bitwise_np (:2645-2654), myCompress_bitwise_mask (:2030-2141) and
// myCompress_bitwise_op (:577-696), whose cost is one add_bit_to_bytes call (+ realloc) per output
// bit (:5456-5489).
//
// The encoder history is the ORIGINAL input (:2095-2097), so every token is a pure function of
// x[i-3..i].  Two launches:
//   encode_count_kernel : per tile of ENC_TILE floats, the total token bit length and the tile's last
//                         31 bits (its successor's first word starts with them)
//   encode_pack_kernel  : workgroup 0 first scans the tile lengths -> every tile's global bit offset G
//                         and publishes them; every tile packs its tokens MSB-first into an LDS bit
//                         buffer (plain word writes, neighbour words merged through DPP), then -- the
//                         offsets long published -- stores them shifted by G mod 32: every word from the
//                         one holding the tile's first bit to its last full word.
// (encode_scan_kernel, the scan as a launch of its own, serves dc_launch_encode_bits.)
// (A single pass with published tile totals was measured slower: a tile waits for the slowest of
// its predecessors' loads, 220-700 us against 140 us; so was a scan folded into the count and pack
// kernels -- a device-scope atomic add of every tile's total into its group's, which the pack then sums:
// count 65 -> 143 us, see DESIGN.md.)
#include "dc_device.h"
#include <algorithm>
#include <stdlib.h>

namespace dc {

constexpr int ENC_TILE = 4096;                  // floats per tile (one offset per tile)
constexpr int ENC_TPB = 256;                    // write kernel: 4 waves per tile
constexpr int ENC_K = ENC_TILE / ENC_TPB;       // 16 consecutive floats per lane
#ifndef DC_CNT_Q
#define DC_CNT_Q 4
#endif
#ifndef DC_CNT_NT
#define DC_CNT_NT 1                     // the count pass streams x past the caches: measured count 85 -> 57 us
#endif
constexpr int CNT_Q = DC_CNT_Q;                 // count kernel: one wave per tile part, CNT_Q float4 per lane
constexpr int CNT_SUB = 256 * CNT_Q;            // floats per count wave
constexpr int CNT_PARTS = ENC_TILE / CNT_SUB;   // count parts per tile (tbits entries)

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
                                             const uint16_t* tab, uint32_t* qsum, bool& neg1) {
#pragma unroll
    for (int q = 0; q < CNT_Q; q++) {
        const float b1 = wave_shr1(f[q].w, h1), b2 = wave_shr1(f[q].z, h2), b3 = wave_shr1(f[q].y, h3);
        h1 = lane63(f[q].w); h2 = lane63(f[q].z); h3 = lane63(f[q].y);
        const float xs[7] = {b3, b2, b1, f[q].x, f[q].y, f[q].z, f[q].w};
        qsum[q] = 0u;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            qsum[q] += (uint32_t)token_len_t<CT>(xs[3 + r], xs[2 + r], xs[1 + r], xs[r], true, P, tab);
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
                                           const uint16_t* tab, long long h, const float4* f, const float* hist, int lane,
                                           uint32_t* psum, unsigned* __restrict__ err, uint32_t* qsum) {
    const long long tb = h * CNT_SUB;
    bool neg1 = false;
    count_tokens<CT>(f, hist[0], hist[1], hist[2], P, tab, qsum, neg1);
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < CNT_Q; q++) sum += qsum[q];
    sum = wave_total(sum);
    if (lane == 0) {
        int vend = CNT_SUB;                                          // elements the vector pass saw
        if (tb + CNT_SUB > n) {                                      // the 0.0f padding's tokens
            const int rem = (int)max(n - tb, 0ll);                   // 0: a part past the end
            vend = rem & ~3;
            sum -= (uint32_t)token_len_t<CT>(0.0f, 0.0f, 0.0f, 0.0f, true, P, tab) * (uint32_t)(CNT_SUB - vend);
            for (int j = vend; j < rem; j++) {                       // the straddling float4
                const long long e = tb + j;
                const float v = x[e];
                neg1 |= v == -1.0f;
                sum += (uint32_t)token_len_t<CT>(v, halo_x(x, idx0, e - 1), halo_x(x, idx0, e - 2),
                                                 halo_x(x, idx0, e - 3), idx0 + e >= 3, P, tab);
            }
        }
        if (CT != 6) {                                               // unpredicted head elements
            for (int j = 0; j < 3 && j < vend && idx0 + tb + j < 3; j++) {
                const long long e = tb + j;
                const float v = x[e], b1 = halo_x(x, idx0, e - 1), b2 = halo_x(x, idx0, e - 2),
                            b3 = halo_x(x, idx0, e - 3);
                sum += (uint32_t)(token_len_t<CT>(v, b1, b2, b3, false, P, tab) - token_len_t<CT>(v, b1, b2, b3, true, P, tab));
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
                                                           unsigned* __restrict__ err, uint32_t* __restrict__ tails,
                                                           uint16_t* __restrict__ psum16) {
    static_assert(CNT_PARTS == 4, "one workgroup of four waves per tile");
    __shared__ uint32_t wsum[4];
    __shared__ uint16_t tab[512];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const long long h = (long long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(wid);
    float4 f[CNT_Q];
    float hist[3];
    uint32_t qsum[CNT_Q];
    load_part(x, n, idx0, h * CNT_SUB, lane, f, hist);
    build_enc_tab<CT>(tab, P, threadIdx.x, 256);
    __syncthreads();
    count_part<CT>(x, n, idx0, P, tab, h, f, hist, lane, wsum + wid, err, qsum);
    // the bit counts of the pack kernel's threads (16 consecutive floats = float4s 4k..4k+3 of a row q:
    // a lane quad), for the tiles it packs without counting (whole, every float predicted)
    const long long tb0 = (long long)blockIdx.x * ENC_TILE;
    if (psum16 && tb0 + ENC_TILE <= n && idx0 + tb0 >= 3) {
#pragma unroll
        for (int q = 0; q < CNT_Q; q++) {
            uint32_t v = qsum[q];
            v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
            v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm 2,3,0,1
            if ((lane & 3) == 0) psum16[blockIdx.x * ENC_TPB + 64 * wid + 16 * q + (lane >> 2)] = (uint16_t)v;
        }
    }
    // the tile's last 31 bits (its successor's first word starts with them): the tokens of its last 16
    // floats (lanes 60..63 of the last wave, last float4 row; >= 48 bits, all predicted), joined in lane 63
    if (tails && wid == 3 && (long long)(blockIdx.x + 1) * ENC_TILE <= n) {
        constexpr int q = CNT_Q - 1;
        const float xs[7] = {wave_shr1(f[q].y, 0.0f), wave_shr1(f[q].z, 0.0f), wave_shr1(f[q].w, 0.0f),
                             f[q].x, f[q].y, f[q].z, f[q].w};
        uint64_t acc = 0;
        uint32_t L = 0;
        if (lane >= 60) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                uint32_t tv;
                int len;
                make_token_t<CT>(xs[3 + r], xs[2 + r], xs[1 + r], xs[r], true, P, tab, tv, len);
                acc = (acc << len) | tv;
                L += (uint32_t)len;
            }
        }
        uint64_t t = 0;
#pragma unroll
        for (int l = 60; l < 64; l++) {
            const uint64_t a = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(acc >> 32), l) << 32) |
                               (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)acc, l);
            const uint32_t sl = (uint32_t)__builtin_amdgcn_readlane((int)L, l);
            t = (sl >= 64u ? 0ull : (t << sl)) | a;
        }
        if (lane == 63) tails[blockIdx.x] = (uint32_t)t & 0x7FFFFFFFu;
    }
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
                                                           unsigned long long* __restrict__ total_bits,
                                                           unsigned long long* __restrict__ total_bits2) {
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
    if (tid == 0) {
        *total_bits = carry;
        if (total_bits2) *total_bits2 = carry;
    }
}

// ------------------------------------------------------------------------------------------------
// Pack kernel (third launch): one workgroup per tile reads its floats, makes the tokens, packs them into
// an LDS bit buffer and stores them at the tile's bit offset G from the scan.  The word holding the
// tile's first bit starts with the last G mod 32 bits of the previous tile (its tail, from the count
// kernel): the tile stores every word from there up to its last full word; the last tile also stores
// its final partial word.  No tile waits for another.
// Registers decide the occupancy (LDS: 17 KB per tile): the lengths are made first (token_len_enc,
// the same decision as make_token_bf) and the token values again while packing.
#ifndef DC_PACK_NT
#define DC_PACK_NT 1                            // x read and the stream written past the caches (streaming)
#endif
constexpr int E3_WORDS = ENC_TILE + 64;                 // bit buffer words (4096 at 32 bits per float)
#ifndef DC_PACK_STG2
#define DC_PACK_STG2 1                          // transpose in two halves: half the staging LDS, 8 tiles per CU
#endif
constexpr int E3_STG = 64 * ENC_K / 16 * 20 / (DC_PACK_STG2 ? 2 : 1);   // a wave's staged floats (rows of 16 + 4 pad)
constexpr int E3_LDS0 = E3_WORDS > 4 * E3_STG ? E3_WORDS : 4 * E3_STG;
constexpr int E3_LDS = E3_LDS0 > 4096 + 256 ? E3_LDS0 : 4096 + 256;   // (+ workgroup 0's scan chunk)
__device__ __forceinline__ uint32_t wave_shr1_u(uint32_t v, uint32_t first) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)first, (int)v, 0x138, 0xF, 0xF, false);
}
typedef float f32x4 __attribute__((ext_vector_type(4)));

// a tile's floats: lane l of wave w gets float4s l + 64q (q < 4) of the wave's 1024 floats, through a buffer
// resource based at the tile (its range: the tile's floats, up to the 16-byte granule of the last one;
// granules past it read 0, and a granule never straddles a page), so offsets stay small for any n
__device__ __forceinline__ void load_tile_x(f32x4 (&f)[ENC_K / 4], const float* __restrict__ x, long long n,
                                            long long tbase, int lane, int wid) {
    const long long m = min(n - tbase, (long long)ENC_TILE);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x + tbase), (short)0, (int)((m + 3) / 4 * 16), 0x00020000);
#pragma unroll
    for (int q = 0; q < ENC_K / 4; q++)
        f[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, 4 * (1024 * wid + 4 * (lane + 64 * q)), 0, DC_PACK_NT ? 2 : 0);
}


// Workgroup 0 of the pack kernel first scans the tile bit counts (no scan launch, no gap): chunks of 2048
// counts (the next one's loads in flight), 8 consecutive per thread through the bit buffer's LDS (a pad
// word per 16), a wave scan and the four wave totals; every offset is stored sc1 (written through), each wave drains its stores, and after
// a barrier one lane publishes the encode's epoch in `flag`.  This is the fence-free hand-off form of
// MI355X_MICROARCH.md (section "Workgroup dispatch ... inter-workgroup visibility", Valid forms, first
// table row): every payload store is an agent-scope (sc1) store, every storing wave runs s_waitcnt
// vmcnt(0) before the workgroup barrier behind which ONE lane stores the flag sc1; the consumer polls the
// flag with sc1 loads and reads every offset with sc1 loads (never L1, never flat), so neither a release
// nor an acquire fence is needed.  The pack relies on workgroup 0 being dispatched first and staying
// resident while the others poll (bounded: a tile whose poll times out sets err bit 4 and stores nothing;
// dc_encode_result then re-encodes with the wait-free three-launch variant, where the scan is a launch of
// its own).  A concurrent process on the same GPU can delay workgroup 0, never wedge the encode.
__device__ void pack_scan_block(const uint32_t* __restrict__ tcnt, uint64_t* __restrict__ toff, unsigned ntiles,
                                int start_bit, unsigned long long* __restrict__ total_bits,
                                unsigned long long* __restrict__ total_bits2, uint32_t* lds, uint32_t* s_w,
                                unsigned* __restrict__ flag, uint32_t epoch) {
    constexpr int PS = 8, PCH = 256 * PS;         // counts per thread and per chunk
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    unsigned long long carry = (unsigned long long)start_bit;
    uint32_t nxt[PS];                             // the next chunk's counts, requested one chunk ahead
#pragma unroll
    for (int k = 0; k < PS; k++) {
        const unsigned t = (unsigned)(k * 256 + tid);
        nxt[k] = t < ntiles ? tcnt[t] : 0u;
    }
    for (unsigned c0 = 0; c0 < ntiles; c0 += PCH) {
#pragma unroll
        for (int k = 0; k < PS; k++) {
            const int i = k * 256 + tid;
            lds[i + (i >> 4)] = nxt[k];
        }
#pragma unroll
        for (int k = 0; k < PS; k++) {
            const unsigned t = c0 + PCH + (unsigned)(k * 256 + tid);
            nxt[k] = t < ntiles ? tcnt[t] : 0u;
        }
        __syncthreads();
        uint32_t c[PS], sum = 0;
#pragma unroll
        for (int i = 0; i < PS; i++) {
            const int j = tid * PS + i;
            c[i] = lds[j + (j >> 4)];
            sum += c[i];
        }
        uint32_t inc = sum;                       // (a chunk's 2048 tiles hold < 2^28 bits)
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t u = __shfl_up(inc, d, 64);
            if (lane >= d) inc += u;
        }
        if (lane == 63) s_w[wid] = inc;
        __syncthreads();
        uint32_t wpre = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < 4; w++) {
            wpre += w < wid ? s_w[w] : 0u;
            tot += s_w[w];
        }
        unsigned long long run = carry + wpre + inc - sum;
#pragma unroll
        for (int i = 0; i < PS; i++) {
            const unsigned t = c0 + (unsigned)(tid * PS + i);
            if (t < ntiles) __hip_atomic_store(&toff[t], run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            run += c[i];
        }
        carry += tot;
        // the chunk's offsets are out: published for its tiles at once (the early tiles wait for the first
        // chunk only)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();                          // (also: lds / s_w are reused)
        // (release at agent scope on top of the sc1 form above: the memory model's own guarantee, ADVICE r03;
        // this variant runs only for A/B, DC_ENC_PASSES=2)
        if (tid == 0) __hip_atomic_store(&flag[c0 / PCH], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (tid == 0) {
        *total_bits = carry;
        if (total_bits2) *total_bits2 = carry;
    }
}

template <int CT>
__global__ __launch_bounds__(ENC_TPB, DC_PACK_STG2 ? 8 : 1) void encode_pack_kernel(
    const float* __restrict__ x, long long n, long long idx0, Params P, uint32_t* __restrict__ out,
    uint64_t* __restrict__ toff, const uint32_t* __restrict__ tcnt, const uint32_t* __restrict__ tails,
    const uint16_t* __restrict__ psum16, unsigned ntiles, int start_bit, unsigned long long* __restrict__ total_bits,
    unsigned long long* __restrict__ total_bits2, unsigned* __restrict__ flag, uint32_t epoch,
    unsigned* __restrict__ err, unsigned long long* __restrict__ dbg, uint32_t* __restrict__ mirror) {
    static_assert(ENC_K == 16 && ENC_TPB == 256, "16 consecutive floats per thread, 4 waves per tile");
#define E3STAMP(ph) do { if (dbg && threadIdx.x == 0 && blockIdx.x < 8192) dbg[blockIdx.x * 8 + (ph)] = __builtin_amdgcn_s_memrealtime(); } while (0)
    E3STAMP(0);
    __shared__ __attribute__((aligned(16))) uint32_t sb[E3_LDS];
    __shared__ uint32_t s_w[ENC_TPB / 64];
    __shared__ uint32_t s_hw[4], s_hi[4], s_tw[4], s_ti[4];           // the waves' first and last words
    __shared__ uint16_t tab[512];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const unsigned tile = blockIdx.x;
    build_enc_tab<CT>(tab, P, tid, ENC_TPB);                          // (read after the barrier below)
    // (flag == nullptr: the offsets come from encode_scan_kernel, launched before -- the wait-free fallback)
    if (tile == 0 && flag) pack_scan_block(tcnt, toff, ntiles, start_bit, total_bits, total_bits2, sb, s_w, flag, epoch);
    const uint32_t tp0 = tile > 0 ? tails[tile - 1] : 0u;
    const uint32_t psum_full = psum16[(long long)tile * ENC_TPB + threadIdx.x];
    const long long tbase = (long long)tile * ENC_TILE;
    const long long base = tbase + (long long)ENC_K * tid;
    const bool full = tbase + ENC_TILE <= n && idx0 + tbase >= 3;
    // ---- the thread's 16 consecutive floats.  Coalesced float4 loads (lane l: float4 l + 64q of the
    // wave's 1024 floats; x through a buffer resource up to the 16-byte granule of its last float:
    // out-of-range floats read 0, a granule never straddles a page), turned into 16 consecutive floats
    // per lane through the wave's part of the bit buffer (element e at word e + 4 (e >> 4): rows of 20
    // words, conflict-free b128 reads; before the packing).  History: the previous thread's last three
    // (DPP), for lane 0 the three floats before the wave's first.
    float h[ENC_K + 3];
    {
        float* stg = reinterpret_cast<float*>(sb) + wid * E3_STG;
        f32x4 f[ENC_K / 4];
        load_tile_x(f, x, n, tbase, lane, wid);
#if DC_PACK_STG2
        // two halves: float4s 0..127 (rows of lanes 0..31), then 128..255 (lanes 32..63) in the same 32 rows
        // (a wave's LDS accesses run in order: the first half's reads precede the second half's writes)
        f32x4 u[ENC_K / 4];
#pragma unroll
        for (int half = 0; half < 2; half++) {
#pragma unroll
            for (int q = 0; q < 2; q++) {
                const int m = lane + 64 * q;
                *reinterpret_cast<f32x4*>(stg + 4 * m + 4 * (m >> 2)) = f[2 * half + q];
            }
            __builtin_amdgcn_wave_barrier();
            if ((lane >> 5) == half)
#pragma unroll
                for (int q = 0; q < ENC_K / 4; q++) u[q] = *reinterpret_cast<const f32x4*>(stg + 20 * (lane & 31) + 4 * q);
            __builtin_amdgcn_wave_barrier();
        }
#pragma unroll
        for (int q = 0; q < ENC_K / 4; q++) {
            h[3 + 4 * q] = u[q].x; h[4 + 4 * q] = u[q].y; h[5 + 4 * q] = u[q].z; h[6 + 4 * q] = u[q].w;
        }
#else
#pragma unroll
        for (int q = 0; q < ENC_K / 4; q++) {
            const int m = lane + 64 * q;
            *reinterpret_cast<f32x4*>(stg + 4 * m + 4 * (m >> 2)) = f[q];
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int q = 0; q < ENC_K / 4; q++) {
            const f32x4 u = *reinterpret_cast<const f32x4*>(stg + 20 * lane + 4 * q);
            h[3 + 4 * q] = u.x; h[4 + 4 * q] = u.y; h[5 + 4 * q] = u.z; h[6 + 4 * q] = u.w;
        }
#endif
        const long long w0 = tbase + 64ll * ENC_K * wid;                   // the wave's first element
        float hw[3];
#pragma unroll
        for (int k = 1; k <= 3; k++) {
            const long long e = w0 - k;
            hw[k - 1] = (e < n && e >= -3 && idx0 + e >= 0) ? x[e] : 0.0f;
        }
        h[2] = wave_shr1(h[3 + ENC_K - 1], hw[0]);
        h[1] = wave_shr1(h[3 + ENC_K - 2], hw[1]);
        h[0] = wave_shr1(h[3 + ENC_K - 3], hw[2]);
    }
    if (!full)
#pragma unroll
        for (int j = 0; j < ENC_K; j++) h[3 + j] = base + j < n ? h[3 + j] : 0.0f;
    // ---- token lengths: whole tiles take the thread's bit count from the count kernel; the first tile
    // of a stream and the last one count here
    uint32_t lp[ENC_K / 4];
#pragma unroll
    for (int q = 0; q < ENC_K / 4; q++) lp[q] = 0u;
    uint32_t mysum = psum_full;
    if (!full) {
        mysum = 0;
#pragma unroll
        for (int j = 0; j < ENC_K; j++) {
            const bool in = base + j < n;
            int len = token_len_t<CT>(h[3 + j], h[2 + j], h[1 + j], h[j], idx0 + base + j >= 3, P, tab);
            len = in ? len : 0;
            lp[j >> 2] |= (uint32_t)len << (8 * (j & 3));
            mysum += (uint32_t)len;
        }
    }
    const uint32_t inc = wave_scan_incl(mysum);
    if (lane == 63) s_w[wid] = inc;
    E3STAMP(1);
    __syncthreads();
    uint32_t wpre = 0, T = 0;
#pragma unroll
    for (int w = 0; w < ENC_TPB / 64; w++) {
        if (w < wid) wpre += s_w[w];
        T += s_w[w];
    }
    const uint32_t off = wpre + inc - mysum;                          // the thread's first tile bit

    // the floats made opaque: otherwise the compiler keeps every predictor term of the length pass
    // alive across the barrier for the value pass (200+ VGPRs, 2 waves per SIMD)
#pragma unroll
    for (int j = 0; j < ENC_K + 3; j++) asm volatile("" : "+v"(h[j]));
    // ---- pack, MSB-first (token values made again here).  Full tiles: every thread holds >= 48 bits,
    // so a word is shared by at most two neighbouring threads: each writes the words it completes, its
    // first merged with the previous lane's unfinished last one (DPP); a wave's first and last words
    // are merged after the barrier
    if (full) {
        uint32_t wi = off >> 5, nb = off & 31u, headw = 0u;
        const uint32_t hi = wi;
        uint64_t acc = 0;
        bool have = false;
#pragma unroll
        for (int j = 0; j < ENC_K; j++) {
            uint32_t tv;
            int len;
            make_token_t<CT>(h[3 + j], h[2 + j], h[1 + j], h[j], true, P, tab, tv, len);
            acc |= (uint64_t)tv << ((64u - nb - (uint32_t)len) & 63u);
            nb += (uint32_t)len;
            if (nb >= 32u) {
                const uint32_t w = (uint32_t)(acc >> 32);
                if (have) sb[wi] = w;
                else headw = w;
                have = true;
                wi++;
                acc <<= 32;
                nb -= 32u;
            }
        }
        const uint32_t tailw = (uint32_t)(acc >> 32);                 // nb bits (0: none)
        const uint32_t pt = wave_shr1_u(tailw, 0u);
        if (lane == 0) { s_hw[wid] = headw; s_hi[wid] = hi; }
        else sb[hi] = headw | pt;
        if (lane == 63) { s_tw[wid] = tailw; s_ti[wid] = nb ? wi : 0xFFFFFFFFu; }
    } else {
        // tile 0 of a stream and the last tile: ORed in token by token over a cleared buffer
        for (int i = tid; i < E3_WORDS / 4; i += ENC_TPB) reinterpret_cast<uint4*>(sb)[i] = make_uint4(0u, 0u, 0u, 0u);
        __syncthreads();
        uint32_t o = off;
#pragma unroll
        for (int j = 0; j < ENC_K; j++) {
            const uint32_t lj = (lp[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            uint32_t tv;
            int len;
            make_token_t<CT>(h[3 + j], h[2 + j], h[1 + j], h[j], idx0 + base + j >= 3, P, tab, tv, len);
            if (lj) {
                const uint64_t v = (uint64_t)tv << ((64u - (o & 31u) - lj) & 63u);
                atomicOr(&sb[o >> 5], (uint32_t)(v >> 32));
                if ((o & 31u) + lj > 32u) atomicOr(&sb[(o >> 5) + 1], (uint32_t)v);
            }
            o += lj;
        }
        if (lane == 0) s_hi[wid] = 0xFFFFFFFFu;
        if (lane == 63) s_ti[wid] = 0xFFFFFFFFu;
    }
    E3STAMP(2);
    __syncthreads();
    // ---- the waves' boundary words: the head of wave w merged with the tail of wave w - 1
    if (tid < 4) {
        const uint32_t hi = s_hi[tid];
        if (hi != 0xFFFFFFFFu) {
            uint32_t w = s_hw[tid];
            if (tid > 0 && s_ti[tid - 1] == hi) w |= s_tw[tid - 1];
            sb[hi] = w;
        }
        if (tid == 3 && s_ti[3] != 0xFFFFFFFFu) sb[s_ti[3]] = s_tw[3];     // the tile's last word
    }
    // the tile's offset from workgroup 0's scan: published long before (its scan takes ~6 us, a tile's
    // loads and tokens longer), polled by one lane, read by all after the barrier (sc1 loads)
    if (tid == 0) {
        s_hw[0] = 1u;
        if (tile != 0 && flag) {
            unsigned spins = 0;
            while (__hip_atomic_load(&flag[tile / 2048u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
                if (++spins > (1u << 22)) { atomicOr(err, 4u); s_hw[0] = 0u; break; }   // (never seen)
                __builtin_amdgcn_s_sleep(8);            // (~500 cycles: thousands of early tiles poll one word)
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");          // (pairs with the flag's release)
        }
    }
    __syncthreads();
    if (s_hw[0] == 0u) return;                                         // no offset: nothing stored
    const unsigned long long Gt = __hip_atomic_load(&toff[tile], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    E3STAMP(3);
    // ---- store the words from the one holding the tile's first bit to its last full one
    const uint32_t sh = (uint32_t)(Gt & 31ull);
    const long long W0 = (long long)(Gt >> 5);
    const int nw = (int)((long long)((Gt + T) >> 5) - W0) + ((tile == ntiles - 1 && ((Gt + T) & 31ull)) ? 1 : 0);
    const int tw = (int)((T + 31u) >> 5);                              // buffer words holding tile bits
    // (a guard, never taken by a correct encode: a tile's bits end within the stream's capacity, 32 bits
    // per float after the start bit -- a stale offset must not send the stores outside the buffer)
    if (Gt + T > (unsigned long long)start_bit + 32ull * (unsigned long long)min(n, tbase + ENC_TILE)) {
        if (tid == 0) atomicOr(err, 2u);
        return;
    }
    for (int i = tid; i < nw; i += ENC_TPB) {
        const uint32_t cur = i < tw ? sb[i] : 0u;                      // (stale past the tile's bits)
        const uint32_t prev = i ? sb[i - 1] : tp0;
        const uint32_t w = sh ? __builtin_amdgcn_alignbit(prev, cur, sh) : cur;
#if defined(DC_ENC_DIAG_NOSTORE)
        if (w == 0x9E3779B9u && i == 12345) out[W0 + i] = 0u;         // (diagnostic build: the words are made, not stored)
#elif DC_PACK_NT
        __builtin_nontemporal_store(__builtin_bswap32(w), out + W0 + i);
#else
        out[W0 + i] = __builtin_bswap32(w);
#endif
        if (mirror) __builtin_nontemporal_store(__builtin_bswap32(w), mirror + W0 + i);
    }
    E3STAMP(4);
#undef E3STAMP
}

// ------------------------------------------------------------------------------------------------
// Single-pass encoder (the default, dc_launch_encode): ONE launch that reads x once.
//
// One workgroup per tile, dispatched in order (per XCD), so a tile's predecessors are running or done
// whenever it waits.  Per tile: the 4096 floats, their tokens made once (values parked in LDS, lengths in
// registers: tokens and history never share the register file), the thread bit counts scanned, the
// tile's total published at once as an AGGREGATE state, the tokens packed into the LDS bit buffer, and
// then -- the packing has given the predecessors time to publish -- the tile's bit offset from a decoupled
// look-back over its predecessors' states (rocPRIM's lookback_scan_state scheme made wide: each lane
// inspects 8 consecutive tiles, so one round trip covers 512 tiles); the INCLUSIVE state is published and
// the words stored shifted by G mod 32.  The word holding a tile's first bit starts with its
// predecessor's last bits, published as a granule of their own beside the aggregate.
//
// States are 8-byte granules written by ONE agent-scope (sc1) store and polled with agent-scope loads
// (MI355X_MICROARCH.md, hand-off granules: the data is the flag, no fence): tag (the encode's epoch, 22
// bits) << 42 | status << 40 | value (40 bits: a bit count or a bit offset).  A stale state of an earlier
// encode never matches the tag (the host clears the array when the epoch wraps).  Every wait is bounded:
// a look-back that times out poisons its tile (status 3, successors give up at once), stores nothing and
// sets err bit 4; the host then re-encodes with the wait-free three-launch path (dc_encode_result).
#ifndef DC_LB_KS
#define DC_LB_KS 4                      // look-back windows of 64 states per round trip, with the scanner
#endif
#ifndef DC_LB_DMA
#define DC_LB_DMA 0                     // the first window into LDS before the pack (lb_dma): 194 vs 147 us, off
#endif
#ifndef DC_LB_EARLY
#define DC_LB_EARLY 0                   // (r06, A/B, off) the first window requested into registers before the pack:
                                        // 156-159 vs 142-143 us (K = 1), 164-165 (K = 2)
#endif
#ifndef DC_LB_K
#define DC_LB_K 8
#endif
#ifndef DC_SCAN_POLL
#define DC_SCAN_POLL 0
#endif
#ifndef DC_LB_SLEEP
#define DC_LB_SLEEP 1
#endif
static_assert(DC_LB_K <= 8 && DC_LB_KS <= 8, "look-back windows read at most LB_PAD words before tile 0");
static_assert(!DC_LB_DMA || DC_LB_KS <= 8, "the LDS window holds at most 512 predecessors");
constexpr long long LB_PAD = 512;                                 // readable words in front of the tile states
constexpr int LB_KW = DC_LB_K;                                    // look-back: tiles per lane per round trip
constexpr unsigned long long ST_VAL = (1ull << 40) - 1;
constexpr unsigned long long ST_MASK = 3ull << 40, ST_AGG = 1ull << 40, ST_INC = 2ull << 40, ST_BAD = 3ull << 40;
constexpr uint32_t ST_TAGM = (1u << 22) - 1;
constexpr unsigned long long LB_WAIT = 2000000ull;                // s_memrealtime ticks (100 MHz): 20 ms
// A wait gives up only when BOTH its wall time exceeds LB_WAIT AND the waiting lane has polled LB_POLLS times
// (r06): the r05 rehearsal with three processes on one GPU ended with encoder status 4 although no tile can wait
// for a later one -- a queue preempted by the other processes' queues (compute wave save / restore) stops every
// wave of the launch, and the wall clock a restored wave reads then jumps past the bound.  A preempted wave does
// not poll, so a count of polls (each >= 1 state round trip, ~1 us) measures the time it actually waited; a
// true deadlock still ends after max(20 ms, LB_POLLS polls) and takes the exact three-launch fallback.
constexpr unsigned LB_POLLS = 8192;
struct WaitBound {
    unsigned long long t0;
    unsigned polls;
    __device__ __forceinline__ void start() { t0 = __builtin_amdgcn_s_memrealtime(); polls = 0; }
    __device__ __forceinline__ bool expired() {           // call once per poll
        return ++polls >= LB_POLLS && __builtin_amdgcn_s_memrealtime() - t0 > LB_WAIT;
    }
};

__device__ __forceinline__ uint64_t st_word(uint32_t tag, unsigned long long status, unsigned long long v) {
    return ((uint64_t)tag << 42) | status | (v & ST_VAL);
}
__device__ __forceinline__ unsigned long long wave_sum64(unsigned long long v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// The help of a waiting tile (enc_lookback): tile ti's bit count computed by one wave from x (lane = 64 floats,
// token_len_t: the length decision of make_token_t), and the tile's last 31 bits (its last 16 tokens, one lane)
// -- exactly what the tile itself publishes.
template <int CT>
__device__ __forceinline__ unsigned long long help_tile_bits(const float* __restrict__ x, long long n, long long idx0, const Params& P,
                                             const uint16_t* tab, long long ti) {
    const int lane = threadIdx.x & 63;
    const long long e0 = ti * ENC_TILE + 64ll * lane;
    float b[3];
#pragma unroll
    for (int k = 1; k <= 3; k++) {
        const long long e = e0 - k;
        b[k - 1] = (e < n && e >= -3 && idx0 + e >= 0) ? x[e] : 0.0f;
    }
    float b1 = b[0], b2 = b[1], b3 = b[2];
    unsigned long long bits = 0;
    for (int j = 0; j < 64; j++) {
        const long long e = e0 + j;
        if (e >= n) break;
        const float v = x[e];
        bits += (unsigned)token_len_t<CT>(v, b1, b2, b3, idx0 + e >= 3, P, tab);
        b3 = b2; b2 = b1; b1 = v;
    }
    return wave_sum64(bits);
}
template <int CT>
__device__ __forceinline__ uint32_t help_tile_tail(const float* __restrict__ x, long long idx0, const Params& P, const uint16_t* tab,
                                   long long ti) {                        // (a full tile: ti + 1 < ntiles)
    const long long e0 = (ti + 1) * ENC_TILE - ENC_K;
    float b1 = x[e0 - 1], b2 = x[e0 - 2], b3 = x[e0 - 3];
    unsigned long long acc = 0;
    for (int j = 0; j < ENC_K; j++) {
        const long long e = e0 + j;
        const float v = x[e];
        uint32_t tv;
        int len;
        make_token_t<CT>(v, b1, b2, b3, idx0 + e >= 3, P, tab, tv, len);
        acc = (acc << len) | tv;
        b3 = b2; b2 = b1; b1 = v;
    }
    return (uint32_t)acc & 0x7FFFFFFFu;
}

// exclusive bit offset of tile t >= 1 (one whole wave; wave-uniform result).  Position p = 64 k + l of the
// window [base - 64 LB_K + 1, base] (tile base - p) is lane l's k-th state, so each of the LB_K loads reads
// 512 contiguous bytes (a strided layout, 64 segments per load, made the look-back traffic exceed the
// codec's); every load is in flight at once.  The states from tile t - 1 down to the nearest INCLUSIVE one
// must all be published.  While one is not, ONE lane polls that state (a whole window re-read per poll by
// ~1800 waiting tiles tripled the encode), then the window is read again.  A window without an inclusive
// state adds its aggregates and the next one is read.  Returns 0, or 1 when a needed state is poisoned or a
// wait timed out.
// lw0 (optional): the first window as loaded into LDS before the tile's pack (lw0[q] = state s0 + q,
// lb_dma below); a state it saw unpublished is polled and the window read again as usual.
// vr (optional): the first window as loaded earlier into registers (vr[k] = lane's k-th state,
// ld_relaxed(st + t - 1 - lane - 64 k), encode_pipe_kernel).
// help (r06): a callable help(ti) -> the bit count of tile ti, computed by this wave from x, or ~0 for no help.
// A state still unpublished after HELP_POLLS polls is computed and published (CAS from the value seen) by the
// waiting tile itself: its forward progress then depends on no other workgroup being scheduled -- with other
// processes' look-back kernels on the same GPU, a predecessor's workgroup can stay undispatched on its XCD
// behind their waiting waves while this one holds a slot of another XCD (r05f: three ranks on one GPU, encoder
// status 4).  The value is the one the owner publishes, so a late owner's store is harmless.
// The help is compiled into its own instantiation (encode_fused_kernel<CT, CRC, true>, chosen by
// dc_set_encode_help / DC_ENC_HELP=1): never triggered, it still cost the hot path 7 us (tiles helping) and 12 us
// (the scanner helping) at 2^26 -- more spilled SGPRs in the token code -- and one process per GPU (the real
// multi-GPU run) does not need it: dispatch there is in order per XCD and only this launch holds the slots.
#ifndef DC_HELP_POLLS
#define DC_HELP_POLLS 256                       // (tests build 0: every unpublished state helped at once)
#endif
constexpr unsigned HELP_POLLS = DC_HELP_POLLS;
struct NoHelp {
    __device__ __forceinline__ unsigned long long operator()(long long) const { return ~0ull; }
};
template <int LB_K, class Help = NoHelp>
__device__ __forceinline__ int enc_lookback(const uint64_t* __restrict__ st, long long t, uint32_t tag,
                                            unsigned long long& excl, uint32_t& stat, int start_bit,
                                            const uint64_t* lw0 = nullptr, long long s0 = 0,
                                            const uint64_t* vr = nullptr, Help help = Help()) {
    const int lane = threadIdx.x & 63;
    long long base = t - 1;
    excl = 0;
    WaitBound wb;
    wb.start();
    bool first = lw0 != nullptr || vr != nullptr;
    for (;;) {
        uint64_t v[LB_K];
        int pinc;                                                         // first inclusive position (64 LB_K: none)
        for (;;) {
            // one address, immediate offsets: positions before tile 0 read the LB_PAD words in front of the
            // states (any value) and are replaced by the virtual inclusive state start_bit
            const uint64_t* p = st + (base - lane);
#pragma unroll
            for (int k = 0; k < LB_K; k++) {
                const long long ti = base - (long long)(64 * k + lane);
                const uint64_t w = first ? (vr ? vr[k] : lw0[ti - s0]) : ld_relaxed(p - 64 * k);
                v[k] = ti >= 0 ? w : st_word(tag, ST_INC, (unsigned long long)start_bit);   // (before tile 0)
            }
            first = false;
            pinc = 64 * LB_K;
            int pinv = 64 * LB_K;                                         // first unpublished position
#pragma unroll
            for (int k = LB_K - 1; k >= 0; k--) {
                const bool live = (uint32_t)(v[k] >> 42) == tag && (v[k] & ST_MASK) != 0;
                const unsigned long long um = __ballot(!live);
                const unsigned long long im = __ballot(live && (v[k] & ST_MASK) != ST_AGG);   // inclusive / poisoned
                if (um) pinv = 64 * k + __ffsll((long long)um) - 1;
                if (im) pinc = 64 * k + __ffsll((long long)im) - 1;
            }
            // every needed state is published (pinv == pinc: the whole window, no inclusive state: go on
            // past it)
            if (pinv >= pinc) break;
            stat++;
            bool gone = false, stuck = false;
            uint64_t seen = 0;
            const long long ti = base - pinv;
            if (lane == (pinv & 63)) {                                    // its lane polls it alone
                for (unsigned k = 0;; k++) {
                    const uint64_t w = ld_relaxed(st + ti);
                    if ((uint32_t)(w >> 42) == tag && (w & ST_MASK) != 0) break;
                    if (k >= HELP_POLLS) { stuck = true; seen = w; break; }
                    if (wb.expired()) { gone = true; break; }
                    stat += 1u << 16;
                    __builtin_amdgcn_s_sleep(DC_LB_SLEEP);
                }
            }
            if (__any(gone)) return 1;
            if (__any(stuck)) {                                           // compute the late tile's count here
                const unsigned long long b = help(ti);
                if (b != ~0ull && lane == (pinv & 63))
                    atomicCAS(reinterpret_cast<unsigned long long*>(const_cast<uint64_t*>(st + ti)),
                              (unsigned long long)seen, (unsigned long long)st_word(tag, ST_AGG, b));
                stat += 1u << 28;
                if (b == ~0ull && wb.expired()) return 1;
            }
        }
        unsigned long long s = 0;
        bool bad = false;
#pragma unroll
        for (int k = 0; k < LB_K; k++) {
            if (64 * k + lane <= pinc) {
                s += v[k] & ST_VAL;
                bad |= (v[k] & ST_MASK) == ST_BAD;
            }
        }
        if (__any(bad)) return 1;
        excl += wave_sum64(s);
        if (pinc < 64 * LB_K) return 0;
        base -= 64 * LB_K;
    }
}

// The first look-back window requested straight into LDS (global_load_lds, agent-coherent sc1: no
// VGPRs held across the pack, where a register window spilled) before the tile packs its words: the
// ~3 us round trip of state loads under the stream then overlaps the pack.  Lane l of load m brings
// states s0 + 128 m + 2 l, +1 (16 bytes); s0 is even (16-byte aligned: st is) and the three loads cover
// the 256 states base - 255 .. base.  Positions before tile 0 read LB_PAD words in front of st.
constexpr int LB_DMA_N = DC_LB_KS / 2 + 1;                        // 128 states per load (+1: s0 rounded down)
__device__ __forceinline__ long long lb_dma(const uint64_t* __restrict__ st, long long base, uint64_t* lw) {
    const long long s0 = (base - 64 * DC_LB_KS) & ~1ll;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int m = 0; m < LB_DMA_N; m++)
        __builtin_amdgcn_global_load_lds(st + s0 + 128 * m + 2 * lane, lw + 128 * m, 16, 0, 16 /* sc1 */);
    return s0;
}

#ifndef DC_TOK_SB
#define DC_TOK_SB 0                     // (experiments: tokens the scheduler may interleave)
#endif
// (r06) the tokens without the LDS table and with ONE wave-uniform prediction branch per 16 tokens: the table
// read + wait + branch of make_token_t made each thread's 16 tokens one dependent chain (16 x ~150 cycles of
// LDS latency, a branch between tokens; the ISA showed ds_read_u16 -> s_waitcnt lgkmcnt(1) -> s_cbranch per
// token); here the raw length is arithmetic (tab[i9] = 32 - l9 | len << 8, l9 = clamp(E + rawadd, 9, 32)) and
// the 16 tokens are independent until the rare prediction fix-up.  Measured r06 (CT7 2^26): encoder 150.8-151.4
// vs 144-145 us with the table form: the extra VALU cost more than the chain (7 waves per SIMD hide the LDS
// latency) -- off.  DC_TOK_ALU=2: the table read kept, one prediction branch per group: 149-152 vs 145-146 us
// (tools/experiments/enc_time.py) -- off as well.
#ifndef DC_TOK_ALU
#define DC_TOK_ALU 0
#endif
#ifndef DC_TOK_G
#define DC_TOK_G 4
#endif
template <int CT>
__device__ __forceinline__ void raw_token_alu(float x, const Params& P, const uint16_t* tab, uint32_t& val, int& len) {
    const uint32_t u = __float_as_uint(x);
    if (CT == 11) { val = u; len = 32; return; }
    const uint32_t i9 = u >> 23;
#if DC_TOK_ALU == 2                                       // (the table read, grouped: one wait per group)
    const uint32_t e = tab[i9];
    uint32_t v = u >> (e & 31u);
    int l = (int)(e >> 8);
    if (CT == 7) {
        const bool f0 = (u >> 15) == P.mask17;
        v ^= f0 ? P.K0 : (i9 == (P.mask17 >> 8) ? P.K1 : 0u);
        l = f0 ? P.lm0 : l;
    }
    val = v;
    len = l;
#else
    const int l9 = min(max((int)(i9 & 0xFFu) + P.rawadd, 9), 32);
    uint32_t v = u >> (uint32_t)(32 - l9);
    int l = l9;
    if (CT == 7) {
        const bool f1 = i9 == (P.mask17 >> 8);
        const bool f0 = (u >> 15) == P.mask17;
        l = f0 ? P.lm0 : (f1 ? P.lm1 : l9);
        v ^= f0 ? P.K0 : (f1 ? P.K1 : 0u);
    }
    val = v;
    len = l;
#endif
}
// |b1 - x| etc. of make_token_t: the predictor distances, and whether a prediction is taken
__device__ __forceinline__ void pred_dists(float x, float b1, float b2, float b3, float& d1, float& d2, float& d3) {
    const float p2 = __fsub_rn(__fmul_rn(2.0f, b1), b2);
    const float p3 = __fadd_rn(__fsub_rn(__fmul_rn(3.0f, b1), __fmul_rn(3.0f, b2)), b3);
    d1 = fabsf(__fsub_rn(b1, x));
    d2 = fabsf(__fsub_rn(p2, x));
    d3 = fabsf(__fsub_rn(p3, x));
}
template <int CT, bool FAST>
__device__ __forceinline__ uint32_t make_tokens16_alu(const float* h, const Params& P, const uint16_t* tab, int g3, int rem,
                                                      uint32_t* tvs,
                                                      uint32_t (&lp)[ENC_K / 4], bool& neg1) {
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < ENC_K / 4; q++) lp[q] = 0u;
    // groups of DC_TOK_G tokens: independent work to cover the VALU latencies, and each group's rare prediction
    // fix-up right after it, so that a float's history dies with its group (one fix-up after all 16 kept the 19
    // history floats live and spilled ~40 VGPRs at 7 workgroups per CU)
#pragma unroll
    for (int g0 = 0; g0 < ENC_K; g0 += DC_TOK_G) {
        uint32_t prm = 0;                                                // the group's tokens that take a prediction
#pragma unroll
        for (int j = g0; j < g0 + DC_TOK_G; j++) {
            const float x = h[3 + j];
            uint32_t v;
            int len;
            raw_token_alu<CT>(x, P, tab, v, len);
            if (CT != 6) {
                float d1, d2, d3;
                pred_dists(x, h[2 + j], h[1 + j], h[j], d1, d2, d3);
                const bool pr = (FAST ? true : j >= g3) && d1 == d1 && fminf(fminf(d1, d2), d3) <= P.thr_le;
                const bool z = fabsf(x) <= P.thr_lt;
                prm |= (pr && !z) ? 1u << j : 0u;
                v = z ? 4u : v;
                len = (pr || z) ? 3 : len;
                neg1 |= x == -1.0f;                                      // the reference's sentinel
            }
            if (!FAST) len = j < rem ? len : 0;                          // past the end: no token
            tvs[ENC_TPB * j] = v;
            lp[j >> 2] |= (uint32_t)len << (8 * (j & 3));
            sum += (uint32_t)len;
        }
        if (CT != 6 && __builtin_expect(__any(prm != 0u), 0)) {         // (rare in ordinary data)
#pragma unroll
            for (int j = g0; j < g0 + DC_TOK_G; j++) {
                if ((prm >> j) & 1u) {
                    float d1, d2, d3;
                    pred_dists(h[3 + j], h[2 + j], h[1 + j], h[j], d1, d2, d3);
                    const float d12 = fminf(d1, d2);
                    tvs[ENC_TPB * j] = d3 < d12 ? 7u : (d2 < d1 ? 6u : 5u);
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    return sum;
}

// (r06) Fewer VALU per token: the encoder is VALU-issue bound (SQ r05l: 1201 VALU per wave x 4 cycles, 7 waves per
// SIMD ~ the launch), and the ISA of make_tokens16 spent ~36 VALU per token, ~6 of them spilling compare masks
// to VGPR lanes (v_writelane / v_readlane: the length selects were sunk below the loop).  Here:
//  * the predictor distances of two tokens per packed instruction (v_pk_add_f32 / v_pk_mul_f32; 3 b computed once
//    per float), no FMA contraction (-ffp-contract=off), the same IEEE operations as make_token_t;
//  * no d1 == d1 test: d1 = |b1 - x| is NaN only when x or b1 is NaN or x = b1 = +-inf, and then d2 and d3 are NaN
//    too (p2 = 2 b1 - b2 and p3 = 3 b1 - 3 b2 + b3 are NaN or an infinity of b1's sign), so min(d1, d2, d3) is NaN
//    and the threshold compare is false either way;
//  * each token's value and length forced into VGPRs where they are made (no mask lives past its token);
//  * the length sum from the packed length bytes (v_sad_u8), not one add per token.
#ifndef DC_ENC_V2
#define DC_ENC_V2 0                     // (A/B, off) bit 0: make_tokens16_v2; bit 1: the OR pack (below)
#endif
typedef float f32x2 __attribute__((ext_vector_type(2)));
template <int CT, bool FAST>
__device__ __forceinline__ uint32_t make_tokens16_v2(const float* h, const Params& P, const uint16_t* tab, int g3, int rem,
                                                     uint32_t* tvs, uint32_t (&lp)[ENC_K / 4], bool& neg1) {
#pragma unroll
    for (int q = 0; q < ENC_K / 4; q++) lp[q] = 0u;
    float dm[ENC_K];
    if (CT != 6) {
        float t3[ENC_K + 2];                                             // 3 h[k], k < 18 (b1 and b2 of every token)
#pragma unroll
        for (int k = 0; k < ENC_K + 2; k += 2) {
            const f32x2 a = {h[k], h[k + 1]};
            const f32x2 m = a * 3.0f;
            t3[k] = m.x; t3[k + 1] = m.y;
        }
#pragma unroll
        for (int j = 0; j < ENC_K; j += 2) {
            const f32x2 x = {h[3 + j], h[4 + j]}, b1 = {h[2 + j], h[3 + j]}, b2 = {h[1 + j], h[2 + j]},
                        b3 = {h[j], h[1 + j]}, c1 = {t3[2 + j], t3[3 + j]}, c2 = {t3[1 + j], t3[2 + j]};
            const f32x2 p2 = (b1 + b1) - b2;                             // __fmul_rn(2, b1) is exact: b1 + b1
            const f32x2 p3 = (c1 - c2) + b3;
            const f32x2 d1 = b1 - x, d2 = p2 - x, d3 = p3 - x;
            dm[j] = fminf(fminf(fabsf(d1.x), fabsf(d2.x)), fabsf(d3.x));
            dm[j + 1] = fminf(fminf(fabsf(d1.y), fabsf(d2.y)), fabsf(d3.y));
        }
    }
#pragma unroll
    for (int j = 0; j < ENC_K; j++) {
        const float xf = h[3 + j];
        const uint32_t u = __float_as_uint(xf);
        uint32_t v;
        int l;
        if (CT == 11) {
            v = u; l = 32;
        } else {
            const uint32_t i9 = u >> 23;
            const uint32_t e = tab[i9];
            v = u >> (e & 31u);
            l = (int)(e >> 8);
            if (CT == 7) {
                const bool f0 = (u >> 15) == P.mask17;
                v ^= f0 ? P.K0 : (i9 == (P.mask17 >> 8) ? P.K1 : 0u);
                l = f0 ? P.lm0 : l;
            }
        }
        if (CT != 6) {
            const bool pr = (FAST ? true : j >= g3) && dm[j] <= P.thr_le;
            const bool z = fabsf(xf) <= P.thr_lt;
            if (__builtin_expect(__any(pr), 0)) {                        // (rare in ordinary data) the predicted code
                float d1, d2, d3;
                pred_dists(xf, h[2 + j], h[1 + j], h[j], d1, d2, d3);
                const float d12 = fminf(d1, d2);
                const uint32_t code = d3 < d12 ? 7u : (d2 < d1 ? 6u : 5u);
                v = pr ? code : v;
            }
            v = z ? 4u : v;
            l = (pr || z) ? 3 : l;
            neg1 |= xf == -1.0f;                                         // the reference's sentinel
        }
        if (!FAST) l = j < rem ? l : 0;                                  // past the end: no token
        asm volatile("" : "+v"(v), "+v"(l));                             // made here: no compare mask outlives it
        tvs[ENC_TPB * j] = v;
        lp[j >> 2] |= (uint32_t)l << (8 * (j & 3));
    }
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < ENC_K / 4; q++) sum = __builtin_amdgcn_sad_u8(lp[q], 0u, sum);
    return sum;
}

// the 16 tokens of a thread: values to tvs[256 j], lengths packed 4 per word in lp, their sum.  Not FAST: the
// thread's elements j >= rem are past the end (no token), those j < g3 precede global index 3 (no prediction)
template <int CT, bool FAST>
__device__ __forceinline__ uint32_t make_tokens16(const float* h, const Params& P, const uint16_t* tab, int g3, int rem,
                                                  uint32_t* tvs, uint32_t (&lp)[ENC_K / 4], bool& neg1) {
    if (DC_ENC_V2 & 1) return make_tokens16_v2<CT, FAST>(h, P, tab, g3, rem, tvs, lp, neg1);
    if (DC_TOK_ALU) return make_tokens16_alu<CT, FAST>(h, P, tab, g3, rem, tvs, lp, neg1);
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < ENC_K / 4; q++) lp[q] = 0u;
#pragma unroll
    for (int j = 0; j < ENC_K; j++) {
        int len;
        uint32_t tv;
        make_token_t<CT>(h[3 + j], h[2 + j], h[1 + j], h[j], FAST ? true : j >= g3, P, tab, tv, len);
        tvs[ENC_TPB * j] = tv;
        if (CT != 6) neg1 |= h[3 + j] == -1.0f;                              // the reference's sentinel
        if (!FAST) len = j < rem ? len : 0;                                  // past the end: no token
        lp[j >> 2] |= (uint32_t)len << (8 * (j & 3));
        sum += (uint32_t)len;
#if DC_TOK_SB
        if ((j % DC_TOK_SB) == DC_TOK_SB - 1) __builtin_amdgcn_sched_barrier(0);
#endif
    }
    return sum;
}

// The scanner (block 0 of the single-pass launch when DC_ENC_SCAN, the default): it publishes every tile's
// INCLUSIVE state as soon as that tile and all its predecessors have published their aggregates.  Each
// round reads the 1024 states after the frontier F (4 consecutive per thread: 32 coalesced bytes), finds
// the first one not yet an aggregate, scans the counts before it (wave scans + wave totals in LDS) and
// stores their inclusive states; F moves past them.  A tile then needs ONE poll of its own state instead
// of a look-back: the chained look-back cost ~3 state round trips (~4.5 us) per tile, as each tile's
// predecessors were looking back at the same time.
// (r06) The scanner's help: a tile whose aggregate is still unpublished after HELP_POLLS scanner rounds is
// counted by the scanner workgroup itself (256 threads x 16 floats, token_len_t) and published -- its aggregate
// (CAS from the value seen) and, for the successor's first word, its tail granule.  The values are the ones the
// tile publishes, so a late tile's own stores are harmless.  With it a tile's look-back depends on no other
// workgroup being dispatched: with other processes' look-back kernels on the GPU a predecessor can stay
// undispatched on its XCD behind their waiting waves (r05f: three ranks on one GPU, encoder status 4).
template <int CT>
__device__ void scanner_help(uint64_t* __restrict__ st, uint64_t* __restrict__ tl, unsigned F, unsigned ntiles,
                             uint32_t tag, uint32_t epoch, uint64_t seen, const float* __restrict__ x, long long n,
                             long long idx0, const Params& P, const uint16_t* tab, unsigned long long* s_red) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const long long e0 = (long long)F * ENC_TILE + (long long)ENC_K * tid;
    float b[3];
#pragma unroll
    for (int k = 1; k <= 3; k++) {
        const long long e = e0 - k;
        b[k - 1] = (e < n && e >= -3 && idx0 + e >= 0) ? x[e] : 0.0f;
    }
    float b1 = b[0], b2 = b[1], b3 = b[2];
    unsigned long long bits = 0;
    for (int j = 0; j < ENC_K; j++) {
        const long long e = e0 + j;
        if (e >= n) break;
        const float v = x[e];
        bits += (unsigned)token_len_t<CT>(v, b1, b2, b3, idx0 + e >= 3, P, tab);
        b3 = b2; b2 = b1; b1 = v;
    }
    bits = wave_sum64(bits);
    if (lane == 0) s_red[wid] = bits;
    __syncthreads();
    if (tid == 0) {
        const unsigned long long T = s_red[0] + s_red[1] + s_red[2] + s_red[3];
        atomicCAS(reinterpret_cast<unsigned long long*>(st + F), (unsigned long long)seen,
                  (unsigned long long)st_word(tag, ST_AGG, T));
        if (F + 1 < ntiles && (ld_relaxed(tl + F) >> 32) != (uint64_t)epoch)
            st_relaxed(tl + F, ((uint64_t)epoch << 32) | help_tile_tail<CT>(x, idx0, P, tab, (long long)F));
    }
    __syncthreads();
}

template <int CT, bool HELP>
__device__ void enc_scanner(uint64_t* __restrict__ st, unsigned ntiles, uint32_t tag, int start_bit,
                            unsigned* __restrict__ err, uint32_t* s_gap, uint32_t* s_kb, uint32_t* s_tot,
                            uint64_t* __restrict__ tl, uint32_t epoch, const float* __restrict__ x, long long n,
                            long long idx0, const Params& P, const uint16_t* tab, unsigned long long* s_red) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    unsigned long long carry = (unsigned long long)start_bit;
    unsigned F = 0, idle = 0;
    WaitBound wb;
    wb.start();
    while (F < ntiles) {
        uint64_t v[4];
        int kb = 4;                                                       // the thread's first state not ready
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const unsigned i = F + 4u * (unsigned)tid + (unsigned)k;
            v[k] = ld_relaxed(st + (i < ntiles ? i : ntiles - 1));
            const bool ok = i < ntiles && (uint32_t)(v[k] >> 42) == tag && (v[k] & ST_MASK) == ST_AGG;
            if (!ok && kb == 4) kb = k;
        }
        const unsigned long long bm = __ballot(kb < 4);
        const int fl = bm ? __ffsll((long long)bm) - 1 : 64;              // the wave's first lane with a gap
        const int fkb = fl < 64 ? __builtin_amdgcn_readlane(kb, fl) : 4;
        if (lane == 0) { s_gap[wid] = (uint32_t)fl; s_kb[wid] = (uint32_t)fkb; }
        __syncthreads();
        unsigned p = 1024;                                                // ready states after F
#pragma unroll
        for (int w = 3; w >= 0; w--)
            if (s_gap[w] < 64u) p = 4u * (64u * (unsigned)w + s_gap[w]) + s_kb[w];
        uint32_t c[4], sum = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            c[k] = 4u * (unsigned)tid + (unsigned)k < p ? (uint32_t)(v[k] & ST_VAL) : 0u;
            sum += c[k];
        }
        const uint32_t inc = wave_scan_incl(sum);
        if (lane == 63) s_tot[wid] = inc;
        __syncthreads();
        uint32_t wpre = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < 4; w++) {
            wpre += w < wid ? s_tot[w] : 0u;
            tot += s_tot[w];
        }
        unsigned long long run = carry + wpre + inc - sum;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            run += c[k];
            const unsigned i = F + 4u * (unsigned)tid + (unsigned)k;
            if (4u * (unsigned)tid + (unsigned)k < p) st_relaxed(st + i, st_word(tag, ST_INC, run));
        }
        carry += tot;
        F += p;
        if (p) {
            wb.start();
            idle = 0;
        } else {
            if (HELP && ++idle >= HELP_POLLS) {                          // tile F is late: count it here
                __syncthreads();                                          // (s_gap / s_kb read above)
                const uint64_t seen = ld_relaxed(st + F);
                const bool pub = (uint32_t)(seen >> 42) == tag && (seen & ST_MASK) == ST_AGG;
                if (!pub) scanner_help<CT>(st, tl, F, ntiles, tag, epoch, seen, x, n, idx0, P, tab, s_red);
                idle = 0;
                continue;
            }
            if (wb.expired()) { if (tid == 0) atomicOr(err, 4u); return; }
            __builtin_amdgcn_s_sleep(2);
        }
        __syncthreads();                                                  // the LDS words are rewritten
    }
}

// (7 workgroups per CU: 72 VGPRs, 2 of them spilled, and ~120 SGPRs spilled to VGPR lanes in the CT7 build;
// the tiles idle through their look-back round trips, so one more resident tile per CU paid: fused
// 147-148 -> 145 us, 754-762 -> 769-777 GB/s; 6 per CU kept every register)
#ifndef DC_FUSED_WAVES
#define DC_FUSED_WAVES 7
#endif
#ifndef DC_STORE_U
#define DC_STORE_U 1                    // (A/B) words per thread per store round: 4 and 8 measured equal, off
#endif
#ifndef DC_STORE_Q
#define DC_STORE_Q 1                    // (r06) 16-byte quads of the stream's grid per thread
#endif
typedef unsigned u32x4q __attribute__((ext_vector_type(4)));
// (A/B, off) After the pack only wave 0 has work left that needs the tile's offset (the look-back, then the
// stores): waves 1-3 may end there, their wave slots taking the next tile's waves while wave 0 waits for its
// look-back round trip.  Measured r05: 148.7-150 us with vs 143.7-145.7 us without (one wave then stores the
// whole tile; the next tile's waves find no free LDS: 9 tiles per CU by LDS, 7 by registers)
#ifndef DC_ENC_EARLY_EXIT
#define DC_ENC_EARLY_EXIT 0
#endif
// CRC (dc_encode_crc_device, the CT9 sender): the raw CRC-32 of the words a tile stores is XOR-ed into the 16 KiB
// block accumulators cblk (dc_device.h's fused CRC; crcf_final_kernel turns them into the stream's zlib CRC):
// thread k takes the 16-word group q0 + k of the stream's word grid (q0 = the group of the tile's first word),
// the tile's stored words in it and zeros for the rest, and shifts its raw CRC to the end of its block.
// SUB (r06): x - min made while loading (dc_encode_sub_device, the halo path) -- its own instantiation, so that the
// default one holds no code for it
template <int CT, bool CRC = false, bool HELP = false, bool SUB = false>
__global__ __launch_bounds__(ENC_TPB, DC_FUSED_WAVES) void encode_fused_kernel(
    const float* __restrict__ x, long long n, long long idx0, Params P, uint32_t* __restrict__ out,
    uint64_t* __restrict__ st, uint64_t* __restrict__ tl, unsigned ntiles, int start_bit,
    unsigned long long* __restrict__ total_bits, unsigned long long* __restrict__ total_bits2, uint32_t epoch,
    unsigned* __restrict__ err, unsigned long long* __restrict__ dbg, int scan, const uint32_t* __restrict__ ctab,
    uint32_t* __restrict__ cblk, uint32_t* __restrict__ mirror) {
    static_assert(ENC_K == 16 && ENC_TPB == 256, "16 consecutive floats per thread, 4 waves per tile");
    // (DC_DEBUG_STAMPS: phase stamps of the first 16384 tiles, s_memrealtime)
#define E1STAMP(ph) do { if (dbg && threadIdx.x == 0 && tile < 16384) dbg[tile * 8 + (ph)] = __builtin_amdgcn_s_memrealtime(); } while (0)
    // sb: first the load transpose (each wave its part), then the tokens (token j of thread t at word
    // 256 j + t), then the bit buffer
    __shared__ __attribute__((aligned(16))) uint32_t sb[E3_WORDS];
    __shared__ uint32_t s_w[4], s_hw[4], s_hi[4], s_tw[4], s_ti[4];
    __shared__ unsigned long long s_G;
    __shared__ uint32_t s_tp, s_ok;
    __shared__ uint16_t tab[512];
    __shared__ __attribute__((aligned(16))) uint64_t lbw[128 * LB_DMA_N];   // the first look-back window
    __shared__ uint32_t cnib[CRC ? 128 : 1];
    __shared__ uint32_t cred[CRC ? 3 * 4 : 1];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t tag = epoch & ST_TAGM;
    if (scan && blockIdx.x == 0) {                                    // the scanner (dispatched first)
        __shared__ unsigned long long s_red[4];
        build_enc_tab<CT>(tab, P, tid, ENC_TPB);                      // (its help counts late tiles)
        __syncthreads();
        enc_scanner<CT, HELP>(st, ntiles, tag, start_bit, err, s_hw, s_hi, s_tw, tl, epoch, x, n, idx0, P, tab, s_red);
        return;
    }
    const unsigned tile = blockIdx.x - (scan ? 1u : 0u);
    E1STAMP(0);
    build_enc_tab<CT>(tab, P, tid, ENC_TPB);                          // (read after the barrier below)
    if (CRC && tid < 128) cnib[tid] = ctab[CRCF_NIB + tid];
    const long long tbase = (long long)tile * ENC_TILE;
    const long long base = tbase + (long long)ENC_K * tid;
    const bool full = tbase + ENC_TILE <= n;
    // ---- the thread's 16 consecutive floats (transposed through the wave's part of sb in two halves,
    // rows of 16 + 4 words) and their history: the previous thread's last three (DPP), for lane 0 the
    // three floats before the wave's first
    float h[ENC_K + 3];
    {
        f32x4 f[ENC_K / 4];
        load_tile_x(f, x, n, tbase, lane, wid);
        float* stg = reinterpret_cast<float*>(sb) + wid * E3_STG;
        f32x4 u[ENC_K / 4];
#pragma unroll
        for (int half = 0; half < 2; half++) {
#pragma unroll
            for (int q = 0; q < 2; q++) {
                const int m = lane + 64 * q;
                *reinterpret_cast<f32x4*>(stg + 4 * m + 4 * (m >> 2)) = f[2 * half + q];
            }
            __builtin_amdgcn_wave_barrier();
            if (half == 0) E1STAMP(7);                                    // (stamps: wave 0's first x granules here)
            if ((lane >> 5) == half)
#pragma unroll
                for (int q = 0; q < ENC_K / 4; q++) u[q] = *reinterpret_cast<const f32x4*>(stg + 20 * (lane & 31) + 4 * q);
            __builtin_amdgcn_wave_barrier();
        }
#pragma unroll
        for (int q = 0; q < ENC_K / 4; q++) {
            h[3 + 4 * q] = u[q].x; h[4 + 4 * q] = u[q].y; h[5 + 4 * q] = u[q].z; h[6 + 4 * q] = u[q].w;
        }
        const long long w0 = tbase + 64ll * ENC_K * wid;                  // the wave's first element
        float hw[3];
#pragma unroll
        for (int k = 1; k <= 3; k++) {
            const long long e = w0 - k;
            hw[k - 1] = (e < n && e >= -3 && idx0 + e >= 0) ? x[e] : 0.0f;
        }
        if (SUB) {                                                         // (dc_encode_sub_device: x - min)
            const float m = P.subp ? *P.subp : P.submin;
            if (__builtin_expect(isfinite(m), 1)) {
#pragma unroll
                for (int j = 0; j < ENC_K; j++) h[3 + j] = sub_fin(h[3 + j], m);
#pragma unroll
                for (int k = 1; k <= 3; k++)
                    if (w0 - k < n && w0 - k >= -3 && idx0 + w0 - k >= 0) hw[k - 1] = sub_fin(hw[k - 1], m);
            } else {                                                       // (a NaN / infinite minimum)
#pragma unroll
                for (int j = 0; j < ENC_K; j++) h[3 + j] = sub_x86(h[3 + j], m);
#pragma unroll
                for (int k = 1; k <= 3; k++)
                    if (w0 - k < n && w0 - k >= -3 && idx0 + w0 - k >= 0) hw[k - 1] = sub_x86(hw[k - 1], m);
            }
        }
        h[2] = wave_shr1(h[3 + ENC_K - 1], hw[0]);
        h[1] = wave_shr1(h[3 + ENC_K - 2], hw[1]);
        h[0] = wave_shr1(h[3 + ENC_K - 3], hw[2]);
    }
    __syncthreads();                                                      // every wave's transpose is done
    // ---- the tokens, once: values to sb, lengths packed in lp
    uint32_t lp[ENC_K / 4], mysum;
    {
        bool neg1 = false;
        if (full && idx0 + tbase >= 3) {
            mysum = make_tokens16<CT, true>(h, P, tab, 0, ENC_K, sb + tid, lp, neg1);
        } else {
            const int rem = (int)min(max(n - base, 0ll), (long long)ENC_K);
            const int g3 = (int)min(max(3 - (idx0 + base), 0ll), (long long)ENC_K);
#pragma unroll
            for (int j = 0; j < ENC_K; j++) h[3 + j] = j < rem ? h[3 + j] : 0.0f;
            mysum = make_tokens16<CT, false>(h, P, tab, g3, rem, sb + tid, lp, neg1);
        }
        if (CT != 6 && __any(neg1) && lane == 0) atomicOr(err, 1u);    // -1.0f: the reference's sentinel
    }
    // ---- the tile's total and the thread's first bit
    E1STAMP(1);
    const uint32_t inc = wave_scan_incl(mysum);
    if (lane == 63) s_w[wid] = inc;
    __syncthreads();
    E1STAMP(2);
    uint32_t tv[ENC_K];
#pragma unroll
    for (int j = 0; j < ENC_K; j++) tv[j] = sb[ENC_TPB * j + tid];
    uint32_t wpre = 0, T = 0;
#pragma unroll
    for (int w = 0; w < ENC_TPB / 64; w++) {
        if (w < wid) wpre += s_w[w];
        T += s_w[w];
    }
    // publish the aggregate (tile 0: its inclusive state) and the tile's last 31 bits (the successor's
    // first word starts with them): the last thread's tokens (>= 48 bits)
    if (tid == 0)
        st_relaxed(st + tile, tile == 0 && !scan ? st_word(tag, ST_INC, (unsigned long long)start_bit + T) : st_word(tag, ST_AGG, T));
    if (tid == ENC_TPB - 1 && tile + 1 < ntiles) {
        uint64_t acc = 0;
#pragma unroll
        for (int j = 0; j < ENC_K; j++) acc = (acc << ((lp[j >> 2] >> (8 * (j & 3))) & 0xFFu)) | tv[j];
        st_relaxed(tl + tile, ((uint64_t)epoch << 32) | ((uint32_t)acc & 0x7FFFFFFFu));
    }
    const uint32_t off = wpre + inc - mysum;                              // the thread's first tile bit
    long long lb_s0 = 0;
    if (DC_LB_DMA && scan && !DC_SCAN_POLL && wid == 0 && tile > 0) lb_s0 = lb_dma(st, (long long)tile - 1, lbw);
    // (r06, DC_LB_EARLY = K > 0) wave 0 requests the first look-back window (K x 64 states) into registers here,
    // before the pack: the barriers wait only for LDS (lgkmcnt), so the state round trip overlaps the pack
    uint64_t lbv[DC_LB_EARLY > 0 ? DC_LB_EARLY : 1];
    if (DC_LB_EARLY && !HELP && !DC_LB_DMA && scan && !DC_SCAN_POLL && wid == 0 && tile > 0) {
        const uint64_t* p = st + ((long long)tile - 1 - lane);
#pragma unroll
        for (int k = 0; k < (DC_LB_EARLY > 0 ? DC_LB_EARLY : 1); k++) lbv[k] = ld_relaxed(p - 64 * k);
    }
    __syncthreads();                                                      // every thread has its tokens back
    // ---- pack, MSB-first.  Full tiles: every thread holds >= 48 bits, so a word is shared by at most
    // two neighbouring threads: each writes the words it completes, its first merged with the previous
    // lane's unfinished last one (DPP); a wave's first and last words are merged after the barrier
    // (r06, DC_ENC_V2) Branch-free instead: the buffer is cleared and every token ORed into the (at most) two
    // words it touches.  A token of l bits at tile bit o ends at e = (o & 31) + l < 64; with sh = (o + l) & 31
    // (v_alignbit's own 5-bit shift), alignbit(0, v, sh) is its part of word o >> 5 when e >= 32 (and
    // alignbit(v, 0, sh) its part of the next word), alignbit(v, 0, sh) its part of word o >> 5 when e < 32.
    // ~8 VALU per token against ~17 for the register word assembly with its per-lane branches.
    if ((DC_ENC_V2 & 2) && full) {
        uint4* sb4 = reinterpret_cast<uint4*>(sb);
#pragma unroll
        for (int i = 0; i < ENC_TILE / 4 / ENC_TPB; i++) sb4[tid + ENC_TPB * i] = make_uint4(0u, 0u, 0u, 0u);
        if (tid < (E3_WORDS - ENC_TILE) / 4) sb4[ENC_TILE / 4 + tid] = make_uint4(0u, 0u, 0u, 0u);
        __syncthreads();
        uint32_t o = off, a = (off >> 3) & ~3u;                           // the token's bit; its word's byte
        char* sbc = reinterpret_cast<char*>(sb);
#pragma unroll
        for (int j = 0; j < ENC_K; j++) {
            const uint32_t l = (lp[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            const uint32_t on = o + l, an = (on >> 3) & ~3u;
            const uint32_t A = __builtin_amdgcn_alignbit(0u, tv[j], on), B = __builtin_amdgcn_alignbit(tv[j], 0u, on);
            const bool big = an != a;
            __hip_atomic_fetch_or(reinterpret_cast<uint32_t*>(sbc + a), big ? A : B, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_or(reinterpret_cast<uint32_t*>(sbc + a + 4), big ? B : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            o = on;
            a = an;
        }
        if (lane == 0) s_hi[wid] = 0xFFFFFFFFu;
        if (lane == 63) s_ti[wid] = 0xFFFFFFFFu;
    } else if (full) {
        uint32_t wi = off >> 5, nb = off & 31u, headw = 0u;
        const uint32_t hi = wi;
        uint64_t acc = 0;
        bool have = false;
#pragma unroll
        for (int j = 0; j < ENC_K; j++) {
            const uint32_t len = (lp[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            acc |= (uint64_t)tv[j] << ((64u - nb - len) & 63u);
            nb += len;
            if (nb >= 32u) {
                const uint32_t w = (uint32_t)(acc >> 32);
                if (have) sb[wi] = w;
                else headw = w;
                have = true;
                wi++;
                acc <<= 32;
                nb -= 32u;
            }
        }
        const uint32_t tailw = (uint32_t)(acc >> 32);                     // nb bits (0: none)
        const uint32_t pt = wave_shr1_u(tailw, 0u);
        if (lane == 0) { s_hw[wid] = headw; s_hi[wid] = hi; }
        else sb[hi] = headw | pt;
        if (lane == 63) { s_tw[wid] = tailw; s_ti[wid] = nb ? wi : 0xFFFFFFFFu; }
    } else {
        // the last tile (some threads hold few or no bits): ORed in token by token over a cleared buffer
        for (int i = tid; i < E3_WORDS / 4; i += ENC_TPB) reinterpret_cast<uint4*>(sb)[i] = make_uint4(0u, 0u, 0u, 0u);
        __syncthreads();
        uint32_t o = off;
#pragma unroll
        for (int j = 0; j < ENC_K; j++) {
            const uint32_t lj = (lp[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            if (lj) {
                const uint64_t v = (uint64_t)tv[j] << ((64u - (o & 31u) - lj) & 63u);
                atomicOr(&sb[o >> 5], (uint32_t)(v >> 32));
                if ((o & 31u) + lj > 32u) atomicOr(&sb[(o >> 5) + 1], (uint32_t)v);
            }
            o += lj;
        }
        if (lane == 0) s_hi[wid] = 0xFFFFFFFFu;
        if (lane == 63) s_ti[wid] = 0xFFFFFFFFu;
    }
    __syncthreads();
    if (DC_ENC_EARLY_EXIT && wid != 0) return;                            // (no barrier after this one)
    // ---- wave 0: the waves' boundary words, then the look-back for the tile's offset
    if (wid == 0) {
        // the predecessor's last bits are requested before the look-back (published with its aggregate,
        // they are there by now: one round trip less after the look-back)
        const uint64_t tl0 = (lane == 0 && tile > 0) ? ld_relaxed(tl + tile - 1) : 0ull;
        if (lane < 4) {
            const uint32_t hi = s_hi[lane];
            if (hi != 0xFFFFFFFFu) {
                uint32_t w = s_hw[lane];
                if (lane > 0 && s_ti[lane - 1] == hi) w |= s_tw[lane - 1];
                sb[hi] = w;
            }
            if (lane == 3 && s_ti[3] != 0xFFFFFFFFu) sb[s_ti[3]] = s_tw[3];   // the tile's last word
        }
        unsigned long long G = (unsigned long long)start_bit;
        uint32_t lbst = 0;
        E1STAMP(3);
        int bad = 0;
        if (scan && DC_SCAN_POLL) {                                      // (A/B: wait for the scanner itself)
            if (lane == 0) {
                WaitBound wb;
                wb.start();
                uint64_t v;
                for (;;) {
                    v = ld_relaxed(st + tile);
                    if ((uint32_t)(v >> 42) == tag && (v & ST_MASK) == ST_INC) break;
                    if (wb.expired()) { bad = 1; break; }
                    lbst += 1u << 16;
                    __builtin_amdgcn_s_sleep(DC_LB_SLEEP);
                }
                G = (v & ST_VAL) - T;
            }
        } else if (scan) {
            // the scanner keeps the inclusive states close behind the published aggregates, ~2-3 us
            // behind this tile's own neighbours (which started with it): a look-back over DC_LB_KS x 64
            // predecessors in one round trip mostly meets one (waiting for the scanner to reach this tile
            // itself cost ~4 us per tile)
#ifdef DC_ENC_DIAG_NOLB
            if (false) {
#else
            if (tile > 0) {
#endif
                if (DC_LB_DMA) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // the window's LDS writes landed
                    bad = enc_lookback<DC_LB_KS>(st, tile, tag, G, lbst, start_bit, lbw, lb_s0);
                } else if (DC_LB_EARLY && !HELP) {
                    bad = enc_lookback<(DC_LB_EARLY > 0 ? DC_LB_EARLY : 1)>(st, tile, tag, G, lbst, start_bit, nullptr, 0, lbv);
                } else {
                    if constexpr (HELP)
                        bad = enc_lookback<DC_LB_KS>(st, tile, tag, G, lbst, start_bit, nullptr, 0, nullptr,
                                                     [&](long long ti) { return help_tile_bits<CT>(x, n, idx0, P, tab, ti); });
                    else
                        bad = enc_lookback<DC_LB_KS>(st, tile, tag, G, lbst, start_bit);
                }
            }
        } else if (tile > 0) {
            bad = enc_lookback<LB_KW>(st, tile, tag, G, lbst, start_bit);
        }
        E1STAMP(4);
#ifdef DC_ENC_DIAG_NOLB
        // (diagnostic build: no look-back -- an in-bounds but wrong offset, 20 bits per float -- to time the rest)
        G = (unsigned long long)start_bit + 20ull * (unsigned long long)tbase;
        bad = 0;
#endif
        if (lane == 0) {
            uint32_t tp = 0;
            if (tile > 0 && !bad) {                                       // the predecessor's last bits
                WaitBound wb;
                wb.start();
                uint64_t v = tl0;
                for (unsigned k = 0; (v >> 32) != (uint64_t)epoch; k++) {
                    v = ld_relaxed(tl + tile - 1);
                    if ((v >> 32) == (uint64_t)epoch) break;
                    if (HELP && k == HELP_POLLS) {                        // the predecessor is late: its tail here
                        v = ((uint64_t)epoch << 32) | help_tile_tail<CT>(x, idx0, P, tab, (long long)tile - 1);
                        st_relaxed(tl + tile - 1, v);
                        break;
                    }
                    if (wb.expired()) { bad = 1; break; }
                    __builtin_amdgcn_s_sleep(1);
                }
                tp = (uint32_t)v;
            }
            // (a guard, never taken by a correct encode: a tile's bits end within the stream's capacity,
            // 32 bits per float after the start bit -- a stale offset must not send the stores outside it)
            if (!bad && G + T > (unsigned long long)start_bit + 32ull * (unsigned long long)min(n, tbase + ENC_TILE)) bad = 2;
            if (tile > 0 && !scan) st_relaxed(st + tile, bad ? st_word(tag, ST_BAD, 0) : st_word(tag, ST_INC, G + T));
            if (bad) atomicOr(err, bad == 2 ? 2u : 4u);
            else if (tile == ntiles - 1) {
                *total_bits = G + T;
                if (total_bits2) *total_bits2 = G + T;
            }
            s_G = G;
            s_tp = tp;
            s_ok = bad ? 0u : 1u;
            if (dbg && tile < 16384) {
                dbg[tile * 8 + 6] = lbst;
                // (slot 7: wave 0's x arrival, E1STAMP(7) above)
            }
        }
    }
    if (DC_ENC_EARLY_EXIT) __builtin_amdgcn_wave_barrier();               // (lane 0's LDS words, same wave)
    else __syncthreads();
    if (!s_ok) return;                                                    // no offset: nothing stored
    // ---- store the words from the one holding the tile's first bit to its last full one
    const unsigned long long Gt = s_G;
    const uint32_t tp0 = s_tp;
    const uint32_t sh = (uint32_t)(Gt & 31ull);
    const long long W0 = (long long)(Gt >> 5);
    const int nw = (int)((long long)((Gt + T) >> 5) - W0) + ((tile == ntiles - 1 && ((Gt + T) & 31ull)) ? 1 : 0);
    const int tw = (int)((T + 31u) >> 5);                                  // buffer words holding tile bits
    constexpr int SW = DC_ENC_EARLY_EXIT ? 64 : ENC_TPB;                    // the storing threads
#if DC_STORE_Q
    // (r06) the stream's 16-byte grid: thread k takes quad Q0 + k (Q0 = W0 / 4): its 4 words from 5 buffer words
    // (v_alignbit by sh, 0 keeps the word), one 16-byte store when the quad lies inside the tile's word range,
    // word stores at the two ends.  The word loop spent ~10 VALU per word (two LDS reads, a select, 64-bit
    // addresses, loop control): the encoder is VALU-bound (SQ: VALU instructions x 4 cycles ~ the kernel time)
    if (!CRC && !mirror) {
        const long long Q0 = W0 >> 2;
        const int nq = (int)(((W0 + nw + 3) >> 2) - Q0);
        const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(out + 4 * Q0, (short)0, nq * 16, 0x00020000);
        for (int k = tid; k < nq; k += ENC_TPB) {
            const int i0 = (int)(4 * (Q0 + k) - W0);                      // the quad's first word in the tile (>= -3)
            uint32_t b[5];
#pragma unroll
            for (int m = 0; m < 5; m++) {
                const int i = i0 - 1 + m;
                b[m] = (i >= 0 && i < tw) ? sb[i] : (i == -1 ? tp0 : 0u);
            }
            u32x4q q;
            q.x = __builtin_bswap32(__builtin_amdgcn_alignbit(b[0], b[1], sh));
            q.y = __builtin_bswap32(__builtin_amdgcn_alignbit(b[1], b[2], sh));
            q.z = __builtin_bswap32(__builtin_amdgcn_alignbit(b[2], b[3], sh));
            q.w = __builtin_bswap32(__builtin_amdgcn_alignbit(b[3], b[4], sh));
            if (i0 >= 0 && i0 + 4 <= nw) {
                __builtin_amdgcn_raw_buffer_store_b128(q, ro, 16 * k, 0, DC_PACK_NT ? 2 : 0);
            } else {
                const uint32_t qv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                for (int m = 0; m < 4; m++)
                    if (i0 + m >= 0 && i0 + m < nw) __builtin_amdgcn_raw_buffer_store_b32(qv[m], ro, 16 * k + 4 * m, 0, DC_PACK_NT ? 2 : 0);
            }
        }
    } else
#endif
    {
#if DC_STORE_U > 1
    // DC_STORE_U words per thread per round: their LDS reads are in flight together (one word per round
    // waited on one LDS round trip each)
    for (int i0 = tid; i0 < nw; i0 += DC_STORE_U * ENC_TPB) {
        uint32_t wv[DC_STORE_U];
#pragma unroll
        for (int u = 0; u < DC_STORE_U; u++) {
            const int i = i0 + u * ENC_TPB;
            const int ic = min(i, E3_WORDS - 1);
            const uint32_t cur = i < tw ? sb[ic] : 0u;                     // (stale past the tile's bits)
            const uint32_t prev = i ? sb[ic - 1] : tp0;
            wv[u] = sh ? __builtin_amdgcn_alignbit(prev, cur, sh) : cur;
        }
#pragma unroll
        for (int u = 0; u < DC_STORE_U; u++) {
            const int i = i0 + u * ENC_TPB;
            if (i < nw) __builtin_nontemporal_store(__builtin_bswap32(wv[u]), out + W0 + i);
            if (mirror && i < nw) __builtin_nontemporal_store(__builtin_bswap32(wv[u]), mirror + W0 + i);
        }
    }
#else
    for (int i = DC_ENC_EARLY_EXIT ? lane : tid; i < nw; i += SW) {
        const uint32_t cur = i < tw ? sb[i] : 0u;                          // (stale past the tile's bits)
        const uint32_t prev = i ? sb[i - 1] : tp0;
        const uint32_t w = sh ? __builtin_amdgcn_alignbit(prev, cur, sh) : cur;
#if defined(DC_ENC_DIAG_NOSTORE)
        if (w == 0x9E3779B9u && i == 12345) out[W0 + i] = 0u;         // (diagnostic build: the words are made, not stored)
#elif DC_PACK_NT
        __builtin_nontemporal_store(__builtin_bswap32(w), out + W0 + i);
#else
        out[W0 + i] = __builtin_bswap32(w);
#endif
        // (the CT9 send: the same words into the receiver's buffer, dc_encode_send_device)
        if (mirror) __builtin_nontemporal_store(__builtin_bswap32(w), mirror + W0 + i);
    }
#endif
    }
    if constexpr (CRC) {
        // the stored words by 16-word groups of the stream's word grid (a tile spans at most 258 groups and
        // three 16 KiB blocks: its raw CRC pieces are XOR-ed per block)
        const long long q0 = W0 >> 4;
        const int ng = (int)(((W0 + nw + 15) >> 4) - q0);
        const long long b0 = q0 >> 8;
        uint32_t vb[3] = {0u, 0u, 0u};
        for (int k = DC_ENC_EARLY_EXIT ? lane : tid; k < ng; k += SW) {
            const long long q = q0 + k;
            uint32_t r = 0;
#pragma unroll 4
            for (int u = 0; u < 16; u++) {
                const int i = (int)(16 * q + u - W0);                      // the tile's word index
                uint32_t wv = 0u;
                if (i >= 0 && i < nw) {
                    const uint32_t cur = i < tw ? sb[i] : 0u;
                    const uint32_t prev = i ? sb[i - 1] : tp0;
                    wv = __builtin_bswap32(sh ? __builtin_amdgcn_alignbit(prev, cur, sh) : cur);
                }
                r = crcf_word(r, wv, cnib);
            }
            const uint32_t v = r ? crcf_mult(ctab[CRCF_KQ + 2 * (255 - (int)(q & 255))], r) : 0u;
            const int bi = (int)((q >> 8) - b0);
            vb[0] ^= bi == 0 ? v : 0u;
            vb[1] ^= bi == 1 ? v : 0u;
            vb[2] ^= bi == 2 ? v : 0u;
        }
#pragma unroll
        for (int j = 0; j < 3; j++) {
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) vb[j] ^= __shfl_xor(vb[j], d, 64);
        }
        if (DC_ENC_EARLY_EXIT) {
            if (lane < 3) {
                const uint32_t v = lane == 0 ? vb[0] : (lane == 1 ? vb[1] : vb[2]);
                if (v) atomicXor(cblk + b0 + lane, v);
            }
        } else {
            if (lane == 0) { cred[wid] = vb[0]; cred[4 + wid] = vb[1]; cred[8 + wid] = vb[2]; }
            __syncthreads();
            if (tid < 3) {
                const uint32_t v = cred[4 * tid] ^ cred[4 * tid + 1] ^ cred[4 * tid + 2] ^ cred[4 * tid + 3];
                if (v) atomicXor(cblk + b0 + tid, v);
            }
        }
    }
    E1STAMP(5);
#undef E1STAMP
}

// ---- the persistent, software-pipelined single pass (mode 1 with DC_ENC_PIPE) ----
// encode_fused_kernel's tile (tools/fused_stamps.py, 2^26 U10 CT7, r04): x loads + tokens 5.4 us, pack 2.3,
// look-back 3.7, store 2.1 -- seven resident tiles per CU, each idling through two ~3 us memory round trips
// (x, then the look-back) with its registers and LDS held.  Here a workgroup keeps two tiles in flight in
// two LDS buffers and loops: while tile i makes its tokens and packs them, the look-back window of tile i-1
// and the x granules of tile i+1 are in flight; then tile i-1 is stored.  Six barriers per tile:
//   top       buffer b is free (its last tile was stored); x of tile i is in registers
//   transpose (wave-local) ; wave 0 requests tile i-1's look-back window and predecessor tail, lane 0 the
//             ticket of tile i+2
//   A         tokens of tile i into buffer b
//   B         x of tile i+1 requested; tokens back into registers; tile i's aggregate and tail published
//   C         pack tile i into buffer b
//   D         wave 0: tile i's wave boundary words; tile i-1's look-back evaluated (its window has been in
//             flight through the tokens and the pack)
//   E         tile i-1 stored from buffer b ^ 1
// Tiles come from a ticket counter: a drawn tile's predecessors are held by running workgroups, each of
// which publishes a tile's aggregate before it waits on anything, so any grid size and any residency make
// progress.  Every workgroup draws until its first failing ticket; the launch's last draw (ticket
// ntiles + tile workgroups - 1) resets the counter to 0 for the next encode.
#ifndef DC_ENC_PIPE
#define DC_ENC_PIPE 0                   // (DC_ENC_PIPE=1 in the environment selects it at run time)
#endif
#ifndef DC_PIPE_WAVES
#define DC_PIPE_WAVES 4                 // workgroups per CU (two 16.6 KB buffers each)
#endif
#ifndef DC_PIPE_STATIC
#define DC_PIPE_STATIC 0                // (A/B) tiles by workgroup index, every workgroup resident, no ticket
#endif
#ifndef DC_PIPE_XTOP
#define DC_PIPE_XTOP 1                  // the next tile's x requested right after the transpose (0: after the tokens)
#endif
constexpr int EP_BUF = E3_WORDS;

// x granules of tile t (load_tile_x's layout) and the three floats before each wave's first (the halo),
// every load unconditional (buffer resources: a granule or float outside the array reads 0), so a wave's
// count of memory instructions after them is fixed and the wait for them is exact.  has = false (no next
// tile): every load is out of range.
__device__ __forceinline__ void pipe_load_x(f32x4 (&f)[ENC_K / 4], float (&hw)[3], const float* __restrict__ x,
                                            long long n, long long idx0, long long tbase, bool has, int lane, int wid) {
    const long long m = has ? min(n - tbase, (long long)ENC_TILE) : 0ll;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x + (has ? tbase : 0)), (short)0, (int)((m + 3) / 4 * 16), 0x00020000);
#pragma unroll
    for (int q = 0; q < ENC_K / 4; q++)
        f[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, 4 * (1024 * wid + 4 * (lane + 64 * q)), 0, DC_PACK_NT ? 2 : 0);
    // the halo: floats tbase + 1024 wid - k (k = 1..3) exist when inside [-min(3, idx0 + tbase), m) of the tile
    const int hc = has ? (int)min(3ll, idx0 + tbase) : 0;
    const __amdgpu_buffer_rsrc_t rh =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x + (has ? tbase : 0) - hc), (short)0, (int)(4 * (m + hc)), 0x00020000);
#pragma unroll
    for (int k = 1; k <= 3; k++)
        hw[k - 1] = __builtin_amdgcn_raw_buffer_load_b32(rh, 4 * (1024 * wid - k + hc), 0, 0);
}

// wave 0: the exclusive bit offset of tile t (look-back; vr: its first window, requested earlier, or null),
// its predecessor's tail (tl0: requested earlier, or 0) -> s_G, s_tp, s_ok; the encode's total at the last tile
__device__ __forceinline__ void pipe_offset(const uint64_t* __restrict__ st, const uint64_t* __restrict__ tl, long long t,
                                            uint32_t Tt, uint32_t tag, uint32_t epoch, int start_bit, long long n,
                                            unsigned ntiles, const uint64_t* vr, uint64_t tl0, unsigned* __restrict__ err,
                                            unsigned long long* __restrict__ total_bits,
                                            unsigned long long* __restrict__ total_bits2, unsigned long long& s_G,
                                            uint32_t& s_tp, uint32_t& s_ok) {
    const int lane = threadIdx.x & 63;
    unsigned long long G = (unsigned long long)start_bit;
    uint32_t lbst = 0;
    int bad = 0;
    if (t > 0) bad = enc_lookback<DC_LB_KS>(st, t, tag, G, lbst, start_bit, nullptr, 0, vr);
    if (lane == 0) {
        uint32_t tp = 0;
        if (t > 0 && !bad) {
            WaitBound wb;
            wb.start();
            uint64_t v = tl0;
            while ((v >> 32) != (uint64_t)epoch) {
                v = ld_relaxed(tl + t - 1);
                if ((v >> 32) == (uint64_t)epoch) break;
                if (wb.expired()) { bad = 1; break; }
                __builtin_amdgcn_s_sleep(1);
            }
            tp = (uint32_t)v;
        }
        // (the guard of encode_fused_kernel: a tile's bits end within the stream's capacity)
        if (!bad && G + Tt > (unsigned long long)start_bit + 32ull * (unsigned long long)min(n, (t + 1) * ENC_TILE)) bad = 2;
        if (bad) atomicOr(err, bad == 2 ? 2u : 4u);
        else if (t == (long long)ntiles - 1) {
            *total_bits = G + Tt;
            if (total_bits2) *total_bits2 = G + Tt;
        }
        s_G = G;
        s_tp = tp;
        s_ok = bad ? 0u : 1u;
    }
}

// waves 1-3: tile t's words (bit buffer sp, Tt bits) from the one holding its first bit, PIPE_NS buffer
// stores per thread whatever the tile's length (words past it are out of the resource's range and dropped):
// a fixed count of memory instructions, so the next tile's x loads (issued before) are waited for exactly
constexpr int PIPE_NS = (E3_WORDS + 1 + 191) / 192;
__device__ __forceinline__ void pipe_store(uint32_t* __restrict__ out, const uint32_t* sp, uint32_t Tt, long long t,
                                           unsigned ntiles, unsigned long long Gt, uint32_t tp0, bool ok) {
    const uint32_t sh = (uint32_t)(Gt & 31ull);
    const long long W0 = (long long)(Gt >> 5);
    const int nw = ok ? (int)((long long)((Gt + Tt) >> 5) - W0) + ((t == (long long)ntiles - 1 && ((Gt + Tt) & 31ull)) ? 1 : 0) : 0;
    const int tw = (int)((Tt + 31u) >> 5);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(out + (ok ? W0 : 0), (short)0, 4 * nw, 0x00020000);
    const int t0 = max((int)threadIdx.x - 64, 0);
#pragma unroll
    for (int j = 0; j < PIPE_NS; j++) {
        const int i = t0 + 192 * j;
        const int ic = min(i, EP_BUF - 1);
        const uint32_t c = i < tw ? sp[ic] : 0u;                           // (stale past the tile's bits)
        const uint32_t pv = i ? sp[max(ic - 1, 0)] : tp0;
        const uint32_t w = sh ? __builtin_amdgcn_alignbit(pv, c, sh) : c;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bswap32(w), ro, 4 * i, 0, DC_PACK_NT ? 2 : 0);
        if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);          // (four at a time: bounded live ranges)
    }
}

template <int CT>
__global__ __launch_bounds__(ENC_TPB, DC_PIPE_WAVES) void encode_pipe_kernel(
    const float* __restrict__ x, long long n, long long idx0, Params P, uint32_t* __restrict__ out,
    uint64_t* __restrict__ st, uint64_t* __restrict__ tl, unsigned ntiles, int start_bit,
    unsigned long long* __restrict__ total_bits, unsigned long long* __restrict__ total_bits2, uint32_t epoch,
    unsigned* __restrict__ err, unsigned* __restrict__ ticket, unsigned ndraw, unsigned long long* __restrict__ dbg) {
    static_assert(ENC_K == 16 && ENC_TPB == 256, "16 consecutive floats per thread, 4 waves per tile");
    // (DC_DEBUG_STAMPS: per tile, s_memrealtime at the top, after barriers A..E and after the stores of the
    // following iteration, by thread 0)
#define EPSTAMP(t, ph) do { if (dbg && tid == 0 && (t) >= 0 && (t) < 16384) dbg[(t) * 8 + (ph)] = __builtin_amdgcn_s_memrealtime(); } while (0)
    __shared__ __attribute__((aligned(16))) uint32_t sbuf[2][EP_BUF];
    __shared__ uint32_t s_w[4], s_hw[4], s_hi[4], s_tw[4], s_ti[4];
    __shared__ uint32_t s_T[2];
    __shared__ unsigned s_nx, s_k0;
    __shared__ unsigned long long s_G;
    __shared__ uint32_t s_tp, s_ok;
    __shared__ uint16_t tab[512];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t tag = epoch & ST_TAGM;
    if (blockIdx.x == 0) {                                            // the scanner (dispatched first)
        __shared__ unsigned long long s_red[4];
        build_enc_tab<CT>(tab, P, tid, ENC_TPB);
        __syncthreads();
        enc_scanner<CT, false>(st, ntiles, tag, start_bit, err, s_hw, s_hi, s_tw, tl, epoch, x, n, idx0, P, tab, s_red);
        return;
    }
    build_enc_tab<CT>(tab, P, tid, ENC_TPB);
    if (DC_PIPE_STATIC) {                                             // (A/B: tile = workgroup + k * grid)
        if (tid == 0) { s_k0 = blockIdx.x - 1; s_nx = blockIdx.x - 1 + (gridDim.x - 1); }
    } else if (tid == 0) {
        unsigned k0 = atomicAdd(ticket, 1u), k1 = ntiles;
        if (k0 == ndraw - 1) atomicExch(ticket, 0u);
        if (k0 < ntiles) {
            k1 = atomicAdd(ticket, 1u);
            if (k1 == ndraw - 1) atomicExch(ticket, 0u);
        }
        s_k0 = k0;
        s_nx = k1;
    }
    __syncthreads();
    long long cur = (long long)s_k0;
    if (cur >= (long long)ntiles) return;
    f32x4 f[ENC_K / 4];
    float hw[3];
    pipe_load_x(f, hw, x, n, idx0, cur * ENC_TILE, true, lane, wid);
    pipe_store(out, sbuf[0], 0u, 0, ntiles, 0ull, 0u, false);         // (no stores: the loop's count)
    long long prev = -1;
    int b = 0;
    for (;;) {
        __syncthreads();                                              // top: buffer b free, s_nx current
        EPSTAMP(cur, 0);
        if (dbg && tid == 0 && cur < 16384) dbg[cur * 8 + 7] = blockIdx.x;
        const long long nxt = (long long)s_nx;
        const bool hasn = nxt < (long long)ntiles;
        uint32_t* sb = sbuf[b];
        const long long tbase = cur * ENC_TILE;
        const long long base = tbase + (long long)ENC_K * tid;
        const bool full = tbase + ENC_TILE <= n;
        // ---- transpose tile cur (wave-local staging in buffer b) and its history
        float h[ENC_K + 3];
        {
            float* stg = reinterpret_cast<float*>(sb) + wid * E3_STG;
            f32x4 u[ENC_K / 4];
#pragma unroll
            for (int half = 0; half < 2; half++) {
#pragma unroll
                for (int q = 0; q < 2; q++) {
                    const int m = lane + 64 * q;
                    *reinterpret_cast<f32x4*>(stg + 4 * m + 4 * (m >> 2)) = f[2 * half + q];
                }
                __builtin_amdgcn_wave_barrier();
                if ((lane >> 5) == half)
#pragma unroll
                    for (int q = 0; q < ENC_K / 4; q++) u[q] = *reinterpret_cast<const f32x4*>(stg + 20 * (lane & 31) + 4 * q);
                __builtin_amdgcn_wave_barrier();
            }
#pragma unroll
            for (int q = 0; q < ENC_K / 4; q++) {
                h[3 + 4 * q] = u[q].x; h[4 + 4 * q] = u[q].y; h[5 + 4 * q] = u[q].z; h[6 + 4 * q] = u[q].w;
            }
            h[2] = wave_shr1(h[3 + ENC_K - 1], hw[0]);
            h[1] = wave_shr1(h[3 + ENC_K - 2], hw[1]);
            h[0] = wave_shr1(h[3 + ENC_K - 3], hw[2]);
        }
        // ---- the next tile's x (in flight through this whole tile), then wave 0: the ticket after it, tile
        // prev's look-back window and its predecessor's tail (positions before tile 0 read the pad in front)
        if (DC_PIPE_XTOP) pipe_load_x(f, hw, x, n, idx0, hasn ? nxt * ENC_TILE : 0ll, hasn, lane, wid);
        uint64_t lbv[DC_LB_KS];
        uint64_t tl0 = 0ull;
        unsigned nk = (unsigned)ntiles;
        if (wid == 0) {
            const uint64_t* p = st + (prev - 1 - lane);
#pragma unroll
            for (int k = 0; k < DC_LB_KS; k++) lbv[k] = ld_relaxed(p - 64 * k);
            tl0 = ld_relaxed(tl + prev - 1);
            if (DC_PIPE_STATIC) nk = (unsigned)min((long long)ntiles, nxt + (long long)(gridDim.x - 1));
            else if (lane == 0 && hasn) nk = atomicAdd(ticket, 1u);
        }
        __syncthreads();                                              // A: every wave's transpose is done
        EPSTAMP(cur, 1);
        // ---- the tokens of tile cur: values to buffer b, lengths packed in lp
        uint32_t lp[ENC_K / 4], mysum;
        {
            bool neg1 = false;
            if (full && idx0 + tbase >= 3) {
                mysum = make_tokens16<CT, true>(h, P, tab, 0, ENC_K, sb + tid, lp, neg1);
            } else {
                const int rem = (int)min(max(n - base, 0ll), (long long)ENC_K);
                const int g3 = (int)min(max(3 - (idx0 + base), 0ll), (long long)ENC_K);
#pragma unroll
                for (int j = 0; j < ENC_K; j++) h[3 + j] = j < rem ? h[3 + j] : 0.0f;
                mysum = make_tokens16<CT, false>(h, P, tab, g3, rem, sb + tid, lp, neg1);
            }
            if (CT != 6 && __any(neg1) && lane == 0) atomicOr(err, 1u);
        }
        const uint32_t inc = wave_scan_incl(mysum);
        if (lane == 63) s_w[wid] = inc;
        __syncthreads();                                              // B
        EPSTAMP(cur, 2);
        if (!DC_PIPE_XTOP) pipe_load_x(f, hw, x, n, idx0, hasn ? nxt * ENC_TILE : 0ll, hasn, lane, wid);
        uint32_t tv[ENC_K];
#pragma unroll
        for (int j = 0; j < ENC_K; j++) tv[j] = sb[ENC_TPB * j + tid];
        uint32_t wpre = 0, T = 0;
#pragma unroll
        for (int w = 0; w < ENC_TPB / 64; w++) {
            if (w < wid) wpre += s_w[w];
            T += s_w[w];
        }
        if (tid == 0) {
            st_relaxed(st + cur, st_word(tag, ST_AGG, T));
            s_T[b] = T;
        }
        if (tid == ENC_TPB - 1 && cur + 1 < (long long)ntiles) {
            uint64_t acc = 0;
#pragma unroll
            for (int j = 0; j < ENC_K; j++) acc = (acc << ((lp[j >> 2] >> (8 * (j & 3))) & 0xFFu)) | tv[j];
            st_relaxed(tl + cur, ((uint64_t)epoch << 32) | ((uint32_t)acc & 0x7FFFFFFFu));
        }
        const uint32_t off = wpre + inc - mysum;
        __syncthreads();                                              // C: every thread has its tokens back
        EPSTAMP(cur, 3);
        // ---- pack tile cur into buffer b (as encode_fused_kernel)
        if (full) {
            uint32_t wi = off >> 5, nb = off & 31u, headw = 0u;
            const uint32_t hi = wi;
            uint64_t acc = 0;
            bool have = false;
#pragma unroll
            for (int j = 0; j < ENC_K; j++) {
                const uint32_t len = (lp[j >> 2] >> (8 * (j & 3))) & 0xFFu;
                acc |= (uint64_t)tv[j] << ((64u - nb - len) & 63u);
                nb += len;
                if (nb >= 32u) {
                    const uint32_t w = (uint32_t)(acc >> 32);
                    if (have) sb[wi] = w;
                    else headw = w;
                    have = true;
                    wi++;
                    acc <<= 32;
                    nb -= 32u;
                }
            }
            const uint32_t tailw = (uint32_t)(acc >> 32);
            const uint32_t pt = wave_shr1_u(tailw, 0u);
            if (lane == 0) { s_hw[wid] = headw; s_hi[wid] = hi; }
            else sb[hi] = headw | pt;
            if (lane == 63) { s_tw[wid] = tailw; s_ti[wid] = nb ? wi : 0xFFFFFFFFu; }
        } else {
            for (int i = tid; i < E3_WORDS / 4; i += ENC_TPB) reinterpret_cast<uint4*>(sb)[i] = make_uint4(0u, 0u, 0u, 0u);
            __syncthreads();
            uint32_t o = off;
#pragma unroll
            for (int j = 0; j < ENC_K; j++) {
                const uint32_t lj = (lp[j >> 2] >> (8 * (j & 3))) & 0xFFu;
                if (lj) {
                    const uint64_t v = (uint64_t)tv[j] << ((64u - (o & 31u) - lj) & 63u);
                    atomicOr(&sb[o >> 5], (uint32_t)(v >> 32));
                    if ((o & 31u) + lj > 32u) atomicOr(&sb[(o >> 5) + 1], (uint32_t)v);
                }
                o += lj;
            }
            if (lane == 0) s_hi[wid] = 0xFFFFFFFFu;
            if (lane == 63) s_ti[wid] = 0xFFFFFFFFu;
        }
        __syncthreads();                                              // D
        EPSTAMP(cur, 4);
        // ---- wave 0: tile cur's boundary words; tile prev's offset (its window has been in flight through
        // the tokens and the pack)
        if (wid == 0) {
            if (lane < 4) {
                const uint32_t hi = s_hi[lane];
                if (hi != 0xFFFFFFFFu) {
                    uint32_t w = s_hw[lane];
                    if (lane > 0 && s_ti[lane - 1] == hi) w |= s_tw[lane - 1];
                    sb[hi] = w;
                }
                if (lane == 3 && s_ti[3] != 0xFFFFFFFFu) sb[s_ti[3]] = s_tw[3];
            }
            if (prev >= 0)
                pipe_offset(st, tl, prev, s_T[b ^ 1], tag, epoch, start_bit, n, ntiles, lbv, tl0, err, total_bits,
                            total_bits2, s_G, s_tp, s_ok);
            if (lane == 0 && hasn) {
                if (!DC_PIPE_STATIC && nk == ndraw - 1) atomicExch(ticket, 0u);
                s_nx = nk;                                            // (read after the next top barrier)
            }
        }
        __syncthreads();                                              // E
        EPSTAMP(cur, 5);
        // ---- waves 1-3: store tile prev (wave 0 issues the same count with an empty range)
        pipe_store(out, sbuf[b ^ 1], s_T[b ^ 1], prev, ntiles, s_G, s_tp, wid > 0 && prev >= 0 && s_ok);
        EPSTAMP(cur, 6);
        prev = cur;
        b ^= 1;
        if (!hasn) break;
        cur = nxt;
    }
    // ---- the workgroup's last tile (prev, in buffer b ^ 1): look-back and store
    __syncthreads();
    if (wid == 0) {
        const uint64_t tl0 = lane == 0 ? ld_relaxed(tl + prev - 1) : 0ull;
        pipe_offset(st, tl, prev, s_T[b ^ 1], tag, epoch, start_bit, n, ntiles, nullptr, tl0, err, total_bits,
                    total_bits2, s_G, s_tp, s_ok);
    }
    __syncthreads();
    pipe_store(out, sbuf[b ^ 1], s_T[b ^ 1], prev, ntiles, s_G, s_tp, wid > 0 && s_ok != 0);
#undef EPSTAMP
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

static long long desc_words_multi(long long nt);
static int g_enc_mode_last = 0;
static int g_enc_crc_fused = 0;                 // 1: the last launch computed the fused CRC pieces
static int g_enc_help = -1;                     // the helping instantiation (DC_ENC_HELP=1 / dc_set_encode_help)
extern "C" int dc_set_encode_help(int on) {
    const int old = g_enc_help < 0 ? 0 : g_enc_help;
    g_enc_help = on ? 1 : 0;
    return old;
}
// encoder variant: 1 = single pass (default), 2 = count + pack (the pack's workgroup 0 scans the tile
// counts, the other tiles wait for its flag), 3 = count + scan launch + pack (no wait anywhere: the
// fallback after a single-pass timeout).  DC_ENC_PASSES=2|3 selects the others.
static int enc_mode_default(void) {
    static int m = 0;
    if (!m) {
        const char* e = getenv("DC_ENC_PASSES");
        m = (e && (atoi(e) == 2 || atoi(e) == 3)) ? atoi(e) : 1;
    }
    return m;
}
extern "C" int dc_encode_mode(void) { return g_enc_mode_last; }
extern "C" int dc_encode_crc_fused_last(void) { return g_enc_crc_fused; }

// mode 0: the default variant.  desc (dc_encode_desc_words): single pass -- tile states (u64) | tail
// granules (u64); two/three launches -- tile offsets (u64) | tile bit counts (u32) | tile tails (u32) |
// per-thread bit counts (u16)
// the CT9 send (dc_encode_send_device): every launch of the next encodes also writes its stream words into this
// buffer (the receiver's), nullptr otherwise
static uint32_t* g_enc_mirror = nullptr;
extern "C" void dc_set_encode_mirror(void* dst) { g_enc_mirror = (uint32_t*)dst; }
// 1 when an encode takes the plain single-pass instantiation (no pipe, chained look-back, helping or multi-pass
// variant is selected): dc_halo_encode2_device runs two such encodes side by side with their own scratch
extern "C" int dc_encode_plain(void) {
    if (g_enc_help < 0) g_enc_help = (getenv("DC_ENC_HELP") && *getenv("DC_ENC_HELP") == '1') ? 1 : 0;
    const char* sc = getenv("DC_ENC_SCAN");
    const char* pp = getenv("DC_ENC_PIPE");
    return enc_mode_default() == 1 && !g_enc_help && !(sc && *sc == '0') && !(pp ? (*pp != '0') : DC_ENC_PIPE) &&
           !g_enc_mirror;
}

extern "C" int dc_launch_encode(const float* x, long long n, long long idx0, const Params* P,
                                uint32_t* out, uint64_t* desc, unsigned* flag, uint32_t epoch, int start_bit, unsigned long long* total_bits, unsigned long long* total_bits2,
                                unsigned* err, unsigned long long* dbg, int mode, const uint32_t* crc_tab, uint32_t* crc_blk,
                                hipStream_t stream) {
    if (n <= 0) return 0;
    if (mode == 0) mode = enc_mode_default();
    g_enc_mode_last = mode;
    g_enc_crc_fused = 0;
    if (g_enc_help < 0) g_enc_help = (getenv("DC_ENC_HELP") && *getenv("DC_ENC_HELP") == '1') ? 1 : 0;
    const unsigned ntiles = (unsigned)((n + ENC_TILE - 1) / ENC_TILE);
    if (mode == 1) {
        const int grid = (int)ntiles;
        dc_mark_phase(0, stream);
        uint64_t* st = desc + ((desc_words_multi(ntiles) + 1) & ~1ll) + LB_PAD;   // 16-byte aligned (lb_dma)
        static int scan = -1;                                            // DC_ENC_SCAN=0: chained look-back
        if (scan < 0) scan = (getenv("DC_ENC_SCAN") && *getenv("DC_ENC_SCAN") == '0') ? 0 : 1;
        static int pipe = -1, cus = 0;                                   // DC_ENC_PIPE=0: one tile per workgroup
        if (pipe < 0) {
            const char* e = getenv("DC_ENC_PIPE");
            pipe = e ? (*e != '0') : DC_ENC_PIPE;
            int dev = 0;
            if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
                cus = 256;
        }
        // (dc_encode_sub_device: only the plain single-pass instantiation subtracts the minimum while loading; for
        // the others the host writes x - min first and encodes that)
        if (P->sub && (crc_blk || !scan || (pipe && flag) || g_enc_help || g_enc_mirror)) return -3;
        g_enc_crc_fused = 0;
        // (the CT9 sender: the stream's CRC pieces while the words are stored; the chained look-back variant
        // has no fused CRC: it encodes plainly and the host takes a CRC pass, dc_encode_crc_fused_last)
        if (crc_blk && scan && !start_bit) {
            g_enc_crc_fused = 1;
            const dim3 gd(grid + 1), bd(ENC_TPB);
            switch (P->ct) {
#define DC_ENC_CRC(C)                                                                                \
    case C:                                                                                          \
        hipLaunchKernelGGL(HIP_KERNEL_NAME(encode_fused_kernel<C, true>), gd, bd, 0, stream, x, n, idx0, *P, out, st, \
                           st + ntiles, ntiles, start_bit, total_bits, total_bits2, epoch, err, dbg, 1, crc_tab, crc_blk, \
                           g_enc_mirror); \
        break;
                DC_ENC_CRC(5) DC_ENC_CRC(6) DC_ENC_CRC(7) DC_ENC_CRC(11)
#undef DC_ENC_CRC
                default: return -2;
            }
            dc_mark_phase(1, stream);
            return hipGetLastError() == hipSuccess ? 0 : -1;
        }
        if (pipe && scan && flag && !g_enc_mirror) {
            // persistent workgroups drawing tiles from a ticket counter (flag word 1088: its own 256-byte
            // line past the pack's 1024 flags, zeroed at init and reset by each launch's last draw)
            const unsigned g = (unsigned)min((long long)ntiles, (long long)DC_PIPE_WAVES * cus - (DC_PIPE_STATIC ? 1 : 0));
            DC_ENC_DISPATCH(encode_pipe_kernel, dim3(g + 1), dim3(ENC_TPB), 0, stream, x, n, idx0, *P, out, st,
                            st + ntiles, ntiles, start_bit, total_bits, total_bits2, epoch, err, flag + 1088, ntiles + g,
                            dbg);
            dc_mark_phase(1, stream);
            return hipGetLastError() == hipSuccess ? 0 : -1;
        }
        if (g_enc_help) {                    // (ranks sharing a GPU: tiles and scanner compute late tiles' counts)
            switch (P->ct) {
#define DC_ENC_HELPK(C)                                                                              \
    case C:                                                                                          \
        hipLaunchKernelGGL(HIP_KERNEL_NAME(encode_fused_kernel<C, false, true>), dim3(grid + scan), dim3(ENC_TPB), 0, \
                           stream, x, n, idx0, *P, out, st, st + ntiles, ntiles, start_bit, total_bits, total_bits2, \
                           epoch, err, dbg, scan, nullptr, nullptr, g_enc_mirror);                   \
        break;
                DC_ENC_HELPK(5) DC_ENC_HELPK(6) DC_ENC_HELPK(7) DC_ENC_HELPK(11)
#undef DC_ENC_HELPK
                default: return -2;
            }
        } else if (P->sub) {                 // (x - min made while loading)
            switch (P->ct) {
#define DC_ENC_SUBK(C)                                                                               \
    case C:                                                                                          \
        hipLaunchKernelGGL(HIP_KERNEL_NAME(encode_fused_kernel<C, false, false, true>), dim3(grid + scan), dim3(ENC_TPB), \
                           0, stream, x, n, idx0, *P, out, st, st + ntiles, ntiles, start_bit, total_bits, total_bits2, \
                           epoch, err, dbg, scan, nullptr, nullptr, g_enc_mirror);                   \
        break;
                DC_ENC_SUBK(5) DC_ENC_SUBK(6) DC_ENC_SUBK(7) DC_ENC_SUBK(11)
#undef DC_ENC_SUBK
                default: return -2;
            }
        } else {
            DC_ENC_DISPATCH(encode_fused_kernel, dim3(grid + scan), dim3(ENC_TPB), 0, stream, x, n, idx0, *P, out, st,
                            st + ntiles, ntiles, start_bit, total_bits, total_bits2, epoch, err, dbg, scan, nullptr,
                            nullptr, g_enc_mirror);
        }
        dc_mark_phase(1, stream);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    if (P->sub) return -3;
    uint32_t* tbits = reinterpret_cast<uint32_t*>(desc + ntiles);
    uint32_t* tails = tbits + ntiles + (ntiles & 1u);
    uint16_t* psum16 = reinterpret_cast<uint16_t*>(tails + ntiles + (ntiles & 1u));
    dc_mark_phase(0, stream);
    DC_ENC_DISPATCH(encode_count_kernel, dim3(ntiles), dim3(256), 0, stream, x, n, idx0, *P, tbits,
                    (long long)ntiles, err, tails, psum16);
    dc_mark_phase(1, stream);                   // (no mark 2: the pack's slot starts at mark 1)
    if (mode == 3) {
        hipLaunchKernelGGL(encode_scan_kernel, dim3(1), dim3(1024), 0, stream, tbits, desc, (long long)ntiles, start_bit,
                           total_bits, total_bits2);
        flag = nullptr;
    }
    DC_ENC_DISPATCH(encode_pack_kernel, dim3(ntiles), dim3(ENC_TPB), 0, stream, x, n, idx0, *P, out, desc, tbits,
                    tails, psum16, ntiles, start_bit, total_bits, total_bits2, flag, epoch, err, dbg, g_enc_mirror);
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
    DC_ENC_DISPATCH(encode_count_kernel, dim3(gc), dim3(256), 0, stream, x, n, idx0, *P, tbits, (long long)ntiles, err,
                    nullptr, nullptr);
    hipLaunchKernelGGL(encode_scan_kernel, dim3(1), dim3(1024), 0, stream, tbits, desc, (long long)ntiles, 0, total_bits,
                       nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" long long dc_encode_tile_count(long long n) { return (n + ENC_TILE - 1) / ENC_TILE; }

// u64 words of the encode descriptor buffer: tile offsets + 32-bit tile counts + 32-bit tile tails +
// 16-bit per-thread counts of the pack kernel
// + the single pass's 2 words per tile (states, tail granules) in a region of their own, which the other
// variants and dc_launch_encode_bits never write (their counts could read as a live tag)
static long long desc_words_multi(long long nt) {
    return nt + (nt + 1) / 2 + (nt + 1) / 2 + 1 + nt * (ENC_TPB / 4);     // offsets, counts, tails, thread counts
}
extern "C" long long dc_encode_desc_words(long long n) {
    const long long nt = dc_encode_tile_count(n);
    return desc_words_multi(nt) + 1 + LB_PAD + 2 * nt;
}
// the epochs a state tag tells apart: the host clears desc when its encode epoch reaches this
extern "C" unsigned dc_encode_epoch_limit(void) { return ST_TAGM; }

}  // namespace dc
