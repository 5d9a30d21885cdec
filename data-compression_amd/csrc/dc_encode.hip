// dc_encode.hip -- single-pass bit-wise encoder for gfx950 (CT 5/6/7/11).
//
// Replaces the per-element serial loop of myCompress_bitwise (impl/dataCompression.c:3310-3444),
// myCompress_bitwise_np (:2645-2654), myCompress_bitwise_mask (:2030-2141) and
// myCompress_bitwise_op (:577-696), whose cost is one add_bit_to_bytes call (+ realloc) per output
// bit (:5456-5489).
//
// One workgroup = one tile of TPB*K consecutive floats.  The encoder history is the ORIGINAL input
// (:2095-2097), so every token is a pure function of x[i-3..i]: each lane builds its K tokens from
// registers, the workgroup scans the token lengths, and a decoupled look-back over per-tile
// descriptors (64-bit granules: flag | epoch | bit count) gives the tile's global bit offset G.
// Word ownership makes the stream race-free without atomics on HBM or a zero pass: a tile writes
// every 32-bit word whose first bit lies in [G, G+T) and completes the last one with the first
// <= 31 bits of the following elements (recomputed locally, <= 11 tokens).  Bits are assembled
// MSB-first in LDS with ds_or and leave as byte-swapped dwords (stream byte 0 = MSB of word 0).
#include "dc_device.h"

namespace dc {

constexpr int ENC_TPB = 256;
constexpr int ENC_K = 16;                       // floats per lane (4 x dwordx4)
constexpr int ENC_TILE = ENC_TPB * ENC_K;       // 4096 floats per tile
constexpr int ENC_LDS_WORDS = ENC_TILE + 48;    // 32 bits/elem max + offset + head slack

// descriptor granule: [63:62] flag (1 aggregate, 2 inclusive) | [61:38] epoch | [37:0] bits
__device__ __forceinline__ uint64_t enc_pack(uint64_t flag, uint32_t epoch, uint64_t v) {
    return (flag << 62) | ((uint64_t)(epoch & 0xFFFFFFu) << 38) | (v & ((1ull << 38) - 1));
}

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

template <int CT>
__global__ __launch_bounds__(ENC_TPB) void encode_kernel(
    const float* __restrict__ x, long long n, long long idx0, Params P, uint32_t* __restrict__ out,
    uint64_t* __restrict__ desc, unsigned* __restrict__ tile_ctr, unsigned ntiles, uint32_t epoch,
    int start_bit, unsigned long long* __restrict__ total_bits, unsigned* __restrict__ err) {
    __shared__ uint32_t s_bits[ENC_LDS_WORDS];
    __shared__ uint32_t s_wsum[ENC_TPB / 64];
    __shared__ unsigned s_tile;
    __shared__ unsigned long long s_G;
    __shared__ uint32_t s_head_val[12];
    __shared__ int s_head_len[12];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (tid == 0) s_tile = atomicInc(tile_ctr, ntiles - 1);       // dynamic id: predecessors run
    for (int i = tid; i < ENC_LDS_WORDS; i += ENC_TPB) s_bits[i] = 0u;
    __syncthreads();
    const unsigned tile = s_tile;
    const long long tbase = (long long)tile * ENC_TILE;
    const long long base = tbase + (long long)tid * ENC_K;

    // ---- load K floats + 3-float halo (history = original inputs)
    float v[ENC_K + 4];
    if (base + ENC_K <= n) {
        const float4* p4 = reinterpret_cast<const float4*>(x + base);
#pragma unroll
        for (int q = 0; q < ENC_K / 4; q++) {
            const float4 t = p4[q];
            v[4 + 4 * q] = t.x; v[5 + 4 * q] = t.y; v[6 + 4 * q] = t.z; v[7 + 4 * q] = t.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < ENC_K; j++) v[4 + j] = (base + j < n) ? x[base + j] : 0.0f;
    }
    const long long gbase = idx0 + base;                          // global element index
#pragma unroll
    for (int j = 1; j <= 3; j++) v[4 - j] = (gbase - j >= 0 && base - j > -4) ? x[base - j] : 0.0f;

    // ---- tokens
    uint32_t tv[ENC_K];
    int tl[ENC_K];
    uint32_t mysum = 0;
    bool neg1 = false;
#pragma unroll
    for (int j = 0; j < ENC_K; j++) {
        if (base + j < n) {
            make_token<CT>(v[4 + j], v[3 + j], v[2 + j], v[1 + j], gbase + j >= 3, P, tv[j], tl[j]);
            neg1 |= (v[4 + j] == -1.0f);
        } else {
            tv[j] = 0u; tl[j] = 0;
        }
        mysum += (uint32_t)tl[j];
    }
    if (CT != 6 && neg1) atomicOr(err, 1u);                      // -1.0f is the reference's sentinel

    // ---- workgroup exclusive scan of bit lengths
    uint32_t inc = mysum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t t = __shfl_up(inc, d, 64);
        if (lane >= d) inc += t;
    }
    if (lane == 63) s_wsum[wid] = inc;

    // ---- head: first <= 31 bits of the elements after this tile (completes our last word)
    const long long nb = tbase + ENC_TILE;                         // first element of next tile
    if (wid == 1 && lane < 12) {
        uint32_t hv = 0u; int hl = 0;
        const long long e = nb + lane;
        if (lane < 11 && e < n) {
            const long long ge = idx0 + e;
            const float xe = x[e];
            const float e1 = x[e - 1], e2 = x[e - 2], e3 = x[e - 3];
            make_token<CT>(xe, e1, e2, e3, ge >= 3, P, hv, hl);
        }
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
    const uint32_t excl = wpre + inc - mysum;

    // ---- decoupled look-back for the tile's global bit offset
    if (wid == 0) {
        unsigned long long G = 0;
        if (tile == 0) {
            if (lane == 0) st_relaxed(&desc[0], enc_pack(2, epoch, (uint64_t)start_bit + T));
            G = (unsigned long long)start_bit;
        } else {
            if (lane == 0) st_relaxed(&desc[tile], enc_pack(1, epoch, T));
            long long look = (long long)tile - 1;
            unsigned long long acc = 0;
            while (true) {
                const long long pred = look - lane;
                uint64_t d = 0;
                int flag = 2;
                uint64_t val = 0;
                if (pred >= 0) {
                    unsigned spins = 0;
                    do {
                        d = ld_relaxed(&desc[pred]);
                        flag = (((d >> 38) & 0xFFFFFFu) == (epoch & 0xFFFFFFu)) ? (int)(d >> 62) : 0;
                        if (flag == 0) __builtin_amdgcn_s_sleep(1);
                    } while (flag == 0 && ++spins < (1u << 26));
                    val = d & ((1ull << 38) - 1);
                    if (flag == 0) { atomicOr(err, 2u); flag = 2; val = 0; }   // bounded spin
                }
                const unsigned long long incl_mask = __ballot(flag == 2);
                if (incl_mask) {
                    const int k = __ffsll((long long)incl_mask) - 1;       // most recent inclusive
                    uint64_t part = (lane <= k) ? val : 0;
#pragma unroll
                    for (int d2 = 32; d2 >= 1; d2 >>= 1) part += __shfl_xor(part, d2, 64);
                    acc += part;
                    break;
                }
                uint64_t part = val;
#pragma unroll
                for (int d2 = 32; d2 >= 1; d2 >>= 1) part += __shfl_xor(part, d2, 64);
                acc += part;
                look -= 64;
            }
            G = acc;
            if (lane == 0) st_relaxed(&desc[tile], enc_pack(2, epoch, G + T));
        }
        if (lane == 0) {
            s_G = G;
            if (tile == ntiles - 1) *total_bits = G + T;
        }
    }
    __syncthreads();
    const unsigned long long G = s_G;
    const uint32_t boff = (uint32_t)(G & 31ull);
    const long long wb = (long long)(G >> 5);

    // ---- assemble MSB-first in LDS
    uint32_t off = boff + excl;
#pragma unroll
    for (int j = 0; j < ENC_K; j++) {
        if (tl[j]) lds_place(s_bits, off, tv[j], tl[j]);
        off += (uint32_t)tl[j];
    }
    if (tid == 0) {
        uint32_t ho = boff + T;
        for (int j = 0; j < 11 && s_head_len[j]; j++) {
            if (ho - boff - T >= 32u) break;
            lds_place(s_bits, ho, s_head_val[j], s_head_len[j]);
            ho += (uint32_t)s_head_len[j];
        }
    }
    __syncthreads();

    // ---- write owned words: first bit in [G, G+T) (tile 0 also owns the start_bit prefix word)
    const unsigned long long Gend = G + T;
    long long w0 = (long long)((G + 31) >> 5);
    if (tile == 0) w0 = 0;
    const long long w1 = (long long)((Gend + 31) >> 5);
    for (long long w = w0 + tid; w < w1; w += ENC_TPB)
        out[w] = __builtin_bswap32(s_bits[w - wb]);
}

// ------------------------------------------------------------------------------------------------
extern "C" int dc_launch_encode(const float* x, long long n, long long idx0, const Params* P,
                                uint32_t* out, uint64_t* desc, unsigned* tile_ctr, uint32_t epoch,
                                int start_bit, unsigned long long* total_bits, unsigned* err,
                                hipStream_t stream) {
    if (n <= 0) return 0;
    const unsigned ntiles = (unsigned)((n + ENC_TILE - 1) / ENC_TILE);
    dim3 grid(ntiles), block(ENC_TPB);
    switch (P->ct) {
        case 5: hipLaunchKernelGGL(encode_kernel<5>, grid, block, 0, stream, x, n, idx0, *P, out, desc, tile_ctr, ntiles, epoch, start_bit, total_bits, err); break;
        case 6: hipLaunchKernelGGL(encode_kernel<6>, grid, block, 0, stream, x, n, idx0, *P, out, desc, tile_ctr, ntiles, epoch, start_bit, total_bits, err); break;
        case 7: hipLaunchKernelGGL(encode_kernel<7>, grid, block, 0, stream, x, n, idx0, *P, out, desc, tile_ctr, ntiles, epoch, start_bit, total_bits, err); break;
        case 11: hipLaunchKernelGGL(encode_kernel<11>, grid, block, 0, stream, x, n, idx0, *P, out, desc, tile_ctr, ntiles, epoch, start_bit, total_bits, err); break;
        default: return -2;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" long long dc_encode_tile_count(long long n) { return (n + ENC_TILE - 1) / ENC_TILE; }

}  // namespace dc
