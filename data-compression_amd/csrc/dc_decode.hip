// dc_decode.hip -- parallel bit-wise decoder for gfx950 (CT 5/6/7/11).
//
// Replaces the bit-serial state machines myDecompress_bitwise (impl/dataCompression.c:2922-3135),
// myDecompress_bitwise_np (:2459-2609), myDecompress_bitwise_mask (:1703-1898) and
// myDecompress_bitwise_op (:698-797).  The stream has no sync markers, so it is cut into chunks of
// CHUNK_BITS and the token boundaries are recovered in parallel:
//
//  1. chunk_paths   : every chunk parses a speculative path P_c from its first bit (entry 0) and
//                     records its exit offset into the next chunk, its token count and which of its
//                     first 32 bit positions lie on P_c.
//  2. group_maps    : the first chunk of every group of GROUP chunks gets its complete entry map
//                     (all 32 possible entries -> exit, count), one lane per entry.
//  3. closure rounds: for every chunk, each exit of the previous chunk's known paths that is not yet
//                     a known entry is parsed alongside P_c until the two paths merge.  Random data
//                     closes in one round; periodic data (e.g. constant input) in a few.
//  4. resolve       : per group, the chunk maps (32 entries, unknown = 63) are composed with a
//                     Hillis-Steele scan in LDS; groups chain by a decoupled look-back whose
//                     aggregate is the group's full 32-entry map (composed with lane shuffles).
//                     Out: every chunk's true entry and first token index.
//  5. decode        : every chunk decodes from its true entry.  The decoder history holds DECODED
//                     values (:1812-1831), so the first tokens of a chunk may depend on the previous
//                     chunk; they are tracked symbolically and left pending.
//  6. fixup         : pending prefixes are re-decoded once the three preceding values are final
//                     (iterated; a serial kernel finishes pathological chains such as ramps of
//                     '111' codes).
// Exactness never depends on speculation succeeding: unknown entries are detected and reported
// so the host can run more closure rounds.
#include "dc_device.h"
#include <algorithm>

namespace dc {

constexpr int UNK = 63;



__global__ void plan_kernel(Plan* plan, const unsigned long long* dev_nbits, unsigned long long host_nbits,
                            long long max_chunks, int ct, long long num) {
    const unsigned long long nbits = dev_nbits ? *dev_nbits : host_nbits;
    Plan p;
    p.nbits = nbits;
    p.nbytes = (long long)((nbits + 7) >> 3);
    long long nc = (long long)((nbits + CHUNK_BITS - 1) / CHUNK_BITS);
    if (nc > max_chunks) nc = max_chunks;
    p.nchunks = nc;
    p.ngroups = (nc + GROUP - 1) / GROUP;
    p.runs = runs_mode(ct, nbits, num);
    *plan = p;
}

// walk the path entering chunk c at relative bit e alongside P_c until merge or chunk end
template <int CT>
__device__ void walk_entry(const uint8_t* s, const Plan& pl, const Params& P, long long c, int e,
                           uint32_t pmask, int pexit, int pcnt, int* out_exit, uint32_t* out_cnt) {
    const long long cs = c * CHUNK_BITS;
    long long ce = cs + CHUNK_BITS;
    const long long cend = ce < (long long)pl.nbits ? ce : (long long)pl.nbits;
    if ((pmask >> e) & 1u) {
        *out_exit = pexit;
        *out_cnt = (uint32_t)(pcnt - __popc(pmask & ((1u << e) - 1u)));
        return;
    }
    BitReader A, Bp;
    A.init(s, pl.nbytes, cs + e);
    uint32_t ca = 0, cb = 0;
    if (CT != 6 && pl.runs) {                                  // A alone to the chunk end, whole runs
        while (A.pos < cend) {
            const uint32_t t = A.peek();
            const int k = (int)t < 0 ? run3(t, A.pos, cend) : 1;
            A.skip(k > 1 ? 3 * k : token_len<CT>(t, P));
            ca += k;
        }
        const long long x = A.pos - ce;
        *out_exit = (x >= 0 && x < 32) ? (int)x : 0;
        *out_cnt = ca;
        return;
    }
    Bp.init(s, pl.nbytes, cs);
    while (A.pos < cend) {
        if (A.pos == Bp.pos) {
            *out_exit = pexit;
            *out_cnt = ca + (uint32_t)pcnt - cb;
            return;
        }
        if (A.pos < Bp.pos || Bp.pos >= cend) {
            A.skip(token_len<CT>(A.peek(), P));
            ca++;
        } else {
            Bp.skip(token_len<CT>(Bp.peek(), P));
            cb++;
        }
    }
    const long long x = A.pos - ce;
    *out_exit = (x >= 0 && x < 32) ? (int)x : 0;
    *out_cnt = ca;
}

// 1. speculative path from each chunk's first bit
template <int CT>
__global__ __launch_bounds__(256) void chunk_paths_kernel(const uint8_t* __restrict__ s, Params P, DecBufs D) {
    const Plan pl = *D.plan;
    for (long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x; c < pl.nchunks;
         c += (long long)gridDim.x * blockDim.x) {
        const long long cs = c * CHUNK_BITS;
        const long long ce = cs + CHUNK_BITS;
        const long long cend = ce < (long long)pl.nbits ? ce : (long long)pl.nbits;
        BitReader br;
        br.init(s, pl.nbytes, cs);
        uint32_t mask = 0, n = 0;
        while (br.pos < cend) {
            const long long r = br.pos - cs;
            if (r < 32) mask |= 1u << r;
            const uint32_t t = br.peek();
            if (CT != 6 && pl.runs && (int)t < 0 && r >= 32) {         // past the mask word: whole runs
                const int k = run3(t, br.pos, cend);
                br.skip(3 * k);
                n += k;
            } else {
                br.skip(token_len<CT>(t, P));
                n++;
            }
        }
        const long long x = br.pos - ce;
        D.p_exit[c] = (uint8_t)((x >= 0 && x < 32) ? x : 0);
        D.p_cnt[c] = (uint16_t)n;
        D.p_mask[c] = mask;
        D.known[c] = 0u;
        D.exitmask[2 * c + 1] = 1u << D.p_exit[c];               // round 1 = P_c itself
    }
}

// 2. complete map of every group's first chunk (one lane per entry)
template <int CT>
__global__ __launch_bounds__(256) void group_maps_kernel(const uint8_t* __restrict__ s, Params P, DecBufs D) {
    const Plan pl = *D.plan;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < pl.ngroups * 32;
         i += (long long)gridDim.x * blockDim.x) {
        const long long g = i >> 5;
        const int e = (int)(i & 31);
        const long long c = g * GROUP;
        int x; uint32_t cnt;
        walk_entry<CT>(s, pl, P, c, e, D.p_mask[c], D.p_exit[c], D.p_cnt[c], &x, &cnt);
        D.fullmap[i] = ((uint32_t)x << 26) | (cnt & 0x3FFFFFFu);
        atomicOr(&D.exitmask[2 * c + 1], 1u << x);                 // all exits known from round 1
    }
}

// 3. one closure round: chunk c adds every exit of chunk c-1's known entries (as of round r-1)
//    that is not yet a known entry of its own.  exitmask is double-buffered by round parity, so a
//    lane never reads a mask its neighbour is writing in the same round.
template <int CT>
__global__ __launch_bounds__(256) void closure_kernel(const uint8_t* __restrict__ s, Params P, DecBufs D, int round) {
    const Plan pl = *D.plan;
    const int rp = round & 1, pp = rp ^ 1;
    for (long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x; c < pl.nchunks;
         c += (long long)gridDim.x * blockDim.x) {
        uint32_t mine = D.exitmask[2 * c + pp];
        if (c != 0 && (c % GROUP) != 0) {                          // group-first chunks are complete
            const uint32_t pmask = D.p_mask[c];
            uint32_t known = D.known[c];
            uint32_t need = D.exitmask[2 * (c - 1) + pp] & ~pmask & ~known;
            while (need) {
                const int e = __ffs(need) - 1;
                need &= need - 1;
                int x; uint32_t cnt;
                walk_entry<CT>(s, pl, P, c, e, pmask, D.p_exit[c], D.p_cnt[c], &x, &cnt);
                D.map[c * 32 + e] = ((uint32_t)x << 26) | (cnt & 0x3FFFFFFu);
                known |= 1u << e;
                mine |= 1u << x;
            }
            D.known[c] = known;
        }
        D.exitmask[2 * c + rp] = mine;
    }
}

// 3b. slow path: complete 32-entry maps for every chunk (one lane per unknown (chunk, entry)).
//     Bounded work (<= 32 walks per chunk) for locally periodic streams where closure rounds would
//     propagate only one chunk per round.
template <int CT>
__global__ __launch_bounds__(256) void full_maps_kernel(const uint8_t* __restrict__ s, Params P, DecBufs D) {
    const Plan pl = *D.plan;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < pl.nchunks * 32;
         i += (long long)gridDim.x * blockDim.x) {
        const long long c = i >> 5;
        const int e = (int)(i & 31);
        if ((c % GROUP) == 0) continue;
        const uint32_t pmask = D.p_mask[c];
        if (((pmask | D.known[c]) >> e) & 1u) continue;
        int x; uint32_t cnt;
        walk_entry<CT>(s, pl, P, c, e, pmask, D.p_exit[c], D.p_cnt[c], &x, &cnt);
        D.map[c * 32 + e] = ((uint32_t)x << 26) | (cnt & 0x3FFFFFFu);
        atomicOr(&D.known[c], 1u << e);
    }
}

// 4. resolve true entries and token offsets
__device__ __forceinline__ uint32_t chunk_map_entry(const DecBufs& D, const Plan& pl, long long gc, int cl, int e) {
    if (gc >= pl.nchunks) return ((uint32_t)e << 26);                    // identity past the end
    if (cl == 0) return D.fullmap[(gc / GROUP) * 32 + e];
    const uint32_t pm = D.p_mask[gc];
    if ((pm >> e) & 1u)
        return ((uint32_t)D.p_exit[gc] << 26) | (uint32_t)(D.p_cnt[gc] - __popc(pm & ((1u << e) - 1u)));
    if ((D.known[gc] >> e) & 1u) return D.map[gc * 32 + e];
    return (uint32_t)UNK << 26;
}

// granule: [63:62] flag (1 A, 2 P) | [61:40] epoch | [39:34] exit | [33:0] count
__device__ __forceinline__ uint64_t gran_pack(uint64_t flag, uint32_t epoch, uint32_t x, unsigned long long cnt) {
    return (flag << 62) | ((uint64_t)(epoch & 0x3FFFFFu) << 40) | ((uint64_t)(x & 63) << 34) |
           (cnt & ((1ull << 34) - 1));
}

__global__ __launch_bounds__(256) void resolve_kernel(DecBufs D, uint32_t epoch) {
    __shared__ uint32_t S[2][32][GROUP];   // [buffer][entry][chunk]: conflict-free lane access
    __shared__ long long s_g;
    __shared__ int s_tin;
    __shared__ unsigned long long s_base;
    const Plan pl = *D.plan;
    const int tid = threadIdx.x, lane = tid & 63;
    while (true) {
        if (tid == 0) s_g = (long long)atomicAdd(&D.ctr[0], 1u);
        __syncthreads();
        const long long g = s_g;
        if (g >= pl.ngroups) break;
        const long long gc = g * GROUP + tid;
        for (int e = 0; e < 32; e++) S[0][e][tid] = chunk_map_entry(D, pl, gc, tid, e);
        __syncthreads();
        int cur = 0;
        for (int d = 1; d < GROUP; d <<= 1) {
            for (int e = 0; e < 32; e++) {
                uint32_t r = S[cur][e][tid];
                if (tid >= d) {
                    const uint32_t a = S[cur][e][tid - d];
                    const uint32_t ax = a >> 26;
                    if (ax == UNK) r = (uint32_t)UNK << 26;
                    else {
                        const uint32_t b = S[cur][ax][tid];
                        r = ((b >> 26) == UNK) ? ((uint32_t)UNK << 26)
                                               : ((b & 0xFC000000u) | ((a + b) & 0x3FFFFFFu));
                    }
                }
                S[cur ^ 1][e][tid] = r;
            }
            cur ^= 1;
            __syncthreads();
        }
        // group map = S[cur][GROUP-1]; chain groups by decoupled look-back (wave 0, lane = entry)
        if (tid < 64) {
            const uint32_t gm = S[cur][lane & 31][GROUP - 1];
            int tin = 0;
            unsigned long long base = 0;
            if (g > 0) {
                if (lane < 32) st_relaxed(&D.gran[g * 32 + lane], gran_pack(1, epoch, gm >> 26, gm & 0x3FFFFFFu));
                int hx = lane & 31;
                unsigned long long hc = 0;
                long long k = g - 1;
                while (true) {
                    // lane 0 polls the predecessor's first granule; A records are then complete
                    uint64_t dv = 0;
                    int flag = 0;
                    if (lane == 0) {
                        unsigned spins = 0;
                        do {
                            dv = ld_relaxed(&D.gran[k * 32]);
                            flag = (((dv >> 40) & 0x3FFFFFu) == (epoch & 0x3FFFFFu)) ? (int)(dv >> 62) : 0;
                            if (flag == 0) __builtin_amdgcn_s_sleep(1);
                        } while (flag == 0 && ++spins < (1u << 24));
                        if (flag == 0) atomicOr(D.err, 16u);
                    }
                    const int flag0 = __shfl(flag, 0, 64);
                    if (flag0 == 1 && lane > 0 && lane < 32) {
                        unsigned spins = 0;
                        int f = 0;
                        do {
                            dv = ld_relaxed(&D.gran[k * 32 + lane]);
                            f = (((dv >> 40) & 0x3FFFFFu) == (epoch & 0x3FFFFFu)) ? (int)(dv >> 62) : 0;
                            if (f == 0) __builtin_amdgcn_s_sleep(1);
                        } while (f == 0 && ++spins < (1u << 24));
                        if (f == 0) atomicOr(D.err, 16u);
                    }
                    const int dx = (int)((dv >> 34) & 63);
                    const unsigned long long dc = dv & ((1ull << 34) - 1);
                    if (flag0 == 2 || flag0 == 0) {
                        const int px = __shfl(dx, 0, 64);
                        const unsigned long long pcnt = __shfl(dc, 0, 64);
                        if (px == UNK || flag0 == 0) { tin = UNK; base = 0; break; }
                        tin = __shfl(hx, px, 64);
                        base = pcnt + __shfl(hc, px, 64);
                        break;
                    }
                    const int nhx_src = dx == UNK ? 0 : dx;
                    const int nhx = __shfl(hx, nhx_src, 64);
                    const unsigned long long nhc = __shfl(hc, nhx_src, 64);
                    hx = (dx == UNK || nhx == UNK) ? UNK : nhx;
                    hc = dc + nhc;
                    k--;
                }
            }
            if (lane == 0) {
                uint32_t fx = UNK;
                unsigned long long fc = base;
                if (tin != UNK) {
                    const uint32_t v = S[cur][tin][GROUP - 1];
                    fx = v >> 26;
                    fc = base + (v & 0x3FFFFFFu);
                }
                st_relaxed(&D.gran[g * 32 + 0], gran_pack(2, epoch, fx, fc));
                s_tin = tin;
                s_base = base;
            }
        }
        __syncthreads();
        if (gc < pl.nchunks) {
            const int tin = s_tin;
            int te = tin;
            unsigned long long off = s_base;
            if (tin != UNK && tid > 0) {
                const uint32_t v = S[cur][tin][tid - 1];
                te = (int)(v >> 26);
                off += v & 0x3FFFFFFu;
            }
            if (te == UNK) atomicOr(D.err, 8u);
            D.entry[gc] = (uint8_t)te;
            D.tokoff[gc] = off;
        }
        __syncthreads();
    }
    // last workgroup out resets the ticket counter for the next call
    if (tid == 0) {
        __threadfence();
        if (atomicAdd(&D.ctr[1], 1u) == gridDim.x - 1) {
            atomicExch(&D.ctr[0], 0u);
            atomicExch(&D.ctr[1], 0u);
        }
    }
}

// 5. decode every chunk from its true entry; prefix tokens that depend on the previous chunk's
//    decoded values stay pending.  kind: 0 concrete, 1..3 incoming b1..b3, 4 derived.
template <int CT>
__global__ __launch_bounds__(256) void decode_kernel(const uint8_t* __restrict__ s, Params P, DecBufs D,
                                                     float* __restrict__ out, long long num) {
    const Plan pl = *D.plan;
    for (long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x; c < pl.nchunks;
         c += (long long)gridDim.x * blockDim.x) {
        const int e = D.entry[c];
        D.done[c] = 0;
        if (e == UNK) { D.pend[c] = 0; continue; }
        const long long cs = c * CHUNK_BITS;
        const long long ce = cs + CHUNK_BITS;
        const long long cend = ce < (long long)pl.nbits ? ce : (long long)pl.nbits;
        unsigned long long k = D.tokoff[c];
        BitReader br;
        br.init(s, pl.nbytes, cs + e);
        float f1 = -1.0f, f2 = -1.0f, f3 = -1.0f;
        int k1 = c == 0 ? 0 : 1, k2 = c == 0 ? 0 : 2, k3 = c == 0 ? 0 : 3;
        int pend = 0, j = 0;
        while (br.pos < cend) {
            const uint32_t t = br.peek();
            const int len = token_len<CT>(t, P);
            int code;
            const uint32_t pat = token_pattern<CT>(t, len, P, &code);
            float v;
            int kind;
            if (code == 0) { v = __uint_as_float(pat); kind = 0; }
            else if (code == 1) { v = f1; kind = k1; }
            else if (code == 2) {
                if (k1 == 0 && k2 == 0) { v = predict_value(2, f1, f2, f3); kind = 0; }
                else { v = 0.0f; kind = 4; }
            } else {
                if (k1 == 0 && k2 == 0 && k3 == 0) { v = predict_value(3, f1, f2, f3); kind = 0; }
                else { v = 0.0f; kind = 4; }
            }
            if (kind == 0) {
                if (k + j < (unsigned long long)num) out[k + j] = v;
            } else {
                pend = j + 1;
            }
            f3 = f2; k3 = k2; f2 = f1; k2 = k1; f1 = v; k1 = kind;
            br.skip(len);
            j++;
        }
        D.pend[c] = (uint16_t)(pend > 65535 ? 65535 : pend);
    }
}

// 6. re-decode pending prefixes whose three preceding values are final
template <int CT>
__device__ bool fix_chunk(const uint8_t* s, const Params& P, const DecBufs& D, const Plan& pl, long long c,
                          float* out, long long num, int it, bool serial, const float* hin = nullptr) {
    const unsigned long long k0 = D.tokoff[c];
    float h[3];
    for (int q = 0; q < 3; q++) {
        const long long idx = (long long)k0 - 1 - q;
        if (idx < 0) { h[q] = hin ? hin[-1 - idx] : -1.0f; continue; }   // before a shard: its incoming b1..b3
        if (idx >= num) { h[q] = 0.0f; continue; }
        long long d = c - 1;
        while (d > 0 && (long long)D.tokoff[d] > idx) d--;
        if (!serial) {
            const bool fin = (idx - (long long)D.tokoff[d] >= (long long)D.pend[d]) ||
                             (D.done[d] != 0 && D.done[d] < it);
            if (!fin) return false;
        }
        h[q] = out[idx];
    }
    float f1 = h[0], f2 = h[1], f3 = h[2];
    const long long cs = c * CHUNK_BITS;
    BitReader br;
    br.init(s, pl.nbytes, cs + D.entry[c]);
    const int np = D.pend[c];
    for (int j = 0; j < np; j++) {
        const uint32_t t = br.peek();
        const int len = token_len<CT>(t, P);
        int code;
        const uint32_t pat = token_pattern<CT>(t, len, P, &code);
        const float v = code == 0 ? __uint_as_float(pat) : predict_value(code, f1, f2, f3);
        if (k0 + j < (unsigned long long)num) out[k0 + j] = v;
        f3 = f2; f2 = f1; f1 = v;
        br.skip(len);
    }
    return true;
}

template <int CT>
__global__ __launch_bounds__(256) void fixup_kernel(const uint8_t* __restrict__ s, Params P, DecBufs D,
                                                    float* __restrict__ out, long long num, int it, int last) {
    const Plan pl = *D.plan;
    for (long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x; c < pl.nchunks;
         c += (long long)gridDim.x * blockDim.x) {
        if (D.pend[c] == 0 || D.done[c] != 0 || D.entry[c] == UNK) continue;
        if (fix_chunk<CT>(s, P, D, pl, c, out, num, it, false)) D.done[c] = (uint16_t)it;
        else if (last) atomicOr(D.err, 32u);
    }
}

template <int CT>
__global__ void fixup_serial_kernel(const uint8_t* __restrict__ s, Params P, DecBufs D, float* __restrict__ out,
                                    long long num) {
    const Plan pl = *D.plan;
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    for (long long c = 0; c < pl.nchunks; c++) {
        if (D.pend[c] == 0 || D.done[c] != 0 || D.entry[c] == UNK) continue;
        fix_chunk<CT>(s, P, D, pl, c, out, num, 0x7FFF, true);
        D.done[c] = 0x7FFF;
    }
}

// a shard's deferred prefixes (dc_decode_shard_fix): chunks [0, nc) in order, the values before the
// shard from hin (b1, b2, b3)
template <int CT>
__global__ void shard_fix_kernel(const uint8_t* __restrict__ s, Params P, DecBufs D, float* __restrict__ out,
                                 long long num, long long nc, const float* __restrict__ hin) {
    const Plan pl = *D.plan;
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    for (long long c = 0; c < pl.nchunks && c < nc; c++) {
        if (D.pend[c] == 0 || D.done[c] != 0 || D.entry[c] == UNK) continue;
        fix_chunk<CT>(s, P, D, pl, c, out, num, 0x7FFF, true, hin);
        D.done[c] = 0x7FFF;
    }
}

// ------------------------------------------------------------------------------------------------
static int g_grid = 2048;

#define DC_DISPATCH(CTV, KER, ...)                                                                   \
    switch (CTV) {                                                                                   \
        case 5: hipLaunchKernelGGL(KER<5>, __VA_ARGS__); break;                                      \
        case 6: hipLaunchKernelGGL(KER<6>, __VA_ARGS__); break;                                      \
        case 7: hipLaunchKernelGGL(KER<7>, __VA_ARGS__); break;                                      \
        case 11: hipLaunchKernelGGL(KER<11>, __VA_ARGS__); break;                                    \
        default: return -2;                                                                          \
    }

extern "C" int dc_launch_decode(const uint8_t* s, const unsigned long long* dev_nbits,
                                unsigned long long host_nbits, long long max_chunks, const Params* P,
                                const DecBufs* D, float* out, long long num, uint32_t epoch, int rounds,
                                int fix_iters, hipStream_t st) {
    const long long max_groups = (max_chunks + GROUP - 1) / GROUP;
    hipLaunchKernelGGL(plan_kernel, dim3(1), dim3(1), 0, st, D->plan, dev_nbits, host_nbits, max_chunks, P->ct, num);
    const int gchunks = (int)std::min<long long>((max_chunks + 255) / 256, g_grid);
    const int ggroups = (int)std::min<long long>((max_groups * 32 + 255) / 256, g_grid);
    DC_DISPATCH(P->ct, chunk_paths_kernel, dim3(gchunks), dim3(256), 0, st, s, *P, *D);
    DC_DISPATCH(P->ct, group_maps_kernel, dim3(ggroups), dim3(256), 0, st, s, *P, *D);
    for (int r = 2; r < 2 + rounds; r++)
        DC_DISPATCH(P->ct, closure_kernel, dim3(gchunks), dim3(256), 0, st, s, *P, *D, r);
    const int gres = (int)std::min<long long>(max_groups, 512);
    hipLaunchKernelGGL(resolve_kernel, dim3(gres > 0 ? gres : 1), dim3(256), 0, st, *D, epoch);
    DC_DISPATCH(P->ct, decode_kernel, dim3(gchunks), dim3(256), 0, st, s, *P, *D, out, num);
    for (int it = 1; it <= fix_iters; it++)
        DC_DISPATCH(P->ct, fixup_kernel, dim3(gchunks), dim3(256), 0, st, s, *P, *D, out, num, it,
                    it == fix_iters ? 1 : 0);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// runs-mode streams the fast path could not chain (tiles entered off their P_0): the parse already left
// every chunk's map of the entries its tile reaches (chunk 0: all 32), so only the composition is left;
// the values then come from the fast decode kernel (dc_launch_decode_fast_resolved)
extern "C" int dc_launch_resolve(long long max_chunks, const DecBufs* D, uint32_t epoch, hipStream_t st) {
    const long long max_groups = (max_chunks + GROUP - 1) / GROUP;
    const int gres = (int)std::min<long long>(max_groups, 512);
    hipLaunchKernelGGL(resolve_kernel, dim3(gres > 0 ? gres : 1), dim3(256), 0, st, *D, epoch);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// extra closure rounds + re-resolve + decode (slow path after an unknown entry was reported)
// slow path after an unresolved entry: complete maps for every chunk, re-resolve, re-decode
extern "C" int dc_launch_decode_more(const uint8_t* s, long long max_chunks, const Params* P, const DecBufs* D,
                                     float* out, long long num, uint32_t epoch, int fix_iters, hipStream_t st) {
    const long long max_groups = (max_chunks + GROUP - 1) / GROUP;
    const int gchunks = (int)std::min<long long>((max_chunks + 255) / 256, g_grid);
    const int gall = (int)std::min<long long>((max_chunks * 32 + 255) / 256, 8192);
    DC_DISPATCH(P->ct, full_maps_kernel, dim3(gall), dim3(256), 0, st, s, *P, *D);
    const int gres = (int)std::min<long long>(max_groups, 512);
    hipLaunchKernelGGL(resolve_kernel, dim3(gres > 0 ? gres : 1), dim3(256), 0, st, *D, epoch);
    DC_DISPATCH(P->ct, decode_kernel, dim3(gchunks), dim3(256), 0, st, s, *P, *D, out, num);
    for (int it = 1; it <= fix_iters; it++)
        DC_DISPATCH(P->ct, fixup_kernel, dim3(gchunks), dim3(256), 0, st, s, *P, *D, out, num, it,
                    it == fix_iters ? 1 : 0);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int dc_launch_shard_fix(const uint8_t* s, const Params* P, const DecBufs* D, float* out, long long num,
                                   long long nchunks, const float* hin, hipStream_t st) {
    DC_DISPATCH(P->ct, shard_fix_kernel, dim3(1), dim3(64), 0, st, s, *P, *D, out, num, nchunks, hin);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int dc_launch_fixup_serial(const uint8_t* s, const Params* P, const DecBufs* D, float* out,
                                      long long num, hipStream_t st) {
    DC_DISPATCH(P->ct, fixup_serial_kernel, dim3(1), dim3(64), 0, st, s, *P, *D, out, num);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Exact sequential decode with the reference's history semantics (decompress_bitwise_float :3143-3190,
// history update :1872-1889): -1.0f marks an empty history slot, so a decoded value of exactly -1.0f
// (or a predicted token before the history is full) changes how the history shifts.  Streams that
// contain such values come only from inputs outside the codec's domain (negative values in CT5/7/11,
// whose sign bit parses as a 3-bit code); the fast path flags them (D.err 128) and this one thread
// decodes the whole stream exactly like the spec decoder, stopping at a truncated token.
template <int CT>
__global__ void decode_serial_kernel(const uint8_t* s, Params P, DecBufs D, float* out, long long num) {
    if (threadIdx.x != 0) return;
    const Plan pl = *D.plan;
    const long long nbits = (long long)pl.nbits;
    BitReader r;
    r.init(s, pl.nbytes, 0);
    float b1 = -1.0f, b2 = -1.0f, b3 = -1.0f;
    if (D.shard == 2 && D.hin) { b1 = D.hin[0]; b2 = D.hin[1]; b3 = D.hin[2]; }   // a shard's incoming values
    long long n = 0;
    while (n < num && r.pos < nbits) {
        const uint32_t tk = r.peek();
        const int len = token_len<CT>(tk, P);
        if (r.pos + len > nbits) break;
        int code;
        const uint32_t pat = token_pattern<CT>(tk, len, P, &code);
        const float v = code == 0 ? __uint_as_float(pat) : predict_value(code, b1, b2, b3);
        out[n++] = v;
        if (b3 == -1.0f) b3 = v;
        else if (b2 == -1.0f) b2 = v;
        else if (b1 == -1.0f) b1 = v;
        else { b3 = b2; b2 = b1; b1 = v; }
        r.skip(len);
    }
}

extern "C" int dc_launch_decode_serial(const uint8_t* s, const Params* P, const DecBufs* D, float* out,
                                       long long num, hipStream_t st) {
    DC_DISPATCH(P->ct, decode_serial_kernel, dim3(1), dim3(64), 0, st, s, *P, *D, out, num);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// after a slow path: does the output hold a -1.0f (history sentinel)?  -> D.err 128
__global__ void find_sentinel_kernel(const float* out, long long num, unsigned* err) {
    bool hit = false;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < num; i += (long long)gridDim.x * blockDim.x)
        hit |= __float_as_uint(out[i]) == 0xBF800000u;
    if (__any(hit) && (threadIdx.x & 63) == 0) atomicOr(err, 128u);
}

extern "C" int dc_launch_find_sentinel(const float* out, long long num, unsigned* err, hipStream_t st) {
    if (num <= 0) return 0;
    const long long g = std::min<long long>((num + 255) / 256, 2048);
    hipLaunchKernelGGL(find_sentinel_kernel, dim3((unsigned)g), dim3(256), 0, st, out, num, err);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" long long dc_decode_chunk_bits(void) { return CHUNK_BITS; }
extern "C" long long dc_decode_group(void) { return GROUP; }

}  // namespace dc
