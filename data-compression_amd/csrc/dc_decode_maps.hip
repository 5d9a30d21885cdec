// dc_decode_maps.hip -- the parse of streams whose token paths merge slowly, for the segment decoder's value
// kernel (decode3_kernel): the chunk entries and token offsets parse3 would record, found from entry -> exit
// maps instead of self-synchronising walks.
//
// parse3 starts every segment's walk 1024 bits early and counts on it meeting the true token path by the
// segment's first chunk; a walk that has not met it is repaired by walking again from the true entry.  Some
// streams' paths take far longer to meet (tools/experiments/sync_kinds.py: a noisy ramp under CT7 at 1e-3 up to
// ~20 kbit, a smooth sine at 1e-5 ~80 kbit, CT11 on normal data ~200 kbit, where U10 takes ~1 kbit): parse3's
// repairs then chain over many segments and it declines the stream (status 512 | 2048).  Those streams were
// decoded by the chunk-map decoder, ~5 ms at 2^24 values.  Here, with no walk longer than a group:
//
// maps_group_kernel   256-bit chunks, 32 lanes per chunk: every bit's next token start into LDS, then lane e
//                     steps from entry bit e (a token starts on one of a chunk's first 32 bits) through that
//                     table -> the chunk's entry -> exit map and token count; 8 chunks a group (one wave), whose
//                     map (the 8 maps composed) goes to gmap and, for each of its 32 entries, its chunks'
//                     records (entry | tokens << 8) to gtab.
// maps_scan_kernel    1024 group maps per workgroup: an inclusive scan of the maps inside each wave (register
//                     maps, four-entry v_perm lookups), the 16 wave totals composed; either every map's entry
//                     from the block's entry (ent_in), or the block's total map (a first pass: the block maps,
//                     scanned by the same kernel on one workgroup to get every block's entry).
// maps_rec_kernel     lane = group: the gtab row of the group's entry -> parse3's records (entry, tokens per
//                     chunk), each decode job's first token relative to its parse job and the parse jobs'
//                     totals -- exactly the rec / rel / ptot decode3_kernel reads.
// decode3_kernel then decodes the values as after parse3.  Every walk is bounded by its group, so the path
// never has to meet: the maps are exact whatever the stream.
#include "dc_device.h"

namespace dc {

constexpr int MP_G = 8;                  // chunks per group
constexpr int MP_B = 1024;               // groups per scan workgroup (one per thread)
constexpr int MP_TOPK = 8;               // block maps per thread in the top scan (<= 8192 blocks: 2^26 chunks)

__device__ __forceinline__ uint32_t mp_word(const uint8_t* __restrict__ s, long long nbytes, long long wi) {
    const long long b = 4 * wi;
    if (b + 4 <= nbytes) return __builtin_bswap32(*reinterpret_cast<const uint32_t*>(s + b));
    uint32_t v = 0;
    for (int k = 0; k < 4; k++) v = (v << 8) | (b + k < nbytes && b + k >= 0 ? (uint32_t)s[b + k] : 0u);
    return v;
}

// One wave per group (a grid of at most MP_GRID waves, each looping over groups): the group's 66 stream words
// (8 chunks + the lookahead) are loaded for the next group while the current one is walked; the wave takes its
// 8 chunks two at a time (lanes 0-31 / 32-63), every bit's next token start computed in registers (the token's
// length from its top 9 bits, token_len_bf) into a per-chunk LDS table, then lane e steps from entry bit e
// through it.  No workgroup barrier: with four waves sharing a group and four barriers per group, waves waited
// 72 % of their cycles (SQ counters, sine @1e-5 at 2^24: 463 us) and the table lookups of the lengths conflicted
// on LDS banks.
#ifndef DC_MP_WPG
#define DC_MP_WPG 1                      // waves per workgroup (independent: each its own groups and LDS)
#endif
constexpr int MP_GRID = DC_MP_WPG > 1 ? 12288 : 8192;   // waves (one-wave workgroups: at most 8 per SIMD)
constexpr int MP_GWORDS = MP_G * 8 + 2;                  // a group's stream words with the last chunk's lookahead
template <int CT>
__global__ __launch_bounds__(64 * DC_MP_WPG) void maps_group_kernel(const uint8_t* __restrict__ s, Params P,
                                                        const unsigned long long* dev_nbits, unsigned long long host_nbits,
                                                        uint8_t* __restrict__ gmap, uint4* __restrict__ gtab, long long ngr,
                                                        long long num, long long max_chunks, unsigned* __restrict__ err) {
    __shared__ uint32_t gwa[DC_MP_WPG][MP_GWORDS + 2];
    __shared__ uint16_t nxa[DC_MP_WPG][2][256];                 // the next token's start from every bit
    __shared__ uint8_t gxa[DC_MP_WPG][MP_G][32], gca[DC_MP_WPG][MP_G][32];
    const int wv = threadIdx.x >> 6;
    uint32_t* gw = gwa[wv];
    uint16_t (*nx)[256] = nxa[wv];
    uint8_t (*gx)[32] = gxa[wv];
    uint8_t (*gc)[32] = gca[wv];
    const unsigned long long nbits = dev_nbits ? *dev_nbits : host_nbits;
    const long long nch = (long long)((nbits + 255) >> 8), nbytes = (long long)((nbits + 7) >> 3);
    const int lane = threadIdx.x & 63, h = lane >> 5, e = lane & 31;
    // a runs-mode stream (decode3 would take it for zero runs, which only parse3 checks) or one longer than
    // the buffers: declined to the chunk-map decoder, as parse3 declines it (status 512 | 1024)
    if (blockIdx.x == 0 && threadIdx.x == 0 && (nch > max_chunks || runs_mode(CT, nbits, num))) atomicOr(err, 512u | 1024u);
    const long long gstride = (long long)gridDim.x * DC_MP_WPG;
    long long gi = (long long)blockIdx.x * DC_MP_WPG + wv;
    uint32_t wa = 0u, wb = 0u;                                   // words lane and 64 + lane of the group
    {
        const long long w0 = gi * MP_G * 8;
        if (gi * MP_G < nch) {
            wa = mp_word(s, nbytes, w0 + lane);
            if (lane < MP_GWORDS - 64) wb = mp_word(s, nbytes, w0 + 64 + lane);
        }
    }
    for (; gi < ngr; gi += gstride) {
        const long long g0 = gi * MP_G;
        if (g0 >= nch) {                                         // (past the stream's end: the identity)
            if (h == 0) gmap[gi * 32 + e] = (uint8_t)e;
            continue;
        }
        __builtin_amdgcn_wave_barrier();                         // (the previous group's LDS reads are done)
        gw[lane] = wa;
        if (lane < MP_GWORDS - 64) gw[64 + lane] = wb;
        {
            const long long gn = gi + gstride, w0 = gn * MP_G * 8;
            wa = 0u; wb = 0u;
            if (gn < ngr && gn * MP_G < nch) {
                wa = mp_word(s, nbytes, w0 + lane);
                if (lane < MP_GWORDS - 64) wb = mp_word(s, nbytes, w0 + 64 + lane);
            }
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll 1
        for (int q = 0; q < MP_G / 2; q++) {
            const int j = 2 * q + h;                             // the group's chunk this half-wave walks
            const long long c = g0 + j;
            // every bit's next token start (8 positions per lane, lengths in registers)
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int p = e + 32 * k;
                const uint32_t w0 = gw[8 * j + k], w1 = gw[8 * j + k + 1];
                const uint32_t t = e ? __builtin_amdgcn_alignbit(w0, w1, 32 - e) : w0;
                nx[h][p] = (uint16_t)(p + token_len_bf<CT>(t, P));
            }
            __builtin_amdgcn_wave_barrier();
            const int lim = c < nch ? (int)min(256ll, (long long)nbits - 256 * c) : 0;
            int pos = e, cnt = 0;
            while (pos < lim) { pos = nx[h][pos]; cnt++; }       // (tokens starting before lim)
            gx[j][e] = c < nch ? (uint8_t)((pos - 256) & 31) : (uint8_t)e;   // (identity past the stream's end)
            gc[j][e] = (uint8_t)cnt;
            __builtin_amdgcn_wave_barrier();
        }
        if (h == 0) {
            // from group entry e: the group's exit, and its chunks' records (entry | tokens << 8) for maps_rec_kernel
            int x = e;
            uint32_t r[MP_G / 2] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int j = 0; j < MP_G; j++) {
                r[j >> 1] |= ((uint32_t)x | ((uint32_t)gc[j][x] << 8)) << (16 * (j & 1));
                x = gx[j][x];
            }
            gmap[gi * 32 + e] = (uint8_t)x;
            gtab[gi * 32 + e] = make_uint4(r[0], r[1], r[2], r[3]);
        }
    }
}

// m: a 32-entry map in 8 registers (byte e = entry e's exit); the map at four entries (the bytes of pw, < 32)
__device__ __forceinline__ uint32_t mp_lookup4(const uint32_t (&m)[8], uint32_t pw) {
    const uint32_t sel = pw & 0x07070707u;
    const uint32_t pr = (pw >> 3) & 0x03030303u;
    uint32_t r = __builtin_amdgcn_perm(m[1], m[0], sel);
#pragma unroll
    for (int pp = 1; pp < 4; pp++) {
        const uint32_t c = __builtin_amdgcn_perm(m[2 * pp + 1], m[2 * pp], sel);
        const uint32_t t = pr ^ (0x01010101u * (uint32_t)pp);
        const uint32_t msk = ((((t | (t >> 1)) & 0x01010101u) ^ 0x01010101u)) * 0xFFu;
        r = (c & msk) | (r & ~msk);
    }
    return r;
}
__device__ __forceinline__ void mp_load(const uint8_t* __restrict__ maps, long long i, long long n, uint32_t (&m)[8]) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(maps);
#pragma unroll
    for (int q = 0; q < 8; q++) m[q] = i < n ? p[i * 8 + q] : 0x03020100u + 0x04040404u * (uint32_t)q;   // (identity)
}
// later o earlier: (m after a) = a's map first, then m -- m[e] <- m[a[e]]
__device__ __forceinline__ void mp_after(uint32_t (&m)[8], const uint32_t (&a)[8]) {
    uint32_t nm[8];
#pragma unroll
    for (int q = 0; q < 8; q++) nm[q] = mp_lookup4(m, a[q]);
#pragma unroll
    for (int q = 0; q < 8; q++) m[q] = nm[q];
}

// Workgroup b scans maps [b K MP_B, (b + 1) K MP_B) (thread i: K consecutive maps composed).  ent_in: the entry
// of the workgroup's first map (ent_in[b], or 0 when null) -> ent_out[map] = the entry of every map; else
// tot_out[b] = the workgroup's total map.
template <int K>
__global__ __launch_bounds__(MP_B) void maps_scan_kernel(const uint8_t* __restrict__ maps, const long long* n_in,
                                                        const uint8_t* __restrict__ ent_in, uint8_t* __restrict__ ent_out,
                                                        uint8_t* __restrict__ tot_out) {
    __shared__ uint32_t tot[MP_B / 64][8];
    __shared__ uint32_t went[MP_B / 64];
    const int i = threadIdx.x, lane = i & 63, wv = i >> 6;
    const long long n = *n_in;
    const long long base = (long long)blockIdx.x * K * MP_B + (long long)i * K;
    if ((long long)blockIdx.x * K * MP_B >= n) return;
    uint32_t m[8];
    mp_load(maps, base, n, m);
#pragma unroll
    for (int k = 1; k < K; k++) {                                // (this thread's maps, in order)
        uint32_t a[8];
        mp_load(maps, base + k, n, a);
        // m so far is earlier: new m = a after m
        uint32_t nm[8];
#pragma unroll
        for (int q = 0; q < 8; q++) nm[q] = mp_lookup4(a, m[q]);
#pragma unroll
        for (int q = 0; q < 8; q++) m[q] = nm[q];
    }
    const uint32_t own[8] = {m[0], m[1], m[2], m[3], m[4], m[5], m[6], m[7]};
    // inclusive scan inside the wave: X_i <- X_i o X_{i-d} (X_{i-d} applied first)
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t pw[8];
#pragma unroll
        for (int q = 0; q < 8; q++) pw[q] = __shfl_up(m[q], d, 64);
        if (lane >= d) mp_after(m, pw);
    }
    if (lane == 63) {
#pragma unroll
        for (int q = 0; q < 8; q++) tot[wv][q] = m[q];
    }
    __syncthreads();
    if (tot_out) {                                               // the workgroup's total: entries through the waves
        if (i < 32) {
            uint32_t x = (uint32_t)i;
            for (int w = 0; w < MP_B / 64; w++) x = (tot[w][x >> 2] >> (8 * (x & 3))) & 31u;
            tot_out[blockIdx.x * 32 + i] = (uint8_t)x;
        }
        return;
    }
    if (i == 0) {                                                // each wave's entry
        uint32_t v = ent_in ? ent_in[blockIdx.x] & 31u : 0u;
        for (int w = 0; w < MP_B / 64; w++) {
            went[w] = v;
            v = (tot[w][v >> 2] >> (8 * (v & 3))) & 31u;
        }
    }
    __syncthreads();
    const uint32_t vin = went[wv];
    // this thread's first map's entry: the inclusive map of the previous lane at the wave's entry
    const uint32_t zin = mp_lookup4(m, vin) & 31u;               // (inclusive through this lane)
    const int yp = __shfl_up((int)zin, 1, 64);
    uint32_t y = lane == 0 ? vin : (uint32_t)yp;
#pragma unroll
    for (int k = 0; k < K; k++) {                                // the entries of this thread's K maps
        if (base + k < n) ent_out[base + k] = (uint8_t)y;
        if (k + 1 < K) {
            uint32_t a[8];
            mp_load(maps, base + k, n, a);
            y = (a[y >> 2] >> (8 * (y & 3))) & 31u;
        }
    }
    (void)own;
}

// lane = group: its chunks' records (entry | tokens << 8) for the group's entry, from the group kernel's table ->
// rec, the tokens of each decode job (64 chunks = 8 groups) and of each parse job (seg decode jobs): rel[decode
// job] = tokens before it in its parse job, ptot[parse job]
__global__ __launch_bounds__(MP_B) void maps_rec_kernel(const unsigned long long* dev_nbits, unsigned long long host_nbits,
                                                       const uint8_t* __restrict__ gent, const uint4* __restrict__ gtab,
                                                       Dec3Bufs D3) {
    __shared__ uint32_t djt[MP_B / 8];                           // tokens per decode job
    const unsigned long long nbits = dev_nbits ? *dev_nbits : host_nbits;
    const long long nch = (long long)((nbits + 255) >> 8);
    const long long g = (long long)blockIdx.x * MP_B + threadIdx.x, c0 = g * MP_G;
    if ((long long)blockIdx.x * MP_B * MP_G >= nch) return;
    uint32_t tot = 0;
    if (c0 < nch) {
        const uint4 q = gtab[g * 32 + (gent[g] & 31u)];
        const uint32_t rec[MP_G / 2] = {q.x, q.y, q.z, q.w};
        uint32_t* r32 = reinterpret_cast<uint32_t*>(D3.rec);
#pragma unroll
        for (int j = 0; j < MP_G / 2; j++) {
            tot += ((rec[j] >> 8) & 0xFFu) + (rec[j] >> 24);
            if (c0 + 2 * j < nch) r32[(c0 >> 1) + j] = c0 + 2 * j + 1 < nch ? rec[j] : rec[j] & 0xFFFFu;
        }
    }
    // decode jobs: 8 consecutive lanes
    uint32_t v = tot;
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    if ((threadIdx.x & 7) == 0) djt[threadIdx.x >> 3] = v;
    __syncthreads();
    const int seg = D3.seg;
    if (threadIdx.x < MP_B / 8) {
        const int j = threadIdx.x;
        const long long dj = (long long)blockIdx.x * (MP_B / 8) + j;
        const int j0 = j - j % seg;                              // the parse job's first decode job here
        uint32_t rel = 0;
        for (int k = j0; k < j; k++) rel += djt[k];
        if (dj * 64 < D3.max_chunks) D3.rel[dj] = rel;
        if (j % seg == seg - 1) D3.ptot[dj / seg] = rel + djt[j];
    }
}

// scratch bytes of the maps parse for streams of up to max_chunks 256-bit chunks
extern "C" long long dc_maps_scratch_bytes(long long max_chunks) {
    const long long ngr = (max_chunks + MP_G - 1) / MP_G + MP_B, nb = ngr / MP_B + 8;
    return ngr * 32 + ngr + nb * 32 + nb + 64 + 16 + ngr * 32 * 16;
}

// the parse-job length (decode jobs) the maps parse writes ptot / rel for: the segment decoder's when it divides a
// scan workgroup's 128 decode jobs, else 16 (dc_launch_decode3_values decodes with the same)
extern "C" int dc_maps_seg(int seg) { return (MP_B / 8) % seg == 0 ? seg : 16; }

extern "C" int dc_launch_maps_parse(const uint8_t* s, const unsigned long long* dev_nbits, unsigned long long host_nbits,
                                    const Params* P, const Dec3Bufs* D3in, long long num, void* scratch, hipStream_t st) {
    Dec3Bufs Dv = *D3in;
    const Dec3Bufs* D3 = &Dv;
    Dv.seg = dc_maps_seg(D3in->seg);
    const long long ngr = (D3->max_chunks + MP_G - 1) / MP_G, nb = (ngr + MP_B - 1) / MP_B;
    if (nb > (long long)MP_TOPK * MP_B || (MP_B / 8) % D3->seg) return -2;
    uint8_t* gmap = (uint8_t*)scratch;
    uint8_t* gent = gmap + (ngr + MP_B) * 32;
    uint8_t* bmap = gent + ngr + MP_B;
    uint8_t* bent = bmap + (nb + 8) * 32;
    long long* cnt = reinterpret_cast<long long*>(((uintptr_t)(bent + nb + 8) + 7) & ~(uintptr_t)7);
    uint4* gtab = reinterpret_cast<uint4*>(((uintptr_t)(cnt + 2) + 15) & ~(uintptr_t)15);   // [group][entry]
    // the group and block counts of this stream (its length may be on the device): one tiny kernel would do;
    // the scans take their counts from device memory, written here from the capacity (groups past the
    // stream's end have identity maps and are never read)
    const long long hc[2] = {ngr, nb};
    if (hipMemcpyAsync(cnt, hc, sizeof hc, hipMemcpyHostToDevice, st) != hipSuccess) return -1;
    const dim3 gg((unsigned)((min(ngr, (long long)MP_GRID) + DC_MP_WPG - 1) / DC_MP_WPG)), gb((unsigned)nb);
    switch (P->ct) {
#define DC_MAPS_CASE(C)                                                                                          \
    case C:                                                                                                      \
        hipLaunchKernelGGL(maps_group_kernel<C>, gg, dim3(64 * DC_MP_WPG), 0, st, s, *P, dev_nbits, host_nbits, gmap, gtab, \
                           ngr, num, D3->max_chunks, D3->err);                                                      \
        break;
        DC_MAPS_CASE(5) DC_MAPS_CASE(6) DC_MAPS_CASE(7) DC_MAPS_CASE(11)
        default: return -2;
    }
    hipLaunchKernelGGL(maps_scan_kernel<1>, gb, dim3(MP_B), 0, st, gmap, cnt, nullptr, nullptr, bmap);
    if (nb <= MP_B)                                              // (the block maps: one per thread)
        hipLaunchKernelGGL(maps_scan_kernel<1>, dim3(1), dim3(MP_B), 0, st, bmap, cnt + 1, nullptr, bent, nullptr);
    else
        hipLaunchKernelGGL(maps_scan_kernel<MP_TOPK>, dim3(1), dim3(MP_B), 0, st, bmap, cnt + 1, nullptr, bent, nullptr);
    hipLaunchKernelGGL(maps_scan_kernel<1>, gb, dim3(MP_B), 0, st, gmap, cnt, bent, gent, nullptr);
#undef DC_MAPS_CASE
    hipLaunchKernelGGL(maps_rec_kernel, gb, dim3(MP_B), 0, st, dev_nbits, host_nbits, gent, gtab, *D3);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace dc
