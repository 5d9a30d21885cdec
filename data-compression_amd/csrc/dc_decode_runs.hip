// dc_decode_runs.hip -- the small-stream decoder: every stream of at most RUNS_MAXC 256-bit chunks
// (256 KiB), among them the Himeno halo planes of BASELINE config 4 (runs-mode streams of '101' copy
// runs, which the segment decoder cannot take: paths read out of phase in a period-3 stream never meet).
// It decodes the grammar of impl/dataCompression.c (myDecompress_bitwise :2922-3135, _np :2459-2630,
// _mask :1703-2027, _op :698-797) in three launches and no host read:
//
// runs_map_kernel     32 lanes per chunk, lane e walks the chunk from entry bit e (a token boundary can
//                     fall on any of the chunk's first 32 bits: tokens are at most 32 bits) and records
//                     the exit (the entry of the next chunk, 0..31) and the tokens it started: the chunk's
//                     entry->exit map and counts.  Runs of 3-bit codes are stepped ten at a time.
// runs_scan_kernel    one workgroup of 1024 threads, thread = a block of consecutive chunks:
//                     (1) the block's entry->exit map (its chunk maps composed), (2) a block scan of the
//                     maps -- function composition is associative -- gives every block its true entry (the
//                     stream starts at bit 0), (3) chunk entries and token counts, a scan of the counts,
//                     (4) pass 1 decodes the block with its incoming history symbolic (each of the three
//                     values before the block: a slot), so its last three values are constants or copies
//                     of a slot -- '101' copies a slot, '100' and raw tokens are constants; a '110'/'111'
//                     prediction from a slot would be a float expression, and if one reaches the block's
//                     last three values the stream goes to the chunk-map decoder -- reading the stream from
//                     LDS (staged once, up to 112 KiB), (5) a block scan of those carries (slot maps compose
//                     associatively) gives every block its concrete incoming history.
// runs_values_kernel  thread = block, 16 workgroups: the block's values from its entry and incoming history
//                     (the stores of one workgroup were the scan kernel's slowest part).
// A stream outside these assumptions (longer than RUNS_MAXC chunks, fewer tokens than values, a carry that
// is a float expression of its slots, a prediction among the stream's first three tokens, the -1.0f
// history sentinel) sets status 512 and is decoded by the chunk-map decoder in dc_decode_finish.
#include "dc_device.h"

namespace dc {

constexpr int RUNS_MAXC = 8192;                 // chunks of 256 bits: 256 KiB of stream
constexpr int RUNS_T = 1024;                    // threads of the decode workgroup
constexpr int RUNS_BMAX = RUNS_MAXC / RUNS_T;   // chunks per thread at most
constexpr uint32_t RUNS_DECLINE = 512u;
constexpr uint32_t RUNS_WHY_SIZE = 1u << 17, RUNS_WHY_SHORT = 1u << 18, RUNS_WHY_EXPR = 1u << 19,
                   RUNS_WHY_SENT = 1u << 20;

typedef unsigned rs_u32x4 __attribute__((ext_vector_type(4)));

// the stream's 32-bit words (MSB-first), bytes past the stream's end read as 0 (as the reference's reader)
__device__ __forceinline__ uint32_t rs_word(const uint8_t* __restrict__ s, long long nbytes, long long wi) {
    const long long b = 4 * wi;
    if (b + 4 <= nbytes) return __builtin_bswap32(*reinterpret_cast<const uint32_t*>(s + b));
    uint32_t v = 0;
    for (int k = 0; k < 4; k++) v = (v << 8) | (b + k < nbytes && b + k >= 0 ? (uint32_t)s[b + k] : 0u);
    return v;
}

struct RunsBufs {
    uint8_t* exitm;                 // [chunk][32] exit bit of the walk entered at bit e
    uint8_t* cntm;                  // [chunk][32] tokens that walk starts in the chunk
    uint4* blk;                     // [block] first chunk's entry | chunks << 8, first token
    float4* bhist;                  // [block] incoming history b1, b2, b3
    uint8_t* bcnt;                  // [block][RUNS_BMAX] tokens of its chunks
    unsigned* err;                  // the decoder status word (shared with the other decoders)
};

template <int CT>
__global__ __launch_bounds__(256) void runs_map_kernel(const uint8_t* __restrict__ s, Params P, RunsBufs R,
                                                       const unsigned long long* dev_nbits,
                                                       unsigned long long host_nbits) {
    __shared__ uint32_t w[8][10];
    const unsigned long long nbits = dev_nbits ? *dev_nbits : host_nbits;
    const long long nch = (long long)((nbits + 255) >> 8), nbytes = (long long)((nbits + 7) >> 3);
    if (nch > RUNS_MAXC) {
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(R.err, RUNS_DECLINE | RUNS_WHY_SIZE);
        return;
    }
    const int h = threadIdx.x >> 5, e = threadIdx.x & 31;
    const long long c = (long long)blockIdx.x * 8 + h;
    if (e < 10) w[h][e] = c < nch ? rs_word(s, nbytes, 8 * c + e) : 0u;
    __syncthreads();
    if (c >= nch) return;
    // tokens that start before the stream's end (the last byte's padding is not a token start of the
    // true path; a walk counting one more there only ever runs past num, see runs_decode_kernel)
    const int lim = (int)min(256ll, (long long)nbits - 256 * c);
    int pos = e, cnt = 0;
    while (pos < lim) {
        const int wi = pos >> 5, sh = pos & 31;
        const uint32_t t = sh ? __builtin_amdgcn_alignbit(w[h][wi], w[h][wi + 1], 32 - sh) : w[h][wi];
        if (CT != 6 && (int)t < 0) {
            const int k = run3i(t, pos, lim);
            pos += 3 * k;
            cnt += k;
        } else {
            pos += token_len_bf<CT>(t, P);
            cnt++;
        }
    }
    R.exitm[c * 32 + e] = (uint8_t)((pos - 256) & 31);
    R.cntm[c * 32 + e] = (uint8_t)cnt;
}

// a history slot of pass 1: kind 0 = the constant v, 1..3 = the k-th value before the block (b1..b3),
// 4 = a float expression of those (a '110'/'111' prediction from a slot)
struct Hs {
    uint32_t k;
    float v;
};

// the stream words a reader needs: from LDS when the whole stream was staged there, else from global
struct RsWords {
    const uint32_t* lw;             // staged words (nullptr: read global), lw[0] = stream word `base`
    const uint8_t* s;
    long long nbytes;
    long long base;
    __device__ __forceinline__ uint32_t at(long long wi) const {
        return lw ? lw[wi - base] : rs_word(s, nbytes, wi);
    }
    __device__ __forceinline__ uint32_t peek(long long pos) const {
        const long long wi = pos >> 5;
        const int sh = (int)(pos & 31);
        const uint32_t w0 = at(wi);
        return sh ? __builtin_amdgcn_alignbit(w0, at(wi + 1), 32 - sh) : w0;
    }
};

// one block's tokens from its first chunk's entry, the incoming history h (pass 1: symbolic slots; the
// values kernel: constants), values to out when STORE (and their history constant).  Returns the history
// after the block.
template <int CT, bool STORE>
__device__ __forceinline__ void block_walk(const RsWords& W, const Params& P, long long c0, long long c1, int entry,
                                           const uint8_t* cn, long long g, long long num, unsigned long long nbits,
                                           Hs& h1, Hs& h2, Hs& h3, bool& sent, float* __restrict__ out) {
    long long pos = 256 * c0 + entry;
    for (int j = 0; j < RUNS_BMAX && g < num; j++) {
        const long long c = c0 + j;
        if (c >= c1) break;
        const int lim = (int)min(256ll, (long long)nbits - 256 * c);
        int left = cn[j];
        while (left > 0 && g < num) {
            const uint32_t t = W.peek(pos);
            int k = CT != 6 ? run_same(t, (int)(pos - 256 * c), lim, left) : 1;
            k = (int)min((long long)k, num - g);
            if (CT != 6 && k > 1) {                             // a run of identical '100' / '101' codes
                const Hs v = (t >> 29) == 4u ? Hs{0u, 0.0f} : h1;
                if ((t >> 29) == 5u && g < 3) sent = true;      // a prediction among the stream's first three
                if (STORE)
                    for (int q = 0; q < k; q++) out[g + q] = v.v;
                h3 = k == 2 ? h1 : v;                           // (two tokens keep the value before them)
                h2 = v; h1 = v;
                pos += 3 * k;
                g += k;
                left -= k;
                continue;
            }
            const int len = token_len_bf<CT>(t, P);
            int code = 0;
            const uint32_t u = token_pattern_bf<CT>(t, len, P, &code);
            Hs v;
            if (code == 0) {
                v = Hs{0u, __uint_as_float(u)};
            } else {
                if (g < 3) sent = true;
                if (code == 1) v = h1;
                else if (h1.k == 0 && h2.k == 0 && (code == 2 || h3.k == 0))
                    v = Hs{0u, predict_value(code, h1.v, h2.v, h3.v)};
                else
                    v = Hs{4u, 0.0f};
            }
            if (v.k == 0 && __float_as_uint(v.v) == 0xBF800000u) sent = true;   // the history sentinel
            if (STORE) out[g] = v.v;
            h3 = h2; h2 = h1; h1 = v;
            pos += len;
            g++;
            left--;
        }
    }
}

constexpr int RUNS_SW = 28 * 1024;              // stream words staged in LDS (112 KiB; larger: global reads)

// one workgroup: block maps and their scan, entries and token offsets, pass 1 (carries), carry scan ->
// per block: first chunk entry, first token, token count, concrete incoming history (RunsBufs.blk)
template <int CT>
__global__ __launch_bounds__(RUNS_T) void runs_scan_kernel(const uint8_t* __restrict__ s, Params P, RunsBufs R,
                                                          const unsigned long long* dev_nbits,
                                                          unsigned long long host_nbits, long long num) {
    __shared__ uint32_t pool[RUNS_SW];                          // block maps (steps 1-2), then the stream
    __shared__ uint32_t ctA[RUNS_T], ctB[RUNS_T];               // token count scan
    __shared__ uint32_t hkA[RUNS_T], hkB[RUNS_T];               // carry kinds (3 x 8 bits)
    __shared__ float hvA[RUNS_T * 3], hvB[RUNS_T * 3];          // carry constants
    __shared__ int bad;
    static_assert(2 * RUNS_T * 8 <= RUNS_SW, "the map double buffer fits the pool");
    const int i = threadIdx.x;
    const unsigned long long nbits = dev_nbits ? *dev_nbits : host_nbits;
    const long long nch = (long long)((nbits + 255) >> 8), nbytes = (long long)((nbits + 7) >> 3);
    if (i == 0) bad = 0;
    __syncthreads();
    if (nch > RUNS_MAXC || (__hip_atomic_load(R.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & RUNS_DECLINE))
        return;
    const int Bc = (int)((nch + RUNS_T - 1) / RUNS_T);          // chunks per thread (<= RUNS_BMAX)
    const long long c0 = (long long)i * Bc, c1 = min(c0 + Bc, nch);

    // (1) the block's map: entry bit e of its first chunk -> entry bit of the chunk after it
    uint8_t bm[32];
#pragma unroll
    for (int e = 0; e < 32; e++) bm[e] = (uint8_t)e;
    for (long long c = c0; c < c1; c++) {
#pragma unroll
        for (int e = 0; e < 32; e++) bm[e] = R.exitm[c * 32 + bm[e]];
    }
    uint32_t* cur = pool;
    uint32_t* nxt = pool + RUNS_T * 8;
#pragma unroll
    for (int q = 0; q < 8; q++)
        cur[i * 8 + q] = (uint32_t)bm[4 * q] | (uint32_t)bm[4 * q + 1] << 8 | (uint32_t)bm[4 * q + 2] << 16 |
                         (uint32_t)bm[4 * q + 3] << 24;
    __syncthreads();
    // (2) inclusive scan of the maps (X_i <- X_i o X_{i-d}: X_{i-d} applied first)
    for (int d = 1; d < RUNS_T; d <<= 1) {
        const uint8_t* mine = reinterpret_cast<const uint8_t*>(cur + i * 8);
#pragma unroll
        for (int q = 0; q < 8; q++) {
            uint32_t v = cur[i * 8 + q];
            if (i >= d) {
                const uint32_t pw = cur[(i - d) * 8 + q];
                v = (uint32_t)mine[pw & 31u] | (uint32_t)mine[(pw >> 8) & 31u] << 8 |
                    (uint32_t)mine[(pw >> 16) & 31u] << 16 | (uint32_t)mine[(pw >> 24) & 31u] << 24;
            }
            nxt[i * 8 + q] = v;
        }
        __syncthreads();
        uint32_t* t = cur; cur = nxt; nxt = t;
    }
    // the block's entry: the maps of every block before it applied to bit 0
    const int y = i == 0 ? 0 : (int)(reinterpret_cast<const uint8_t*>(cur + (i - 1) * 8)[0]);
    __syncthreads();                                            // (the pool takes the stream next)

    // the stream into LDS when it fits (coalesced 16-byte loads), for pass 1's walks
    const long long nw = (long long)((nbits + 31) >> 5) + 2;
    const bool staged = nw <= RUNS_SW;
    if (staged) {
        for (long long q = i; q < nw; q += RUNS_T) pool[q] = rs_word(s, nbytes, q);
    }
    // (3) chunk entries and token counts (needed by pass 1 and the values kernel)
    uint8_t cn[RUNS_BMAX];
    uint32_t nblk = 0;
    {
        int x = y;
#pragma unroll
        for (int j = 0; j < RUNS_BMAX; j++) {
            const long long c = c0 + j;
            cn[j] = 0;
            if (c < c1) {
                cn[j] = R.cntm[c * 32 + x];
                x = R.exitm[c * 32 + x];
                nblk += cn[j];
            }
        }
    }
    uint32_t* ca = ctA;
    uint32_t* cb = ctB;
    ca[i] = nblk;
    __syncthreads();
    for (int d = 1; d < RUNS_T; d <<= 1) {
        cb[i] = ca[i] + (i >= d ? ca[i - d] : 0u);
        __syncthreads();
        uint32_t* t = ca; ca = cb; cb = t;
    }
    const long long T0 = (long long)ca[i] - nblk;               // the block's first token
    const long long total = ca[RUNS_T - 1];
    if (total < num) {                                          // fewer tokens than values: the reference
        if (i == 0) atomicOr(R.err, RUNS_DECLINE | RUNS_WHY_SHORT);   // reads zeros past the end -> other path
        return;
    }
    // (4) pass 1: the block with symbolic incoming history -> its carry (last three values)
    RsWords W{staged ? pool : nullptr, s, nbytes, 0};
    Hs h1 = {1u, 0.f}, h2 = {2u, 0.f}, h3 = {3u, 0.f};
    bool sent = false;
    if (c0 < c1) block_walk<CT, false>(W, P, c0, c1, y, cn, T0, num, nbits, h1, h2, h3, sent, nullptr);
    if (h1.k == 4u || h2.k == 4u || h3.k == 4u) atomicOr(&bad, 1);
    if (sent) atomicOr(&bad, 2);
    // (5) scan of the carries: slot map composition (later o earlier)
    uint32_t* ka = hkA;
    uint32_t* kb = hkB;
    float* va = hvA;
    float* vb = hvB;
    ka[i] = h1.k | h2.k << 8 | h3.k << 16;
    va[3 * i] = h1.v; va[3 * i + 1] = h2.v; va[3 * i + 2] = h3.v;
    __syncthreads();
    if (bad) {
        if (i == 0) atomicOr(R.err, RUNS_DECLINE | ((bad & 1) ? RUNS_WHY_EXPR : 0u) | ((bad & 2) ? RUNS_WHY_SENT : 0u));
        return;
    }
    for (int d = 1; d < RUNS_T; d <<= 1) {
        uint32_t kk = ka[i];
        float v0 = va[3 * i], v1 = va[3 * i + 1], v2 = va[3 * i + 2];
        if (i >= d) {
            const uint32_t ek = ka[i - d];
            float r[3] = {v0, v1, v2};
            uint32_t nk = 0;
#pragma unroll
            for (int q = 0; q < 3; q++) {
                const uint32_t sk = (kk >> (8 * q)) & 0xFFu;
                if (sk >= 1u && sk <= 3u) {                     // a copy of the earlier carry's slot sk
                    nk |= ((ek >> (8 * (sk - 1))) & 0xFFu) << (8 * q);
                    r[q] = va[3 * (i - d) + (sk - 1)];
                } else {
                    nk |= sk << (8 * q);
                }
            }
            kk = nk; v0 = r[0]; v1 = r[1]; v2 = r[2];
        }
        kb[i] = kk;
        vb[3 * i] = v0; vb[3 * i + 1] = v1; vb[3 * i + 2] = v2;
        __syncthreads();
        uint32_t* t = ka; ka = kb; kb = t;
        float* tv = va; va = vb; vb = tv;
    }
    // the block's incoming history: every block before it (the stream starts with none -- a prediction
    // there declined above -- so remaining slot references read 0)
    float b1 = 0.f, b2 = 0.f, b3 = 0.f;
    if (i > 0) {
        const uint32_t kk = ka[i - 1];
        b1 = ((kk & 0xFFu) == 0u) ? va[3 * (i - 1)] : 0.f;
        b2 = (((kk >> 8) & 0xFFu) == 0u) ? va[3 * (i - 1) + 1] : 0.f;
        b3 = (((kk >> 16) & 0xFFu) == 0u) ? va[3 * (i - 1) + 2] : 0.f;
    }
    R.blk[i] = make_uint4((uint32_t)y | (uint32_t)(c1 > c0 ? c1 - c0 : 0) << 8, (uint32_t)T0, 0u, 0u);
    R.bhist[i] = make_float4(b1, b2, b3, 0.0f);
#pragma unroll
    for (int j = 0; j < RUNS_BMAX; j++) R.bcnt[i * RUNS_BMAX + j] = cn[j];
}

// thread = block: its values from its first chunk's entry with the concrete incoming history
template <int CT>
__global__ __launch_bounds__(64) void runs_values_kernel(const uint8_t* __restrict__ s, Params P, RunsBufs R,
                                                        const unsigned long long* dev_nbits,
                                                        unsigned long long host_nbits, float* __restrict__ out,
                                                        long long num) {
    constexpr int ROW = 8 * RUNS_BMAX + 2;                      // a block's stream words (+ 2 past its end)
    __shared__ uint32_t kw[64 * ROW];
    const unsigned long long nbits = dev_nbits ? *dev_nbits : host_nbits;
    const long long nch = (long long)((nbits + 255) >> 8), nbytes = (long long)((nbits + 7) >> 3);
    if (nch > RUNS_MAXC || (__hip_atomic_load(R.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & RUNS_DECLINE))
        return;
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= RUNS_T) return;
    const int Bc = (int)((nch + RUNS_T - 1) / RUNS_T);
    const long long c0 = (long long)i * Bc;
    const uint4 b = R.blk[i];
    const int nc = (int)(b.x >> 8);
    if (nc <= 0) return;
    // the block's words into this lane's LDS row (independent loads, all in flight), read back per token
    uint32_t* row = kw + threadIdx.x * ROW;
    for (int q = 0; q < 8 * nc + 2; q++) row[q] = rs_word(s, nbytes, 8 * c0 + q);
    const float4 hb = R.bhist[i];
    uint8_t cn[RUNS_BMAX];
#pragma unroll
    for (int j = 0; j < RUNS_BMAX; j++) cn[j] = R.bcnt[i * RUNS_BMAX + j];
    Hs h1 = {0u, hb.x}, h2 = {0u, hb.y}, h3 = {0u, hb.z};
    bool sent = false;
    RsWords W{row, s, nbytes, 8 * c0};
    block_walk<CT, true>(W, P, c0, c0 + nc, (int)(b.x & 0xFFu), cn, (long long)b.y, num, nbits, h1, h2, h3, sent, out);
    if (sent) atomicOr(R.err, RUNS_DECLINE | RUNS_WHY_SENT);
}

extern "C" int dc_launch_decode_runs(const uint8_t* s, const unsigned long long* dev_nbits, unsigned long long host_nbits,
                                     long long max_chunks, const Params* P, uint8_t* maps, unsigned* err, float* out,
                                     long long num, hipStream_t st) {
    if (max_chunks > RUNS_MAXC + 8 || max_chunks < 1) return -2;     // (the stream's own length is checked on the device)
    RunsBufs R;
    const size_t mb = (size_t)(RUNS_MAXC + 8) * 32;
    R.exitm = maps;
    R.cntm = maps + mb;
    R.blk = reinterpret_cast<uint4*>(maps + 2 * mb);
    R.bhist = reinterpret_cast<float4*>(maps + 2 * mb + 16 * RUNS_T);
    R.bcnt = maps + 2 * mb + 32 * RUNS_T;
    R.err = err;
    const int g1 = (int)((max_chunks + 7) / 8);
    dc_mark_phase(4, st);
    switch (P->ct) {
#define DC_RUNS_CASE(C)                                                                                        \
    case C:                                                                                                    \
        hipLaunchKernelGGL(runs_map_kernel<C>, dim3(g1), dim3(256), 0, st, s, *P, R, dev_nbits, host_nbits);   \
        hipLaunchKernelGGL(runs_scan_kernel<C>, dim3(1), dim3(RUNS_T), 0, st, s, *P, R, dev_nbits, host_nbits, \
                           num);                                                                               \
        dc_mark_phase(5, st);                                                                                  \
        hipLaunchKernelGGL(runs_values_kernel<C>, dim3(RUNS_T / 64), dim3(64), 0, st, s, *P, R, dev_nbits,     \
                           host_nbits, out, num);                                                              \
        break;
        DC_RUNS_CASE(5)
        DC_RUNS_CASE(6)
        DC_RUNS_CASE(7)
        DC_RUNS_CASE(11)
#undef DC_RUNS_CASE
        default: return -2;
    }
    dc_mark_phase(7, st);
    dc_mark_next_set();
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
extern "C" long long dc_decode_runs_max_chunks(void) { return RUNS_MAXC; }
extern "C" size_t dc_decode_runs_scratch_bytes(void) {
    return (size_t)(RUNS_MAXC + 8) * 32 * 2 + (size_t)RUNS_T * (16 + 16 + RUNS_BMAX);
}

}  // namespace dc
