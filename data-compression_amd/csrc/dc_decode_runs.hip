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
    uint8_t* pm;                    // [chunk][32] group-first entry -> the chunk's entry (8-chunk groups)
    uint8_t* gmap;                  // [group][32] group-first entry -> the next group's entry
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
    // tokens that start before the stream's end (the last byte's padding is not a token start of the
    // true path; a walk counting one more there only ever runs past num, see runs_decode_kernel)
    const int lim = c < nch ? (int)min(256ll, (long long)nbits - 256 * c) : 0;   // (past the stream: no walk)
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
    if (c >= nch) pos = 256 + e;                                // (identity past the stream's end)
    const uint8_t ex = (uint8_t)((pos - 256) & 31);
    if (c < nch) {
        R.exitm[c * 32 + e] = ex;
        R.cntm[c * 32 + e] = (uint8_t)cnt;
    }
    // the workgroup's 8 chunks are a group: every chunk's prefix map inside the group (entry of the
    // group's first chunk -> the chunk's entry) and the group's map, so the scan kernel scans groups
    __shared__ uint8_t gx[8][32];
    gx[h][e] = ex;
    __syncthreads();
    if (h == 0) {
        int x = e;
        const long long g0 = (long long)blockIdx.x * 8;
        for (int j = 0; j < 8; j++) {
            if (g0 + j < nch) R.pm[(g0 + j) * 32 + e] = (uint8_t)x;
            x = gx[j][x];
        }
        R.gmap[blockIdx.x * 32 + e] = (uint8_t)x;
    }
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
    int pad;                        // 1: word w staged at w + w/8 (the scan kernel's whole-stream copy)
    __device__ __forceinline__ uint32_t at(long long wi) const {
        if (!lw) return rs_word(s, nbytes, wi);
        const long long q = wi - base;
        return lw[pad ? q + (q >> 3) : q];
    }
    __device__ __forceinline__ uint32_t peek(long long pos) const {
        const long long wi = pos >> 5;
        const int sh = (int)(pos & 31);
        const uint32_t w0 = at(wi);
        return sh ? __builtin_amdgcn_alignbit(w0, at(wi + 1), 32 - sh) : w0;
    }
};

// (r06) the values kernel's scatter mode: value g of a Himeno halo plane goes to its element of the array, plus the
// plane's minimum (the plane_scatter_kernel pass fused into the decode, impl/himenoBMTxps.c:699-706)
struct RunsScatter {
    float* p;
    const float* dmin;
    int mj, mk, ijk, v, B;
};

// one block's tokens from its first chunk's entry, the incoming history h (pass 1: symbolic slots; the
// values kernel: constants), values stored when STORE (1: out[g]; 2: the plane element of S, + mn) and their
// history constant.  Returns the history after the block.
template <int CT, int STORE>
__device__ __forceinline__ void block_walk(const RsWords& W, const Params& P, long long c0, long long c1, int entry,
                                           const uint8_t* cn, long long g, long long num, unsigned long long nbits,
                                           Hs& h1, Hs& h2, Hs& h3, bool& sent, float* __restrict__ out,
                                           const RunsScatter& S = RunsScatter{}, float mn = 0.0f) {
    auto put = [&](long long e, float x) {
        if (STORE == 1) {
            out[e] = x;
        } else if (STORE == 2) {
            const int a = (int)e / S.B;                     // (a plane holds < 2^31 values)
            S.p[plane_index(a, (int)e - a * S.B, S.ijk, S.v, S.mj, S.mk)] = __fadd_rn(x, mn);
        }
    };
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
                    for (int q = 0; q < k; q++) put(g + q, v.v);
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
            if (STORE) put(g, v.v);
            h3 = h2; h2 = h1; h1 = v;
            pos += len;
            g++;
            left--;
        }
    }
}

#ifdef DC_RUNS_PROF
__device__ unsigned long long g_runs_prof[16];
#define RSTAMP(k) do { if (threadIdx.x == 0) g_runs_prof[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define RSTAMP(k) do {} while (0)
#endif
extern "C" int dc_runs_prof_read(unsigned long long* out) {
#ifdef DC_RUNS_PROF
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_runs_prof), sizeof g_runs_prof) == hipSuccess ? 0 : -1;
#else
    (void)out;
    return -1;
#endif
}

constexpr int RUNS_SW = 28 * 1024;              // stream words staged in LDS (112 KiB; larger: global reads)

// one workgroup: block maps and their scan, entries and token offsets, pass 1 (carries), carry scan ->
// per block: first chunk entry, first token, token count, concrete incoming history (RunsBufs.blk)
template <int CT>
__global__ __launch_bounds__(RUNS_T) void runs_scan_kernel(const uint8_t* __restrict__ s, Params P, RunsBufs R,
                                                          const unsigned long long* dev_nbits,
                                                          unsigned long long host_nbits, long long num) {
    __shared__ uint32_t pool[RUNS_SW];                          // block maps (steps 1-2), then the stream
    __shared__ uint32_t ctA[RUNS_T / 64], ctB[RUNS_T / 64 + 1];    // wave token totals, their offsets
    __shared__ uint32_t hkA[RUNS_T / 64];                           // wave carries: kinds (3 x 8 bits)
    __shared__ float hvA[RUNS_T / 64 * 3], hvB[RUNS_T / 64 * 3];    // their constants, wave histories
    __shared__ int bad;
    static_assert(2 * RUNS_T * 8 <= RUNS_SW, "the map double buffer fits the pool");
    const int i = threadIdx.x;
    RSTAMP(0);
    const unsigned long long nbits = dev_nbits ? *dev_nbits : host_nbits;
    const long long nch = (long long)((nbits + 255) >> 8), nbytes = (long long)((nbits + 7) >> 3);
    if (i == 0) bad = 0;
    __syncthreads();
    if (nch > RUNS_MAXC || (__hip_atomic_load(R.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & RUNS_DECLINE))
        return;
    const int Bc = (int)((nch + RUNS_T - 1) / RUNS_T);          // chunks per thread (<= RUNS_BMAX)
    const long long c0 = (long long)i * Bc, c1 = min(c0 + Bc, nch);

    // (1)+(2) every group's entry.  Inside a wave: an inclusive scan of the group maps over its 64 lanes
    // by shuffles (X_g <- X_g o X_{g-d}, X_{g-d} applied first; no barrier), the lane's map in registers
    // and four entries of X_{g-d} at a time looked up in it with v_perm (byte e of the map is byte (e & 7)
    // of register pair e >> 3: four perms give every pair's candidate, a per-byte select keeps the right
    // one).  Across waves only one value is needed: the entry of each wave's first group, which thread 0
    // carries through the wave totals (one byte lookup each).  A block's entry is then its group's entry
    // through the chunk's prefix map inside the group (runs_map_kernel): one lookup.
    RSTAMP(1);
    const long long ngr = (nch + 7) / 8;
    const int nwv = (int)((ngr + 63) / 64);                     // waves with groups
    uint32_t m[8];
    {
        const uint32_t* gm = reinterpret_cast<const uint32_t*>(R.gmap);
#pragma unroll
        for (int q = 0; q < 8; q++) m[q] = i < ngr ? gm[i * 8 + q] : 0x03020100u + 0x04040404u * (uint32_t)q;
    }
    auto lookup4 = [&](uint32_t pw) {                            // m at four entries (bytes of pw, < 32)
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
    };
    const int lane = i & 63, wv = i >> 6;
    if (wv < nwv) {                                             // (wave-uniform)
        for (int d = 1; d < 64; d <<= 1) {
            uint32_t pw[8];
#pragma unroll
            for (int q = 0; q < 8; q++) pw[q] = __shfl_up(m[q], d, 64);
            if (lane >= d) {
                uint32_t nm[8];
#pragma unroll
                for (int q = 0; q < 8; q++) nm[q] = lookup4(pw[q]);
#pragma unroll
                for (int q = 0; q < 8; q++) m[q] = nm[q];
            }
        }
    }
    uint32_t* tot = pool;                                       // the wave totals, then their entries
    uint8_t* gent = reinterpret_cast<uint8_t*>(pool + 256);     // every group's entry
    if (lane == 63 && wv < nwv) {
#pragma unroll
        for (int q = 0; q < 8; q++) tot[wv * 8 + q] = m[q];
    }
    __syncthreads();
    if (i == 0) {
        uint32_t v = 0;                                         // the stream's first token: bit 0
        for (int w = 0; w < nwv; w++) {
            tot[128 + w] = v;
            v = (tot[w * 8 + (v >> 2)] >> (8 * (v & 3))) & 0xFFu;
        }
    }
    __syncthreads();
    if (wv < nwv) {
        const uint32_t vin = tot[128 + wv];
        const uint32_t zin = lookup4(vin) & 0xFFu;              // this lane's inclusive map at the wave's entry
        const int yp = __shfl_up((int)zin, 1, 64);
        if (i < ngr) gent[i] = (uint8_t)(lane == 0 ? (int)vin : yp);
    }
    __syncthreads();
    const int y = c0 < c1 ? (int)R.pm[c0 * 32 + gent[c0 >> 3]] : 0;   // the block's entry
    __syncthreads();                                            // (the pool takes the stream next)
    RSTAMP(2);
    // the stream into LDS when it fits (coalesced 16-byte loads), for pass 1's walks
    // (word w at w + w/8: the lanes' blocks lie 8 words apart, unpadded they would share banks)
    const long long nw = (long long)((nbits + 31) >> 5) + 2;
    const bool staged = nw + (nw >> 3) + 1 <= RUNS_SW;
    if (staged) {
        for (long long q = i; q < nw; q += RUNS_T) pool[q + (q >> 3)] = rs_word(s, nbytes, q);
    }
    RSTAMP(3);
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
    // token offsets: DPP wave scans, the 16 wave totals scanned by thread 0
    const uint32_t cinc = wave_scan_incl(nblk);
    if (lane == 63) ctA[wv] = cinc;
    __syncthreads();
    if (i == 0) {
        uint32_t acc = 0;
        for (int w = 0; w < RUNS_T / 64; w++) { ctB[w] = acc; acc += ctA[w]; }
        ctB[RUNS_T / 64] = acc;
    }
    __syncthreads();
    const long long T0 = (long long)ctB[wv] + cinc - nblk;      // the block's first token
    const long long total = ctB[RUNS_T / 64];
    if (total < num) {                                          // fewer tokens than values: the reference
        if (i == 0) atomicOr(R.err, RUNS_DECLINE | RUNS_WHY_SHORT);   // reads zeros past the end -> other path
        return;
    }
    RSTAMP(4);
    // (4) pass 1: the block with symbolic incoming history -> its carry (last three values)
    RsWords W{staged ? pool : nullptr, s, nbytes, 0, 1};
    Hs h1 = {1u, 0.f}, h2 = {2u, 0.f}, h3 = {3u, 0.f};
    bool sent = false;
    if (c0 < c1) block_walk<CT, 0>(W, P, c0, c1, y, cn, T0, num, nbits, h1, h2, h3, sent, nullptr);
    if (h1.k == 4u || h2.k == 4u || h3.k == 4u) atomicOr(&bad, 1);
    if (sent) atomicOr(&bad, 2);
    RSTAMP(5);
    // (5) the blocks' incoming histories: an inclusive scan of the carries (slot maps: later o earlier)
    // inside each wave by shuffles, thread 0 carrying the concrete history through the wave totals, and
    // each block's incoming history = its predecessor's inclusive carry applied to its wave's history
    __syncthreads();
    if (bad) {
        if (i == 0) atomicOr(R.err, RUNS_DECLINE | ((bad & 1) ? RUNS_WHY_EXPR : 0u) | ((bad & 2) ? RUNS_WHY_SENT : 0u));
        return;
    }
    uint32_t kk = h1.k | h2.k << 8 | h3.k << 16;
    float cv[3] = {h1.v, h2.v, h3.v};
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t ek = (uint32_t)__shfl_up((int)kk, d, 64);
        float ev[3];
#pragma unroll
        for (int q = 0; q < 3; q++) ev[q] = __shfl_up(cv[q], d, 64);
        if (lane >= d) {
            uint32_t nk = 0;
#pragma unroll
            for (int q = 0; q < 3; q++) {
                const uint32_t sk = (kk >> (8 * q)) & 0xFFu;
                if (sk >= 1u && sk <= 3u) {                     // a copy of the earlier carry's slot sk
                    nk |= ((ek >> (8 * (sk - 1))) & 0xFFu) << (8 * q);
                    cv[q] = sk == 1u ? ev[0] : (sk == 2u ? ev[1] : ev[2]);
                } else {
                    nk |= sk << (8 * q);
                }
            }
            kk = nk;
        }
    }
    if (lane == 63) {
        hkA[wv] = kk;
        hvA[3 * wv] = cv[0]; hvA[3 * wv + 1] = cv[1]; hvA[3 * wv + 2] = cv[2];
    }
    __syncthreads();
    if (i == 0) {                                               // the stream starts with no history (zeros)
        float H[3] = {0.f, 0.f, 0.f};
        for (int w = 0; w < RUNS_T / 64; w++) {
            hvB[3 * w] = H[0]; hvB[3 * w + 1] = H[1]; hvB[3 * w + 2] = H[2];
            const uint32_t tk = hkA[w];
            float nh[3];
#pragma unroll
            for (int q = 0; q < 3; q++) {
                const uint32_t sk = (tk >> (8 * q)) & 0xFFu;
                nh[q] = sk == 0u ? hvA[3 * w + q] : H[sk - 1];
            }
            H[0] = nh[0]; H[1] = nh[1]; H[2] = nh[2];
        }
    }
    __syncthreads();
    const float Hw[3] = {hvB[3 * wv], hvB[3 * wv + 1], hvB[3 * wv + 2]};
    float z[3];
#pragma unroll
    for (int q = 0; q < 3; q++) {
        const uint32_t sk = (kk >> (8 * q)) & 0xFFu;
        z[q] = sk == 0u ? cv[q] : (sk == 1u ? Hw[0] : (sk == 2u ? Hw[1] : Hw[2]));
    }
    float b1 = __shfl_up(z[0], 1, 64), b2 = __shfl_up(z[1], 1, 64), b3 = __shfl_up(z[2], 1, 64);
    if (lane == 0) { b1 = Hw[0]; b2 = Hw[1]; b3 = Hw[2]; }
    RSTAMP(6);
    R.blk[i] = make_uint4((uint32_t)y | (uint32_t)(c1 > c0 ? c1 - c0 : 0) << 8, (uint32_t)T0, 0u, 0u);
    R.bhist[i] = make_float4(b1, b2, b3, 0.0f);
#pragma unroll
    for (int j = 0; j < RUNS_BMAX; j++) R.bcnt[i * RUNS_BMAX + j] = cn[j];
}

// thread = block: its values from its first chunk's entry with the concrete incoming history
template <int CT, bool SCAT>
__global__ __launch_bounds__(64) void runs_values_kernel(const uint8_t* __restrict__ s, Params P, RunsBufs R,
                                                        const unsigned long long* dev_nbits,
                                                        unsigned long long host_nbits, float* __restrict__ out,
                                                        long long num, RunsScatter S) {
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
    RsWords W{row, s, nbytes, 8 * c0, 0};
    block_walk<CT, SCAT ? 2 : 1>(W, P, c0, c0 + nc, (int)(b.x & 0xFFu), cn, (long long)b.y, num, nbits, h1, h2, h3,
                                 sent, out, S, SCAT ? *S.dmin : 0.0f);
    if (sent) atomicOr(R.err, RUNS_DECLINE | RUNS_WHY_SENT);
}

static int launch_runs(const uint8_t* s, const unsigned long long* dev_nbits, unsigned long long host_nbits,
                       long long max_chunks, const Params* P, uint8_t* maps, unsigned* err, float* out, long long num,
                       const RunsScatter* S, hipStream_t st) {
    if (max_chunks > RUNS_MAXC + 8 || max_chunks < 1) return -2;     // (the stream's own length is checked on the device)
    RunsBufs R;
    const size_t mb = (size_t)(RUNS_MAXC + 8) * 32;
    R.exitm = maps;
    R.cntm = maps + mb;
    R.blk = reinterpret_cast<uint4*>(maps + 2 * mb);
    R.bhist = reinterpret_cast<float4*>(maps + 2 * mb + 16 * RUNS_T);
    R.bcnt = maps + 2 * mb + 32 * RUNS_T;
    R.pm = maps + 2 * mb + 32 * RUNS_T + RUNS_BMAX * RUNS_T;
    R.gmap = R.pm + mb;
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
        if (S)                                                                                                 \
            hipLaunchKernelGGL((runs_values_kernel<C, true>), dim3(RUNS_T / 64), dim3(64), 0, st, s, *P, R,     \
                               dev_nbits, host_nbits, out, num, *S);                                           \
        else                                                                                                   \
            hipLaunchKernelGGL((runs_values_kernel<C, false>), dim3(RUNS_T / 64), dim3(64), 0, st, s, *P, R,    \
                               dev_nbits, host_nbits, out, num, RunsScatter{});                                \
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
extern "C" int dc_launch_decode_runs(const uint8_t* s, const unsigned long long* dev_nbits, unsigned long long host_nbits,
                                     long long max_chunks, const Params* P, uint8_t* maps, unsigned* err, float* out,
                                     long long num, hipStream_t st) {
    return launch_runs(s, dev_nbits, host_nbits, max_chunks, P, maps, err, out, num, nullptr, st);
}
// (r06) a Himeno halo plane decoded straight into its array: value e of the A x B plane ijk at index v to its element of
// the [.][mj][mk] array p, plus *d_min (as dc_launch_decode_runs followed by dc_launch_plane_scatter, one launch less)
extern "C" int dc_launch_decode_runs_scatter(const uint8_t* s, const unsigned long long* dev_nbits,
                                             unsigned long long host_nbits, long long max_chunks, const Params* P,
                                             uint8_t* maps, unsigned* err, long long num, float* p, const float* d_min,
                                             int mj, int mk, int ijk, int v, int B, hipStream_t st) {
    if (!p || !d_min || B <= 0 || num >= (1ll << 31)) return -2;
    const RunsScatter S{p, d_min, mj, mk, ijk, v, B};
    return launch_runs(s, dev_nbits, host_nbits, max_chunks, P, maps, err, nullptr, num, &S, st);
}
extern "C" long long dc_decode_runs_max_chunks(void) { return RUNS_MAXC; }
extern "C" size_t dc_decode_runs_scratch_bytes(void) {
    return (size_t)(RUNS_MAXC + 8) * 32 * 3 + (size_t)RUNS_T * (16 + 16 + RUNS_BMAX) + (size_t)(RUNS_MAXC / 8 + 8) * 32;
}

}  // namespace dc
