// dc_decode_fast.hip -- LDS-staged three-kernel decoder: the fast path of the bit-wise decoders of
// impl/dataCompression.c (myDecompress_bitwise :2922, _np :2459, _mask :1703, _op :698).
//
// A tile = GROUP chunks of CHUNK_BITS = one workgroup, one lane per chunk.  Each kernel reads the
// tile's stream bytes from HBM once, with coalesced 16-byte loads, into LDS rows padded to 33 words
// (lanes reading the same offset of their own chunks hit different banks; word w sits at w + w/32).
// All parsing runs out of LDS through a branch-free 3-word window reader with a prefetched word.
//
// parse_kernel : speculative path P_c per chunk; the tile's first chunk gets its complete 32-entry
//                map; every other chunk walks the exits of its predecessor's known entries until they
//                merge with P_c (closure rounds inside the workgroup).  The true path through a tile is
//                a "standard" chain (entry of chunk c = exit of P_{c-1}) with rare deviations, which
//                one lane resolves by hopping over the failure points.  Per tile it stores the chunk
//                records and the tile map (32 entries -> exit, token count).  Tiles never wait on
//                each other.
// tile_scan    : one workgroup chains the tiles: in practice every tile map has a constant exit (all
//                32 entries merge long before the tile ends), so tile t's entry is tile t-1's exit and
//                a block scan of the counts gives every tile's first token index.
// decode_kernel: re-resolves the chunk entries of its tile from the tile entry, decodes every chunk
//                from its true entry (history = DECODED values, tracked symbolically where it depends
//                on the previous chunk), scans the chunk carry functions in LDS, chains tiles through a
//                history look-back when a pending prefix needs it, and re-decodes pending prefixes.
// Anything outside these assumptions (closure overflow, an unresolved entry, arithmetic prediction
// chains across chunks) is reported in D.err and finished by the exact multi-kernel path.
#include "dc_device.h"
#include <algorithm>
#include <stdlib.h>

namespace dc {

constexpr int LROW = CHUNK_BITS / 32;          // stream words per chunk
// LDS rows are padded to 33 words (stream word w sits at w + w/32): ds_read_b32 banks are
// (address/4) mod 32 per 32-lane half, and the lanes of a wave walk their chunks at nearly the same
// word offset, so unpadded rows put a whole half-wave on one or two banks (SQ_LDS_BANK_CONFLICT
// was ~ half of the LDS cycles); padded, lane c's word w is on bank (c + w) mod 32.
#ifndef DC_PAD
#define DC_PAD 1
#endif
__host__ __device__ constexpr int padw(int n) { return DC_PAD ? n + (n >> 5) + 1 : n; }
constexpr int LWORDS = padw(GROUP * LROW + 8);  // + the words after the tile
#ifndef DC_OV
#define DC_OV 1024
#endif
constexpr int OV = DC_OV;                       // overlap: P_c starts OV bits before its chunk
constexpr int OVW = OV / 32;
constexpr int PWORDS = padw(GROUP * LROW + 8 + OVW);
#ifndef DC_PARSE_LUT
#define DC_PARSE_LUT 1
#endif
#if DC_PARSE_LUT
#define PLEN(t) ((int)S.tl[(t) >> 23])
#else
#define PLEN(t) token_len_bf<CT>((t), P)
#endif
#ifndef DC_DEC_NT
#define DC_DEC_NT 1                              // decode stages the stream with nontemporal loads (its last read)
#endif
#ifndef DC_KMAX
#define DC_KMAX 3                               // 3: the three phases of a period-3 run ('101' chains)
#endif
constexpr int KMAX = DC_KMAX;                        // extra known entries per chunk (besides P_c's own)
constexpr int RMAX = 12;                       // closure rounds inside a tile
constexpr int CW = CHUNK_BITS / 32;            // words per chunk
constexpr int UNKE = 63;

#define STAMP(ph) do { if (D.dbg && threadIdx.x == 0 && t < 4096) D.dbg[t * 16 + (ph)] = __builtin_amdgcn_s_memrealtime(); } while (0)

__device__ __forceinline__ int lidx(int w) { return DC_PAD ? w + (w >> 5) : w; }
__device__ __forceinline__ uint32_t ldw(const uint32_t* L, int w) {
    // byte offset (w + w / 32) * 4: one v_add_lshl_u32 after the shift
    const uint32_t off = ((uint32_t)lidx(w)) << 2;
    return *(const uint32_t*)((const char*)L + off);
}

// branch-free MSB-first reader: w0:w1 hold the next 64 bits from bit sh of w0, w2 the next word.
// Every step is fetch() (issues the LDS read of the word after w2, at the top of the step) ... step()
// (shifts it in).  The read is not loop-carried, so the compiler needs no back-edge copy of an
// in-flight register -- with a loop-carried prefetch it placed an lgkmcnt(0) wait on every step.
struct Rd {
    uint32_t a, b, c, nx;                      // the 64-bit window (a:b) is read from bit 32 - s of a
    int s, w3, pos;                            // s in [0, 31]; w3 = word index of the next fetch; pos = stream bit
    __device__ __forceinline__ void init(const uint32_t* L, int p) {
        const int wi = (p - 1) >> 5;           // a word boundary is bit 32 of a (s = 0), never bit 0
        s = 32 * (wi + 1) - p;
        a = ldw(L, max(wi, 0)); b = ldw(L, wi + 1); c = ldw(L, wi + 2);
        w3 = wi + 3;
        pos = p;
    }
    __device__ __forceinline__ void fetch(const uint32_t* L) { nx = ldw(L, w3); }
    __device__ __forceinline__ uint32_t peek() const {
        return __builtin_amdgcn_alignbit(a, b, (uint32_t)s);           // ((a:b) >> s), low word
    }
    __device__ __forceinline__ void step(int len) {
        uint32_t d;
        const bool adv = __builtin_usub_overflow((uint32_t)s, (uint32_t)len, &d);   // borrow = next word
        s = (int)(d & 31u);
        pos += len;
        a = adv ? b : a;
        b = adv ? c : b;
        c = adv ? nx : c;
        w3 += adv ? 1 : 0;
    }
};

// stage stream words [tw, tw + nw) into padded LDS rows (zeros outside the stream; tw may be < 0)
__device__ __forceinline__ void stage_words(uint32_t* L, const uint8_t* s, long long nbytes, long long tw, int nw,
                                            bool nt = false) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(s);
    const long long nwfull = nbytes >> 2;
    if (tw >= 0 && tw + nw <= nwfull && ((reinterpret_cast<uintptr_t>(s) & 15u) == 0) && (tw & 3) == 0 && (nw & 3) == 0) {
        const uint4* w4 = reinterpret_cast<const uint4*>(w + tw);
        const int n4 = nw >> 2;
        constexpr int QF = CW * GROUP / 4 / GROUP;           // full rounds of GROUP uint4
        uint4 r[QF + 1];
#pragma unroll
        for (int q = 0; q <= QF; q++) {
            const int i = threadIdx.x + q * GROUP;
            if (q < QF || i < n4) {
                if (nt) {
                    typedef unsigned u4v __attribute__((ext_vector_type(4)));
                    const u4v w = __builtin_nontemporal_load(reinterpret_cast<const u4v*>(w4 + i));
                    r[q] = make_uint4(w.x, w.y, w.z, w.w);
                } else {
                    r[q] = w4[i];
                }
            }
        }
#pragma unroll
        for (int q = 0; q <= QF; q++) {
            const int i4 = threadIdx.x + q * GROUP;
            if (q < QF || i4 < n4) {
                const int i = 4 * i4;
                uint32_t* d = L + lidx(i);
                d[0] = __builtin_bswap32(r[q].x);
                d[1] = __builtin_bswap32(r[q].y);
                d[2] = __builtin_bswap32(r[q].z);
                d[3] = __builtin_bswap32(r[q].w);
            }
        }
        return;
    }
    for (int i = threadIdx.x; i < nw; i += blockDim.x) {
        const long long gw = tw + i;
        uint32_t v = 0;
        if (gw < 0) {
            v = 0;
        } else if (gw < nwfull) {
            v = __builtin_bswap32(w[gw]);
        } else if (4 * gw < nbytes) {
            for (int k = 0; k < 4; k++) {
                const long long bi = 4 * gw + k;
                v = (v << 8) | (bi < nbytes ? (uint32_t)s[bi] : 0u);
            }
        }
        L[lidx(i)] = v;
    }
}

// the tile's words [tw, tw + GROUP*CW + 4)
__device__ __forceinline__ void stage_tile(uint32_t* L, const uint8_t* s, long long nbytes, long long tw) {
    stage_words(L, s, nbytes, tw, GROUP * CW + 4, DC_DEC_NT);        // the decode is the stream's last reader
}

// walk entry e of chunk c (LDS bits [cs, cend)) alongside P_c (whose first boundary in the chunk is
// pmask's lowest bit); the reader that is behind steps.  Returns the exit relative to the next chunk
// and the number of tokens starting in the chunk.
template <int CT>
__device__ __forceinline__ void walk_lds(const uint32_t* L, const uint8_t* tl, int cs, int cend, int e,
                                         uint32_t pmask, int pexit, int pcnt, int* out_exit, int* out_cnt,
                                         bool runs) {
    if ((pmask >> e) & 1u) {
        *out_exit = pexit;
        *out_cnt = pcnt - __popc(pmask & ((1u << e) - 1u));
        return;
    }
    Rd A, B;
    A.init(L, cs + e);
    if (CT != 6 && runs) {                     // runs mode: A alone to the chunk end, whole runs per step
        int ca = 0;
        while (A.pos < cend) {
            A.fetch(L);
            const uint32_t tk = A.peek();
            const int L = (int)tl[tk >> 23];
            const int k = (int)tk < 0 ? run3i(tk, A.pos, cend) : run_per3(tk, L, A.pos, cend);
            A.step(k > 1 ? ((int)tk < 0 ? 3 : L) * k : L);
            ca += k;
        }
        const int x = A.pos - (cs + CHUNK_BITS);
        *out_exit = (x >= 0 && x < 32) ? x : 0;
        *out_cnt = ca;
        return;
    }
    B.init(L, cs + (pmask ? __ffs(pmask) - 1 : 32));
    int ca = 0, cb = 0;
    bool merged = false;
    while (A.pos < cend) {
        if (A.pos == B.pos) { merged = true; break; }
        const bool sa = A.pos < B.pos || B.pos >= cend;
        const uint32_t nx = ldw(L, sa ? A.w3 : B.w3);
        const uint32_t tk = sa ? A.peek() : B.peek();
        const int len = tl[tk >> 23];
        if (sa) { A.nx = nx; A.step(len); ca++; } else { B.nx = nx; B.step(len); cb++; }
    }
    if (merged) { *out_exit = pexit; *out_cnt = ca + pcnt - cb; return; }
    const int x = A.pos - (cs + CHUNK_BITS);
    *out_exit = (x >= 0 && x < 32) ? x : 0;
    *out_cnt = ca;
}

// ------------------------------------------------------------------------------------------------
struct ParseShared {
    uint32_t L[PWORDS];
    uint8_t tl[512];                           // token length by the first 9 bits (build_lut_len)
    uint32_t ke[GROUP * KMAX];                 // entry<<16 | exit<<10 | cnt
    union {                                    // closure rounds, then the tile chain
        uint8_t nkr[2][GROUP];                 // known-entry count of every chunk, by round parity
        uint16_t devcnt[GROUP];
    };
    uint32_t pm[GROUP];
    uint64_t bad[GROUP / 64];
    uint16_t n[GROUP];
    uint8_t x[GROUP], nk[GROUP], stdexit[GROUP], dev[GROUP];
    uint32_t wsum[GROUP / 64];
    uint32_t x0m;                              // runs mode: exits of all 32 entries of chunk 0
    int texit;
#ifdef DC_PARSE_PAD
    uint32_t occpad[DC_PARSE_PAD / 4];          // occupancy experiment: extra LDS per workgroup
#endif
};

__device__ __forceinline__ int next_bad(const uint64_t* bad, int c, int nact) {
    for (int w = c >> 6; w < GROUP / 64; w++) {
        uint64_t m = bad[w];
        if (w == (c >> 6)) m &= ~0ull << (c & 63);
        if (m) { const int f = w * 64 + __ffsll((long long)m) - 1; return f < nact ? f : nact; }
    }
    return nact;
}

// map of chunk c at entry e from the LDS state of the parse kernel
__device__ __forceinline__ bool lookup_entry(const ParseShared& S, int c, int e, int* ex, int* cn) {
    const uint32_t pm = S.pm[c];
    if ((pm >> e) & 1u) { *ex = S.x[c]; *cn = S.n[c] - __popc(pm & ((1u << e) - 1u)); return true; }
    for (int k = 0; k < S.nk[c]; k++) {
        const uint32_t v = S.ke[c * KMAX + k];
        if ((int)(v >> 16) == e) { *ex = (int)((v >> 10) & 63); *cn = (int)(v & 1023); return true; }
    }
    return false;
}

__device__ __forceinline__ Plan make_plan(const unsigned long long* dev_nbits, unsigned long long host_nbits,
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
    return p;
}

// the parse also derives the plan (sizes from the bit length, on the device so encode -> decode needs no
// host round trip) and publishes it for the later kernels
template <int CT>
__global__ __launch_bounds__(GROUP) void parse_kernel(const uint8_t* __restrict__ s, Params P, DecBufs D,
                                                    const unsigned long long* dev_nbits, unsigned long long host_nbits,
                                                    long long max_chunks, long long num) {
    __shared__ ParseShared S;
    const Plan pl = make_plan(dev_nbits, host_nbits, max_chunks, CT, num);
    if (blockIdx.x == 0 && threadIdx.x == 0) *D.plan = pl;
    const int c = threadIdx.x, lane = c & 63, wid = c >> 6;
    build_lut_len<CT>(S.tl, P, c, GROUP);                             // visible after the first barrier
    for (long long t = blockIdx.x; t < pl.ngroups; t += gridDim.x) {
        const long long tbit = t * (long long)GROUP * CHUNK_BITS;
        STAMP(0);
        // LDS bit OV = the tile's first stream bit; the OV bits before it let P_0 synchronise
        stage_words(S.L, s, pl.nbytes, (tbit >> 5) - OVW, GROUP * CW + OVW + 4);
        const long long gc = t * GROUP + c;
        const long long rem = (long long)pl.nbits - tbit;
        const int nact = (int)min((long long)GROUP, (rem + CHUNK_BITS - 1) / CHUNK_BITS);
        const bool act = c < nact;
        const int cs = OV + c * CHUNK_BITS;
        const int cend = OV + (int)min((long long)(c * CHUNK_BITS + CHUNK_BITS), rem);
        __syncthreads();
        STAMP(1);

        // ---- round 1: P_c from OV bits before the chunk (from bit 0 for the stream's first chunk);
        // self-synchronisation makes P_c the true path inside the chunk in almost every case
        uint32_t pm = 0;
        int n = 0, x = 0;
        if (act) {
            Rd r;
            // (tile 0: never before the stream's first bit, which is a true boundary)
            r.init(S.L, gc == 0 ? cs : (t == 0 ? max(cs - OV, OV) : cs - OV));
            const unsigned long long q0 = D.dbg ? __builtin_amdgcn_s_memtime() : 0;
            if (CT != 6 && pl.runs) {
                while (r.pos < cs) {
                    r.fetch(S.L);
                    const uint32_t tk = r.peek();
                    const int L = PLEN(tk);
                    r.step((int)tk < 0 ? 3 * run3i(tk, r.pos, cs) : L * run_per3(tk, L, r.pos, cs));
                }
            } else {
                while (r.pos < cs) { r.fetch(S.L); r.step(PLEN(r.peek())); }
            }
            if (D.dbg && t < 4096 && (c & 63) == 0)                  // per-wave cycles (diagnostic)
                D.dbg[t * 16 + 12 + (c >> 6)] = (__builtin_amdgcn_s_memtime() - q0) << 16;
            const int pend = min(cs + 32, cend);                      // boundaries in the first word
            while (r.pos < pend) {
                r.fetch(S.L);
                pm |= 1u << (r.pos - cs);
                r.step(PLEN(r.peek()));
                n++;
            }
            if (CT != 6 && pl.runs) {
                while (r.pos < cend) {
                    r.fetch(S.L);
                    const uint32_t tk = r.peek();
                    const int L = PLEN(tk);
                    const int k = (int)tk < 0 ? run3i(tk, r.pos, cend) : run_per3(tk, L, r.pos, cend);
                    r.step(k > 1 ? ((int)tk < 0 ? 3 : L) * k : L);
                    n += k;
                }
            } else {
                while (r.pos < cend) {
                    r.fetch(S.L);
                    r.step(PLEN(r.peek()));
                    n++;
                }
            }
            const int xx = r.pos - (cs + CHUNK_BITS);
            x = (xx >= 0 && xx < 32) ? xx : 0;
        }
        S.pm[c] = pm; S.n[c] = (uint16_t)n; S.x[c] = (uint8_t)x;
        if (c == 0) S.x0m = 0;
        __syncthreads();
        STAMP(2);

        // ---- runs mode: the complete 32-entry map of chunk 0 (one lane per entry), so that a tile
        // entered off P_0 (period-3 streams never resynchronise) can be resolved exactly by composing
        // chunk maps (dc_launch_decode_resolve) instead of re-deriving every map
        if (CT != 6 && pl.runs) {
            if (c < 32) {
                int ex, cn;
                walk_lds<CT>(S.L, S.tl, OV, OV + (int)min((long long)CHUNK_BITS, rem), c, S.pm[0], S.x[0], S.n[0],
                             &ex, &cn, true);
                D.fullmap[t * 32 + c] = ((uint32_t)ex << 26) | (uint32_t)cn;
                atomicOr(&S.x0m, 1u << ex);
            }
            __syncthreads();
        }

        // ---- round 2: P_{c-1}'s exit into chunk c, where P_c has no boundary there (rare)
        int nk = 0;
        if (act && c > 0) {
            const int e = S.x[c - 1];
            if (!((pm >> e) & 1u)) {
                int ex, cn;
                walk_lds<CT>(S.L, S.tl, cs, cend, e, pm, x, n, &ex, &cn, pl.runs);
                S.ke[c * KMAX] = ((uint32_t)e << 16) | ((uint32_t)ex << 10) | (uint32_t)cn;
                nk = 1;
            }
        }
        S.nk[c] = (uint8_t)nk;
        S.nkr[0][c] = (uint8_t)nk;
        __syncthreads();
        STAMP(3);

        // ---- closure rounds: add every exit of the predecessor's known entries
        int round = 3;
        for (; round <= RMAX; round++) {
            const int rp = round & 1, pp = rp ^ 1;
            int added = 0;
            if (act && c > 0) {
                uint32_t known = pm;
                for (int k = 0; k < nk; k++) known |= 1u << (S.ke[c * KMAX + k] >> 16);
                // exits of the predecessor's entries known at the end of the previous round
                uint32_t emp = 1u << S.x[c - 1];
                if (CT != 6 && pl.runs && c == 1) emp |= S.x0m;
                const int nkp = S.nkr[pp][c - 1];
                for (int k = 0; k < nkp; k++) emp |= 1u << ((S.ke[(c - 1) * KMAX + k] >> 10) & 63u);
                uint32_t need = emp & ~known;
                while (need) {
                    const int e = __ffs(need) - 1;
                    need &= need - 1;
                    if (nk >= KMAX) { atomicOr(D.err, 64u); break; }
                    int ex, cn;
                    walk_lds<CT>(S.L, S.tl, cs, cend, e, pm, x, n, &ex, &cn, pl.runs);
                    S.ke[c * KMAX + nk] = ((uint32_t)e << 16) | ((uint32_t)ex << 10) | (uint32_t)cn;
                    nk++;
                        added = 1;
                }
            }
            S.nkr[rp][c] = (uint8_t)nk;
            S.nk[c] = (uint8_t)nk;
            if (!__syncthreads_or(added)) break;
        }
        if (round > RMAX && c == 0) atomicOr(D.err, 64u);
        STAMP(4);

        // ---- standard chain data: entry of chunk c = exit of P_{c-1}
        int scnt = 0, sex = x;
        bool ok = true;
        if (act && c > 0) {
            int ex, cn;
            if (lookup_entry(S, c, S.x[c - 1], &ex, &cn)) { scnt = cn; sex = ex; ok = (ex == x); }
            else atomicOr(D.err, 8u);
        }
        S.stdexit[c] = (uint8_t)sex;
        const unsigned long long bm = __ballot(!ok);
        if (lane == 0) S.bad[wid] = bm;
        __syncthreads();

        // ---- tile chain: every tile entry that is a boundary of P_0 continues as P_0 and leaves chunk 0
        // at x_0; from there one lane follows the chain, hopping over standard runs and recording the
        // chunks where it deviates from them
        S.dev[c] = 0xFF;
        __syncthreads();
        if (c == 0) {
            int e = S.x[0], cc = 1;
            bool good = true;
            while (cc < nact) {
                if (e == S.x[cc - 1]) {
                    const int fb = next_bad(S.bad, cc, nact);
                    if (fb >= nact) { e = S.x[nact - 1]; break; }
                    e = S.stdexit[fb];
                    cc = fb + 1;
                } else {
                    int ex, cn;
                    if (!lookup_entry(S, cc, e, &ex, &cn)) { good = false; break; }
                    S.dev[cc] = (uint8_t)e;
                    S.devcnt[cc] = (uint16_t)cn;
                    e = ex;
                    cc++;
                }
            }
            S.texit = good ? e : UNKE;
        }
        __syncthreads();
        // chain entry and token count of every chunk (chunk 0's depend on the tile entry: tile_fix)
        const bool dv = S.dev[c] != 0xFF;
        const int centry = c == 0 ? 0 : (dv ? S.dev[c] : S.x[c - 1]);
        const uint32_t ccnt = (c == 0 || !act) ? 0u : (dv ? S.devcnt[c] : (uint32_t)scnt);
        uint32_t inc2 = ccnt;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t tv = __shfl_up(inc2, d, 64);
            if (lane >= d) inc2 += tv;
        }
        if (lane == 63) S.wsum[wid] = inc2;
        __syncthreads();
        uint32_t wp2 = 0;
        for (int w = 0; w < wid; w++) wp2 += S.wsum[w];
        if (act) {
            D.entry[gc] = (uint8_t)centry;
            D.tokoff[gc] = wp2 + inc2 - ccnt;                 // tile-relative, chunks 1..c-1
        }
        if (c == GROUP - 1) {
            D.tmap[t * 4 + 0] = S.pm[0];
            D.tmap[t * 4 + 1] = (uint32_t)S.n[0] | ((uint32_t)S.x[0] << 16) | ((uint32_t)S.texit << 24);
            D.tmap[t * 4 + 2] = wp2 + inc2;                   // tokens of chunks 1..nact-1
        }
        // ---- chunk records for the decode kernel
        if (act) {
            D.p_exit[gc] = (uint8_t)x;
            D.p_cnt[gc] = (uint16_t)n;
            D.p_mask[gc] = pm;
            D.cmeta[gc] = (uint32_t)scnt | ((uint32_t)sex << 10) | ((uint32_t)nk << 16) | ((ok ? 1u : 0u) << 20);
            // extra entries in the exact path's format (map by entry + known mask), which resolve_kernel reads
            uint32_t kn = 0;
            for (int k = 0; k < nk; k++) {
                const uint32_t v = S.ke[c * KMAX + k];
                const int e = (int)(v >> 16);
                kn |= 1u << e;
                D.map[gc * 32 + e] = (((v >> 10) & 63u) << 26) | (v & 1023u);
            }
            D.known[gc] = c == 0 ? 0u : kn;
        }
        __syncthreads();
        STAMP(7);
    }
}

// map of chunk gc at entry e from the parse kernel's global records
__device__ __forceinline__ bool lookup_global(const DecBufs& D, long long gc, int e, int* ex, int* cn) {
    const uint32_t pm = D.p_mask[gc];
    if ((pm >> e) & 1u) { *ex = D.p_exit[gc]; *cn = D.p_cnt[gc] - __popc(pm & ((1u << e) - 1u)); return true; }
    if ((D.known[gc] >> e) & 1u) {
        const uint32_t v = D.map[gc * 32 + e];
        *ex = (int)(v >> 26); *cn = (int)(v & 0x3FFFFFFu);
        return true;
    }
    return false;
}

// ------------------------------------------------------------------------------------------------
// tile_fix: tile t's entry E is tile t-1's exit, which is the same for every entry of tile t-1 that
// is a boundary of its P_0 -- so every tile's entry is known at once.  When E is not a boundary of
// tile t's own P_0 (P_0 had not synchronised by the tile start: a few % of tiles), one wave stages the
// tile's first chunks and walks from E, chunk by chunk, until it joins the tile chain; the walked
// chunks get their entries and offsets overridden.  One wave per tile.
constexpr int FIXW = 8192 / CHUNK_BITS;                   // chunks a fix-up walk may cover (8 Kbit)
struct FixShared {
    uint32_t L[4][padw(FIXW * LROW + 8)];
    uint8_t tl[512];
};

template <int CT>
__global__ __launch_bounds__(256) void tile_fix_kernel(const uint8_t* __restrict__ s, Params P, DecBufs D) {
    __shared__ FixShared S;
    const Plan pl = *D.plan;
    const long long nt = pl.ngroups;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const long long t = (long long)blockIdx.x * 4 + wv;
    build_lut_len<CT>(S.tl, P, threadIdx.x, 256);
    __syncthreads();
    if (t >= nt) return;
    const int E = t == 0 ? 0 : (int)(D.tmap[(t - 1) * 4 + 1] >> 24);
    const uint32_t pm0 = D.tmap[t * 4 + 0], r1 = D.tmap[t * 4 + 1];
    const int n0 = (int)(r1 & 0xFFFF), x0 = (int)((r1 >> 16) & 0xFF), X = (int)(r1 >> 24);
    const long long tbit = t * (long long)GROUP * CHUNK_BITS;
    const long long rem = (long long)pl.nbits - tbit;
    const int nact = (int)min((long long)GROUP, (rem + CHUNK_BITS - 1) / CHUNK_BITS);
    if (E == UNKE || (X == UNKE && t + 1 < nt)) {
        if (lane == 0) { atomicOr(D.err, 8u); D.tentry[t] = UNKE; D.tmap[t * 4 + 3] = 0; }
        return;
    }
    if ((pm0 >> E) & 1u) {
        if (lane == 0) {
            D.tentry[t] = (uint32_t)E | ((uint32_t)(n0 - __popc(pm0 & ((1u << E) - 1u))) << 6);
            D.tmap[t * 4 + 3] = 0;
        }
        return;
    }
    // rare: stage the first FIXW chunks of the tile (wave-local LDS), walk from E
    uint32_t* L = S.L[wv];
    const uint32_t* w = reinterpret_cast<const uint32_t*>(s);
    const long long nwfull = pl.nbytes >> 2;
    for (int i = lane; i < FIXW * CW + 4; i += 64) {
        const long long gw = (tbit >> 5) + i;
        uint32_t v = 0;
        if (gw < nwfull) v = __builtin_bswap32(w[gw]);
        else if (4 * gw < pl.nbytes)
            for (int k = 0; k < 4; k++) { const long long bi = 4 * gw + k; v = (v << 8) | (bi < pl.nbytes ? (uint32_t)s[bi] : 0u); }
        L[lidx(i)] = v;
    }
    __builtin_amdgcn_s_waitcnt(0);                      // the wave's own LDS stores land in order
    __builtin_amdgcn_wave_barrier();
    if (lane != 0) return;
    const int cend0 = (int)min((long long)CHUNK_BITS, rem);
    int ex, c0;
    walk_lds<CT>(L, S.tl, 0, cend0, E, pm0, x0, n0, &ex, &c0, pl.runs);
    const long long g0 = t * GROUP;
    int k = 1;
    uint32_t acc = 0;
    int kjoin = nact;
    long long delta = 0;
    bool ok = true;
    while (k < nact) {
        if (ex == (int)D.entry[g0 + k]) {                          // joined the tile chain
            kjoin = k;
            delta = (long long)acc - (long long)D.tokoff[g0 + k];
            break;
        }
        if (k >= FIXW) { ok = false; break; }
        const long long gk = g0 + k;
        int nx, cn;
        if (!lookup_global(D, gk, ex, &nx, &cn)) {
            const int cs = k * CHUNK_BITS;
            const int ce = (int)min((long long)(cs + CHUNK_BITS), rem);
            walk_lds<CT>(L, S.tl, cs, ce, ex, D.p_mask[gk], D.p_exit[gk], D.p_cnt[gk], &nx, &cn, pl.runs);
        }
        D.entry[gk] = (uint8_t)ex;
        D.tokoff[gk] = acc;
        acc += (uint32_t)cn;
        ex = nx;
        k++;
    }
    if (k == nact) {                                               // walked to the tile end
        kjoin = nact;
        delta = (long long)acc - (long long)D.tmap[t * 4 + 2];
        if (ex != X && t + 1 < nt) ok = false;                       // the next tile's entry would change
    }
    if (!ok) { atomicOr(D.err, 8u); D.tentry[t] = UNKE; D.tmap[t * 4 + 3] = 0; return; }
    D.tentry[t] = (uint32_t)E | ((uint32_t)c0 << 6) | ((uint32_t)kjoin << 16);
    D.tmap[t * 4 + 3] = (uint32_t)(int)delta;
}

// tile_scan: first token index of every tile (one workgroup, block scan of the tile counts)
__global__ __launch_bounds__(1024) void tile_scan_kernel(DecBufs D) {
    __shared__ unsigned long long wtot[16];
    const Plan pl = *D.plan;
    const long long nt = pl.ngroups;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const long long per = (nt + 1023) / 1024;
    const long long t0 = tid * per, t1 = min(nt, t0 + per);
    auto count = [&](long long t) -> unsigned long long {
        const uint32_t te = D.tentry[t];
        if ((te & 63) == UNKE) return 0ull;
        return (unsigned long long)((te >> 6) & 1023) + (unsigned long long)((long long)D.tmap[t * 4 + 2] + (int)D.tmap[t * 4 + 3]);
    };
    unsigned long long sum = 0;
    for (long long t = t0; t < t1; t++) sum += count(t);
    unsigned long long inc = sum;                    // wave scan, then the 16 wave totals
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long u = __shfl_up(inc, d, 64);
        if (lane >= d) inc += u;
    }
    if (lane == 63) wtot[wid] = inc;
    __syncthreads();
    unsigned long long wpre = 0;
#pragma unroll
    for (int w = 0; w < 16; w++) wpre += w < wid ? wtot[w] : 0ull;
    unsigned long long part_tid = wpre + inc;
    unsigned long long run = part_tid - sum;
    for (long long t = t0; t < t1; t++) {
        D.tbase[t] = run;
        run += count(t);
    }
    if (t1 == nt && t0 < t1) D.tbase[nt] = run;             // total: the last tile's end
    if (nt == 0 && tid == 0) D.tbase[0] = 0;
}

// ------------------------------------------------------------------------------------------------
// decode.  kinds: 0 concrete, 1..3 = the chunk's (tile's) incoming b1..b3, 4 derived (serial)
// Output ring: every lane keeps its last RING decoded values in LDS at slot (idx + a0) & (RING-1),
// where a0 aligns the slots to 64-byte sectors of `out`.  Complete sectors leave as four 16-byte
// stores issued back to back (HBM sees whole sectors instead of scattered partial lines); the values
// before the chunk's first and after its last sector boundary leave as plain dword stores.
#ifndef DC_RING
#define DC_RING 16
#endif
constexpr int RING = DC_RING;
#ifndef DC_SECT
#define DC_SECT 8
#endif
constexpr int SECT = DC_SECT;
static_assert(SECT == 2 || SECT % 4 == 0, "sectors of 2 or 4k floats");

// Indices are relative to the chunk's first output index k0 (32-bit): token j sits in ring slot
// (j + r0) & (RING - 1) with r0 = (k0 + a0) & (RING - 1); sectors start at j = h + SECT*i, h = the
// values before the first sector boundary; lim = num - k0 bounds every store.
__device__ __forceinline__ void store_sector(const float* ring, float* outk, int s0, int r0, int lim) {
#ifdef DC_NOSTORE
    if (lim >= 0) return;
#endif
    const int sl = (s0 + r0) & (RING - 1);
    if (s0 + SECT <= lim) {
        if constexpr (SECT % 4 == 0) {
            const float4* r4 = reinterpret_cast<const float4*>(ring + sl);
            float4* o4 = reinterpret_cast<float4*>(outk + s0);
#pragma unroll
            for (int q = 0; q < SECT / 4; q++) o4[q] = r4[q];
        } else {
            *reinterpret_cast<float2*>(outk + s0) = *reinterpret_cast<const float2*>(ring + sl);
        }
    } else {
        for (int i = 0; i < SECT && s0 + i < lim; i++) outk[s0 + i] = ring[sl + i];
    }
}

// at a flush point (j values decoded): the head (values before the first sector boundary) once it
// is complete, then the complete sector (at most one is pending: a lane adds <= SECT values between
// flush points)
__device__ __forceinline__ void flush_ring(const float* ring, float* outk, int r0, int& fl, int j, bool& hdone, int lim) {
    if (!hdone && j >= fl) {
        for (int ii = 0; ii < fl; ii++)
            if (ii < lim) outk[ii] = ring[(ii + r0) & (RING - 1)];
        hdone = true;
    }
    if (fl + SECT <= j) {
        store_sector(ring, outk, fl, r0, lim);
        fl += SECT;
    }
}

// runs-mode flush after every step: the head once complete, then every complete sector.  A lane then
// holds < SECT unflushed values before a step, so a step may add up to RING - SECT + 1 values.
constexpr int RUNK = RING - SECT;                  // values one run step may add
__device__ __forceinline__ void flush_ring_all(const float* ring, float* outk, int r0, int& fl, int j, bool& hdone, int lim) {
    if (!hdone && j >= fl) {
        for (int ii = 0; ii < fl; ii++)
            if (ii < lim) outk[ii] = ring[(ii + r0) & (RING - 1)];
        hdone = true;
    }
    while (hdone && fl + SECT <= j) {
        store_sector(ring, outk, fl, r0, lim);
        fl += SECT;
    }
}
__device__ __forceinline__ void ring_put(float* ring, int j, int r0, int kr, float v) {
#pragma unroll
    for (int q = 0; q < RUNK; q++)
        if (q < kr) ring[(j + q + r0) & (RING - 1)] = v;
}

// Phase-B flushes with the global stores one flush behind the LDS reads: the sector read at flush k
// sits in registers and leaves at flush k+1, so no flush waits on its own LDS read.
struct PendSector {
    float4 a, b;
    int s0;
    bool have;
};
__device__ __forceinline__ void pend_store(PendSector& p, float* outk, int lim) {
    if (!p.have) return;
    if (p.s0 + SECT <= lim) {
        float4* o4 = reinterpret_cast<float4*>(outk + p.s0);
        o4[0] = p.a;
        o4[1] = p.b;
    } else {
        const float v[8] = {p.a.x, p.a.y, p.a.z, p.a.w, p.b.x, p.b.y, p.b.z, p.b.w};
        for (int i = 0; i < SECT && p.s0 + i < lim; i++) outk[p.s0 + i] = v[i];
    }
    p.have = false;
}
__device__ __forceinline__ void flush_ring_deferred(const float* ring, float* outk, int r0, int& fl, int j, bool& hdone,
                                                    int lim, PendSector& p) {
    if (!hdone && j >= fl) {
        for (int ii = 0; ii < fl; ii++)
            if (ii < lim) outk[ii] = ring[(ii + r0) & (RING - 1)];
        hdone = true;
    }
    if (fl + SECT <= j) {
        pend_store(p, outk, lim);
        const float4* r4 = reinterpret_cast<const float4*>(ring + ((fl + r0) & (RING - 1)));
        p.a = r4[0];
        p.b = r4[1];
        p.s0 = fl;
        p.have = true;
        fl += SECT;
    }
}

struct DecodeShared {
    uint32_t L[LWORDS];
    TokLut T;                                      // token length / pattern tables (build_lut)
    union {
        float ring[GROUP * RING];                  // decode pass output rings
        struct {                                   // carry scan (in place, two barriers a step)
            uint8_t kd[3][GROUP];
            float fv[3][GROUP];
        } k;
    } u;
    float tin[3];
    int need, cplx, defer, badin;
    long long tile;
#ifdef DC_DEC_PAD
    uint32_t occpad[DC_DEC_PAD / 4];            // occupancy experiment: extra LDS per workgroup
#endif
};

__device__ __forceinline__ uint64_t hpack(uint64_t flag, uint32_t epoch, uint32_t kind, float v) {
    return (flag << 62) | ((uint64_t)(epoch & 0x3FFFFFu) << 40) | ((uint64_t)(kind & 0xFF) << 32) | (uint64_t)__float_as_uint(v);
}
__device__ __forceinline__ int hflag(uint64_t v, uint32_t epoch) {
    return (((v >> 40) & 0x3FFFFFu) == (epoch & 0x3FFFFFu)) ? (int)(v >> 62) : 0;
}

template <int CT>
__global__ __launch_bounds__(GROUP) void decode_kernel_fast(const uint8_t* __restrict__ s, Params P, DecBufs D,
                                                            float* __restrict__ out, long long num, uint32_t epoch) {
    __shared__ DecodeShared S;
    const Plan pl = *D.plan;
    const int c = threadIdx.x;
    // a runs-mode stream whose tile chain failed (tile_fix reported an unknown entry) is resolved exactly
    // by dc_decode_finish (resolve_kernel, then this kernel again): nothing to decode now
    // (the tile loop is skipped, not the epilogue: the ticket counters below must still be reset)
    const bool skip_all = pl.runs && (__hip_atomic_load(D.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 8u);
    build_lut<CT>(S.T, P, c, GROUP);                                  // visible after the first barrier
    while (!skip_all) {
        if (c == 0) S.tile = (long long)atomicAdd(&D.ctr[4], 1u);
        __syncthreads();
        const long long t = S.tile;
        if (t >= pl.ngroups) break;
        const long long tbit = t * (long long)GROUP * CHUNK_BITS;
        STAMP(8);
        const long long gc = t * GROUP + c;
        // the tile's chain records are loaded before the stream is staged (one memory round trip)
        const uint32_t te = D.tentry[t];
        const unsigned long long base = D.tbase[t];
        const int tmx = (int)D.tmap[t * 4 + 3];
        const int e_rec = D.entry[gc];
        const unsigned long long off_rec = D.tokoff[gc];
        stage_tile(S.L, s, pl.nbytes, tbit >> 5);
        const long long rem = (long long)pl.nbits - tbit;
        const int nact = (int)min((long long)GROUP, (rem + CHUNK_BITS - 1) / CHUNK_BITS);
        const bool act = c < nact;
        const int cs = c * CHUNK_BITS;
        const int cend = (int)min((long long)(cs + CHUNK_BITS), rem);
        if (c == 0) { S.need = 0; S.cplx = 0; S.defer = 0; S.badin = 0; }
        // ---- entry and first token index of every chunk (parse kernel chain + tile_fix overrides)
        const int ein = (int)(te & 63), c0 = (int)((te >> 6) & 1023), kjoin = (int)(te >> 16);
        int e = UNKE;
        unsigned long long k0 = 0;
        if (act && ein != UNKE) {
            if (c == 0) {
                e = ein;
                k0 = base;
            } else {
                e = e_rec;
                const long long rel = (long long)off_rec + (c >= kjoin ? (long long)tmx : 0ll);
                k0 = base + (unsigned long long)(c0 + rel);
            }
            D.entry[gc] = (uint8_t)e;
            D.tokoff[gc] = k0;
        }
        if (act && ein == UNKE) { D.entry[gc] = UNKE; atomicOr(D.err, 8u); }
        __syncthreads();
        STAMP(9);

        // ---- pass 1: decode from the true entry; concrete values are stored immediately
        const bool first = (gc == 0) && D.shard == 0;    // a shard's first chunk has symbolic history
        float f1 = -1.0f, f2 = -1.0f, f3 = -1.0f;
        int k1 = first ? 0 : 1, k2 = first ? 0 : 2, k3 = first ? 0 : 3;
        int pend = 0;
        bool sent = false;
        const int a0 = (int)((reinterpret_cast<uintptr_t>(out) >> 2) & (SECT - 1));
        float* ring = S.u.ring + c * RING;
        const bool dec = act && e != UNKE;
        float* outk = out + (long long)k0;
        if (dec) {
            const long long k0l = (long long)k0;
            const int r0 = (int)((k0l + a0) & (RING - 1));
            int fl = (int)((SECT - ((k0l + a0) & (SECT - 1))) & (SECT - 1));   // first sector start
            bool hdone = false;                                      // head (partial first sector) stored
            const long long liml = num - k0l;
            const int lim = liml > 0x7FFFFFFFll ? 0x7FFFFFFF : (int)max(liml, 0ll);
            Rd r;
            r.init(S.L, cs + e);
            int j = 0, it = 0;
            const bool runs = CT != 6 && pl.runs;
            // phase A: history still (partly) symbolic, or the stream's first three tokens.  In runs mode
            // a run of identical '100' / '101' codes is one step (Himeno planes start their chunks inside
            // '101' runs, symbolic until the row's raw token)
            while (r.pos < cend && ((k1 | k2 | k3) != 0 || (first && j < 3))) {
                r.fetch(S.L);
                const uint32_t tk = r.peek();
                const uint32_t meta = S.T.meta[tk >> 23];
                uint32_t pat = lut_pattern(S.T, tk, meta);
                int code = 0;
                if (CT != 6) {
                    const bool c3 = (int)tk < 0;
                    code = c3 ? (int)__builtin_amdgcn_ubfe(tk, 29u, 2u) : 0;
                    pat = c3 ? 0u : pat;
                }
                const int kr = (runs && !(first && j < 3)) ? run_same(tk, r.pos, cend, RUNK) : 1;
                const float p2 = predict2(f1, f2), p3 = predict3(f1, f2, f3);
                const float v = code == 0 ? __uint_as_float(pat) : (code == 1 ? f1 : (code == 2 ? p2 : p3));
                const int kind = code == 0 ? 0 : (code == 1 ? k1 : (code == 2 ? ((k1 | k2) ? 4 : 0) : ((k1 | k2 | k3) ? 4 : 0)));
                if (kind != 0) pend = j + kr;                        // re-decoded by the fix-up
                // history sentinel (-1.0f) or a prediction before the stream's history is full: exact path
                sent |= (kind == 0 && __float_as_uint(v) == 0xBF800000u) || (first && j < 3 && code != 0);
                if (runs) {
                    ring_put(ring, j, r0, kr, v);
                    f3 = kr >= 3 ? v : (kr == 2 ? f1 : f2); k3 = kr >= 3 ? kind : (kr == 2 ? k1 : k2);
                    f2 = kr >= 2 ? v : f1; k2 = kr >= 2 ? kind : k1;
                    f1 = v; k1 = kind;
                    r.step(kr > 1 ? 3 * kr : (int)(meta >> 8));
                    j += kr;
                    flush_ring_all(ring, outk, r0, fl, j, hdone, lim);
                    continue;
                }
                ring[(j + r0) & (RING - 1)] = v;
                f3 = f2; k3 = k2; f2 = f1; k2 = k1; f1 = v; k1 = kind;
                r.step((int)(meta >> 8));
                j++;
                if (++it == SECT) {                                  // uniform among the active lanes
                    it = 0;
                    flush_ring(ring, outk, r0, fl, j, hdone, lim);
                }
            }
            flush_ring(ring, outk, r0, fl, j, hdone, lim);
            it = 0;
            const bool chk_all = (CT == 6 && P.B >= 23) || (CT == 7 && (P.mask17 >> 16) != 0u && P.mm == 23);
            int sentv = 0;
            // phase B in runs mode: one lane-divergent loop, a run of identical '100' / '101' codes per step
            if (runs) {
                while (r.pos < cend) {
                    r.fetch(S.L);
                    const uint32_t tk = r.peek();
                    const uint32_t meta = S.T.meta[tk >> 23];
                    const uint32_t pat = lut_pattern(S.T, tk, meta);
                    const uint32_t cc = __builtin_amdgcn_ubfe(tk, 29u, 3u);    // 4..7 = '100'..'111'
                    const int kr = run_same(tk, r.pos, cend, RUNK);
                    float v = cc < 4u ? __uint_as_float(pat) : (cc == 5u ? f1 : 0.0f);
                    if (cc >= 6u) {
                        v = cc == 6u ? predict2(f1, f2) : predict3(f1, f2, f3);
                        sentv |= __float_as_uint(v) == 0xBF800000u ? 1 : 0;
                    }
                    if (chk_all) sentv |= __float_as_uint(v) == 0xBF800000u ? 1 : 0;
                    ring_put(ring, j, r0, kr, v);
                    f3 = kr >= 3 ? v : (kr == 2 ? f1 : f2);
                    f2 = kr >= 2 ? v : f1;
                    f1 = v;
                    r.step(kr > 1 ? 3 * kr : (int)(meta >> 8));
                    j += kr;
                    flush_ring_all(ring, outk, r0, fl, j, hdone, lim);
                }
            }
            // phase B: concrete history (kinds stay 0 from here on).  Runs in uniform blocks of SECT
            // steps with per-lane predication (a finished lane steps by 0 and keeps its history), so
            // the only branches are the block loop, the flush and the rare prediction branch.  Only
            // '110'/'111' predictions can make the -1.0f sentinel here unless chk_all (CT6 or a
            // negative mask with 23 kept mantissa bits: patterns without a midpoint bit).
            PendSector ps;
            ps.have = false;
            ps.s0 = 0;
            while (__any(r.pos < cend)) {
#pragma unroll
                for (int u = 0; u < SECT; u++) {
                    r.fetch(S.L);
                    const uint32_t tk = r.peek();
                    const uint32_t meta = S.T.meta[tk >> 23];
                    const uint32_t pat = lut_pattern(S.T, tk, meta);
                    const bool on = r.pos < cend;
                    float v;
                    if (CT == 6) {
                        v = __uint_as_float(pat);
                    } else {
                        const uint32_t cc = __builtin_amdgcn_ubfe(tk, 29u, 3u);    // 4..7 = '100'..'111'
                        v = cc < 4u ? __uint_as_float(pat) : (cc == 5u ? f1 : 0.0f);
                        if (__builtin_expect(__any(on && cc >= 6u), 0)) {       // predictions: wave-uniform branch
                            const float p2 = predict2(f1, f2), p3 = predict3(f1, f2, f3);
                            v = cc == 6u ? p2 : (cc == 7u ? p3 : v);
                            sentv |= (on && cc >= 6u && __float_as_uint(v) == 0xBF800000u) ? 1 : 0;
                        }
                    }
                    if (chk_all) sentv |= (on && __float_as_uint(v) == 0xBF800000u) ? 1 : 0;
                    ring[(j + r0) & (RING - 1)] = v;
                    f3 = on ? f2 : f3; f2 = on ? f1 : f2; f1 = on ? v : f1;
                    r.step(on ? (int)(meta >> 8) : 0);
                    j += on ? 1 : 0;
                }
                flush_ring_deferred(ring, outk, r0, fl, j, hdone, lim, ps);
            }
            pend_store(ps, outk, lim);
            sent |= sentv != 0;
            flush_ring(ring, outk, r0, fl, j, hdone, lim);
            const int t0 = hdone ? fl : 0;                           // tail, or a chunk inside one sector
            for (int ii = t0; ii < j; ii++)
                if (ii < lim) outk[ii] = ring[(ii + r0) & (RING - 1)];
        }
        if (sent) atomicOr(D.err, 128u);
        sent = false;
        if (!act || e == UNKE) { k1 = 1; k2 = 2; k3 = 3; }
        __syncthreads();                                   // resolution arrays are dead from here
        S.u.k.kd[0][c] = (uint8_t)k1; S.u.k.kd[1][c] = (uint8_t)k2; S.u.k.kd[2][c] = (uint8_t)k3;
        S.u.k.fv[0][c] = f1; S.u.k.fv[1][c] = f2; S.u.k.fv[2][c] = f3;
        // the scan only serves pending prefixes and a tile whose last chunk ends on symbolic history: when
        // no chunk left a prefix pending and the last chunk's history is concrete, F_last is that history
        const int lastc = nact - 1;
        const bool anypend = __syncthreads_or(act && pend > 0);
        const bool noscan = !anypend && S.u.k.kd[0][lastc] == 0 && S.u.k.kd[1][lastc] == 0 && S.u.k.kd[2][lastc] == 0;
        const int fsrc = noscan ? lastc : GROUP - 1;        // where the tile's outgoing history is read
        STAMP(10);
        // ---- inclusive scan of carry functions: F_c = f_c o ... o f_0
        for (int d = 1; d < (noscan ? 1 : GROUP); d <<= 1) {
            int kk[3];
            float vv[3];
#pragma unroll
            for (int i = 0; i < 3; i++) {
                const int k0i = S.u.k.kd[i][c];
                kk[i] = k0i;
                vv[i] = S.u.k.fv[i][c];
                if (c >= d && k0i >= 1 && k0i <= 3) {
                    kk[i] = S.u.k.kd[k0i - 1][c - d];
                    vv[i] = S.u.k.fv[k0i - 1][c - d];
                }
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 3; i++) {
                S.u.k.kd[i][c] = (uint8_t)kk[i];
                S.u.k.fv[i][c] = vv[i];
            }
            __syncthreads();
        }
        int ik[3];
        float iv[3];
        for (int i = 0; i < 3; i++) {
            ik[i] = c == 0 ? i + 1 : S.u.k.kd[i][c - 1];
            iv[i] = c == 0 ? 0.0f : S.u.k.fv[i][c - 1];
        }
        if (pend > 0) {
            bool needs = false, cx = false;
            for (int i = 0; i < 3; i++) { needs |= (ik[i] >= 1 && ik[i] <= 3); cx |= (ik[i] == 4); }
            if (needs) S.need = 1;
            if (cx) S.cplx = 1;
        }
        const int tk0 = S.u.k.kd[0][fsrc], tk1 = S.u.k.kd[1][fsrc], tk2 = S.u.k.kd[2][fsrc];
        if (c == 0) {
            for (int i = 0; i < 3; i++)
                st_relaxed(&D.hist[t * 6 + i], hpack(1, epoch, S.u.k.kd[i][fsrc], S.u.k.fv[i][fsrc]));
            if (tk0 == 0 && tk1 == 0 && tk2 == 0)
                for (int i = 0; i < 3; i++)
                    st_relaxed(&D.hist[t * 6 + 3 + i], hpack(2, epoch, 0, S.u.k.fv[i][fsrc]));
            if (tk0 == 4 || tk1 == 4 || tk2 == 4) S.cplx = 1;
        }
        __syncthreads();
        const int need = S.need, cplx = S.cplx;
        if (cplx) {
            if (c == 0) {
                atomicOr(D.err, 32u);
                for (int i = 0; i < 3; i++) st_relaxed(&D.hist[t * 6 + 3 + i], hpack(2, epoch, 4, 0.0f));
            }
            if (act) { D.pend[gc] = (uint16_t)min(pend, 65535); D.done[gc] = 0; }
            __syncthreads();
            continue;
        }
        // ---- tile incoming (history look-back), lanes 0..2 = b1..b3
        if (need && c < 3) {
            float val = -1.0f;
            int j = c;
            long long k = t - 1;
            unsigned spins = 0;
            bool bad = false;
            while (k >= 0) {
                const uint64_t pv = ld_relaxed(&D.hist[k * 6 + 3 + j]);
                if (hflag(pv, epoch) == 2) {
                    if (((pv >> 32) & 0xFF) == 4) bad = true;
                    val = __uint_as_float((uint32_t)pv);
                    break;
                }
                const uint64_t av = ld_relaxed(&D.hist[k * 6 + j]);
                if (hflag(av, epoch) == 1) {
                    const int kind = (int)((av >> 32) & 0xFF);
                    if (kind == 0) { val = __uint_as_float((uint32_t)av); break; }
                    if (kind >= 1 && kind <= 3) { j = kind - 1; k--; continue; }
                }
                if (++spins > (1u << 24)) { bad = true; atomicOr(D.err, 16u); break; }
                __builtin_amdgcn_s_sleep(1);
            }
            if (k < 0 && !bad) {                             // before the stream: a shard's incoming values
                if (D.shard == 2) val = D.hin[j];
                else if (D.shard == 1) S.defer = 1;
            }
            if (bad) { atomicOr(D.err, 32u); S.badin = 1; }
            S.tin[c] = val;
        }
        __syncthreads();
        const bool defer = need && S.defer;                  // incoming values unknown yet (shard, mode 1)
        // the incoming history came from a tile left to the serial fix-up (kind 4): so is this tile
        const bool badin = need && S.badin;
        if (need && c == 0 && !(tk0 == 0 && tk1 == 0 && tk2 == 0)) {
            const int kk[3] = {tk0, tk1, tk2};
            for (int i = 0; i < 3; i++)
                st_relaxed(&D.hist[t * 6 + 3 + i],
                           (defer || badin) ? hpack(2, epoch, 4, 0.0f)
                                            : hpack(2, epoch, 0, kk[i] == 0 ? S.u.k.fv[i][fsrc] : S.tin[kk[i] - 1]));
        }
        if (badin) {                                         // every pending prefix: dc_launch_fixup_serial
            if (act) { D.pend[gc] = (uint16_t)min(pend, 65535); D.done[gc] = 0; }
            __syncthreads();
            continue;
        }
        // deferred: prefixes that depend on the shard's incoming values wait for dc_decode_shard_fix
        const bool dchunk = defer && act && pend > 0 &&
                            ((ik[0] >= 1 && ik[0] <= 3) || (ik[1] >= 1 && ik[1] <= 3) || (ik[2] >= 1 && ik[2] <= 3));
        if (dchunk) atomicOr(D.err, 256u);
        // ---- fix-up: re-decode the pending prefix with concrete history
        if (act && pend > 0 && !dchunk) {
            float g1 = ik[0] == 0 ? iv[0] : S.tin[ik[0] - 1];
            float g2 = ik[1] == 0 ? iv[1] : S.tin[ik[1] - 1];
            float g3 = ik[2] == 0 ? iv[2] : S.tin[ik[2] - 1];
            Rd r;
            r.init(S.L, cs + e);
            const bool runs = CT != 6 && pl.runs;
            for (int jj = 0; jj < pend;) {
                r.fetch(S.L);
                const uint32_t tk = r.peek();
                const uint32_t meta = S.T.meta[tk >> 23];
                const int len = (int)(meta >> 8);
                uint32_t pat = lut_pattern(S.T, tk, meta);
                int code = 0;
                if (CT != 6) {
                    const bool c3 = (int)tk < 0;
                    code = c3 ? (int)__builtin_amdgcn_ubfe(tk, 29u, 2u) : 0;
                    pat = c3 ? 0u : pat;
                }
                // runs mode: a run of identical '100' / '101' codes inside the prefix is one step
                const int kr = runs ? min(run_same(tk, 0, 30, 10), pend - jj) : 1;
                const float v = code == 0 ? __uint_as_float(pat) : predict_value(code, g1, g2, g3);
                for (int q = 0; q < kr; q++)
                    if (k0 + jj + q < (unsigned long long)num) outk[jj + q] = v;
                sent |= __float_as_uint(v) == 0xBF800000u;
                g3 = kr >= 3 ? v : (kr == 2 ? g1 : g2);
                g2 = kr >= 2 ? v : g1;
                g1 = v;
                r.step(kr > 1 ? 3 * kr : len);
                jj += kr;
            }
        }
        if (act) { D.pend[gc] = (uint16_t)min(pend, 65535); D.done[gc] = (pend && !dchunk) ? 1 : 0; }
        if (sent) atomicOr(D.err, 128u);
        __syncthreads();
        STAMP(11);
    }
    if (c == 0) {
        __threadfence();
        if (atomicAdd(&D.ctr[5], 1u) == gridDim.x - 1) { atomicExch(&D.ctr[4], 0u); atomicExch(&D.ctr[5], 0u); }
    }
}

// ------------------------------------------------------------------------------------------------
#define DC_DISPATCH_F(CTV, KER, ...)                                                                 \
    switch (CTV) {                                                                                   \
        case 5: hipLaunchKernelGGL(KER<5>, __VA_ARGS__); break;                                      \
        case 6: hipLaunchKernelGGL(KER<6>, __VA_ARGS__); break;                                      \
        case 7: hipLaunchKernelGGL(KER<7>, __VA_ARGS__); break;                                      \
        case 11: hipLaunchKernelGGL(KER<11>, __VA_ARGS__); break;                                    \
        default: return -2;                                                                          \
    }

// resident decode workgroups (persistent grid; tiles are claimed from an atomic counter in order)
static int decode_grid(int ct) {
    static int cache[12];
    const int ci = (ct > 0 && ct < 12) ? ct : 0;
    if (cache[ci]) return cache[ci];
    int dev = 0, ncu = 256, per = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const void* f = ct == 5 ? (const void*)decode_kernel_fast<5> : ct == 6 ? (const void*)decode_kernel_fast<6>
                  : ct == 7 ? (const void*)decode_kernel_fast<7> : (const void*)decode_kernel_fast<11>;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, f, GROUP, 0) != hipSuccess || per < 1) per = 1;
    cache[ci] = per * ncu;
    const char* e = getenv("DC_DECODE_GRID");                 // experiment override
    if (e && atoi(e) > 0) cache[ci] = atoi(e);
    return cache[ci];
}

// after resolve_kernel (exact entries and global first-token indices of every chunk): the tile records
// the fast decode reads -- tile entry, token base, chunk offsets relative to it, no tile_fix join
__global__ __launch_bounds__(GROUP) void tiles_from_resolved_kernel(DecBufs D) {
    const Plan pl = *D.plan;
    for (long long t = blockIdx.x; t < pl.ngroups; t += gridDim.x) {
        const long long g0 = t * GROUP, gc = g0 + threadIdx.x;
        const unsigned long long base = D.tokoff[g0];
        if (threadIdx.x > 0 && gc < pl.nchunks) D.tokoff[gc] -= base;
        if (threadIdx.x == 0) {
            D.tentry[t] = (uint32_t)D.entry[g0] & 63u;       // UNK (63) stays UNKE: the decode reports it
            D.tbase[t] = base;
            D.tmap[t * 4 + 3] = 0;
        }
    }
}

extern "C" int dc_launch_decode_fast_resolved(const uint8_t* s, long long max_chunks, const Params* P,
                                              const DecBufs* D, float* out, long long num, uint32_t epoch,
                                              hipStream_t st) {
    const long long max_groups = (max_chunks + GROUP - 1) / GROUP;
    const int g = (int)std::min<long long>(max_groups > 0 ? max_groups : 1, 4096);
    hipLaunchKernelGGL(tiles_from_resolved_kernel, dim3(g), dim3(GROUP), 0, st, *D);
    const int gdec = (int)std::min<long long>(max_groups > 0 ? max_groups : 1, decode_grid(P->ct));
    DC_DISPATCH_F(P->ct, decode_kernel_fast, dim3(gdec), dim3(GROUP), 0, st, s, *P, *D, out, num, epoch);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int dc_launch_decode_fast(const uint8_t* s, const unsigned long long* dev_nbits,
                                     unsigned long long host_nbits, long long max_chunks, const Params* P,
                                     const DecBufs* D, float* out, long long num, uint32_t epoch, hipStream_t st) {
    const long long max_groups = (max_chunks + GROUP - 1) / GROUP;
    static const long long parse_grid = [] {                  // DC_PARSE_GRID: experiment override
        const char* e = getenv("DC_PARSE_GRID");
        return (e && atoll(e) > 0) ? atoll(e) : 256ll * 16;   // swept 1024..16384: 4096 best (parse 161 -> 154 us)
    }();
    const int gparse = (int)std::min<long long>(max_groups > 0 ? max_groups : 1, parse_grid);
    dc_mark_phase(4, st);
    DC_DISPATCH_F(P->ct, parse_kernel, dim3(gparse), dim3(GROUP), 0, st, s, *P, *D, dev_nbits, host_nbits, max_chunks, num);
    dc_mark_phase(5, st);
    DC_DISPATCH_F(P->ct, tile_fix_kernel, dim3((unsigned)((max_groups + 3) / 4 > 0 ? (max_groups + 3) / 4 : 1)), dim3(256), 0, st,
                  s, *P, *D);
    hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, st, *D);
    const int gdec = (int)std::min<long long>(max_groups > 0 ? max_groups : 1, decode_grid(P->ct));
    dc_mark_phase(6, st);
    DC_DISPATCH_F(P->ct, decode_kernel_fast, dim3(gdec), dim3(GROUP), 0, st, s, *P, *D, out, num, epoch);
    dc_mark_phase(7, st);
    dc_mark_next_set();
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace dc
