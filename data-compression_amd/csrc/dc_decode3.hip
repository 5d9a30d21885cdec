// dc_decode3.hip -- segment decoder: the fast path of the bit-wise decoders of impl/dataCompression.c
// (myDecompress_bitwise :2922, _np :2459, _mask :1703, _op :698) for streams of ordinary density.
//
// The token walk is one dependent chain per reader: each step reads the next stream word and a table
// entry from LDS and is ~250 cycles of latency on gfx950.  Throughput therefore needs many chains per
// SIMD and few LDS bank conflicts, with as few walks per token as possible:
//
// parse3_kernel  one wave per parse job.  Lane l walks SEGMENT l of the job (seg 256-bit chunks, tens
//                of thousands of bits; 4, 8 or 16 chunks by stream size) after a 1024-bit pre-walk
//                (self-synchronisation), reading the stream through a per-lane LDS ring of
//                16 words refilled 128 bits at a time with loads issued two phases ahead.  The ring is
//                stored [word][lane], so every ds_read_b32 of a wave hits 32 distinct banks whatever the
//                lanes' offsets.  At every chunk boundary the lane records the chunk's entry offset and
//                token count (16 bits).  Links are checked afterwards: a segment's first entry must
//                equal the previous segment's exit (in-wave shuffle; across jobs the previous job's
//                exit, published after its main walk and in-job repairs and waited for -- no chain: an
//                exit never waits for another job; a wait past its bound, never seen, hands the stream
//                to the chunk-map decoder).  A broken link (the pre-walk had not synchronised, ~0.24% of
//                CT7 segments at 1e-3, tools/sync_sim.py) is repaired by re-walking from the true entry
//                until the path meets the recorded entries again (~1.25 chunks on average).  The
//                wave's token counts are scanned into job-relative first-token offsets of every decode job.
// decode3_kernel one wave per decode job of 64 chunks: lane = chunk, decoded from its recorded entry for
//                its recorded token count (the job's first token: the wave's running sum of the parse
//                jobs' totals, advanced by a prefetched window per job -- no scan launch).  Values go to a wave-private LDS buffer at their job-relative
//                index (aligned to the output's 16-byte grid) and leave as whole float4 stores.
//                Predicted codes ('101'/'110'/'111', rare in ordinary data) read their history from that
//                buffer; the first tokens of a chunk that need the previous chunk's values are left
//                pending and re-decoded lane by lane afterwards (the job's first chunk takes the previous
//                job's last three values, published as epoch-tagged granules).
// A stream outside these assumptions (runs mode: mostly 3-bit codes; a repair that does not converge;
// more tokens per job than the buffer holds; the -1.0f history sentinel) sets status 512 and is decoded
// by the chunk-map decoder of dc_decode_fast.hip instead (dc_decode_finish).
#include "dc_device.h"
#include <algorithm>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

namespace dc {

#ifndef DC_WALK2
#define DC_WALK2 0
#endif
#ifndef DC_EXIT_EARLY
#define DC_EXIT_EARLY 1                 // 8/16-chunk segments: a job's exit published right after its main walk
#endif
#ifndef DC_P3_PW4
#define DC_P3_PW4 1024
#endif
// pre-walk: 1024 bits (4 chunks, one region line) before every segment (DC_PARSE_PL6=2: 2048 for CT6 --
// 12% instead of 94% of its jobs repair, but the longer walk cost more: config 2 parse3 98 vs 92 us)
#ifndef DC_PARSE_PL6
#define DC_PARSE_PL6 1
#endif
constexpr int D3_SEG = 16;             // chunks per parse segment (4 region lines); 8 for small streams

constexpr int D3_RING = 16;            // ring words per lane (four 128-bit phases; a power of two: the fetch wraps)
constexpr int D3_CAP = 1024 + 16;      // decode job output buffer (floats per wave)
constexpr int D3_CAP_DENSE = 2048 + 32; // the dense instantiation's (< ~16 bits per value, e.g. CT7 at 1e-2: 3
                                        // workgroups per CU by LDS instead of 4; dc_launch_decode3's `dense`)
constexpr uint32_t D3_DECLINE = 512u;
#ifndef D3_MAX_ROUNDS
#define D3_MAX_ROUNDS 8                 // repair rounds of a parse job before the stream is declined (64: a
                                        // stream that never resynchronises, e.g. a noisy ramp, spent ~1 ms
                                        // per decode in them; U10 at 1e-3 / 1e-6 never needs more than 8)
#endif
// s_memrealtime ticks (100 MHz): 2 ms.  Jobs are dispatched in order on each XCD but not across XCDs, so with
// another kernel running beside (bench.py's pipelined pass: the next step's encode) a job's predecessor can
// start more than 200 us after it -- the old bound declined such streams (status 0xa00 with 20-chunk
// segments); the bound only guards against a wait that never ends, which has not been seen.  (r06) 20 ms: two
// ranks sharing one GPU (the gloo rehearsal of the multi-rank bench) still hit 2 ms beside the other process's
// encode (status 0xa00 after the timed steps); a real hang ends all the same
constexpr unsigned long long D3_LINK_WAIT = 2000000;
// why (diagnostic bits beside 512): 1024 runs mode / capacity, 2048 unresolved link, 4096 fewer tokens
// than values, 8192 a job denser than its buffer, 16384 the history sentinel or an early prediction
constexpr uint32_t D3_WHY_RUNS = 1024u, D3_WHY_LINK = 2048u, D3_WHY_SHORT = 4096u, D3_WHY_DENSE = 8192u,
                   D3_WHY_SENT = 16384u, D3_WHY_SHARD = 65536u;   // (32768: D3_ZMISS)

// DC_DEC3_PROF builds (make XDEFS=-DDC_DEC3_PROF B=build_p L=lib_p): per-section shader-clock totals
// summed over waves into g_prof3 (read with dc_dec3_prof_read; tools/dec3_prof.py)
#ifdef DC_DEC3_PROF
__device__ unsigned long long g_prof3[32];
#define P3_DECL() unsigned long long p3a[16] = {0}
#define P3_T(v) const long long v = clock64()
#define P3_ADD(i, val) (p3a[i] += (unsigned long long)(val))
#define P3_MAX(i, val) (((threadIdx.x & 63) == 0) ? (void)atomicMax(&g_prof3[i], (unsigned long long)(val)) : (void)0)
#define P3_FLUSH()                                                                                     \
    do {                                                                                               \
        if ((threadIdx.x & 63) == 0)                                                                   \
            for (int i_ = 0; i_ < 16; i_++)                                                            \
                if (p3a[i_]) atomicAdd(&g_prof3[i_], p3a[i_]);                                         \
    } while (0)
#define P3_PARAM , unsigned long long* p3a
#define P3_ARG , p3a
#else
#define P3_PARAM
#define P3_ARG
#define P3_DECL() do {} while (0)
#define P3_T(v) do {} while (0)
#define P3_ADD(i, val) do {} while (0)
#define P3_MAX(i, val) do {} while (0)
#define P3_FLUSH() do {} while (0)
#endif

__device__ __forceinline__ uint32_t bsw(uint32_t v) { return __builtin_bswap32(v); }

// 4 stream words from word gw (a multiple of 4), MSB-first, through a buffer resource whose range is
// the buffer's readable capacity (capw words, a multiple of 4, every stream byte inside it): groups
// outside it -- before the stream (a negative offset wraps past the range) or past the capacity -- read
// as 0 in hardware, so the load is one unconditional buffer_load_dwordx4 that stays in flight until its
// words are used (a branchy or select-guarded global load made the compiler wait at once).  Bytes past
// the stream's end read as 0, as the reference's reader sees them.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t stream_rsrc(const uint8_t* s, long long capw) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(s), (short)0, (int)(capw * 4), 0x00020000);
}
__device__ __forceinline__ uint32_t keep_bytes(uint32_t w, int rem) {     // rem = stream bytes left at w
    return (uint32_t)(0xFFFFFFFF00000000ull >> (8 * min(max(rem, 0), 4))) & w;
}
// (stream offsets fit 31 bits: the host takes this decoder only for capacities below 2 GiB).  The raw
// load and its finishing (byte order, the stream's end) are separate, so that nothing touches the loaded
// registers before the words are needed and the load stays in flight.
__device__ __forceinline__ uint4 load_raw4(__amdgpu_buffer_rsrc_t rs, long long gw) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(uint32_t)(gw * 4), 0, 0);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 finish4(uint4 v, long long nbytes, long long gw) {
    uint4 w = make_uint4(bsw(v.x), bsw(v.y), bsw(v.z), bsw(v.w));
    const int r0 = (int)nbytes - (int)(uint32_t)(gw * 4);
    if (r0 < 16) {                            // the group holding the stream's last byte (or past it: 0 already)
        w.x = keep_bytes(w.x, r0);
        w.y = keep_bytes(w.y, r0 - 4);
        w.z = keep_bytes(w.z, r0 - 8);
        w.w = keep_bytes(w.w, r0 - 12);
    }
    return w;
}
__device__ __forceinline__ uint4 load_w4(__amdgpu_buffer_rsrc_t rs, long long nbytes, long long gw) {
    return finish4(load_raw4(rs, gw), nbytes, gw);
}

__device__ __forceinline__ bool declined_now(const Dec3Bufs& D3) {
    return (__hip_atomic_load(D3.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & D3_DECLINE) != 0;
}

struct Geo3 {
    unsigned long long nbits;
    long long nbytes, nchunks, nseg, npjobs, ndjobs;
};
template <int SEG>
__device__ __forceinline__ Geo3 geo3(const unsigned long long* dev_nbits, unsigned long long host_nbits) {
    constexpr int seg = SEG;
    Geo3 g;
    g.nbits = dev_nbits ? *dev_nbits : host_nbits;
    g.nbytes = (long long)((g.nbits + 7) >> 3);
    g.nchunks = (long long)((g.nbits + 255) >> 8);
    g.nseg = (g.nchunks + seg - 1) / seg;
    g.npjobs = (g.nseg + 63) / 64;
    g.ndjobs = (g.nchunks + 63) / 64;
    return g;
}

// ------------------------------------------------------------------------------------------------
// parse: the per-lane ring reader.  Ring word i of lane l lives at LDS dword (i mod 16)*64 + l; ring word 0
// is segment-relative word 4*kbase of the current epoch.  The fetch address wraps inside the 16 words
// ((addr + 256) & 0xFFF keeps the lane's byte offset, < 256), so no mirror words are needed: 4 KB of ring
// per wave (was 5 KB with a 4-word mirror), which holds 6 parse waves per SIMD instead of 5.
constexpr uint32_t D3_RMASK = (uint32_t)(D3_RING * 256 - 1);
struct Ring3 {
    uint32_t* L;
    uint32_t lc;                                    // lane * 4
    uint32_t a, b, c, s, addr;                      // window (a:b) from bit 32 - s of a, c, next fetch address
    int pos;                                        // segment-relative bit
    __device__ __forceinline__ uint32_t R(int i) const { return L[((i & (D3_RING - 1)) << 6) + (int)(lc >> 2)]; }
    __device__ __forceinline__ void init(int p, int kbase) {
        const int wi = (p - 1) >> 5;                // word holding bit p - 1 (floor for p <= 0)
        const int li = wi - 4 * kbase;
        s = (uint32_t)(32 * (wi + 1) - p);
        a = R(max(li, 0)); b = R(li + 1); c = R(li + 2);
        addr = (((uint32_t)(li + 3) << 8) | lc) & D3_RMASK;
        pos = p;
    }
    __device__ __forceinline__ void put(int slot, uint4 v) {
        L[((slot * 4 + 0) << 6) + (lc >> 2)] = v.x; L[((slot * 4 + 1) << 6) + (lc >> 2)] = v.y;
        L[((slot * 4 + 2) << 6) + (lc >> 2)] = v.z; L[((slot * 4 + 3) << 6) + (lc >> 2)] = v.w;
    }
    // walk until pos >= pend; tokens stepped
    __device__ __forceinline__ int walk(int pend, const uint8_t* tl) {
        int n = 0;
#if DC_WALK2
        // two steps per loop round, the second predicated (a lane past pend steps by 0): one exit test and
        // one exec update per two tokens
        while (pos < pend) {
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const uint32_t nx = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(L) + addr);
                const uint32_t t = __builtin_amdgcn_alignbit(a, b, s);
                int len = tl[t >> 23];
                if (u == 1) len = pos < pend ? len : 0;
                uint32_t d;
                const bool adv = __builtin_usub_overflow(s, (uint32_t)len, &d);
                s = d & 31u;
                pos += len;
                a = adv ? b : a;
                b = adv ? c : b;
                c = adv ? nx : c;
                addr = (addr + (adv ? 256u : 0u)) & D3_RMASK;
                n += len > 0 ? 1 : 0;
            }
        }
        return n;
#endif
        while (pos < pend) {
            const uint32_t nx = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(L) + addr);
            const uint32_t t = __builtin_amdgcn_alignbit(a, b, s);
            const int len = tl[t >> 23];
            uint32_t d;
            const bool adv = __builtin_usub_overflow(s, (uint32_t)len, &d);
            s = d & 31u;
            pos += len;
            a = adv ? b : a;
            b = adv ? c : b;
            c = adv ? nx : c;
            addr = (addr + (adv ? 256u : 0u)) & D3_RMASK;
            n++;
        }
        return n;
    }
};

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
    (void)lane;
    return wave_scan_incl(v);                       // DPP, no LDS round trips
}

// The lane's region is read one 128-byte line (8 phases, 4 chunks) at a time through 8 staged uint4
// (VGPRs): a line's first half is requested right after the staging it reuses went to the ring, 5
// phases before it is needed, and its halves close together -- each stream line leaves HBM once (16-byte
// loads spread over 8 phases let L2 drop the line between them: 8x the stream in fetch).  Region line
// L covers segment phases 8(L-1) .. 8(L-1)+7 (line 0: the 1024-bit pre-walk).
struct Stage8 {
    uint4 S[8];
};
__device__ __forceinline__ void stage_half(Stage8& st, int h0, __amdgpu_buffer_rsrc_t rs, long long gw) {
#pragma unroll
    for (int h = 0; h < 4; h++) st.S[h0 + h] = load_raw4(rs, gw + 4 * h);
}

// walk region lines L0 .. L1-1; the reader starts at segment bit pinit (a lane that is not live walks
// nothing).  `start(c, kbase)` runs before chunk c is walked (c < 0 in the pre-walk), `end(c, count)`
// after it.
// EARLY (the repair rounds): the walk ends at the first chunk entry at which no lane is left walking; a lane
// that is not live loads nothing (its requests point past the buffer's range: 0, no memory traffic).
template <bool EARLY, class Start, class End>
__device__ __forceinline__ int run_lines(Ring3& r, __amdgpu_buffer_rsrc_t rs, long long nbytes, long long gw0, int L0,
                                          int L1, int lim, int pinit, bool live, const uint8_t* tl, Start start,
                                          End end) {
    Stage8 st;
    const long long gl = (EARLY && !live) ? (1ll << 29) : gw0;        // the lane's load base
    const long long w0 = gw0 + 32ll * (L0 - 1);
    stage_half(st, 0, rs, gl + 32ll * (L0 - 1));
    stage_half(st, 4, rs, gl + 32ll * (L0 - 1) + 16);
    r.put(0, finish4(st.S[0], nbytes, w0));
    r.put(1, finish4(st.S[1], nbytes, w0 + 4));
    int kbase = 8 * (L0 - 1);
    r.init(pinit, kbase);
    if (!live) r.pos = 1 << 30;
    for (int L = L0; L < L1; L++) {
        int n0 = 0;
#pragma unroll
        for (int h = 0; h < 8; h++) {
            const int k = 8 * (L - 1) + h;
            if ((h & 1) == 0) {
                start(k >> 1, kbase);
                // (repairs: ~1.25 chunks on average -- stop at the first chunk entry where every lane has
                // met its recorded path, not at the end of the line)
                if (EARLY && h > 0 && !__any(r.pos < (1 << 30))) return L - L0 + 1;
            }
            const int n = r.walk(min(128 * (k + 1), lim), tl);
            r.put((h + 2) & 3, finish4(st.S[(h + 2) & 7], nbytes, gw0 + 4ll * (k + 2)));
            if (h == 1) stage_half(st, 0, rs, gl + 32ll * L);
            if (h == 5) stage_half(st, 4, rs, gl + 32ll * L + 16);
            if ((h & 3) == 3) kbase += 4;
            if (h & 1) end(k >> 1, n0 + n);
            else n0 = n;
        }
        if (EARLY && !__any(r.pos < (1 << 30))) return L - L0 + 1;   // every lane met its recorded path
    }
    return L1 - L0;
}

// A runs-mode stream (mostly 3-bit codes) that is nothing but num '100' codes -- every value within the
// bound of 0, e.g. a constant input after toSmallDataset (BASELINE config 3) -- decodes to num zeros
// (impl/dataCompression.c:1712-1716: '100' -> 0).  parse3 checks the first 3*num stream bits against the
// period-3 pattern 100100... (grid-stride over 32-bit words, MSB-first) and flags any difference;
// decode3 then writes the zeros at streaming speed, or hands the stream to the chunk-map decoder.
constexpr uint32_t D3_ZMISS = 32768u;
__device__ __forceinline__ void zero_run_check(__amdgpu_buffer_rsrc_t rs, const Geo3& G, long long num, unsigned* err,
                                               unsigned flag = D3_ZMISS) {
    const unsigned long long need = 3ull * (unsigned long long)num;
    if (need > G.nbits) {                                     // fewer bits than num tokens: not this case
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(err, flag);
        return;
    }
    const long long nw = (long long)((need + 31) >> 5);
    bool bad = false;
    const long long step = (long long)gridDim.x * blockDim.x * 4;
    for (long long w0 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4; w0 < nw; w0 += step) {
        const uint4 q = load_w4(rs, G.nbytes, w0);
        const uint32_t v[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const long long w = w0 + i;
            const uint32_t ph = (uint32_t)((2 * w) % 3);                   // (32 w) mod 3
            const uint32_t pat = ph == 0 ? 0x92492492u : (ph == 1 ? 0x24924924u : 0x49249249u);
            const long long rem = (long long)need - 32 * w;               // bits of the word to check
            const uint32_t m = rem >= 32 ? 0xFFFFFFFFu : (rem <= 0 ? 0u : ~(0xFFFFFFFFu >> rem));
            bad |= ((v[i] ^ pat) & m) != 0u;
        }
    }
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(err, flag);
}

// One parse job (64 segments, lane = segment): the main walk, the links, the records, the token offsets.
// Returns the job's token total (every lane).  PUB (fused3d_kernel): the records and the decode jobs' offsets
// are read by other CUs in the same launch, so they are stored sc1 (write-through, MI355X_MICROARCH.md
// "Valid forms"), the offsets into frel's per-fused-job rows
template <int SEG>
__device__ __forceinline__ long long frel_index(long long dj) {
    constexpr long long JPF = 4 * SEG, RELP = (4 * SEG + 31) & ~31;
    return (dj / JPF) * RELP + dj % JPF;
}
template <int CT, int SEG, bool PUB = false>
__device__ __forceinline__ uint32_t parse3_job(Ring3& r, uint16_t* recs, const uint8_t* tl, const Geo3& G,
                                               __amdgpu_buffer_rsrc_t rs, __amdgpu_buffer_rsrc_t rrec,
                                               const Dec3Bufs& D3, unsigned job, uint32_t epoch, int lane P3_PARAM) {
    constexpr int seg = SEG;
    constexpr int PL = CT == 6 ? DC_PARSE_PL6 : 1;              // pre-walk lines (1024 bits each)
    const long long sidx = (long long)job * 64 + lane;              // this lane's segment
    const long long sbit = sidx * seg * 256;
    const bool act = sidx < G.nseg;
    const int lim = act ? (int)min((long long)G.nbits - sbit, (long long)seg * 256 + 64) : -(1 << 30);
    const long long gw0 = sbit >> 5;
    const long long c0 = sidx * seg;                                   // first chunk of the segment
    P3_T(t0);

    // ---- main walk: the pre-walk line (1024 bits before the segment), then the segment's lines
    uint32_t tot = 0;
    int e0 = 0, ec = 0;
    // (DC_P3_PW4: the pre-walk's bits for 4-chunk segments -- small streams, whose parse is one walk; the walk
    // starts inside line 0, the phases before it step nothing)
    constexpr int PW = (SEG == 4 && PL == 1) ? DC_P3_PW4 : 1024 * PL;
    run_lines<false>(r, rs, G.nbytes, gw0, 1 - PL, seg / 4 + 1, lim, -PW, act, tl,
              [&](int c, int kbase) {
                  if (c == 0 && sidx == 0) r.init(0, kbase);             // the stream's first bit
                  ec = r.pos - 256 * c;
              },
              [&](int c, int cnt) {
                  if (c >= 0) {
                      recs[c * 64 + lane] = (uint16_t)((uint32_t)(ec & 31) | ((uint32_t)cnt << 8));
                      tot += (uint32_t)cnt;
                      if (c == 0) e0 = ec;
                  }
              });
    const int X = r.pos - 256 * seg;                                 // entry of the next segment
    // the job's exit: 8- and 16-chunk segments publish it right after the main walk (a repair that
    // moves it is rare enough to decline the stream for), 4-chunk segments after the in-job repairs;
    // CT6 always after them (its long tokens at small bounds resynchronise slowly: U10 at 1e-6 declined
    // at every size, `tools/seg_time.py`; late publication costs ~1 us at 2^26, 3-5 us for CT11, which
    // keeps the early one)
    constexpr bool EARLY_EXIT = seg >= 8 && DC_EXIT_EARLY && CT != 6;
    if (EARLY_EXIT && lane == 63) st_relaxed(&D3.pexit[job], ((uint64_t)epoch << 32) | (uint32_t)X);
    P3_T(t1);
    P3_ADD(0, t1 - t0);
    P3_ADD(4, act ? tot : 0u);

    // ---- links within the job: a segment's first entry = the previous segment's exit.  A lane whose
    // entry is not re-walks from that exit, rewriting its records until the path meets a recorded
    // entry again; a path that reaches the segment end without meeting it moves the exit, and the
    // successor is checked again (rounds; a moved exit of the last segment declines)
    // (the link into the job: checked at once if the previous job has published its exit, else after
    // the in-job links with a bounded wait)
    int xin = __shfl_up(X, 1, 64), ecur = e0, Xcur = X, rounds = 0;
    bool link0 = false;
    if (lane == 0 && act && sidx > 0) {
        const uint64_t v = ld_relaxed(&D3.pexit[job - 1]);
        if ((v >> 32) == (uint64_t)epoch) { xin = (int)(uint32_t)v; link0 = true; }
    }
    bool bad = act && (lane > 0 || link0) && ecur != xin;
    for (int pass = 0; pass < 2; pass++) {
    if (pass == 1) {                            // the job's first link: wait (bounded) for the exit
        // the job's exit, after the links within the job are repaired (a repair that reaches the end
        // of the last segment moves it -- with 4-chunk segments not rare enough to decline the stream
        // for): it depends on nothing outside the job, so no job waits for more than one main walk
        // and one round of in-job repairs
        if (!EARLY_EXIT && lane == 63) st_relaxed(&D3.pexit[job], ((uint64_t)epoch << 32) | (uint32_t)Xcur);
        bool chk = false;
        if (lane == 0 && act && sidx > 0 && !link0) {
            // the previous job is resident (a lower workgroup, or this grid's previous round) and
            // publishes its exit after its main walk (and in-job repairs, 4-chunk segments)
            const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
            P3_T(tw0);
            uint64_t v;
            while (((v = ld_relaxed(&D3.pexit[job - 1])) >> 32) != (uint64_t)epoch &&
                   __builtin_amdgcn_s_memrealtime() - w0 < D3_LINK_WAIT)
                __builtin_amdgcn_s_sleep(2);
            if ((v >> 32) == (uint64_t)epoch) { xin = (int)(uint32_t)v; link0 = true; chk = true; }
            else atomicOr(D3.err, D3_DECLINE | D3_WHY_LINK);   // (never seen: the chunk-map decoder takes it)
            P3_T(tw1);
            P3_ADD(1, tw1 - tw0);
        }
        bad = chk && ecur != xin;
    }
    while (__any(bad)) {
        if (++rounds > D3_MAX_ROUNDS) { if (lane == 0) atomicOr(D3.err, D3_DECLINE | D3_WHY_LINK); break; }
        bool live = bad;
        P3_T(tr0);
        const int nl = run_lines<true>(r, rs, G.nbytes, gw0, 1, seg / 4 + 1, lim, bad ? xin : 0, bad, tl,
                  [&](int c, int) {
                      const int old = (int)(recs[c * 64 + lane] & 31u);
                      if (live && c > 0 && r.pos - 256 * c == old && 256 * c < lim) {
                          live = false;                                 // met the recorded path
                          r.pos = 1 << 30;
                      }
                      ec = r.pos - 256 * c;
                  },
                  [&](int c, int cnt) {
                      if (live) {
                          const uint32_t old = recs[c * 64 + lane];
                          recs[c * 64 + lane] = (uint16_t)((uint32_t)(ec & 31) | ((uint32_t)cnt << 8));
                          tot += (uint32_t)cnt - (old >> 8);
                          if (c == 0) ecur = ec;
                      }
                  });
        P3_T(tr1);
        P3_ADD(6, tr1 - tr0);
        P3_ADD(7, nl);
        (void)nl;
        const bool whole = 256 * seg < lim;                              // a successor segment exists
        const int Xn = live ? r.pos - 256 * seg : Xcur;
        const bool moved = live && whole && Xn != Xcur;
        Xcur = Xn;
        if (moved && lane == 63 && (pass == 1 || EARLY_EXIT)) atomicOr(D3.err, D3_DECLINE | D3_WHY_LINK);   // (published)
        const int xp = __shfl_up(Xcur, 1, 64);
        const bool mp = __shfl_up((int)moved, 1, 64) != 0;
        bad = lane >= 1 && act && mp && ecur != xp;
        xin = bad ? xp : xin;
    }
    }
    P3_T(t2);
    P3_ADD(2, t2 - t1);
    P3_MAX(16, t2 - t0);
    P3_MAX(17, t1 - t0);
    P3_MAX(18, t2 - t1);
    P3_ADD(3, rounds);
    P3_ADD(5, 1);

    // ---- the segment's records: 32 bytes per lane, one contiguous 2 KB block per wave
    if (act) {
        uint32_t w[seg / 2];
#pragma unroll
        for (int i = 0; i < seg / 2; i++)
            w[i] = (uint32_t)recs[(2 * i) * 64 + lane] | ((uint32_t)recs[(2 * i + 1) * 64 + lane] << 16);
#pragma unroll
        for (int i = 0; i < seg / 8; i++) {
            const u32x4 v = {w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]};
            __builtin_amdgcn_raw_buffer_store_b128(v, rrec, (int)(2 * c0 + 16 * i), 0, PUB ? 16 : 0);
        }
        if constexpr (seg % 8 == 4) {                  // (4 chunks left: 4-chunk segments, the fused kernel's 20)
            const u32x2 v = {w[seg / 2 - 2], w[seg / 2 - 1]};
            __builtin_amdgcn_raw_buffer_store_b64(v, rrec, (int)(2 * c0 + 16 * (seg / 8)), 0, PUB ? 16 : 0);
        }
    }

    // ---- token offsets: the job's total and every decode job's first token relative to the job
    const uint32_t inc = wave_incl_scan(tot, lane);
    if (lane == 63) D3.ptot[job] = inc;
    auto put_rel = [&](long long dj, uint32_t v) {
        if (dj * 64 < D3.max_chunks) {
            if constexpr (PUB) __hip_atomic_store(&D3.frel[frel_index<SEG>(dj)], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else D3.rel[dj] = v;
        }
    };
    if constexpr (64 % seg == 0) {                     // decode jobs start on segment boundaries
        if (((lane * seg) & 63) == 0) put_rel((long long)job * seg + (lane * seg) / 64, inc - tot);
    } else {                                           // (seg < 64: at most one decode job starts in a segment)
        const int k = (int)((64 - ((lane * seg) & 63)) & 63);        // its chunk within the segment
        if (k < seg) {
            uint32_t pre = inc - tot;
            for (int c = 0; c < k; c++) pre += (uint32_t)(recs[c * 64 + lane] >> 8);
            put_rel(((long long)job * 64 * seg + (long long)lane * seg + k) / 64, pre);
        }
    }
    return (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
}

template <int CT, int SEG>
__global__ __launch_bounds__(64) void parse3_kernel(const uint8_t* __restrict__ s, Params P, Dec3Bufs D3,
                                                    const unsigned long long* dev_nbits, unsigned long long host_nbits,
                                                    long long num, uint32_t epoch) {
    constexpr int seg = SEG;
    static_assert(SEG % 4 == 0 && SEG <= 64, "whole region lines; at most one decode job start per segment");
    __shared__ uint32_t ring[D3_RING * 64];
    __shared__ uint16_t recs[seg * 64];                          // [chunk][lane]: the wave's records
    __shared__ uint8_t tl[512];
    const int lane = threadIdx.x;
    build_lut_len<CT>(tl, P, lane, 64);
    const Geo3 G = geo3<SEG>(dev_nbits, host_nbits);
    const __amdgpu_buffer_rsrc_t rs = stream_rsrc(s, D3.capw);
    const __amdgpu_buffer_rsrc_t rrec =
        __builtin_amdgcn_make_buffer_rsrc(D3.rec, (short)0, (int)min(2 * (D3.max_chunks + 4096), 0x7FFFFF00ll), 0x00020000);   // (the pool pads rec by 4096 chunks)
    const bool over = G.nchunks > D3.max_chunks, runs = !over && runs_mode(CT, G.nbits, num);
    const bool decline = over || runs;
    if (over && blockIdx.x == 0 && lane == 0) atomicOr(D3.err, D3_DECLINE | D3_WHY_RUNS);
    if (D3.shard && blockIdx.x == 0 && lane == 0) D3.spend[0] = 0u;     // (decode3 runs after this kernel)
    if (runs) zero_run_check(rs, G, num, D3.err);      // decode3 fills zeros, or hands the stream over
    __syncthreads();
    Ring3 r;
    r.L = ring;
    r.lc = (uint32_t)lane << 2;
    P3_DECL();
    // jobs by a fixed stride (a shared ticket counter serialised every wave on one L2 line)
    for (unsigned job = blockIdx.x; !decline && (long long)job < G.npjobs; job += gridDim.x) {
        parse3_job<CT, SEG>(r, recs, tl, G, rs, rrec, D3, job, epoch, lane P3_ARG);
    }
    P3_FLUSH();
}

// ------------------------------------------------------------------------------------------------
// decode
struct Lut3 {
    uint16_t meta[512];                 // sh | len << 8
    uint2 kv[512];                      // pattern = ((t >> sh) & x) | y; 3-bit codes: {0, 0}
};

template <int CT>
__device__ __forceinline__ void build_lut3(Lut3& T, const Params& P, int tid, int nthr) {
    build_lut_meta<CT>(T.meta, P, tid, nthr);
    for (int i = tid; i < 512; i += nthr) {
        const uint32_t t = (uint32_t)i << 23;
        uint32_t keep, add;
        if (CT != 6 && (int)t < 0) {
            keep = 0u; add = 0u;                     // '1xx': zero, or a prediction (filled in by the caller)
        } else if (CT == 11) {
            keep = 0xFFFFFFFFu; add = 0u;
        } else {
            const int len = token_len_bf<6>(t, P);   // raw length 9 + m(E)
            const uint32_t y = len >= 32 ? 0u : 0xFFFFFFFFu >> len;
            keep = ~y; add = y & ~(y >> 1);
            if (CT == 7 && (t & P.hm) == P.hm) {
                const bool f1 = (t >> P.fsh) & 1u;
                keep = f1 ? P.k1 : P.k0;
                add = f1 ? P.c1 : P.c0;
            }
        }
        T.kv[i] = make_uint2(keep, add);
    }
}

struct Rd3 {                                        // reader over a lane's 12 staged words, [word][lane]
    const uint32_t* L;
    uint32_t a, b, c, s, addr;
    __device__ __forceinline__ void init(const uint32_t* Lw, int lane, int p) {   // p in [0, 32)
        L = Lw;
        const int wi = (p - 1) >> 5;                   // -1 or 0
        s = (uint32_t)(32 * (wi + 1) - p);
        a = L[(max(wi, 0) << 6) + lane]; b = L[((wi + 1) << 6) + lane]; c = L[((wi + 2) << 6) + lane];
        addr = ((uint32_t)(wi + 3) << 8) | ((uint32_t)lane << 2);
    }
    __device__ __forceinline__ uint32_t fetch() const {
        return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(L) + addr);
    }
    __device__ __forceinline__ uint32_t peek() const { return __builtin_amdgcn_alignbit(a, b, s); }
    __device__ __forceinline__ void step(uint32_t nx, int len) {
        uint32_t d;
        const bool adv = __builtin_usub_overflow(s, (uint32_t)len, &d);
        s = d & 31u;
        a = adv ? b : a;
        b = adv ? c : b;
        c = adv ? nx : c;
        addr += adv ? 256u : 0u;
    }
};

// the previous decode job's k-th last value (k = 1..3), published by that job's wave
__device__ __forceinline__ float prev_job_value(const Dec3Bufs& D3, long long job, int k, uint32_t epoch) {
    const uint64_t* p = &D3.hist[(job - 1) * 3 + (k - 1)];
    unsigned spins = 0;
    uint64_t v;
    while (((v = ld_relaxed(p)) >> 32) != (uint64_t)epoch) {
        if (++spins > (1u << 22) || declined_now(D3)) { atomicOr(D3.err, D3_DECLINE | 16u); return 0.0f; }
        __builtin_amdgcn_s_sleep(1);
    }
    return __uint_as_float((uint32_t)v);
}

// a decode job's inputs, requested one job ahead (the job's records, its token offset, 12 stream words
// per lane) so that their latency hides behind the previous job's walk and stores
#ifndef DC_DEC3_NT
#define DC_DEC3_NT 1                                // the decoded floats stored past the caches (streaming)
#endif
constexpr int D3_OOB = 0x7FFFFFF0;                  // a buffer offset past every range below: reads 0, drops writes
                                                    // (ranges end below 0x7FFFFF00)
struct Pre3 {
    uint32_t rc, rl;
    uint32_t pt[4];                                 // parse-job token totals of the job's window (below)
    uint4 v0, v1, v2;
};
__device__ __forceinline__ __amdgpu_buffer_rsrc_t any_rsrc(const void* p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}
// (the first token of parse job pj is the sum of ptot[0..pj): a wave keeps that sum for the parse job of
// its previous decode job, plo, and adds the window ptot[plo..pj) -- 256 totals, 4 per lane, when the
// grid's stride is 4096 decode jobs -- so no scan kernel and no wait on another wave)
template <int SEG>
__device__ __forceinline__ Pre3 prefetch3(__amdgpu_buffer_rsrc_t rr, __amdgpu_buffer_rsrc_t rt, __amdgpu_buffer_rsrc_t rl,
                                          __amdgpu_buffer_rsrc_t rs, const Geo3& G, unsigned job, long long plo,
                                          int lane) {
    Pre3 q;
    const long long g = (long long)job * 64 + lane;
    const bool ok = (long long)job < G.ndjobs;
    const long long phi = ok ? (long long)(job / SEG) : plo;
    q.rc = __builtin_amdgcn_raw_buffer_load_b16(rr, g < G.nchunks ? (int)(2 * g) : D3_OOB, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const long long k = plo + 4 * lane + i;
        q.pt[i] = __builtin_amdgcn_raw_buffer_load_b32(rt, k < phi ? (int)(4 * k) : D3_OOB, 0, 0);
    }
    q.rl = __builtin_amdgcn_raw_buffer_load_b32(rl, ok ? (int)(4 * job) : D3_OOB, 0, 0);
    q.v0 = load_raw4(rs, 8 * g);
    q.v1 = load_raw4(rs, 8 * g + 4);
    q.v2 = load_raw4(rs, 8 * g + 8);
    return q;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) { return wave_total(v); }

// One decode job (64 chunks, lane = chunk) whose first token is `base`: the walk into the wave's buffer, the
// pending prefixes, the history granules, the float4 stores.
template <int CT, int CAP>
__device__ __forceinline__ void decode3_job(const Lut3& T, uint32_t* L, float* ob, const Geo3& G, __amdgpu_buffer_rsrc_t rs,
                                            __amdgpu_buffer_rsrc_t ro, bool chk_all, const Dec3Bufs& D3, const Pre3& cur,
                                            unsigned job, unsigned long long base, float* __restrict__ out, long long num,
                                            uint32_t epoch, int lane P3_PARAM) {
    P3_T(u0);
    const long long g = (long long)job * 64 + lane;
    const int e = (int)(cur.rc & 31u), n = (int)(cur.rc >> 8);
    const uint32_t inc = wave_incl_scan((uint32_t)n, lane);
    const int off = (int)inc - n;
    const int Tn = (int)__builtin_amdgcn_readlane(inc, 63);
    // the stream's last decode job: a stream with fewer tokens than num is left to the other decoder
    // (it reads past the stream as the reference does)
    if ((long long)job == G.ndjobs - 1 && (long long)(base + (unsigned long long)Tn) < num && lane == 0)
        atomicOr(D3.err, D3_DECLINE | D3_WHY_SHORT);
    const int al = (int)(base & 3ull);
    P3_T(u1);
    P3_ADD(8, u1 - u0);
    // (no `continue` after a lane-conditional store here: the structurizer then peeled the loop head
    // for lanes 1..63 with lane 0 inactive, and their readfirstlane claimed job 0 again, forever)
    const bool fits = al + Tn <= CAP;
    if (!fits) atomicOr(D3.err, D3_DECLINE | D3_WHY_DENSE);        // every lane: OR is idempotent
    bool sent = false;
    if (fits) {
    {   // stage the chunk's 8 words + 4 words of the next chunk
        const uint4 v0 = finish4(cur.v0, G.nbytes, 8 * g), v1 = finish4(cur.v1, G.nbytes, 8 * g + 4),
                    v2 = finish4(cur.v2, G.nbytes, 8 * g + 8);
        L[(0 << 6) + lane] = v0.x; L[(1 << 6) + lane] = v0.y; L[(2 << 6) + lane] = v0.z; L[(3 << 6) + lane] = v0.w;
        L[(4 << 6) + lane] = v1.x; L[(5 << 6) + lane] = v1.y; L[(6 << 6) + lane] = v1.z; L[(7 << 6) + lane] = v1.w;
        L[(8 << 6) + lane] = v2.x; L[(9 << 6) + lane] = v2.y; L[(10 << 6) + lane] = v2.z; L[(11 << 6) + lane] = v2.w;
    }
    P3_T(u2);
    P3_ADD(9, u2 - u1);
    const int o0 = al + off;
    int pend = 0;
    {
        Rd3 r;
        r.init(L, lane, e);
        int o = o0;
        for (int t = 0; t < n; t++) {
            const uint32_t nx = r.fetch();
            const uint32_t tk = r.peek();
            const uint32_t idx = tk >> 23;
            const uint32_t meta = T.meta[idx];
            const uint2 kv = T.kv[idx];
            uint32_t v = ((tk >> (meta & 31u)) & kv.x) | kv.y;
            if (CT != 6) {
                const uint32_t cc = tk >> 29;                            // 5..7: '101' '110' '111'
                if (__builtin_expect(__any(cc >= 5u), 0)) {
                    if (cc >= 5u) {
                        const int need = (int)cc - 4;
                        if (t < need || t - need < pend || (g == 0 && t < 3)) {
                            pend = t + 1;                                // needs the previous chunk's values
                            // a prediction among the stream's first 3 (a shard's: its incoming values)
                            sent |= g == 0 && t < 3 && D3.shard != 1;
                            v = 0u;
                        } else {
                            const float pv = predict_value(need, ob[o - 1], ob[o - 2], ob[o - 3]);
                            v = __float_as_uint(pv);
                            sent |= v == 0xBF800000u;
                        }
                    }
                }
            }
            ob[o] = __uint_as_float(v);
            o++;
            r.step(nx, (int)(meta >> 8));
        }
    }
    P3_T(u3);
    P3_ADD(10, u3 - u2);
    // ---- pending prefixes, in rounds: a lane re-decodes its prefix once no lane before it still holds an
    // unresolved prefix that reaches its three history values (U: the furthest end of those prefixes) --
    // usually every pending lane in the first round (a noisy ramp has ~40% of its chunks start with a
    // prediction; lane by lane, that serial loop was 80% of its decode)
    unsigned long long pm = __ballot(pend > 0);
    P3_ADD(14, __popcll(pm));
    P3_ADD(15, Tn);
    while (pm) {
        const bool mine = ((pm >> lane) & 1ull) != 0ull;
        int U = mine ? o0 + pend : -(1 << 30);
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {                          // inclusive max over lanes <= this one
            const int u = __shfl_up(U, d, 64);
            if (lane >= d) U = max(U, u);
        }
        U = __shfl_up(U, 1, 64);                                      // exclusive
        if (lane == 0) U = -(1 << 30);
        const bool go = mine && U <= max(o0 - 3, al);
        pm &= ~__ballot(go);
        __builtin_amdgcn_wave_barrier();
        if (go) {
            float h[3];
#pragma unroll
            for (int k = 1; k <= 3; k++) {
                const int i = o0 - k;
                // (job 0 has no predecessor: a prediction among its first tokens declined above)
                h[k - 1] = i >= al ? ob[i] : (job > 0 ? prev_job_value(D3, job, al - i, epoch) : 0.0f);
            }
            float b1 = h[0], b2 = h[1], b3 = h[2];
            if (D3.shard == 1 && g == 0) {
                // a shard's first chunk: its prefix waits for the values before the shard (zeros here,
                // re-decoded by shard3_fix_kernel).  Values after the prefix never read it; if the
                // prefix reaches the chunk's last three (read by the next chunk), hand the shard over
                D3.spend[0] = (uint32_t)pend;
                if (pend > n - 3) atomicOr(D3.err, D3_DECLINE | D3_WHY_SHARD);
            }
            Rd3 r;
            r.init(L, lane, e);
            for (int t = 0; t < pend; t++) {
                const uint32_t nx = r.fetch();
                const uint32_t tk = r.peek();
                const uint32_t idx = tk >> 23;
                const uint32_t meta = T.meta[idx];
                const uint2 kv = T.kv[idx];
                uint32_t v = ((tk >> (meta & 31u)) & kv.x) | kv.y;
                const uint32_t cc = tk >> 29;
                if (CT != 6 && cc >= 5u) {
                    v = __float_as_uint(predict_value((int)cc - 4, b1, b2, b3));
                    sent |= v == 0xBF800000u;
                }
                ob[o0 + t] = __uint_as_float(v);
                b3 = b2; b2 = b1; b1 = __uint_as_float(v);
                r.step(nx, (int)(meta >> 8));
            }
        }
    }
    P3_T(u4);
    P3_ADD(11, u4 - u3);
    // ---- publish the job's last three values (the next job's first chunk may need them)
    if (lane < 3 && Tn >= 3)
        st_relaxed(&D3.hist[(long long)job * 3 + lane], ((uint64_t)epoch << 32) | __float_as_uint(ob[al + Tn - 1 - lane]));
    }
    P3_T(u4s);
    // ---- store: the job's values as whole float4s of the output's 16-byte grid (a fixed count of
    // buffer stores, lanes outside the job writing past the range), the partial float4s at its two
    // ends float by float (lanes 0..3: the first, 4..7: the last)
    const int span = al + Tn;
    const int Q = (span + 3) >> 2;
    const long long gi0 = (long long)(base - (unsigned long long)al);
    bool sv = false;
    const float4* ob4 = reinterpret_cast<const float4*>(ob);
#pragma unroll
    for (int i = 0; i < (CAP + 3) / 4 / 64 + 1; i++) {
        const int q = lane + 64 * i;
        const float4 v = ob4[min(q, CAP / 4 - 1)];
        const long long gi = gi0 + 4 * q;
        const bool full = fits && q < Q && 4 * q >= al && 4 * q + 4 <= span && gi + 4 <= num;
        if (chk_all && q < Q)
            sv |= __float_as_uint(v.x) == 0xBF800000u || __float_as_uint(v.y) == 0xBF800000u ||
                  __float_as_uint(v.z) == 0xBF800000u || __float_as_uint(v.w) == 0xBF800000u;
        const u32x4 raw = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
#ifndef DC_DEC3_NOSTORE
        __builtin_amdgcn_raw_buffer_store_b128(raw, ro, full ? (int)(4 * gi) : D3_OOB, 0, DC_DEC3_NT ? 2 : 0);
#else                                   // (diagnostic build: the values are computed, never stored)
        if (raw.x == 0x12345678u && full && gi == 0) out[0] = v.y + v.z + v.w;
#endif
    }
    {
        const int qe = lane < 4 ? 0 : Q - 1;
        const int idx = 4 * qe + (lane & 3);
        const long long gi = gi0 + idx;
        const bool qfull = 4 * qe >= al && 4 * qe + 4 <= span && gi0 + 4 * qe + 4 <= num;
        const bool ok = fits && lane < 8 && !qfull && idx >= al && idx < span && gi < num;
        const float v = ob[min(max(idx, 0), CAP - 1)];
        (void)ok;
#ifndef DC_DEC3_NOSTORE
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), ro, ok ? (int)(4 * gi) : D3_OOB, 0, DC_DEC3_NT ? 2 : 0);
#endif
    }
    if (__any(sent || sv) && lane == 0) atomicOr(D3.err, D3_DECLINE | D3_WHY_SENT);
    P3_T(u5);
    P3_ADD(12, u5 - u4s);
    P3_ADD(13, 1);
}

// four waves per SIMD (<= 128 VGPRs): round 5's dense buffer template, shard flags and pending rounds had taken the
// kernel to 129-145 VGPRs, three waves per SIMD, and decode3 from 97 to 115 us at 2^26 U10
#ifndef DC_D3_MINW
#define DC_D3_MINW 4
#endif
template <int CT, int SEG, int CAP>
__global__ __launch_bounds__(256, DC_D3_MINW) void decode3_kernel(const uint8_t* __restrict__ s, Params P, Dec3Bufs D3,
                                                     const unsigned long long* dev_nbits, unsigned long long host_nbits,
                                                     float* __restrict__ out, long long num, uint32_t epoch) {
    __shared__ Lut3 T;
    __shared__ uint32_t stg[4][12 * 64];
    __shared__ __attribute__((aligned(16))) float obuf[4][CAP];
    build_lut3<CT>(T, P, threadIdx.x, 256);
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const Geo3 G = geo3<SEG>(dev_nbits, host_nbits);
    const __amdgpu_buffer_rsrc_t rs = stream_rsrc(s, D3.capw);
    const __amdgpu_buffer_rsrc_t rr = any_rsrc(D3.rec, 0x7FFFFF00), rt = any_rsrc(D3.ptot, 0x7FFFFF00),
                                 rl = any_rsrc(D3.rel, 0x7FFFFF00), ro = any_rsrc(out, (int)(num * 4));
    const unsigned err0 = __hip_atomic_load(D3.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool declined = (err0 & D3_DECLINE) != 0;
    if (!declined && G.nchunks <= D3.max_chunks && runs_mode(CT, G.nbits, num)) {
        // a runs-mode stream: num zeros if parse3 found nothing but '100' codes, else the chunk-map decoder's
        if (err0 & D3_ZMISS) {
            if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(D3.err, D3_DECLINE | D3_WHY_RUNS);
            return;
        }
        const u32x4 z4 = {0u, 0u, 0u, 0u};
        const __amdgpu_buffer_rsrc_t rz = any_rsrc(out, (int)(num * 4));
        for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; 4 * i < num; i += (long long)gridDim.x * blockDim.x)
            if (4 * i + 4 <= num) __builtin_amdgcn_raw_buffer_store_b128(z4, rz, (int)(16 * i), 0, DC_DEC3_NT ? 2 : 0);
            else for (long long j = 4 * i; j < num; j++) out[j] = 0.0f;
        return;
    }
    // patterns without a midpoint bit can equal the -1.0f history sentinel: check every value then
    const bool chk_all = (CT == 6 && P.B >= 23) || (CT == 7 && (P.mask17 >> 16) != 0u && P.mm == 23);
    uint32_t* L = stg[w];
    float* ob = obuf[w];
    P3_DECL();
    // jobs by a fixed stride (a shared ticket counter serialised every wave on one L2 line: 80k jobs
    // at ~13 ns each).  A job waits only for its predecessor's published values, rarely, and every
    // predecessor belongs to an earlier wave of the same round or to an earlier round.
    const unsigned stride = gridDim.x * 4;
    unsigned long long pcar = 0;                    // first token of parse job plo
    long long plo = 0;
    auto process = [&](const Pre3& cur, unsigned job) {
        const long long pj = (long long)(job / SEG);
        uint32_t wsum = wave_sum(cur.pt[0] + cur.pt[1] + cur.pt[2] + cur.pt[3]);
        for (long long k0 = plo + 256; k0 < pj; k0 += 256) {     // a window longer than one prefetch (rare)
            uint32_t v = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const long long k = k0 + 4 * lane + i;
                v += k < pj ? D3.ptot[k] : 0u;
            }
            wsum += wave_sum(v);
        }
        pcar += wsum;
        plo = pj;
        const unsigned long long base = pcar + cur.rl;
        decode3_job<CT, CAP>(T, L, ob, G, rs, ro, chk_all, D3, cur, job, base, out, num, epoch, lane P3_ARG);
    };
    // two jobs per round, their inputs in two register sets: each job's loads are in flight during the
    // other's walk and stores (one set copied into the other would wait for the loads -- and for every
    // store issued since, as stores count in the same counter)
    unsigned job = blockIdx.x * 4 + w;
    if (!declined && (long long)job < G.ndjobs) {
        Pre3 A = prefetch3<SEG>(rr, rt, rl, rs, G, job, 0, lane), B;
        // as many (dropped, distinct) stores after the first prefetch as a job issues after its
        // successor's: the loop's entry then looks like its back edge to the wait-count placement,
        // which otherwise waits for every store of the previous job before using a job's inputs
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("" ::: "memory");
        const u32x4 z4 = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int i = 0; i < (CAP + 3) / 4 / 64 + 1; i++)
            __builtin_amdgcn_raw_buffer_store_b128(z4, ro, D3_OOB - 64 * (i + 1), 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(0u, ro, D3_OOB, 0, 0);
        for (;;) {
            B = prefetch3<SEG>(rr, rt, rl, rs, G, job + stride, (long long)(job / SEG), lane);
            process(A, job);
            job += stride;
            if ((long long)job >= G.ndjobs) break;
            A = prefetch3<SEG>(rr, rt, rl, rs, G, job + stride, (long long)(job / SEG), lane);
            process(B, job);
            job += stride;
            if ((long long)job >= G.ndjobs) break;
        }
    }
    P3_FLUSH();
}

// ------------------------------------------------------------------------------------------------
// fused3_kernel (opt-in: DC_FUSED3=1; ordinary density, whole streams): parse and decode in one launch, the
// prototype VERDICT r04 asked for.  A workgroup of 4 waves takes fused job J = parse jobs 4J..4J+3 (256 SEG
// chunks): wave w parses job 4J+w exactly as parse3_kernel does (parse3_job), the workgroup publishes its token
// total (ftag[J], epoch-tagged) and sums the totals of the fused jobs between its previous one and J (published
// by the other workgroups after their parse; waited for, bounded) for the tokens before J; then the 4 waves
// decode J's 4 SEG decode jobs (decode job 4 SEG J + 4i + w) exactly as decode3_kernel does (decode3_job),
// their stream words and records fresh in the caches.  The parse rings and the decode buffers share one LDS
// union, so the launch holds decode3's 4 workgroups per CU -- 16 waves, where parse3 alone holds 24: the host
// takes the shortest segment (16, 20 or 32 chunks) whose parse jobs all fit in one round of resident waves, as
// parse3's do (a second round of parse jobs runs after the first round's decode, alone).  `stamps` (or null):
// per fused job the workgroup's s_memrealtime at its start, parse end, prefix known and decode end.
__device__ __forceinline__ unsigned long long wave_sum64(unsigned long long v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}
template <int CT, int SEG, int CAP>
__global__ __launch_bounds__(256, DC_D3_MINW) void fused3_kernel(const uint8_t* __restrict__ s, Params P, Dec3Bufs D3,
                                                                const unsigned long long* dev_nbits,
                                                                unsigned long long host_nbits, float* __restrict__ out,
                                                                long long num, uint32_t epoch,
                                                                unsigned long long* __restrict__ stamps) {
    static_assert(SEG % 4 == 0 && SEG <= 64, "whole region lines; at most one decode job start per segment");
    struct PS { uint32_t ring[4][D3_RING * 64]; uint16_t recs[4][SEG * 64]; };
    struct DS { uint32_t stg[4][12 * 64]; float obuf[4][CAP]; };
    union US { PS p; DS d; };
    __shared__ __attribute__((aligned(16))) US U;
    __shared__ Lut3 T;
    __shared__ uint8_t tl[512];
    __shared__ uint32_t sj[8];
    build_lut_len<CT>(tl, P, threadIdx.x, 256);
    build_lut3<CT>(T, P, threadIdx.x, 256);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const Geo3 G = geo3<SEG>(dev_nbits, host_nbits);
    const __amdgpu_buffer_rsrc_t rs = stream_rsrc(s, D3.capw);
    const __amdgpu_buffer_rsrc_t rrec =
        __builtin_amdgcn_make_buffer_rsrc(D3.rec, (short)0, (int)min(2 * (D3.max_chunks + 4096), 0x7FFFFF00ll), 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = any_rsrc(D3.rec, 0x7FFFFF00), rl = any_rsrc(D3.rel, 0x7FFFFF00),
                                 ro = any_rsrc(out, (int)(num * 4));
    const bool over = G.nchunks > D3.max_chunks, runs = !over && runs_mode(CT, G.nbits, num);
    if (over) {
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(D3.err, D3_DECLINE | D3_WHY_RUNS);
        return;
    }
    if (runs) {
        // a runs-mode stream of nothing but '100' codes: zeros, written while every workgroup checks its part of
        // the pattern -- a difference anywhere declines it, and the chunk-map decoder writes the output again
        zero_run_check(rs, G, num, D3.err, D3_ZMISS | D3_DECLINE | D3_WHY_RUNS);
        const u32x4 z4 = {0u, 0u, 0u, 0u};
        for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; 4 * i < num; i += (long long)gridDim.x * blockDim.x)
            if (4 * i + 4 <= num) __builtin_amdgcn_raw_buffer_store_b128(z4, ro, (int)(16 * i), 0, DC_DEC3_NT ? 2 : 0);
            else for (long long j = 4 * i; j < num; j++) out[j] = 0.0f;
        return;
    }
    __syncthreads();
    const bool chk_all = (CT == 6 && P.B >= 23) || (CT == 7 && (P.mask17 >> 16) != 0u && P.mm == 23);
    Ring3 r;
    r.L = U.p.ring[w];
    r.lc = (uint32_t)lane << 2;
    P3_DECL();
    const long long nfj = (G.npjobs + 3) / 4;
    unsigned long long pcar = 0;                               // tokens before fused job jn
    long long jn = 0;
    for (long long J = blockIdx.x; J < nfj; J += gridDim.x) {
        const unsigned long long ts0 = __builtin_amdgcn_s_memrealtime();
        // ---- parse: wave w takes parse job 4J + w
        const long long pj = 4 * J + w;
        uint32_t tot = 0;
        if (pj < G.npjobs) tot = parse3_job<CT, SEG>(r, U.p.recs[w], tl, G, rs, rrec, D3, (unsigned)pj, epoch, lane P3_ARG);
        if (lane == 0) sj[w] = tot;
        __syncthreads();                                       // (records, rel and totals written; rings free)
        const unsigned long long ts1 = __builtin_amdgcn_s_memrealtime();
        // ---- the tokens before J: this workgroup's carry plus the fused jobs jn .. J-1 of the other workgroups
        if (w == 0) {
            const uint32_t ft = sj[0] + sj[1] + sj[2] + sj[3];
            if (lane == 0) st_relaxed(&D3.ftag[J], ((uint64_t)epoch << 32) | ft);
            unsigned long long acc = 0;
            bool ok = true;
            for (long long k = jn + lane; k < J; k += 64) {
                const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
                uint64_t v;
                while (((v = ld_relaxed(&D3.ftag[k])) >> 32) != (uint64_t)epoch) {
                    if (__builtin_amdgcn_s_memrealtime() - w0 > D3_LINK_WAIT) { ok = false; break; }
                    __builtin_amdgcn_s_sleep(2);
                }
                acc += (uint32_t)v;
            }
            if (!ok) atomicOr(D3.err, D3_DECLINE | D3_WHY_LINK);
            pcar += wave_sum64(acc);
            if (lane == 0) {
                sj[4] = (uint32_t)pcar; sj[5] = (uint32_t)(pcar >> 32);
                sj[6] = declined_now(D3) ? 1u : 0u;            // (no decode after a decline: its records are partial)
            }
            pcar += ft;
        }
        jn = J + 1;
        __syncthreads();
        const unsigned long long S0 = (unsigned long long)sj[4] | ((unsigned long long)sj[5] << 32);
        const uint32_t pre[4] = {0u, sj[0], sj[0] + sj[1], sj[0] + sj[1] + sj[2]};
        const unsigned long long ts2 = __builtin_amdgcn_s_memrealtime();
        // ---- decode: decode jobs 64J + 4i + w (the job's successor is the next wave's, its predecessor the
        // previous wave's: the history granules are published in step)
        for (int i = 0; i < SEG && !sj[6]; i++) {
            const long long dj = 4ll * SEG * J + 4 * i + w;
            if (dj >= G.ndjobs) break;
            const long long g = dj * 64 + lane;
            Pre3 cur;
            cur.rc = __builtin_amdgcn_raw_buffer_load_b16(rr, g < G.nchunks ? (int)(2 * g) : D3_OOB, 0, 0);
            cur.rl = __builtin_amdgcn_raw_buffer_load_b32(rl, (int)(4 * dj), 0, 0);
            cur.v0 = load_raw4(rs, 8 * g);
            cur.v1 = load_raw4(rs, 8 * g + 4);
            cur.v2 = load_raw4(rs, 8 * g + 8);
            const unsigned long long base = S0 + pre[(4 * i + w) / SEG] + cur.rl;
            decode3_job<CT, CAP>(T, U.d.stg[w], U.d.obuf[w], G, rs, ro, chk_all, D3, cur, (unsigned)dj, base, out, num,
                                 epoch, lane P3_ARG);
        }
        const unsigned long long ts3 = __builtin_amdgcn_s_memrealtime();
        if (stamps && threadIdx.x == 0) {
            stamps[4 * J] = ts0; stamps[4 * J + 1] = ts1; stamps[4 * J + 2] = ts2; stamps[4 * J + 3] = ts3;
        }
        __syncthreads();                                       // (the decode buffers read: the next parse's rings)
    }
    P3_FLUSH();
}

// ------------------------------------------------------------------------------------------------
// fused3d_kernel (DC_FUSED3=2): fused3_kernel's parse, then the decode jobs split between the parsing workgroup
// and every other wave.  Round 5's fused3 lost its single stream read to scheduling: every workgroup decoded its
// own fused job, so a workgroup whose parse ended late decoded late, and the launch ended in a 45-us tail with
// fewer and fewer workgroups decoding (r05_fused3.txt: parse 46-75 us, decode 65-98 us per workgroup).  Here:
//   parse   workgroup J parses fused job J (4 parse jobs, one per wave; J += gridDim.x when one round does not
//           hold them) and publishes its records, the decode jobs' offsets (frel) and {its token total (ftag[J]),
//           the tokens before its parse jobs 1..3 (fsub[J])} -- records and offsets stored sc1, every storing
//           wave drained, one lane's sc1 granules behind the workgroup barrier (MI355X_MICROARCH.md "Valid
//           forms", first row);
//   static  the first DC_F3D_STATIC quarters of J's rounds of 4 decode jobs are decoded by J's own waves
//           (jobs 4 i + w, as fused3_kernel: the records and stream words its parse just read);
//   dynamic the remaining rounds of every fused job are tickets (one round's 4 jobs) in 8 queues (queue q: the
//           fused jobs J = q mod 8, in order; a wave starts at its workgroup's queue blockIdx % 8 -- the blocks
//           of one XCD -- and moves on to the others when it runs dry), so the launch ends with every wave busy.
// A wave keeps the tokens before its last fused job and adds the totals in between (polled, epoch-tagged).
// 8 queue heads (the guide's dequeue: one returning atomic per ticket; one head saturates near 88 per us).  The
// launch's last wave (a done counter) zeroes the heads.  First measured with every round dynamic (r06): 210 vs
// 195 us for parse3 + decode3 -- every wave waited for the slowest parse and paid ~2 round trips per ticket.
constexpr int F3D_B = 4;                            // decode jobs per ticket (~4 us each at 2^26)
#ifndef DC_F3D_STATIC
#define DC_F3D_STATIC 3                             // quarters of a fused job's decode rounds its own workgroup takes
#endif
constexpr int F3D_QW = 32;                          // words between queue heads (a 128-B line each)
template <int CT, int SEG, int CAP>
__global__ __launch_bounds__(256, DC_D3_MINW) void fused3d_kernel(const uint8_t* __restrict__ s, Params P, Dec3Bufs D3,
                                                                 const unsigned long long* dev_nbits,
                                                                 unsigned long long host_nbits, float* __restrict__ out,
                                                                 long long num, uint32_t epoch,
                                                                 unsigned long long* __restrict__ stamps, int sq) {
    static_assert(SEG % 4 == 0 && SEG <= 64 && F3D_B == 4, "whole region lines; a ticket = one round's 4 jobs");
    // SR of a fused job's SEG rounds of 4 decode jobs are decoded by its own workgroup, the rest handed out
    constexpr int JPF = 4 * SEG;
    const int SR = SEG * sq / 4, TPF = SEG - SR;
    struct PS { uint32_t ring[4][D3_RING * 64]; uint16_t recs[4][SEG * 64]; };
    struct DS { uint32_t stg[4][12 * 64]; float obuf[4][CAP]; };
    union US { PS p; DS d; };
    __shared__ __attribute__((aligned(16))) US U;
    __shared__ Lut3 T;
    __shared__ uint8_t tl[512];
    __shared__ uint32_t sj[4];
    build_lut_len<CT>(tl, P, threadIdx.x, 256);
    build_lut3<CT>(T, P, threadIdx.x, 256);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const Geo3 G = geo3<SEG>(dev_nbits, host_nbits);
    const __amdgpu_buffer_rsrc_t rs = stream_rsrc(s, D3.capw);
    const __amdgpu_buffer_rsrc_t rrec =
        __builtin_amdgcn_make_buffer_rsrc(D3.rec, (short)0, (int)min(2 * (D3.max_chunks + 4096), 0x7FFFFF00ll), 0x00020000);
    const __amdgpu_buffer_rsrc_t rsub = any_rsrc(D3.fsub, 0x7FFFFF00), ro = any_rsrc(out, (int)(num * 4));
    const bool over = G.nchunks > D3.max_chunks, runs = !over && runs_mode(CT, G.nbits, num);
    if (over) {                                                // (no ticket drawn: the heads stay zero)
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(D3.err, D3_DECLINE | D3_WHY_RUNS);
        return;
    }
    if (runs) {
        zero_run_check(rs, G, num, D3.err, D3_ZMISS | D3_DECLINE | D3_WHY_RUNS);
        const u32x4 z4 = {0u, 0u, 0u, 0u};
        for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; 4 * i < num; i += (long long)gridDim.x * blockDim.x)
            if (4 * i + 4 <= num) __builtin_amdgcn_raw_buffer_store_b128(z4, ro, (int)(16 * i), 0, DC_DEC3_NT ? 2 : 0);
            else for (long long j = 4 * i; j < num; j++) out[j] = 0.0f;
        return;
    }
    __syncthreads();
    const bool chk_all = (CT == 6 && P.B >= 23) || (CT == 7 && (P.mask17 >> 16) != 0u && P.mm == 23);
    Ring3 r;
    r.L = U.p.ring[w];
    r.lc = (uint32_t)lane << 2;
    P3_DECL();
    const long long nfj = (G.npjobs + 3) / 4;
    const unsigned long long ts0 = __builtin_amdgcn_s_memrealtime();
    // ---- parse: fused jobs J = blockIdx.x, + gridDim.x, ... (one round when the grid holds them all), wave w
    // taking parse job 4J + w; a parse waits only for its predecessor's exit, which a lower workgroup of the
    // same round (or the previous round) publishes after its main walk: no wait on any decode
    for (long long J = blockIdx.x; J < nfj; J += gridDim.x) {
        const long long pj = 4 * J + w;
        uint32_t tot = 0;
        if (pj < G.npjobs)
            tot = parse3_job<CT, SEG, true>(r, U.p.recs[w], tl, G, rs, rrec, D3, (unsigned)pj, epoch, lane P3_ARG);
        if (lane == 0) sj[w] = tot;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       // this wave's records and offsets have left
        __syncthreads();                                       // (after the last: the rings become decode buffers)
        if (threadIdx.x == 0) {
            const uint32_t c1 = sj[0], c2 = c1 + sj[1], c3 = c2 + sj[2];
            const u32x4 v = {epoch, c1, c2, c3};
            __builtin_amdgcn_raw_buffer_store_b128(v, rsub, (int)(16 * J), 0, 16);   // sc1 granule
            st_relaxed(&D3.ftag[J], ((uint64_t)epoch << 32) | (c3 + sj[3]));
        }
        __syncthreads();                                       // (sj is rewritten by the next round)
    }
    const unsigned long long ts1 = __builtin_amdgcn_s_memrealtime();
    // ---- the tokens before fused job J (polled totals; a wave keeps the sum for its last fused job Jc)
    long long Jc = 0;
    unsigned long long pc = 0;
    bool bad = false;
    auto prefix_to = [&](long long J2) {
        if (J2 < Jc) { Jc = 0; pc = 0; }
        if (J2 > Jc) {
            unsigned long long acc = 0;
            for (long long k = Jc + lane; k < J2; k += 64) {
                const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
                uint64_t v;
                while (((v = ld_relaxed(&D3.ftag[k])) >> 32) != (uint64_t)epoch) {
                    if (__builtin_amdgcn_s_memrealtime() - w0 > D3_LINK_WAIT) { bad = true; break; }
                    __builtin_amdgcn_s_sleep(2);
                }
                acc += (uint32_t)v;
            }
            pc += wave_sum64(acc);
            Jc = J2;
        }
    };
    // the tokens before each parse job of J2 (lane 0 polls J2's granule), wave-uniform
    auto subs = [&](long long J2, uint32_t (&c)[4]) {
        uint32_t c1 = 0, c2 = 0, c3 = 0;
        if (lane == 0) {
            const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
            u32x4 v;
            while ((v = __builtin_amdgcn_raw_buffer_load_b128(rsub, (int)(16 * J2), 0, 16)).x != epoch) {
                if (__builtin_amdgcn_s_memrealtime() - w0 > D3_LINK_WAIT) { bad = true; break; }
                __builtin_amdgcn_s_sleep(2);
            }
            c1 = v.y; c2 = v.z; c3 = v.w;
        }
        c[0] = 0u;
        c[1] = (uint32_t)__builtin_amdgcn_readfirstlane((int)c1);
        c[2] = (uint32_t)__builtin_amdgcn_readfirstlane((int)c2);
        c[3] = (uint32_t)__builtin_amdgcn_readfirstlane((int)c3);
    };
    auto job = [&](long long J2, long long dj, const uint32_t (&c)[4]) {
        const long long g = dj * 64 + lane;
        Pre3 cur;
        cur.rc = __builtin_amdgcn_raw_buffer_load_b16(rrec, g < G.nchunks ? (int)(2 * g) : D3_OOB, 0, 16);
        cur.rl = __hip_atomic_load(&D3.frel[frel_index<SEG>(dj)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        cur.v0 = load_raw4(rs, 8 * g);
        cur.v1 = load_raw4(rs, 8 * g + 4);
        cur.v2 = load_raw4(rs, 8 * g + 8);
        const int pi = (int)((dj - JPF * J2) / SEG);
        const unsigned long long base = pc + (pi == 0 ? 0u : pi == 1 ? c[1] : pi == 2 ? c[2] : c[3]) + cur.rl;
        decode3_job<CT, CAP>(T, U.d.stg[w], U.d.obuf[w], G, rs, ro, chk_all, D3, cur, (unsigned)dj, base, out, num,
                             epoch, lane P3_ARG);
    };
    // ---- static part: the workgroup's own fused jobs, decode jobs 4 i + w of rounds i < SR, as fused3_kernel
    // (their records and stream words fresh from this workgroup's parse, no ticket)
    for (long long J2 = blockIdx.x; J2 < nfj && !bad; J2 += gridDim.x) {
        prefix_to(J2);
        uint32_t c[4];
        subs(J2, c);
        if (__any(bad)) { bad = true; break; }
        for (int i = 0; i < SR; i++) {
            const long long dj = JPF * J2 + 4 * i + w;
            if (dj >= G.ndjobs) break;
            job(J2, dj, c);
        }
    }
    // ---- dynamic part: the rounds i >= SR of every fused job, as tickets of F3D_B decode jobs (one round's
    // four); queue q holds the fused jobs q, q + 8, ... (TPF tickets each)
    auto ntk = [&](int q) -> unsigned { return q < nfj ? (unsigned)(((nfj - q + 7) / 8) * TPF) : 0u; };
    auto deq = [&](int q) -> unsigned {
        unsigned t = 0;
        if (lane == 0) t = __hip_atomic_fetch_add(&D3.fq[F3D_QW * q], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return (unsigned)__builtin_amdgcn_readfirstlane((int)t);
    };
    unsigned qdone = 0;
    int q = (int)(blockIdx.x & 7);
    unsigned t = deq(q);
    bad = __any(bad);
    while (!bad) {
        if (t >= ntk(q)) {                                     // queue q has run dry: the next one
            qdone |= 1u << q;
            if (qdone == 0xFFu) break;
            do { q = (q + 1) & 7; } while ((qdone >> q) & 1u);
            t = deq(q);
            continue;
        }
        const long long J2 = q + 8ll * (t / TPF);
        const long long dj0 = JPF * J2 + 4ll * SR + (long long)F3D_B * (t % TPF);
        const unsigned tn = deq(q);                            // the next ticket
        prefix_to(J2);
        uint32_t c[4];
        subs(J2, c);
        bad = __any(bad);
        if (bad) break;
        for (int b = 0; b < F3D_B; b++) {
            const long long dj = dj0 + b;
            if (dj >= G.ndjobs) break;
            job(J2, dj, c);
        }
        t = tn;
    }
    if (bad && lane == 0) atomicOr(D3.err, D3_DECLINE | D3_WHY_LINK);
    if (stamps && lane == 0) {                                 // per wave: start, parse end, decode end
        stamps[16 * blockIdx.x + 4 * w] = ts0; stamps[16 * blockIdx.x + 4 * w + 1] = ts1;
        stamps[16 * blockIdx.x + 4 * w + 2] = __builtin_amdgcn_s_memrealtime();
    }
    // ---- the launch's last wave zeroes the queue heads for the next launch (every wave of the grid gets here
    // once, after its last draw)
    if (lane == 0) {
        const unsigned d = __hip_atomic_fetch_add(&D3.fq[F3D_QW * 8], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d == 4u * gridDim.x - 1u) {
#pragma unroll
            for (int k = 0; k <= 8; k++) __hip_atomic_store(&D3.fq[F3D_QW * k], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    P3_FLUSH();
}

// A shard's first pending tokens (D3.spend[0] of its first chunk, which starts at stream bit 0), decoded
// again from the three values before the shard (hin: b1, b2, b3 = the previous shard's last three values,
// last first), one token after another as impl/dataCompression.c:1900-2027 reads them.
template <int CT>
__global__ __launch_bounds__(64) void shard3_fix_kernel(const uint8_t* __restrict__ s, Params P, Dec3Bufs D3,
                                                       const float* __restrict__ hin, float* __restrict__ out,
                                                       long long num) {
    if (threadIdx.x != 0) return;
    const int np = (int)min((long long)D3.spend[0], num);
    if (np <= 0) return;
    const __amdgpu_buffer_rsrc_t rs = stream_rsrc(s, D3.capw);
    float b1 = hin[0], b2 = hin[1], b3 = hin[2];
    // (the prefix lies in the chunk's first 288 bits; finish4 takes the byte count as an int, so the stream's
    // readable capacity bounds it -- 1 << 40 truncated to 0 and zeroed every word)
    const long long nb = D3.capw * 4;
    uint4 w = load_w4(rs, nb, 0);
    uint32_t win[12] = {w.x, w.y, w.z, w.w};
    w = load_w4(rs, nb, 4);
    win[4] = w.x; win[5] = w.y; win[6] = w.z; win[7] = w.w;
    w = load_w4(rs, nb, 8);
    win[8] = w.x; win[9] = w.y; win[10] = w.z; win[11] = w.w;
    int pos = 0;
    bool sent = false;
    for (int t = 0; t < np; t++) {
        const int wi = pos >> 5, sh = pos & 31;
        if (wi + 1 >= 12) break;                    // (never: a chunk's tokens start within its 256 bits)
        const uint32_t tk = sh ? __builtin_amdgcn_alignbit(win[wi], win[wi + 1], 32 - sh) : win[wi];
        const int len = token_len_bf<CT>(tk, P);
        int code = 0;
        uint32_t v = token_pattern_bf<CT>(tk, len, P, &code);
        if (code > 0) {
            v = __float_as_uint(predict_value(code, b1, b2, b3));
            sent |= v == 0xBF800000u;
        }
        out[t] = __uint_as_float(v);
        b3 = b2; b2 = b1; b1 = __uint_as_float(v);
        pos += len;
    }
    if (sent) atomicOr(D3.err, D3_DECLINE | D3_WHY_SENT);
}

// ------------------------------------------------------------------------------------------------
#define DC_DISPATCH_3(CTV, SEGV, KER, ...)                                                           \
    switch ((CTV) * 100 + (SEGV)) {                                                                  \
        case 504: hipLaunchKernelGGL(HIP_KERNEL_NAME(KER<5, 4>), __VA_ARGS__); break;                \
        case 604: hipLaunchKernelGGL(HIP_KERNEL_NAME(KER<6, 4>), __VA_ARGS__); break;                \
        case 704: hipLaunchKernelGGL(HIP_KERNEL_NAME(KER<7, 4>), __VA_ARGS__); break;                \
        case 1104: hipLaunchKernelGGL(HIP_KERNEL_NAME(KER<11, 4>), __VA_ARGS__); break;              \
        case 508: hipLaunchKernelGGL(HIP_KERNEL_NAME(KER<5, 8>), __VA_ARGS__); break;                \
        case 608: hipLaunchKernelGGL(HIP_KERNEL_NAME(KER<6, 8>), __VA_ARGS__); break;                \
        case 708: hipLaunchKernelGGL(HIP_KERNEL_NAME(KER<7, 8>), __VA_ARGS__); break;                \
        case 1108: hipLaunchKernelGGL(HIP_KERNEL_NAME(KER<11, 8>), __VA_ARGS__); break;              \
        case 516: hipLaunchKernelGGL(HIP_KERNEL_NAME(KER<5, 16>), __VA_ARGS__); break;               \
        case 616: hipLaunchKernelGGL(HIP_KERNEL_NAME(KER<6, 16>), __VA_ARGS__); break;               \
        case 716: hipLaunchKernelGGL(HIP_KERNEL_NAME(KER<7, 16>), __VA_ARGS__); break;               \
        case 1116: hipLaunchKernelGGL(HIP_KERNEL_NAME(KER<11, 16>), __VA_ARGS__); break;             \
        case 520: hipLaunchKernelGGL(HIP_KERNEL_NAME(KER<5, 20>), __VA_ARGS__); break;               \
        case 620: hipLaunchKernelGGL(HIP_KERNEL_NAME(KER<6, 20>), __VA_ARGS__); break;               \
        case 720: hipLaunchKernelGGL(HIP_KERNEL_NAME(KER<7, 20>), __VA_ARGS__); break;               \
        case 1120: hipLaunchKernelGGL(HIP_KERNEL_NAME(KER<11, 20>), __VA_ARGS__); break;             \
        case 524: hipLaunchKernelGGL(HIP_KERNEL_NAME(KER<5, 24>), __VA_ARGS__); break;               \
        case 624: hipLaunchKernelGGL(HIP_KERNEL_NAME(KER<6, 24>), __VA_ARGS__); break;               \
        case 724: hipLaunchKernelGGL(HIP_KERNEL_NAME(KER<7, 24>), __VA_ARGS__); break;               \
        case 1124: hipLaunchKernelGGL(HIP_KERNEL_NAME(KER<11, 24>), __VA_ARGS__); break;             \
        default: return -2;                                                                          \
    }

// decode3_kernel<CT, SEG, CAP>: the kernel of a (CT, segment length) for a job buffer of CAP values
template <int CAP>
static const void* decode3_fn(int ct, int seg) {
#define D3F(C)                                                                                       \
    (seg == 4 ? (const void*)decode3_kernel<C, 4, CAP> : seg == 8 ? (const void*)decode3_kernel<C, 8, CAP> \
     : seg == 20 ? (const void*)decode3_kernel<C, 20, CAP> : seg == 24 ? (const void*)decode3_kernel<C, 24, CAP> \
                 : (const void*)decode3_kernel<C, 16, CAP>)
    return ct == 5 ? D3F(5) : ct == 6 ? D3F(6) : ct == 7 ? D3F(7) : D3F(11);
#undef D3F
}
template <int CAP>
static int launch_decode3_cap(int ct, int seg, int grid, hipStream_t st, const uint8_t* s, const Params& P,
                              const Dec3Bufs& D3, const unsigned long long* dev_nbits, unsigned long long host_nbits,
                              float* out, long long num, uint32_t epoch) {
#define D3C(CTV, SEGV)                                                                              \
    case CTV * 100 + SEGV:                                                                           \
        hipLaunchKernelGGL(HIP_KERNEL_NAME(decode3_kernel<CTV, SEGV, CAP>), dim3(grid), dim3(256), 0, st, s, P, D3, \
                           dev_nbits, host_nbits, out, num, epoch);                                  \
        break;
    switch (ct * 100 + seg) {
        D3C(5, 4) D3C(6, 4) D3C(7, 4) D3C(11, 4) D3C(5, 8) D3C(6, 8) D3C(7, 8) D3C(11, 8)
        D3C(5, 16) D3C(6, 16) D3C(7, 16) D3C(11, 16) D3C(5, 20) D3C(6, 20) D3C(7, 20) D3C(11, 20)
        D3C(5, 24) D3C(6, 24) D3C(7, 24) D3C(11, 24)
        default: return -2;
    }
#undef D3C
    return 0;
}

static int resident3(const void* f, int threads) {
    int dev = 0, ncu = 256, per = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, f, threads, 0) != hipSuccess || per < 1) per = 1;
    return per * ncu;
}

// segment length (chunks) for a stream of up to max_chunks chunks: 16; 8 for streams too small to fill
// the GPU with 16-chunk segments (<= 2.5 M chunks of capacity, 80 MB: the parse's walk per lane is then
// 1024 + 2048 bits instead of 1024 + 4096, and there are twice the jobs); 4 below 1 M chunks (32 MB:
// 1024 + 1024 bits, four times the jobs -- still one round of parse waves, and a small stream's parse is
// the length of one walk).  Short segments need tokens short enough (bound exponent B <= 12, e.g. 1e-3:
// tokens of <= ~21 bits) for a repaired path to meet the recorded one within the segment -- at 1e-6 a
// job's last segment could move its exit and decline the stream.  CT6 (no 3-bit codes: its paths run
// side by side for longer, tools/sync_sim.py: 4% of 1024-bit pre-walks unsynchronised, 0.4% not met
// within 4 chunks) takes 8 chunks or more; CT11 (32-bit verbatim tokens, a path
// read out of phase stays out of phase until a 3-bit code realigns it) takes 8 or more.  The host sizes the scratch for
// 4-chunk segments (DC_DEC3_SEG=4|8|16|20|24 forces one)
static int g_seg_forced = -1;
static int seg_forced() {
    if (g_seg_forced < 0) {
        const char* e = getenv("DC_DEC3_SEG");
        const int f = e ? atoi(e) : 0;
        g_seg_forced = (f == 4 || f == 8 || f == 16 || f == 20 || f == 24) ? f : 0;
    }
    return g_seg_forced;
}
// tests: force a segment length (4, 8 or 16; 0: by size); returns the previous setting
extern "C" int dc_set_decode3_seg(int seg) {
    const int old = seg_forced();
    g_seg_forced = (seg == 4 || seg == 8 || seg == 16 || seg == 20 || seg == 24) ? seg : 0;
    return old;
}
extern "C" int dc_decode3_seg(long long max_chunks, int B, int ct) {
    const int forced = seg_forced();
    if (forced) return forced;
    if (B > 12) return D3_SEG;
    if (max_chunks <= 1000000ll && (ct == 5 || ct == 7)) return 4;
    // 8-chunk segments: a job exit that a repair moves after it was published declines the stream, and the
    // chance grows with the job count.  U10 at the default bound (tools/seg_time.py): CT11 declined from 2^24
    // floats (its 32-bit tokens resynchronise slowly), CT6 from 2^25; CT5 / CT7 never up to 2^26
    if (ct == 11) return D3_SEG;
    if (ct == 6) return max_chunks <= 1100000ll ? 8 : D3_SEG;
    // CT5 / CT7 above 2.5 M chunks of capacity: 20-chunk segments -- fewer parse waves than parse3's 24 per CU
    // are resident (2^26 U10: 3971 jobs instead of 4964), each walks 20 % more bits but faster (parse3 88.6-89.1
    // -> 83.3 us, bench 767-775 -> 782-786 GB/s, tools/gpu_seg_ab.sh; 24 chunks: 86.6-87.1 us)
    return max_chunks <= 2500000ll ? 8 : 20;
}

// DC_DEC3_DEBUG=1: wait for every kernel (at most 2 s each) and report one that does not finish
static void dbg_wait(const char* what, hipStream_t st) {
    static int on = -1;
    if (on < 0) on = getenv("DC_DEC3_DEBUG") ? 1 : 0;
    if (!on) return;
    for (int i = 0; i < 2000; i++) {
        if (hipStreamQuery(st) == hipSuccess) return;
        usleep(1000);
    }
    fprintf(stderr, "[dcamd] %s has not finished after 2 s\n", what);
    fflush(stderr);
}

// DC_DEC3_DEBUG: a snapshot of the decoder state while a kernel is still running (another stream)
static void dbg_dump(const Dec3Bufs* D3) {
    static int on = -1;
    if (on < 0) on = getenv("DC_DEC3_DEBUG") ? 1 : 0;
    if (!on) return;
    hipStream_t s2;
    if (hipStreamCreateWithFlags(&s2, hipStreamNonBlocking) != hipSuccess) return;
    unsigned err = 0;
    uint64_t hist[12] = {0};
    uint32_t rel[4] = {0}, pt[4] = {0};
    uint16_t rec[16] = {0};
    (void)hipMemcpyAsync(&err, D3->err, 4, hipMemcpyDeviceToHost, s2);
    (void)hipMemcpyAsync(hist, D3->hist, sizeof hist, hipMemcpyDeviceToHost, s2);
    (void)hipMemcpyAsync(rel, D3->rel, sizeof rel, hipMemcpyDeviceToHost, s2);
    (void)hipMemcpyAsync(pt, D3->ptot, sizeof pt, hipMemcpyDeviceToHost, s2);
    (void)hipMemcpyAsync(rec, D3->rec, sizeof rec, hipMemcpyDeviceToHost, s2);
    (void)hipStreamSynchronize(s2);
    fprintf(stderr, "[dcamd] err 0x%x seg %d\n", err, D3->seg);
    for (int i = 0; i < 4; i++)
        fprintf(stderr, "  job %d hist %llx %llx %llx rel %u ptot %u\n", i, (unsigned long long)hist[3 * i],
                (unsigned long long)hist[3 * i + 1], (unsigned long long)hist[3 * i + 2], rel[i], pt[i]);
    for (int i = 0; i < 16; i++) fprintf(stderr, " rec%d=%u/%u", i, rec[i] & 31u, rec[i] >> 8);
    fprintf(stderr, "\n");
    fflush(stderr);
    (void)hipStreamDestroy(s2);
}

// resident grids per (CT, segment length, buffer) instantiation: every job of a call must be resident at once
// (parse3's link wait, decode3's history wait), so each grid is sized from its own kernel's occupancy
static int decode3_grids(const Params* P, const Dec3Bufs* D3, int dense, int* g1_out, int* g3_out) {
    static int gp[5][12], gd[2][5][12];
    const int ci = (P->ct > 0 && P->ct < 12) ? P->ct : 0;
    if (D3->seg != 4 && D3->seg != 8 && D3->seg != 16 && D3->seg != 20 && D3->seg != 24) return -2;
    if (P->ct != 5 && P->ct != 6 && P->ct != 7 && P->ct != 11) return -2;
    const int si = D3->seg == 16 ? 1 : D3->seg == 4 ? 2 : D3->seg == 20 ? 3 : D3->seg == 24 ? 4 : 0, di = dense ? 1 : 0;
    if (!gp[si][ci]) {
        const void* fp;
#define DC_PICK3(KER, SEGV) (P->ct == 5 ? (const void*)KER<5, SEGV> : P->ct == 6 ? (const void*)KER<6, SEGV>   \
                             : P->ct == 7 ? (const void*)KER<7, SEGV> : (const void*)KER<11, SEGV>)
        if (si == 1) fp = DC_PICK3(parse3_kernel, 16);
        else if (si == 2) fp = DC_PICK3(parse3_kernel, 4);
        else if (si == 3) fp = DC_PICK3(parse3_kernel, 20);
        else if (si == 4) fp = DC_PICK3(parse3_kernel, 24);
        else fp = DC_PICK3(parse3_kernel, 8);
#undef DC_PICK3
        gp[si][ci] = resident3(fp, 64);
    }
    if (!gd[di][si][ci])
        gd[di][si][ci] = resident3(dense ? decode3_fn<D3_CAP_DENSE>(P->ct, D3->seg) : decode3_fn<D3_CAP>(P->ct, D3->seg), 256);
    const long long maxseg = (D3->max_chunks + D3->seg - 1) / D3->seg;
    const long long maxpj = (maxseg + 63) / 64, maxdj = (D3->max_chunks + 63) / 64;
    int g1 = (int)std::max<long long>(1, std::min<long long>(maxpj, gp[si][ci]));
    int g3 = (int)std::max<long long>(1, std::min<long long>((maxdj + 3) / 4, gd[di][si][ci]));
    {   // (experiments, DESIGN section 9: the occupancy a fused parse + decode launch would leave each phase)
        // DC_P3_PER_CU / DC_D3_PER_CU cap the resident parse waves / decode workgroups per CU
        static int p3cap = -1, d3cap = -1, ncu = 256;
        if (p3cap < 0) {
            const char* a = getenv("DC_P3_PER_CU");
            const char* b = getenv("DC_D3_PER_CU");
            p3cap = a ? atoi(a) : 0;
            d3cap = b ? atoi(b) : 0;
            int dev = 0;
            (void)hipGetDevice(&dev);
            (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        }
        if (p3cap > 0) g1 = std::min(g1, p3cap * ncu);
        if (d3cap > 0) g3 = std::min(g3, d3cap * ncu);
    }
    *g1_out = g1;
    *g3_out = g3;
    return 0;
}

// DC_FUSED3=1: fused3_kernel instead of parse3 + decode3 (16-chunk segments, ordinary density, whole streams);
// DC_FUSED3_STAMPS=1 records its per-job phase stamps (dc_fused3_stamps)
static unsigned long long* g_f3_stamps = nullptr;
static long long g_f3_nfj = 0;
static int g_f3_on = -1;
static int fused3_on() {
    if (g_f3_on < 0) { const char* e = getenv("DC_FUSED3"); g_f3_on = (e && (*e == '1' || *e == '2')) ? *e - '0' : 0; }
    return g_f3_on;
}
// tests / experiments: 1 selects fused3_kernel, 2 fused3d_kernel (dynamic decode jobs), 0 the two launches;
// returns the previous setting
extern "C" int dc_set_fused3(int on) {
    const int old = fused3_on();
    g_f3_on = (on == 1 || on == 2) ? on : 0;
    return old;
}
static int g_f3_seg = 0;
static long long g_f3_hint_cap = -1, g_f3_hint_nch = 0;
extern "C" void dc_decode3_size_hint(long long max_chunks, long long nchunks) {
    g_f3_hint_cap = max_chunks;
    g_f3_hint_nch = nchunks;
}
static int launch_fused3(const uint8_t* s, const unsigned long long* dev_nbits, unsigned long long host_nbits,
                         const Params* P, const Dec3Bufs* D3, float* out, long long num, uint32_t epoch, int dyn,
                         hipStream_t st) {
    const void* fp = dyn ? (P->ct == 5 ? (const void*)fused3d_kernel<5, 16, D3_CAP> : P->ct == 6 ? (const void*)fused3d_kernel<6, 16, D3_CAP>
                            : P->ct == 7 ? (const void*)fused3d_kernel<7, 16, D3_CAP> : (const void*)fused3d_kernel<11, 16, D3_CAP>)
                         : (P->ct == 5 ? (const void*)fused3_kernel<5, 16, D3_CAP> : P->ct == 6 ? (const void*)fused3_kernel<6, 16, D3_CAP>
                            : P->ct == 7 ? (const void*)fused3_kernel<7, 16, D3_CAP> : (const void*)fused3_kernel<11, 16, D3_CAP>);
    static int resv[2][12];
    int* res = resv[dyn ? 1 : 0];
    const int ci = P->ct;
    if (!res[ci]) res[ci] = resident3(fp, 256);             // (the same registers and LDS for every SEG)
    // the segment length by a model of the launch (fused jobs in rounds of res[ci] workgroups; per round a job's
    // parse ~2.35 us per 4 chunks walked -- the pre-walk line and the segment's lines -- its decode ~4.4 us per
    // decode job and wave, ~10 us of prefix wait; measured at 2^26 U10) on the stream's chunks
    // (its capacity when the length is on the device only); DC_FUSED3_SEG forces one
    // (the length of the last stream of this capacity when this one's is on the device only: a stream decoded
    // over and over, like the bench's, then gets the segment length of its own size)
    const long long nch = host_nbits ? (long long)((host_nbits + 255) / 256)
                        : (g_f3_hint_cap == D3->max_chunks && g_f3_hint_nch > 0 ? g_f3_hint_nch : D3->max_chunks);
    int seg = 16;
    double best = 1e30;
    for (int sg : {16, 20, 24, 32, 64}) {
        const long long fj = (((nch + sg - 1) / sg + 63) / 64 + 3) / 4;
        // (dynamic decode: the decode work is spread over every wave, so the shortest segment whose parse is one
        // round wins -- the parse walk is the part no other workgroup can take over)
        const double t = dyn ? (fj <= res[ci] ? (double)sg : 1e6 + sg)
                             : (double)((fj + res[ci] - 1) / res[ci]) * (2.35 * (sg / 4 + 1) * 4 + 4.4 * sg + 10.0);
        if (t < best) { best = t; seg = sg; }
    }
    if (const char* e = getenv("DC_FUSED3_SEG")) {
        const int f = atoi(e);
        if (f == 16 || f == 20 || f == 24 || f == 32 || f == 64) seg = f;
    }
    g_f3_seg = seg;
    const long long maxpj = ((D3->max_chunks + seg - 1) / seg + 63) / 64, nfj = (maxpj + 3) / 4;
    const int grid = (int)std::max<long long>(1, std::min<long long>(nfj, res[ci]));
    static int sq = -1;                                    // fused3d: quarters of the rounds decoded statically
    if (sq < 0) {
        const char* e = getenv("DC_F3D_STATIC");
        sq = (e && *e >= '0' && *e <= '4') ? *e - '0' : DC_F3D_STATIC;
    }
    unsigned long long* stamps = nullptr;
    if (getenv("DC_FUSED3_STAMPS")) {                      // (fused3d: 16 words per workgroup, 4 per wave)
        const long long nst = dyn ? 4 * (long long)grid : nfj;
        if (nst > g_f3_nfj) {
            if (g_f3_stamps) (void)hipFree(g_f3_stamps);
            if (hipMalloc((void**)&g_f3_stamps, (size_t)nst * 4 * 8) != hipSuccess) return -1;
            g_f3_nfj = nst;
        }
        stamps = g_f3_stamps;
        (void)hipMemsetAsync(stamps, 0, (size_t)g_f3_nfj * 4 * 8, st);
    }
#define F3L(C, S) do {                                                                               \
        if (dyn) hipLaunchKernelGGL(HIP_KERNEL_NAME(fused3d_kernel<C, S, D3_CAP>), dim3(grid), dim3(256), 0, st, s, \
                                    *P, *D3, dev_nbits, host_nbits, out, num, epoch, stamps, sq);    \
        else hipLaunchKernelGGL(HIP_KERNEL_NAME(fused3_kernel<C, S, D3_CAP>), dim3(grid), dim3(256), 0, st, s, *P, \
                                *D3, dev_nbits, host_nbits, out, num, epoch, stamps);                \
    } while (0)
#define F3C(C)                                                                                       \
    do {                                                                                             \
        if (seg == 16) F3L(C, 16);                                                                   \
        else if (seg == 20) F3L(C, 20);                                                              \
        else if (seg == 24) F3L(C, 24);                                                              \
        else if (seg == 32) F3L(C, 32);                                                              \
        else F3L(C, 64);                                                                             \
    } while (0)
    switch (P->ct) {
        case 5: F3C(5); break;
        case 6: F3C(6); break;
        case 7: F3C(7); break;
        case 11: F3C(11); break;
        default: return -2;
    }
#undef F3C
#undef F3L
    return 0;
}
// the stamps of the last fused launch (4 per fused job: start, parse end, prefix known, decode end; 100 MHz)
extern "C" int dc_fused3_last_seg(void) { return g_f3_seg; }
extern "C" long long dc_fused3_stamps(unsigned long long* out, long long max_jobs) {
    if (!g_f3_stamps) return 0;
    const long long n = std::min(max_jobs, g_f3_nfj);
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpy(out, g_f3_stamps, (size_t)n * 4 * 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return n;
}

static int g_f3_last = 0;
extern "C" int dc_decode3_last_fused(void) { return g_f3_last; }
extern "C" void dc_decode3_clear_fused(void) { g_f3_last = 0; }
extern "C" int dc_launch_decode3(const uint8_t* s, const unsigned long long* dev_nbits, unsigned long long host_nbits,
                                 const Params* P, const Dec3Bufs* D3, float* out, long long num, uint32_t epoch,
                                 int dense, hipStream_t st) {
    int g1 = 0, g3 = 0;
    if (decode3_grids(P, D3, dense, &g1, &g3)) return -2;
    g_f3_last = fused3_on() && D3->seg >= 16 && !dense && !D3->shard;
    if (g_f3_last) {
        dc_mark_phase(4, st);
        dc_mark_phase(5, st);                   // (the timing slots: an empty parse, the launch as decode's)
        if (launch_fused3(s, dev_nbits, host_nbits, P, D3, out, num, epoch, fused3_on() == 2, st)) return -2;
        dbg_wait("fused3_kernel", st);
        dc_mark_phase(7, st);
        dc_mark_next_set();
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    dc_mark_phase(4, st);
    DC_DISPATCH_3(P->ct, D3->seg, parse3_kernel, dim3(g1), dim3(64), 0, st, s, *P, *D3, dev_nbits, host_nbits, num, epoch);
    dbg_wait("parse3_kernel", st);
    dc_mark_phase(5, st);                       // (no mark 6: decode3's slot starts at mark 5)
    if (dense) launch_decode3_cap<D3_CAP_DENSE>(P->ct, D3->seg, g3, st, s, *P, *D3, dev_nbits, host_nbits, out, num, epoch);
    else launch_decode3_cap<D3_CAP>(P->ct, D3->seg, g3, st, s, *P, *D3, dev_nbits, host_nbits, out, num, epoch);
    dbg_wait("decode3_kernel", st);
    if (getenv("DC_DEC3_DEBUG") && hipStreamQuery(st) != hipSuccess) dbg_dump(D3);
    dc_mark_phase(7, st);
    dc_mark_next_set();
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// decode3 alone, after a parse that filled rec / rel / ptot another way (dc_launch_maps_parse)
extern "C" int dc_launch_decode3_values(const uint8_t* s, const unsigned long long* dev_nbits, unsigned long long host_nbits,
                                        const Params* P, const Dec3Bufs* D3in, float* out, long long num, uint32_t epoch,
                                        int dense, hipStream_t st) {
    Dec3Bufs Dv = *D3in;
    Dec3Bufs* D3 = &Dv;
    Dv.seg = dc_maps_seg(D3in->seg);                   // (the maps parse's parse jobs)
    int g1 = 0, g3 = 0;
    if (decode3_grids(P, D3, dense, &g1, &g3)) return -2;
    if (dense) launch_decode3_cap<D3_CAP_DENSE>(P->ct, D3->seg, g3, st, s, *P, *D3, dev_nbits, host_nbits, out, num, epoch);
    else launch_decode3_cap<D3_CAP>(P->ct, D3->seg, g3, st, s, *P, *D3, dev_nbits, host_nbits, out, num, epoch);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int dc_launch_shard3_fix(const uint8_t* s, const Params* P, const Dec3Bufs* D3, const float* hin, float* out,
                                    long long num, hipStream_t st) {
    switch (P->ct) {
        case 5: hipLaunchKernelGGL(shard3_fix_kernel<5>, dim3(1), dim3(64), 0, st, s, *P, *D3, hin, out, num); break;
        case 6: hipLaunchKernelGGL(shard3_fix_kernel<6>, dim3(1), dim3(64), 0, st, s, *P, *D3, hin, out, num); break;
        case 7: hipLaunchKernelGGL(shard3_fix_kernel<7>, dim3(1), dim3(64), 0, st, s, *P, *D3, hin, out, num); break;
        case 11: hipLaunchKernelGGL(shard3_fix_kernel<11>, dim3(1), dim3(64), 0, st, s, *P, *D3, hin, out, num); break;
        default: return -2;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int dc_dec3_prof_read(unsigned long long* out, int reset) {
#ifdef DC_DEC3_PROF
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof3), sizeof g_prof3) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long z[32] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof3), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
#else
    (void)out; (void)reset;
    return -1;
#endif
}

}  // namespace dc
