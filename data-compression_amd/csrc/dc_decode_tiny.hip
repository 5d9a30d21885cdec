// dc_decode_tiny.hip -- the decoder of small streams in ONE workgroup (r06, VERDICT r05 next-5: the reference's
// payloads are small, impl/pingpong.c:169-209 sends 2^14 floats).  The segment decoder's two launches spend ~20 us
// at 2^14 on one long dependent token walk per lane (a 1024-bit pre-walk plus a 1024-bit segment, five waves on the
// whole GPU) and a cross-job exit hand-off.  A stream of at most 2^19 bits (64 KiB: 2^14 floats at any bound) and
// at most 2^14 values fits one CU's LDS together with its decoded values, so here:
//   load     the stream into LDS (byte-swapped words, one zero word in front), the token tables
//   walk     thread i takes segment i (512 bits): a speculative walk from 512 bits before it (self-synchronisation,
//            thread 0 from bit 0) to its first token boundary, then through the segment: entry, exit, token count
//   links    rounds: a thread whose entry is not its predecessor's exit walks again from that exit (a round per
//            link of a chain; chains longer than TY_ROUNDS decline)
//   offsets  a block scan of the counts: each segment's first value index
//   values   each thread decodes its tokens into the LDS value array; a prediction whose history lies in the
//            previous segment makes the prefix up to it pending
//   pending  rounds: a pending prefix is decoded again once the previous segment holds no pending value
//   store    the values to HBM as float4s
// The same grammar and arithmetic as decode3_job (impl/dataCompression.c:1703-2027 for CT7, :2922-3135 CT5, ...):
// the token tables of dc_device.h (build_lut), predict_value with the x86 NaN rules.  Declines (the host then takes
// the chunk-map decoder, as for a declined segment decode): a stream longer than 2^19 bits or with fewer tokens
// than values, a prediction among the first three values or a decoded -1.0f (the reference's history sentinel),
// link or pending chains longer than TY_ROUNDS rounds (runs-mode streams: constant or copy-run data).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "dc_device.h"
#include "dc_shared.h"

namespace dc {

constexpr int TY_T = 1024;                        // threads = segments
constexpr int TY_SEGB = 512;                      // bits per segment
constexpr long long TY_MAXBITS = (long long)TY_T * TY_SEGB;    // 2^19
constexpr int TY_NUM = 16384;                     // values
constexpr int TY_W = TY_T * TY_SEGB / 32 + 8;     // stream words + the zero word in front + pad
// LDS word of logical stream word j (j = 0: the zero word): one pad word per 16, so that the 64 lanes of a wave,
// 16 words (a segment) apart, read 64 different banks (unpadded every lane of a wave hit two banks)
__device__ __forceinline__ int wix(int j) { return j + (j >> 4); }
constexpr int TY_WP = TY_W + TY_W / 16 + 2;
#ifndef DC_TY_PW
#define DC_TY_PW 512                              // pre-walk bits
#endif
constexpr int TY_ROUNDS = 48;
constexpr uint32_t TY_DECLINE = 512u, TY_WHY_RUNS = 1024u, TY_WHY_SHORT = 4096u, TY_WHY_SENT = 16384u;

// MSB-first reader over the LDS words Wd (Wd[0] = 0, stream word k at Wd[k + 1]): the window (a:b) from bit s of
// the word before b, c the next word, the word after c requested one step ahead (as decode3's Rd3)
struct TyRd {
    const uint32_t* Wd;
    uint32_t a, b, c, s;
    int wn;
    int p;                                        // the stream bit of the window's start
    __device__ __forceinline__ void init(const uint32_t* W, int pos) {
        Wd = W;
        const int wi = (pos - 1) >> 5;            // the word holding bit pos - 1 (-1 for pos 0)
        s = (uint32_t)(32 * (wi + 1) - pos);      // 0..31 (0: the window starts at b)
        a = W[wix(wi + 1)]; b = W[wix(wi + 2)]; c = W[wix(wi + 3)];
        wn = wi + 4;
        p = pos;
    }
    __device__ __forceinline__ uint32_t fetch() const { return Wd[wix(wn)]; }
    __device__ __forceinline__ uint32_t peek() const { return __builtin_amdgcn_alignbit(a, b, s); }
    __device__ __forceinline__ void step(uint32_t nx, int len) {
        uint32_t d;
        const bool adv = __builtin_usub_overflow(s, (uint32_t)len, &d);
        s = d & 31u;
        a = adv ? b : a;
        b = adv ? c : b;
        c = adv ? nx : c;
        wn += adv ? 1 : 0;
        p += len;
    }
};

// 16-byte stream groups through a buffer resource over the readable capacity (groups past it read 0), words
// byte-swapped (MSB-first) and the bytes past the stream's end cleared
typedef unsigned ty_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ty_load4(__amdgpu_buffer_rsrc_t rs, int q) {
    const ty_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * q, 0, 0);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t ty_word(uint32_t v, long long nbytes, long long byte0) {
    const long long rem = nbytes - byte0;                                  // stream bytes left at this word
    const uint32_t w = __builtin_bswap32(v);
    return rem >= 4 ? w : (rem <= 0 ? 0u : w & (uint32_t)(0xFFFFFFFF00000000ull >> (8 * rem)));
}

// walk from the reader's position while it is below `end`: the tokens stepped.  DC_TY_ALU: the length computed
// (token_len_bf) instead of read from the LDS table -- a lone chain per thread, so the table read's latency is
// the step's
#ifndef DC_TY_ALU
#define DC_TY_ALU 0
#endif
template <int CT>
__device__ __forceinline__ int ty_walk(TyRd& r, int end, const uint16_t* meta, const Params& P) {
    int n = 0;
    while (r.p < end) {
        const uint32_t nx = r.fetch();
        const uint32_t t = r.peek();
        r.step(nx, DC_TY_ALU ? token_len_bf<CT>(t, P) : (int)(meta[t >> 23] >> 8));
        n++;
    }
    return n;
}

#ifdef DC_TY_STAMPS                                // (diagnostic builds: phase stamps of the last launch)
__device__ unsigned long long ty_stamps[16];
#define TYS(k) do { if (threadIdx.x == 0) ty_stamps[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
extern "C" int dc_tiny_stamps(unsigned long long* h) {
    return hipMemcpyFromSymbol(h, HIP_SYMBOL(ty_stamps), sizeof(ty_stamps), 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#else
#define TYS(k) do {} while (0)
#endif

template <int CT>
__global__ __launch_bounds__(TY_T, 1) void tiny_decode_kernel(const uint8_t* __restrict__ s, long long capw,
                                                              const unsigned long long* dev_nbits,
                                                              unsigned long long host_nbits, Params P,
                                                              float* __restrict__ out, long long num,
                                                              unsigned* __restrict__ err) {
    __shared__ __attribute__((aligned(16))) uint32_t W[TY_WP];
    __shared__ __attribute__((aligned(16))) float OB[TY_NUM];
    __shared__ TokLut T;
    __shared__ int X[TY_T];                        // exits (absolute bits); then the pending counts
    __shared__ uint32_t wsum[TY_T / 64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    TYS(0);
    const unsigned long long nb64 = dev_nbits ? *dev_nbits : host_nbits;
    if (nb64 > (unsigned long long)TY_MAXBITS || num < 1 || num > TY_NUM) {      // (uniform)
        if (tid == 0) atomicOr(err, TY_DECLINE | TY_WHY_SHORT);
        return;
    }
    const int nbits = (int)nb64;
    const long long nbytes = (nb64 + 7) >> 3;
    build_lut<CT>(T, P, tid, TY_T);
    {   // the stream: 16-byte groups (every load in flight at once), bytes past the stream read as 0
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(s), (short)0, (int)(capw * 4), 0x00020000);
        constexpr int QN = (TY_W - 8) / 4 / TY_T;                                  // 4 groups per thread
        uint4 v[QN];
#pragma unroll
        for (int k = 0; k < QN; k++) v[k] = ty_load4(rs, tid + TY_T * k);
#pragma unroll
        for (int k = 0; k < QN; k++) {
            const int q = tid + TY_T * k;
            const long long b0 = 16ll * q;
            W[wix(1 + 4 * q)] = ty_word(v[k].x, nbytes, b0);
            W[wix(2 + 4 * q)] = ty_word(v[k].y, nbytes, b0 + 4);
            W[wix(3 + 4 * q)] = ty_word(v[k].z, nbytes, b0 + 8);
            W[wix(4 + 4 * q)] = ty_word(v[k].w, nbytes, b0 + 12);
        }
        if (tid == 0) W[0] = 0u;
        if (tid < 7) W[wix(TY_W - 7 + tid)] = 0u;
    }
    __syncthreads();
    TYS(1);
    // ---- walk: entry, exit, count of segment tid
    const int sb = tid * TY_SEGB;
    const bool act = sb < nbits;
    const int end = min(sb + TY_SEGB, nbits);
    TyRd r;
    r.init(W, tid == 0 ? 0 : max(sb - DC_TY_PW, 0));
    int e = 0, x = 0, cnt = 0;
    if (act) {
        ty_walk<CT>(r, sb, T.meta, P);
        e = r.p;
        cnt = ty_walk<CT>(r, end, T.meta, P);
        x = r.p;
    }
    X[tid] = x;
    __syncthreads();
    TYS(2);
    // ---- links: a segment's entry must be its predecessor's exit
    for (int round = 0;; round++) {
        const int xin = tid > 0 ? X[tid - 1] : 0;
        const bool bad = act && tid > 0 && e != xin;
        if (!__syncthreads_or(bad)) {
            TYS(8 + 0 * round);
#ifdef DC_TY_STAMPS
            if (tid == 0) ty_stamps[10] = round;
#endif
            break;
        }
        if (round >= TY_ROUNDS) {
            if (tid == 0) atomicOr(err, TY_DECLINE | TY_WHY_RUNS);
            return;                                                                // (uniform)
        }
        if (bad) {
            r.init(W, xin);
            e = xin;
            cnt = e < end ? ty_walk<CT>(r, end, T.meta, P) : 0;
            x = max(r.p, e);
        }
        X[tid] = x;
        __syncthreads();
    }
    // ---- each segment's first value index: a block scan of the counts
    const uint32_t inc = wave_scan_incl((uint32_t)cnt);
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < TY_T / 64; w++) {
        pre += w < wid ? wsum[w] : 0u;
        tot += wsum[w];
    }
    TYS(3);
    if ((long long)tot < num) {                                                    // (uniform)
        if (tid == 0) atomicOr(err, TY_DECLINE | TY_WHY_SHORT);
        return;
    }
    const int o0 = (int)(pre + inc) - cnt;
    const int nt = (int)min((long long)cnt, max(num - o0, 0ll));                    // the values kept
    // ---- values
    bool sent = false;
    int pend = 0;
    if (nt > 0) {
        r.init(W, e);
        for (int t = 0; t < nt; t++) {
            const uint32_t nx = r.fetch();
            const uint32_t tk = r.peek();
            const uint32_t meta = T.meta[tk >> 23];
            uint32_t v = lut_pattern(T, tk, meta);
            if (CT != 6) {
                const uint32_t cc = tk >> 29;                                      // 4: '100' (0), 5..7: predictions
                if (cc >= 4u) v = 0u;
                if (cc >= 5u) {
                    const int need = (int)cc - 4, o = o0 + t;
                    if (o < 3) sent = true;                                        // reads the reference's sentinel
                    else if (t < need || t - need < pend) pend = t + 1;            // history in the previous segment
                    else v = __float_as_uint(predict_value(need, OB[o - 1], OB[o - 2], OB[o - 3]));
                }
            }
            sent |= v == 0xBF800000u;                                              // (a -1.0f value: the sentinel)
            OB[o0 + t] = __uint_as_float(v);
            r.step(nx, (int)(meta >> 8));
        }
    }
    __syncthreads();                                                                // (X read by every thread)
    TYS(4);
    X[tid] = pend;
    __syncthreads();
    // ---- pending prefixes, one link of a chain per round
    for (int round = 0;; round++) {
        const bool go = pend > 0 && (tid == 0 || X[tid - 1] == 0);
        if (!__syncthreads_or(pend > 0)) {
#ifdef DC_TY_STAMPS
            if (tid == 0) ty_stamps[11] = round;
#endif
            break;
        }
        if (round >= TY_ROUNDS) {
            if (tid == 0) atomicOr(err, TY_DECLINE | TY_WHY_RUNS);
            return;
        }
        if (go) {
            float b1 = OB[o0 - 1], b2 = OB[o0 - 2], b3 = OB[o0 - 3];              // (o0 >= 3: a prediction before
            r.init(W, e);                                                          //  value 3 declined above)
            for (int t = 0; t < pend; t++) {
                const uint32_t nx = r.fetch();
                const uint32_t tk = r.peek();
                const uint32_t meta = T.meta[tk >> 23];
                uint32_t v = lut_pattern(T, tk, meta);
                const uint32_t cc = tk >> 29;
                if (cc >= 4u) v = 0u;
                if (cc >= 5u) v = __float_as_uint(predict_value((int)cc - 4, b1, b2, b3));
                sent |= v == 0xBF800000u;
                OB[o0 + t] = __uint_as_float(v);
                b3 = b2; b2 = b1; b1 = __uint_as_float(v);
                r.step(nx, (int)(meta >> 8));
            }
            pend = 0;
        }
        __syncthreads();
        X[tid] = pend;
        __syncthreads();
    }
    if (__syncthreads_or(sent)) {
        if (tid == 0) atomicOr(err, TY_DECLINE | TY_WHY_SENT);
        return;
    }
    TYS(5);
    // ---- store: whole float4s, then the tail
    const int n4 = (int)(num >> 2);
    float4* o4 = reinterpret_cast<float4*>(out);
    const float4* b4 = reinterpret_cast<const float4*>(OB);
    for (int q = tid; q < n4; q += TY_T) o4[q] = b4[q];
    if (tid < (int)(num & 3)) out[4 * n4 + tid] = OB[4 * n4 + tid];
    TYS(6);
}

extern "C" long long dc_tiny_max_values(void) { return TY_NUM; }
extern "C" long long dc_tiny_max_bits(void) { return TY_MAXBITS; }

// d_out 16-byte aligned, num <= TY_NUM; capb: the stream buffer's readable bytes
extern "C" int dc_launch_decode_tiny(const uint8_t* s, long long capb, const unsigned long long* dev_nbits,
                                     unsigned long long host_nbits, const Params* P, float* out, long long num,
                                     unsigned* err, hipStream_t st) {
    if (num < 1 || num > TY_NUM || ((uintptr_t)out & 15u) || ((uintptr_t)s & 3u) || capb < 16) return -2;
    const long long capw = min(capb, (long long)(TY_W - 8) * 4) / 16 * 4;
    dc_mark_phase(4, st);
    dc_mark_phase(5, st);                          // (the timing slots: an empty parse, the launch as decode's)
    switch (P->ct) {
        case 5: hipLaunchKernelGGL(tiny_decode_kernel<5>, dim3(1), dim3(TY_T), 0, st, s, capw, dev_nbits, host_nbits, *P, out, num, err); break;
        case 6: hipLaunchKernelGGL(tiny_decode_kernel<6>, dim3(1), dim3(TY_T), 0, st, s, capw, dev_nbits, host_nbits, *P, out, num, err); break;
        case 7: hipLaunchKernelGGL(tiny_decode_kernel<7>, dim3(1), dim3(TY_T), 0, st, s, capw, dev_nbits, host_nbits, *P, out, num, err); break;
        case 11: hipLaunchKernelGGL(tiny_decode_kernel<11>, dim3(1), dim3(TY_T), 0, st, s, capw, dev_nbits, host_nbits, *P, out, num, err); break;
        default: return -2;
    }
    dc_mark_phase(7, st);
    dc_mark_next_set();
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace dc
