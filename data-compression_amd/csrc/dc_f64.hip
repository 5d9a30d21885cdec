// dc_f64.hip -- the DOUBLE bit-wise codecs on gfx950 (CT 5/6/7/11) and their pre-passes.
//
// Replaces myCompress_bitwise_double (impl/dataCompression.c:3189), _np (:2633), _mask (:1590),
// _op (:355) and the decoders myDecompress_bitwise_double (:2656), _np (:2286), _mask (:1199),
// _op (:476); toSmallDataset_double (:3522) and med_dataset_double (:3564).
//
// Grammar (the float one widened): '100' zero, '101'/'110'/'111' predictions (history = ORIGINAL
// inputs in the encoder, DECODED values in the decoder), raw token = the top 12+m bits of the double,
// m = clamp(B + E - 1023, 0, 52) (compress_bitwise_double :3446-3477), CT7 masked tokens
// '0' 1^type {0|1} + tail against mask[1+11+8] (compress_bitwise_double_mask :1493-1588), CT11 verbatim
// 64 bits.  A token is at most 64 bits and its length is a function of its first 12 bits.
// Double arithmetic uses explicit round-to-nearest intrinsics (no FMA contraction, as on x86 SSE2).
//
// Encoder: count (tile bit lengths) -> scan (tile offsets; zeroes every tile's first word) -> write
//   (tokens ORed into an LDS bit buffer, interior words stored, the two shared boundary words ORed
//   with global atomics).  Inputs holding the -1.0 history sentinel (:3191) go to an exact serial
//   kernel.
// Decoder (tokens are not self-delimiting from an arbitrary bit):
//   map    : one lane per 2048-bit chunk parses the path from the chunk's bit 0 (P0, boundaries kept in
//            LDS) and, for every other entry offset 1..63, walks until it lands on a P0 boundary:
//            chunk map entry -> (exit offset into the next chunk, tokens started in the chunk);
//   compose: maps of 64 consecutive nodes are composed (one lane per entry), level after level until
//            one root remains;  descend: from the root (entry 0, token 0) every node's true entry and
//            first token index are assigned top-down;
//   decode : one lane per chunk decodes from its entry; values that depend on the previous chunk are
//            tracked symbolically (kind 1..3 = incoming b1..b3, 4 = derived) and left pending;
//   fix    : pending prefixes are re-decoded from the three preceding outputs -- in parallel where the
//            previous chunk ends concrete, then one ordered pass for chains crossing whole chunks;
//   exact  : a stream whose first three tokens hold a prediction or that decodes to the -1.0 history
//            sentinel (:2722-2740) is re-decoded by one thread with the reference's history semantics.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <stdlib.h>
#include <string.h>
#include "dc_shared.h"
#include "../../include/dc_gpu.h"

namespace dc64 {

struct P64 {
    int ct, B, type, mm, mm0;
    double bound;
    uint32_t mask20;
};

constexpr int ETILE = 1024;                 // encoder elements per tile
constexpr int ETPB = 256;                   // encoder threads per tile (4 consecutive elements each)
constexpr int CB = 2048;                    // decoder chunk bits
constexpr int MAPW = CB / 32;               // P0 boundary mask words per chunk
constexpr int FAN = 64;                     // compose fan-in
constexpr unsigned ERR_SERIAL = 1u;

__device__ __forceinline__ uint64_t d2u(double d) { return (uint64_t)__double_as_longlong(d); }
__device__ __forceinline__ double u2d(uint64_t u) { return __longlong_as_double((long long)u); }
__device__ __forceinline__ int mbits(int B, int E) { return min(max(B + E - 1023, 0), 52); }
__device__ __forceinline__ uint32_t bswap(uint32_t v) { return __builtin_bswap32(v); }

// NaN results follow x86 SSE2 as gcc orders the operations (the reference's host): 2*b1 - b2 returns
// the first NaN of b1, b2 (quieted); 3*b1 - 3*b2 + b3 is evaluated as b3 + (3*b1 - 3*b2), so a NaN b3
// wins; a NaN made from non-NaN operands (inf - inf) is the x86 default NaN 0xFFF8000000000000.
// Only streams decoded outside the codec's domain reach this (an encoder never predicts with NaNs).
__device__ __noinline__ double x86_nan(double b1, double b2, double b3, bool use3) {
    const uint64_t q = 0x0008000000000000ull;
    if (use3 && b3 != b3) return u2d(d2u(b3) | q);
    if (b1 != b1) return u2d(d2u(b1) | q);
    if (b2 != b2) return u2d(d2u(b2) | q);
    return u2d(0xFFF8000000000000ull);
}
__device__ __forceinline__ double pred2(double b1, double b2) {
    const double v = __dsub_rn(__dmul_rn(2.0, b1), b2);
    return v != v ? x86_nan(b1, b2, 0.0, false) : v;
}
__device__ __forceinline__ double pred3(double b1, double b2, double b3) {
    const double v = __dadd_rn(__dsub_rn(__dmul_rn(3.0, b1), __dmul_rn(3.0, b2)), b3);
    return v != v ? x86_nan(b1, b2, b3, true) : v;
}

// ---------------------------------------------------------------------------------------------- encoder
// token of x (myCompress_bitwise_double :3229-3300 and its _np/_mask/_op twins); b1..b3 = ORIGINAL inputs
template <int CT>
__device__ __forceinline__ void make_token(double x, double b1, double b2, double b3, bool pred, const P64& P,
                                           uint64_t& val, int& len) {
    const uint64_t u = d2u(x);
    if (CT != 6) {
        if (fabs(x) < P.bound) { val = 4; len = 3; return; }                       // '100'
        if (pred) {
            const double d1 = fabs(__dsub_rn(b1, x)), d2 = fabs(__dsub_rn(pred2(b1, b2), x));
            const double d3 = fabs(__dsub_rn(pred3(b1, b2, b3), x));
            double dmin = d1; uint64_t code = 5;
            if (d2 < dmin) { dmin = d2; code = 6; }
            if (d3 < dmin) { dmin = d3; code = 7; }
            if (dmin <= P.bound) { val = code; len = 3; return; }
        }
        if (CT == 11) { val = u; len = 64; return; }
    }
    const int m = mbits(P.B, (int)((u >> 52) & 0x7FF));
    if (CT == 7 && (u >> 52) == (uint64_t)(P.mask20 >> 8)) {                    // :1523-1575
        const uint64_t head = ((1ull << P.type) - 1ull) << 1;
        if (((u >> 44) & 0xFF) == (P.mask20 & 0xFF)) {
            const int tl = m > 8 ? m - 8 : 0;
            val = (head << tl) | (tl ? ((u >> (52 - m)) & ((1ull << tl) - 1ull)) : 0ull);
            len = P.type + 2 + tl;
        } else {
            val = ((head | 1ull) << m) | (m ? ((u >> (52 - m)) & ((1ull << m) - 1ull)) : 0ull);
            len = P.type + 2 + m;
        }
        return;
    }
    val = u >> (52 - m);
    len = 12 + m;
}

// element e's token with its history (encoder: original inputs, no prediction before element 3)
template <int CT>
__device__ __forceinline__ void token_at(const double* __restrict__ x, long long e, const P64& P, uint64_t& val, int& len) {
    const double v = x[e];
    const bool pred = e >= 3;
    const double b1 = pred ? x[e - 1] : 0.0, b2 = pred ? x[e - 2] : 0.0, b3 = pred ? x[e - 3] : 0.0;
    make_token<CT>(v, b1, b2, b3, pred, P, val, len);
}

// the tokens of the 4 consecutive elements e0..e0+3 from one load of x[e0-3 .. e0+3]
template <int CT>
__device__ __forceinline__ void tokens4(const double* __restrict__ x, long long n, long long e0, const P64& P,
                                        uint64_t* val, int* len, bool* neg1) {
    double w[7];
    if (e0 >= 3 && e0 + 4 <= n) {
#pragma unroll
        for (int i = 0; i < 7; i++) w[i] = x[e0 - 3 + i];
    } else {
#pragma unroll
        for (int i = 0; i < 7; i++) {
            const long long e = e0 - 3 + i;
            w[i] = (e >= 0 && e < n) ? x[e] : 0.0;
        }
    }
    bool m1 = false;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        val[k] = 0; len[k] = 0;
        if (e0 + k < n) {
            make_token<CT>(w[3 + k], w[2 + k], w[1 + k], w[k], e0 + k >= 3, P, val[k], len[k]);
            m1 |= w[3 + k] == -1.0;
        }
    }
    *neg1 = m1;
}

template <int CT>
__global__ __launch_bounds__(ETPB) void enc_count(const double* __restrict__ x, long long n, P64 P,
                                                 uint32_t* __restrict__ tbits, unsigned* __restrict__ err) {
    __shared__ uint32_t part[ETPB / 64];
    const long long t = blockIdx.x;
    const long long e0 = t * ETILE + 4 * threadIdx.x;
    uint64_t vv[4];
    int ll[4];
    bool neg1 = false;
    tokens4<CT>(x, n, e0, P, vv, ll, &neg1);
    uint32_t sum = (uint32_t)(ll[0] + ll[1] + ll[2] + ll[3]);
    if (neg1) atomicOr(err, ERR_SERIAL);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) sum += __shfl_xor(sum, d, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = sum;
    __syncthreads();
    if (threadIdx.x == 0) tbits[t] = part[0] + part[1] + part[2] + part[3];
}

// exclusive scan of the tile lengths (one workgroup, 1024 tiles per round); zeroes every tile's first
// stream word and the last one (the write kernel ORs the words it shares with its neighbours)
__global__ __launch_bounds__(1024) void enc_scan(const uint32_t* __restrict__ tbits, long long ntiles, int start_bit,
                                                 unsigned long long* __restrict__ toff, uint32_t* __restrict__ out,
                                                 unsigned long long* __restrict__ total) {
    __shared__ unsigned long long ws[16];
    __shared__ unsigned long long carry;
    if (threadIdx.x == 0) carry = (unsigned long long)start_bit;
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (long long b = 0; b < ntiles; b += 1024) {
        const long long t = b + threadIdx.x;
        const unsigned long long v = t < ntiles ? tbits[t] : 0ull;
        unsigned long long s = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long o = __shfl_up(s, d, 64);
            if (lane >= d) s += o;
        }
        if (lane == 63) ws[wv] = s;
        __syncthreads();
        unsigned long long wpre = 0;
        for (int i = 0; i < wv; i++) wpre += ws[i];
        const unsigned long long c0 = carry;
        const unsigned long long off = c0 + wpre + s - v;
        if (t < ntiles) {
            toff[t] = off;
            out[off >> 5] = 0u;
        }
        __syncthreads();
        if (threadIdx.x == 1023) carry = off + v;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const unsigned long long end = carry;
        if (end > (unsigned long long)start_bit) out[(end - 1) >> 5] = 0u;
        *total = end - (unsigned long long)start_bit;
    }
}

// the same scan in three launches for many tiles: block scans (1024 tiles each), a scan of the block
// sums, then offsets + start bit, zeroing of every tile's first word and the stream's last word
__global__ __launch_bounds__(1024) void enc_scan_part(const uint32_t* __restrict__ tbits, long long ntiles,
                                                      unsigned long long* __restrict__ toff,
                                                      unsigned long long* __restrict__ psum) {
    __shared__ unsigned long long ws[16];
    const long long t = blockIdx.x * 1024ll + threadIdx.x;
    const unsigned long long v = t < ntiles ? tbits[t] : 0ull;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned long long s = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long o = __shfl_up(s, d, 64);
        if (lane >= d) s += o;
    }
    if (lane == 63) ws[wv] = s;
    __syncthreads();
    unsigned long long pre = 0, tot = 0;
    for (int i = 0; i < 16; i++) { if (i < wv) pre += ws[i]; tot += ws[i]; }
    if (t < ntiles) toff[t] = pre + s - v;
    if (threadIdx.x == 0) psum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void scan_top(unsigned long long* __restrict__ psum, long long nb) {
    __shared__ unsigned long long ws[16];
    __shared__ unsigned long long carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (long long b = 0; b <= nb; b += 1024) {                  // psum[nb] = the total
        const long long i = b + threadIdx.x;
        const unsigned long long v = i < nb ? psum[i] : 0ull;
        unsigned long long s = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long o = __shfl_up(s, d, 64);
            if (lane >= d) s += o;
        }
        if (lane == 63) ws[wv] = s;
        __syncthreads();
        unsigned long long pre = 0;
        for (int k = 0; k < wv; k++) pre += ws[k];
        const unsigned long long off = carry + pre + s - v;
        if (i <= nb) psum[i] = off;
        __syncthreads();
        if (threadIdx.x == 1023) carry = off + v;
        __syncthreads();
    }
}

__global__ __launch_bounds__(1024) void enc_scan_add(long long ntiles, int start_bit, const unsigned long long* __restrict__ psum,
                                                     unsigned long long* __restrict__ toff, uint32_t* __restrict__ out,
                                                     unsigned long long* __restrict__ total) {
    const long long t = blockIdx.x * 1024ll + threadIdx.x;
    if (t < ntiles) {
        const unsigned long long off = toff[t] + psum[blockIdx.x] + (unsigned long long)start_bit;
        toff[t] = off;
        out[off >> 5] = 0u;
    }
    if (t == 0) {
        const long long nb = (ntiles + 1023) / 1024;
        const unsigned long long end = psum[nb] + (unsigned long long)start_bit;
        if (end > (unsigned long long)start_bit) out[(end - 1) >> 5] = 0u;
        *total = end - (unsigned long long)start_bit;
    }
}

__device__ __forceinline__ void lds_or(uint32_t* L, uint32_t off, uint64_t val, int len) {   // len 1..64
    const uint32_t w = off >> 5, b = off & 31u;
    const int end = (int)b + len;                                     // 1..95
    // the token occupies bits [b, end) of the 96-bit window L[w..w+2]
    const uint64_t hi = end <= 64 ? (val << (64 - end)) : (val >> (end - 64));
    const uint32_t lo = end > 64 ? (uint32_t)(val << (96 - end)) : 0u;
    const uint32_t a0 = (uint32_t)(hi >> 32), a1 = (uint32_t)hi;
    if (a0) atomicOr(&L[w], a0);
    if (a1) atomicOr(&L[w + 1], a1);
    if (lo) atomicOr(&L[w + 2], lo);
}

template <int CT>
__global__ __launch_bounds__(ETPB) void enc_write(const double* __restrict__ x, long long n, P64 P,
                                                 const unsigned long long* __restrict__ toff,
                                                 uint32_t* __restrict__ out) {
    __shared__ uint32_t L[ETILE * 2 + 8];
    __shared__ uint32_t wsum[ETPB / 64];
    const long long t = blockIdx.x;
    for (int i = threadIdx.x; i < ETILE * 2 + 8; i += ETPB) L[i] = 0u;
    const long long e0 = t * ETILE + 4 * threadIdx.x;
    uint64_t val[4];
    int len[4];
    bool neg1;                                        // (reported by the count pass)
    tokens4<CT>(x, n, e0, P, val, len, &neg1);
    const uint32_t sum = (uint32_t)(len[0] + len[1] + len[2] + len[3]);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t s = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(s, d, 64);
        if (lane >= d) s += o;
    }
    if (lane == 63) wsum[wv] = s;
    __syncthreads();
    uint32_t pre = s - sum, tot = 0;
    for (int i = 0; i < ETPB / 64; i++) {
        if (i < wv) pre += wsum[i];
        tot += wsum[i];
    }
    const unsigned long long G = toff[t];
    uint32_t off = (uint32_t)(G & 31ull) + pre;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (len[k]) lds_or(L, off, val[k], len[k]);
        off += (uint32_t)len[k];
    }
    __syncthreads();
    if (tot == 0) return;
    const unsigned long long gw0 = G >> 5, gw1 = (G + tot - 1) >> 5;
    for (unsigned long long w = gw0 + threadIdx.x; w <= gw1; w += ETPB) {
        const uint32_t v = L[w - gw0];
        // a word is shared with the previous / next tile only if the tile starts / ends inside it
        const bool shared = (w == gw0 && (G & 31ull)) || (w == gw1 && ((G + tot) & 31ull));
        if (shared) { if (v) atomicOr(&out[w], bswap(v)); }
        else out[w] = bswap(v);
    }
}

// exact serial encoder (one thread): the reference's sentinel history (:3191-3227), used when an input
// equals -1.0; writes whole bytes, zeroing the stream as it goes
template <int CT>
__global__ void enc_serial(const double* __restrict__ x, long long n, P64 P, int start_bit, uint8_t* __restrict__ out,
                           unsigned long long* __restrict__ total, const unsigned* __restrict__ err) {
    if (threadIdx.x != 0 || blockIdx.x != 0 || !(*err & ERR_SERIAL)) return;
    double b1 = -1.0, b2 = -1.0, b3 = -1.0;
    unsigned long long bits = (unsigned long long)start_bit;
    uint32_t acc = 0;                 // bits of the current byte, MSB first
    int nacc = start_bit;             // the caller ORs the kept head bits of its first byte
    long long ob = 0;
    for (long long i = 0; i < n; i++) {
        const double v = x[i];
        uint64_t val; int len;
        if (CT == 6) {
            make_token<CT>(v, 0, 0, 0, false, P, val, len);
        } else if (b3 == -1.0 || b2 == -1.0 || b1 == -1.0) {
            make_token<CT>(v, 0, 0, 0, false, P, val, len);
            if (b3 == -1.0) b3 = v; else if (b2 == -1.0) b2 = v; else b1 = v;
        } else {
            make_token<CT>(v, b1, b2, b3, true, P, val, len);
            b3 = b2; b2 = b1; b1 = v;
        }
        for (int k = len - 1; k >= 0; k--) {
            acc = (acc << 1) | (uint32_t)((val >> k) & 1ull);
            if (++nacc == 8) { out[ob++] = (uint8_t)acc; acc = 0; nacc = 0; }
        }
        bits += (unsigned long long)len;
    }
    if (nacc) out[ob] = (uint8_t)(acc << (8 - nacc));
    *total = bits - (unsigned long long)start_bit;
}

// ---------------------------------------------------------------------------------------------- decoder
struct Plan64 {
    unsigned long long nbits;
    long long nbytes, nwords, nchunks;
};

__global__ void dec_plan(Plan64* pl, const unsigned long long* dev_nbits, unsigned long long host_nbits, long long max_chunks,
                         unsigned* err) {
    const unsigned long long nb = dev_nbits ? *dev_nbits : host_nbits;
    Plan64 p;
    p.nbits = nb;
    p.nbytes = (long long)((nb + 7) >> 3);
    p.nwords = (long long)((nb + 31) >> 5);
    p.nchunks = std::min((long long)((nb + CB - 1) / CB), max_chunks);
    if (p.nchunks == 0) *err = ERR_SERIAL;           // empty stream: the exact decoder reports it
    *pl = p;
}

// stream bytes -> big-endian 32-bit words, 4 zero words of padding past the end
__global__ void dec_stage(const uint8_t* __restrict__ s, const Plan64* __restrict__ pl, uint32_t* __restrict__ W,
                          long long max_words) {
    const long long nb = pl->nbytes, nw = pl->nwords + 4;
    for (long long w = blockIdx.x * (long long)blockDim.x + threadIdx.x; w < nw && w < max_words;
         w += (long long)gridDim.x * blockDim.x) {
        uint32_t v = 0;
        const long long b = 4 * w;
        if (b + 4 <= nb && ((reinterpret_cast<uintptr_t>(s) & 3) == 0)) {
            v = bswap(*reinterpret_cast<const uint32_t*>(s + b));
        } else {
            for (int k = 0; k < 4; k++) v = (v << 8) | (b + k < nb ? (uint32_t)s[b + k] : 0u);
        }
        W[w] = v;
    }
}

__device__ __forceinline__ uint64_t peek(const uint32_t* __restrict__ W, unsigned long long p) {
    const unsigned long long w = p >> 5;
    const int s = (int)(p & 31);
    const uint64_t a = ((uint64_t)W[w] << 32) | W[w + 1];
    return s ? (a << s) | ((uint64_t)W[w + 2] >> (32 - s)) : a;
}

template <int CT>
__device__ __forceinline__ int tok_len(uint64_t win, const P64& P) {
    if (CT != 6 && (win >> 63)) return 3;
    if (CT == 11) return 64;
    if (CT == 7) {
        const uint32_t ones = (1u << P.type) - 1u;
        if (((uint32_t)(win >> (63 - P.type)) & ones) == ones)
            return P.type + 2 + (((win >> (62 - P.type)) & 1ull) ? P.mm : P.mm0);
    }
    return 12 + mbits(P.B, (int)((win >> 52) & 0x7FF));
}

// value of a non-code token (decompress_bitwise_double :2895-2918, _mask :1418-1488; CT11 verbatim)
template <int CT>
__device__ __forceinline__ double tok_value(uint64_t win, int len, const P64& P) {
    if (CT == 11) return u2d(win);
    if (CT == 7) {
        const uint32_t ones = (1u << P.type) - 1u;
        if (((uint32_t)(win >> (63 - P.type)) & ones) == ones) {
            const int flag = (int)((win >> (62 - P.type)) & 1ull);
            const int tl = len - (P.type + 2);
            const uint64_t tail = tl ? ((win << (P.type + 2)) >> (64 - tl)) : 0ull;
            uint64_t u;
            if (!flag) {
                u = (uint64_t)P.mask20 << 44;
                if (tl) u |= tail << (44 - tl);
                if (20 + tl < 64) u |= 1ull << (43 - tl);
            } else {
                u = (uint64_t)(P.mask20 >> 8) << 52;
                if (tl) u |= tail << (52 - tl);
                if (12 + tl < 64) u |= 1ull << (51 - tl);
            }
            return u2d(u);
        }
    }
    if (len >= 64) return u2d(win);
    return u2d((win & ~((1ull << (64 - len)) - 1ull)) | (1ull << (63 - len)));
}

// A workgroup of 64 lanes handles 64 consecutive chunks: their stream words (plus the 8 that follow,
// for walks past the last chunk) are staged in LDS, one pad word per 64 so that lanes walking their
// chunks at about the same offset hit different banks.
constexpr int GW = 64 * MAPW + 8;
constexpr int SW = GW + GW / 64 + 2;
constexpr int MB = 512;                     // P0 boundaries kept for the first MB bits of a chunk
__device__ __forceinline__ int sidx(int w) { return w + (w >> 6); }
__device__ __forceinline__ uint64_t peekS(const uint32_t* S, uint32_t q) {
    const int w = (int)(q >> 5), s = (int)(q & 31);
    const uint64_t a = ((uint64_t)S[sidx(w)] << 32) | S[sidx(w + 1)];
    return s ? (a << s) | ((uint64_t)S[sidx(w + 2)] >> (32 - s)) : a;
}
__device__ __forceinline__ void stage_group(uint32_t* S, const uint32_t* __restrict__ W, long long w0, long long wlim) {
    for (int i = threadIdx.x; i < GW; i += blockDim.x) {
        const long long w = w0 + i;
        S[sidx(i)] = w < wlim ? W[w] : 0u;
    }
}

// chunk maps, entry-major: map[e * mstride + c] = exit | count << 8 for every entry e of chunk c.  One
// lane per chunk parses P0 from the chunk's bit 0 (boundaries of its first MB bits kept); every other
// entry walks until it lands on a P0 boundary (then it shares P0's remaining tokens and exit) or
// leaves the chunk.
template <int CT>
__global__ __launch_bounds__(64) void dec_map(const uint32_t* __restrict__ W, const Plan64* __restrict__ pl, P64 P,
                                              uint32_t* __restrict__ map, long long mstride) {
    __shared__ uint32_t S[SW];
    __shared__ uint32_t M[64 * (MB / 32 + 1)];
    const long long g0 = blockIdx.x * 64ll;
    const long long nc = pl->nchunks;
    if (g0 >= nc) return;
    stage_group(S, W, g0 * MAPW, pl->nwords + 4);
    const long long c = g0 + threadIdx.x;
    uint32_t* mk = M + threadIdx.x * (MB / 32 + 1);
#pragma unroll
    for (int i = 0; i < MB / 32; i++) mk[i] = 0u;
    __syncthreads();
    if (c >= nc) return;
    const long long avail = (long long)pl->nbits - g0 * CB;            // stream bits from the group start
    const uint32_t lim = (uint32_t)std::min(avail, (long long)(64 * CB + 64));
    const uint32_t cs = threadIdx.x * CB, ce = cs + CB;
    uint32_t p = cs, cnt0 = 0;
    while (p < ce) {
        const int l = tok_len<CT>(peekS(S, p), P);
        if (p + (uint32_t)l > lim) { p = ce; break; }                  // the stream's last (padding) bits
        const uint32_t r = p - cs;
        if (r < MB) mk[r >> 5] |= 1u << (r & 31);
        cnt0++;
        p += (uint32_t)l;
    }
    const uint32_t exit0 = p - ce;
    map[c] = exit0 | (cnt0 << 8);
    for (int e = 1; e < 64; e++) {
        uint32_t q = (uint32_t)e, cnt = 0, ex = 0;
        while (true) {
            if (q >= CB) { ex = q - CB; break; }
            if (cs + q >= lim) { ex = 0; break; }
            if (q < MB && ((mk[q >> 5] >> (q & 31)) & 1u)) {            // joined P0: its remaining tokens
                uint32_t before = __popc(mk[q >> 5] & ((1u << (q & 31)) - 1u));
                for (uint32_t i = 0; i < (q >> 5); i++) before += __popc(mk[i]);
                cnt += cnt0 - before;
                ex = exit0;
                break;
            }
            const int l = tok_len<CT>(peekS(S, cs + q), P);
            if (cs + q + (uint32_t)l > lim) { ex = 0; break; }
            cnt++;
            q += (uint32_t)l;
        }
        map[(long long)e * mstride + c] = ex | (cnt << 8);
    }
}

// compose FAN consecutive node maps (level l-1) into one map (level l); one lane per entry
// ---- fast path: speculative entries.  Lane c pre-walks the previous chunk from its bit 0 (any start
// synchronises with the true token boundaries with high probability within one chunk of random data)
// and so arrives at chunk c with a speculative entry se[c]; it then walks chunk c: exit sx[c], tokens
// sn[c].  The entries are right when every link holds: sx[c-1] == se[c] (chunk 0 starts at bit 0).
#ifndef DC64_OVB
#define DC64_OVB 2048
#endif
constexpr int OVB = DC64_OVB;
#ifndef DC64_RING
#define DC64_RING 0                              // 1: 64-byte output sectors through a padded LDS ring
#endif                // pre-walk overlap (bits)
constexpr int OVW = OVB / 32;
constexpr int GWS = OVW + 64 * MAPW + 8;
constexpr int SWS = GWS + GWS / 64 + 2;

template <int CT>
__global__ __launch_bounds__(64) void dec_spec(const uint32_t* __restrict__ W, const Plan64* __restrict__ pl, P64 P,
                                               uint8_t* __restrict__ se, uint8_t* __restrict__ sx,
                                               uint16_t* __restrict__ sn) {
    __shared__ uint32_t S[SWS];
    const long long g0 = blockIdx.x * 64ll;
    const long long nc = pl->nchunks;
    if (g0 >= nc) return;
    const long long w0 = g0 * MAPW - OVW, wlim = pl->nwords + 4;
    for (int i = threadIdx.x; i < GWS; i += 64) {
        const long long w = w0 + i;
        S[sidx(i)] = (w >= 0 && w < wlim) ? W[w] : 0u;
    }
    __syncthreads();
    const long long c = g0 + threadIdx.x;
    if (c >= nc) return;
    const long long avail = (long long)pl->nbits - (g0 * CB - OVB);         // stream bits from S's origin
    const uint32_t lim = (uint32_t)std::min(avail, (long long)(OVB + 64 * CB + 64));
    const uint32_t cs = OVB + threadIdx.x * CB, ce = cs + CB;
    uint32_t p = c == 0 ? cs : cs - OVB;
    while (p < cs) p += (uint32_t)tok_len<CT>(peekS(S, p), P);
    const uint32_t e = p - cs;
    uint32_t n = 0;
    while (p < ce) {
        const int l = tok_len<CT>(peekS(S, p), P);
        if (p + (uint32_t)l > lim) { p = ce; break; }
        n++;
        p += (uint32_t)l;
    }
    se[c] = (uint8_t)e;
    sx[c] = (uint8_t)(p - ce);
    sn[c] = (uint16_t)n;
}

// broken links: bad[c] = sx[c-1] != se[c]; *ctr counts them, list[] holds them (any order)
__global__ __launch_bounds__(256) void dec_links(const Plan64* __restrict__ pl, const uint8_t* __restrict__ se,
                                                 const uint8_t* __restrict__ sx, uint8_t* __restrict__ bad,
                                                 unsigned* __restrict__ ctr, unsigned* __restrict__ list) {
    const long long c = blockIdx.x * 256ll + threadIdx.x;
    if (c >= pl->nchunks) return;
    const bool b = c > 0 && sx[c - 1] != se[c];
    bad[c] = b ? 1 : 0;
    if (b) list[atomicAdd(ctr, 1u)] = (unsigned)c;
}

// one repair round: a chunk with a broken link whose predecessor's link holds takes the predecessor's
// exit as its entry and walks again (chains of broken links advance one chunk per round).  One
// workgroup per listed chunk: its words are staged in LDS, lane 0 walks.
template <int CT>
__global__ __launch_bounds__(64) void dec_relink(const uint32_t* __restrict__ W, const Plan64* __restrict__ pl, P64 P,
                                                 uint8_t* __restrict__ se, uint8_t* __restrict__ sx,
                                                 uint16_t* __restrict__ sn, const uint8_t* __restrict__ bad,
                                                 const unsigned* __restrict__ ctr, const unsigned* __restrict__ list) {
    __shared__ uint32_t S[MAPW + 8];
    const unsigned nl = *ctr;
    const long long wlim = pl->nwords + 4;
    for (unsigned i = blockIdx.x; i < nl; i += gridDim.x) {
        const long long c = list[i];
        if (c <= 0 || c >= pl->nchunks || !bad[c] || bad[c - 1]) continue;     // uniform in the workgroup
        __syncthreads();
        for (int k = threadIdx.x; k < MAPW + 8; k += 64) {
            const long long w = c * MAPW + k;
            S[k] = w < wlim ? W[w] : 0u;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            const long long avail = (long long)pl->nbits - c * CB;
            const uint32_t lim = (uint32_t)std::min(avail, (long long)(CB + 64));
            const int t = sx[c - 1];
            uint32_t p = (uint32_t)t, n = 0;
            while (p < (uint32_t)CB) {
                const uint32_t w = p >> 5, sh = p & 31;
                const uint64_t a = ((uint64_t)S[w] << 32) | S[w + 1];
                const uint64_t win = sh ? (a << sh) | ((uint64_t)S[w + 2] >> (32 - sh)) : a;
                const int l = tok_len<CT>(win, P);
                if (p + (uint32_t)l > lim) { p = CB; break; }
                n++;
                p += (uint32_t)l;
            }
            se[c] = (uint8_t)t;
            sx[c] = (uint8_t)(p - CB);
            sn[c] = (uint16_t)n;
        }
    }
}

// exclusive scan of the chunk token counts -> first token index of every chunk (3 launches)
__global__ __launch_bounds__(1024) void cnt_scan_part(const Plan64* __restrict__ pl, const uint16_t* __restrict__ sn,
                                                      unsigned long long* __restrict__ base,
                                                      unsigned long long* __restrict__ psum) {
    __shared__ unsigned long long ws[16];
    const long long c = blockIdx.x * 1024ll + threadIdx.x;
    if (blockIdx.x * 1024ll >= pl->nchunks) return;
    const unsigned long long v = c < pl->nchunks ? sn[c] : 0ull;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned long long s = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long o = __shfl_up(s, d, 64);
        if (lane >= d) s += o;
    }
    if (lane == 63) ws[wv] = s;
    __syncthreads();
    unsigned long long pre = 0, tot = 0;
    for (int i = 0; i < 16; i++) { if (i < wv) pre += ws[i]; tot += ws[i]; }
    if (c < pl->nchunks) base[c] = pre + s - v;
    if (threadIdx.x == 0) psum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void cnt_scan_top(const Plan64* __restrict__ pl, unsigned long long* __restrict__ psum) {
    __shared__ unsigned long long ws[16];
    __shared__ unsigned long long carry;
    const long long nb = (pl->nchunks + 1023) / 1024;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (long long b = 0; b < nb; b += 1024) {
        const long long i = b + threadIdx.x;
        const unsigned long long v = i < nb ? psum[i] : 0ull;
        unsigned long long s = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long o = __shfl_up(s, d, 64);
            if (lane >= d) s += o;
        }
        if (lane == 63) ws[wv] = s;
        __syncthreads();
        unsigned long long pre = 0;
        for (int k = 0; k < wv; k++) pre += ws[k];
        const unsigned long long off = carry + pre + s - v;
        if (i < nb) psum[i] = off;
        __syncthreads();
        if (threadIdx.x == 1023) carry = off + v;
        __syncthreads();
    }
}

__global__ __launch_bounds__(1024) void cnt_scan_add(const Plan64* __restrict__ pl, const unsigned long long* __restrict__ psum,
                                                     unsigned long long* __restrict__ base) {
    const long long c = blockIdx.x * 1024ll + threadIdx.x;
    if (c < pl->nchunks) base[c] += psum[blockIdx.x];
}

// (level-1 input = the entry-major chunk maps: node i entry e at in[e * nin_max + i])
template <typename T>
__global__ __launch_bounds__(64) void dec_compose(const T* __restrict__ in, long long nin_max,
                                                  const Plan64* __restrict__ pl, long long div,
                                                  unsigned long long* __restrict__ outm) {
    const bool emaj = sizeof(T) == 4;
    const long long g = blockIdx.x;
    const long long nin = (pl->nchunks + div - 1) / div;         // nodes at the input level
    if (g * FAN >= nin) return;
    int e = (int)threadIdx.x;
    unsigned long long cnt = 0;
    const long long end = std::min(nin, (g + 1) * FAN);
    for (long long i = g * FAN; i < end; i++) {
        const unsigned long long m = (unsigned long long)(emaj ? in[(long long)e * nin_max + i] : in[i * 64 + e]);
        e = (int)(m & 63ull);
        cnt += m >> 8;
    }
    outm[g * 64 + threadIdx.x] = (unsigned long long)e | (cnt << 8);
}

// assign entry / first token of the FAN children of every node (one thread per node)
template <typename T>
__global__ void dec_descend(const T* __restrict__ cmap, const Plan64* __restrict__ pl, long long div_child,
                            const uint8_t* __restrict__ pent, const unsigned long long* __restrict__ pbase,
                            uint8_t* __restrict__ cent, unsigned long long* __restrict__ cbase, long long npar_max,
                            int root, long long mstride) {
    const bool emaj = sizeof(T) == 4;           // chunk maps are entry-major
    const long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    const long long nchild = (pl->nchunks + div_child - 1) / div_child;
    if (g >= npar_max || g * FAN >= nchild) return;
    int e = root ? 0 : pent[g];
    unsigned long long k = root ? 0ull : pbase[g];
    const long long end = std::min(nchild, (g + 1) * FAN);
    for (long long i = g * FAN; i < end; i++) {
        cent[i] = (uint8_t)e;
        cbase[i] = k;
        const unsigned long long m = (unsigned long long)(emaj ? cmap[(long long)e * mstride + i] : cmap[i * 64 + e]);
        e = (int)(m & 63ull);
        k += m >> 8;
    }
}

// decode every chunk from its true entry; history kinds: 0 concrete, 1..3 incoming b1..b3, 4 derived
template <int CT>
__global__ __launch_bounds__(64) void dec_chunks(const uint32_t* __restrict__ W, const Plan64* __restrict__ pl, P64 P,
                                                 const uint8_t* __restrict__ cent,
                                                 const unsigned long long* __restrict__ cbase, double* __restrict__ out,
                                                 long long num, uint16_t* __restrict__ pend, uint8_t* __restrict__ thru,
                                                 unsigned* __restrict__ err) {
    __shared__ uint32_t S[SW];
#if DC64_RING
    __shared__ double RING[64 * 17];
#endif
    const long long g0 = blockIdx.x * 64ll;
    if (g0 >= pl->nchunks) return;
    stage_group(S, W, g0 * MAPW, pl->nwords + 4);
    __syncthreads();
    const long long c = g0 + threadIdx.x;
    if (c >= pl->nchunks) return;
    const long long avail = (long long)pl->nbits - g0 * CB;
    const uint32_t nb = (uint32_t)std::min(avail, (long long)(64 * CB + 64));
    const uint32_t cs = threadIdx.x * CB, ce = cs + CB;
    uint32_t p = cs + cent[c];
    const long long k0 = (long long)cbase[c];
#if DC64_RING
    double* ring = RING + threadIdx.x * 17;               // 16 doubles + 1 pad (2-way LDS conflicts)
#endif
    double f1 = -1.0, f2 = -1.0, f3 = -1.0;
    int q1 = c ? 1 : 0, q2 = c ? 2 : 0, q3 = c ? 3 : 0;
    int pd = 0;
    bool bad = false;
    long long j = 0;
    // outputs leave as whole 32-byte sectors (4 doubles, two 16-byte stores) from a 4-register buffer;
    // pending values are written too (dec_fix rewrites them) -- the partial head / tail sectors, shared
    // with the neighbouring chunks, element by element
    const bool al = (reinterpret_cast<uintptr_t>(out) & 31) == 0;
    double r0 = 0.0, r1 = 0.0, r2 = 0.0, r3 = 0.0;
    auto put = [&](long long i) {
        const int sl = (int)(i & 3);
        out[i] = sl == 0 ? r0 : sl == 1 ? r1 : sl == 2 ? r2 : r3;
    };
    while (p < ce && k0 + j < num) {
        const uint64_t win = peekS(S, p);
        const int l = tok_len<CT>(win, P);
        if (p + (uint32_t)l > nb) break;
        double v;
        int q = 0;
        if (CT != 6 && (win >> 63)) {
            const int code = (int)((win >> 61) & 3ull);
            if (code == 0) v = 0.0;
            else if (code == 1) { v = f1; q = q1; }
            else if (code == 2) { v = pred2(f1, f2); q = (q1 | q2) ? 4 : 0; }
            else { v = pred3(f1, f2, f3); q = (q1 | q2 | q3) ? 4 : 0; }
            if (c == 0 && j < 3 && code != 0) bad = true;                  // prediction against sentinels
        } else {
            v = tok_value<CT>(win, l, P);
        }
        if (q) pd = (int)j + 1;
        else bad |= d2u(v) == 0xBFF0000000000000ull;                       // the -1.0 history sentinel
        const long long g = k0 + j;
#if DC64_RING
        if (al) {
            ring[g & 15] = v;
            if ((g & 7) == 7) {
                if (g - 7 >= k0) {
                    const int b = (int)((g - 7) & 15);
                    double2* o2 = reinterpret_cast<double2*>(out + (g - 7));
                    o2[0] = make_double2(ring[b], ring[b + 1]);
                    o2[1] = make_double2(ring[b + 2], ring[b + 3]);
                    o2[2] = make_double2(ring[b + 4], ring[b + 5]);
                    o2[3] = make_double2(ring[b + 6], ring[b + 7]);
                } else {
                    for (long long i = k0; i <= g; i++) out[i] = ring[i & 15];
                }
            }
        } else if (!q) {
            out[g] = v;
        }
#else
        if (al) {
            const int sl = (int)(g & 3);
            r0 = sl == 0 ? v : r0; r1 = sl == 1 ? v : r1; r2 = sl == 2 ? v : r2; r3 = sl == 3 ? v : r3;
            if (sl == 3) {
                if (g - 3 >= k0) {
                    double2* o2 = reinterpret_cast<double2*>(out + (g - 3));
                    o2[0] = make_double2(r0, r1);
                    o2[1] = make_double2(r2, r3);
                } else {
                    for (long long i = k0; i <= g; i++) put(i);
                }
            }
        } else if (!q) {
            out[g] = v;
        }
#endif
        f3 = f2; q3 = q2; f2 = f1; q2 = q1; f1 = v; q1 = q;
        p += (uint32_t)l;
        j++;
    }
    if (al && j > 0) {                                                     // the partial last sector
        const long long gl = k0 + j - 1;
#if DC64_RING
        if ((gl & 7) != 7)
            for (long long i = std::max(k0, gl & ~7ll); i <= gl; i++) out[i] = ring[i & 15];
#else
        if ((gl & 3) != 3)
            for (long long i = std::max(k0, gl & ~3ll); i <= gl; i++) put(i);
#endif
    }
    pend[c] = (uint16_t)pd;
    thru[c] = (uint8_t)((q1 | q2 | q3) ? 1 : 0);
    if (c == pl->nchunks - 1 && k0 + j < num) bad = true;                 // fewer tokens than num
    if (bad) atomicOr(err, ERR_SERIAL);
}

template <int CT>
__device__ __forceinline__ bool redecode_prefix(const uint32_t* __restrict__ W, const P64& P, unsigned long long p, int pd,
                                                double* __restrict__ out, long long k0) {
    double g1 = out[k0 - 1], g2 = out[k0 - 2], g3 = out[k0 - 3];
    bool bad = false;
    for (int j = 0; j < pd; j++) {
        const uint64_t win = peek(W, p);
        const int l = tok_len<CT>(win, P);
        double v;
        if (CT != 6 && (win >> 63)) {
            const int code = (int)((win >> 61) & 3ull);
            v = code == 0 ? 0.0 : code == 1 ? g1 : code == 2 ? pred2(g1, g2) : pred3(g1, g2, g3);
        } else {
            v = tok_value<CT>(win, l, P);
        }
        out[k0 + j] = v;
        bad |= d2u(v) == 0xBFF0000000000000ull;
        g3 = g2; g2 = g1; g1 = v;
        p += (unsigned long long)l;
    }
    return bad;
}

// pending prefixes whose previous chunk ends with three concrete values
template <int CT>
__global__ __launch_bounds__(256) void dec_fix(const uint32_t* __restrict__ W, const Plan64* __restrict__ pl, P64 P,
                                               const uint8_t* __restrict__ cent, const unsigned long long* __restrict__ cbase,
                                               double* __restrict__ out, const uint16_t* __restrict__ pend,
                                               const uint8_t* __restrict__ thru, unsigned* __restrict__ err) {
    const long long c = blockIdx.x * 256ll + threadIdx.x;
    if (c <= 0 || c >= pl->nchunks || pend[c] == 0) return;
    if (thru[c - 1]) { atomicAdd(err + 1, 1u); return; }             // left to the ordered pass
    const long long k0 = (long long)cbase[c];
    if (k0 < 3) { atomicOr(err, ERR_SERIAL); return; }
    if (redecode_prefix<CT>(W, P, (unsigned long long)c * CB + cent[c], pend[c], out, k0)) atomicOr(err, ERR_SERIAL);
}

// chains crossing whole chunks, in stream order (one wave scans the flags 64 chunks at a time)
template <int CT>
__global__ __launch_bounds__(64) void dec_fix_serial(const uint32_t* __restrict__ W, const Plan64* __restrict__ pl, P64 P,
                                                     const uint8_t* __restrict__ cent,
                                                     const unsigned long long* __restrict__ cbase, double* __restrict__ out,
                                                     const uint16_t* __restrict__ pend, const uint8_t* __restrict__ thru,
                                                     unsigned* __restrict__ err) {
    const long long nc = pl->nchunks;
    if (err[1] == 0) return;                                         // no chain crosses a whole chunk
    for (long long b = 1; b < nc; b += 64) {
        const long long c = b + threadIdx.x;
        const bool need = c < nc && pend[c] != 0 && thru[c - 1];
        uint64_t bal = __ballot(need);
        if (threadIdx.x == 0) {
            while (bal) {
                const int i = __ffsll((unsigned long long)bal) - 1;
                bal &= bal - 1;
                const long long cc = b + i;
                const long long k0 = (long long)cbase[cc];
                if (k0 < 3) { atomicOr(err, ERR_SERIAL); continue; }
                if (redecode_prefix<CT>(W, P, (unsigned long long)cc * CB + cent[cc], pend[cc], out, k0))
                    atomicOr(err, ERR_SERIAL);
                __threadfence();
            }
        }
        __syncthreads();
    }
}

// exact serial decoder with the reference's history semantics (sentinel fill order :2722-2740)
template <int CT>
__global__ void dec_exact(const uint32_t* __restrict__ W, const Plan64* __restrict__ pl, P64 P, double* __restrict__ out,
                          long long num, const unsigned* __restrict__ err, unsigned long long* __restrict__ ndec) {
    if (threadIdx.x != 0 || blockIdx.x != 0 || !(*err & ERR_SERIAL)) return;
    const unsigned long long nb = pl->nbits;
    double b1 = -1.0, b2 = -1.0, b3 = -1.0;
    unsigned long long p = 0;
    long long n = 0;
    while (n < num && p < nb) {
        const uint64_t win = peek(W, p);
        const int l = tok_len<CT>(win, P);
        if (p + (unsigned long long)l > nb) break;
        double v;
        if (CT != 6 && (win >> 63)) {
            const int code = (int)((win >> 61) & 3ull);
            v = code == 0 ? 0.0 : code == 1 ? b1 : code == 2 ? pred2(b1, b2) : pred3(b1, b2, b3);
        } else {
            v = tok_value<CT>(win, l, P);
        }
        out[n++] = v;
        if (b3 == -1.0) b3 = v;
        else if (b2 == -1.0) b2 = v;
        else if (b1 == -1.0) b1 = v;
        else { b3 = b2; b2 = b1; b1 = v; }
        p += (unsigned long long)l;
    }
    *ndec = (unsigned long long)n;
}

// ---------------------------------------------------------------------------------------------- pre-passes
// toSmallDataset_double: the first minimum under '<' (NaN never replaces; x[0] NaN stays), then x - min
__global__ __launch_bounds__(256) void min_part(const double* __restrict__ x, long long n, double* __restrict__ pv,
                                                long long* __restrict__ pi) {
    __shared__ double sv[256];
    __shared__ long long si[256];
    double bv = 0.0;
    long long bi = -1;
    for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const double v = x[i];
        if (v == v && (bi < 0 || v < bv)) { bv = v; bi = i; }
    }
    sv[threadIdx.x] = bv; si[threadIdx.x] = bi;
    __syncthreads();
    for (int d = 128; d >= 1; d >>= 1) {
        if ((int)threadIdx.x < d) {
            const double ov = sv[threadIdx.x + d];
            const long long oi = si[threadIdx.x + d];
            const double mv = sv[threadIdx.x];
            const long long mi = si[threadIdx.x];
            if (oi >= 0 && (mi < 0 || ov < mv || (!(mv < ov) && oi < mi))) { sv[threadIdx.x] = ov; si[threadIdx.x] = oi; }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) { pv[blockIdx.x] = sv[0]; pi[blockIdx.x] = si[0]; }
}

__global__ void min_final(const double* __restrict__ x, const double* __restrict__ pv, const long long* __restrict__ pi,
                          int np, double* __restrict__ dmin) {
    if (threadIdx.x != 0) return;
    double bv = 0.0;
    long long bi = -1;
    for (int k = 0; k < np; k++) {
        const long long oi = pi[k];
        const double ov = pv[k];
        if (oi >= 0 && (bi < 0 || ov < bv || (!(bv < ov) && oi < bi))) { bv = ov; bi = oi; }
    }
    const double x0 = x[0];
    *dmin = (x0 != x0 || bi < 0) ? x0 : x[bi];
}

// a - b as the reference's x86 build computes it (SSE subsd): a NaN operand propagates quieted, the first one
// when both are, and an invalid result (inf - inf) is the default NaN 0xFFF8000000000000
__device__ __forceinline__ double sub_x86(double a, double b) {
    const unsigned long long q = 0x0008000000000000ull;
    if (__builtin_expect(a != a, 0)) return __longlong_as_double((long long)((unsigned long long)__double_as_longlong(a) | q));
    if (__builtin_expect(b != b, 0)) return __longlong_as_double((long long)((unsigned long long)__double_as_longlong(b) | q));
    const double r = __dsub_rn(a, b);
    return r != r ? __longlong_as_double((long long)0xFFF8000000000000ull) : r;
}
__global__ void sub_min(const double* __restrict__ x, long long n, const double* __restrict__ dmin, double* __restrict__ y) {
    const double m = *dmin;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        y[i] = sub_x86(x[i], m);
}

}  // namespace dc64

// ================================================================================================ host
using namespace dc64;

extern "C" int dc_set_error(int code, const char* msg);

namespace {
struct Ctx64 {
    // encoder
    uint32_t* tbits = nullptr; unsigned long long* toff = nullptr; unsigned long long* psum = nullptr;
    long long enc_cap = 0;
    unsigned long long* d_total = nullptr; unsigned* d_err = nullptr;
    // decoder
    void* pool = nullptr; size_t pool_cap = 0;
    Plan64* plan = nullptr;
    unsigned long long* h = nullptr;        // pinned: [0] total bits [1] err [2] ndec
    // pre-passes
    double* pv = nullptr; long long* pi = nullptr; double* d_f = nullptr; int* d_i = nullptr;
    void* med_scr = nullptr; size_t med_cap = 0;          // exact mean scratch (dc_med_scratch_bytes64)
    int dec_pending = 0, dec_ct = 0, map_fallback = 0;
    long long dbg_words = 0, dbg_chunks = 0;
    unsigned* ctr = nullptr;
    long long dec_num = 0;
};
Ctx64 C64;

#define H64(call)                                                                  \
    do {                                                                           \
        hipError_t e_ = (call);                                                    \
        if (e_ != hipSuccess) return dc_set_error(DC_ERR_HIP, hipGetErrorString(e_)); \
    } while (0)

int ensure64(hipStream_t* st) {
    int rc = dc_init(0);                        // no-op once the library is initialised
    if (rc) return rc;
    *st = (hipStream_t)dc_get_stream();
    if (!C64.d_total) {
        H64(hipMalloc((void**)&C64.d_total, 64));
        H64(hipMalloc((void**)&C64.d_err, 64));
        H64(hipMalloc((void**)&C64.plan, sizeof(Plan64)));
        H64(hipHostMalloc((void**)&C64.h, 8 * sizeof(unsigned long long), 0));
        H64(hipMalloc((void**)&C64.pv, 1024 * sizeof(double)));
        H64(hipMalloc((void**)&C64.pi, 1024 * sizeof(long long)));
        H64(hipMalloc((void**)&C64.d_f, 64));
        H64(hipMalloc((void**)&C64.d_i, 64));
        H64(hipMalloc((void**)&C64.ctr, 64));
    }
    return DC_OK;
}

int bound_binary(double bound) {                           // to_absErrorBound_binary :5512
    for (int n = 0; n < 100; n++) if (bound >= ldexp(1.0, -n)) return n;
    return 100;
}

int make_p64(P64* P, int ct, int type, uint32_t mask20) {
    if (!(ct == 5 || ct == 6 || ct == 7 || ct == 11)) return dc_set_error(DC_ERR_ARG, "double codec: ct must be 5, 6, 7 or 11");
    if (ct == 7 && (type < 1 || type > 10)) return dc_set_error(DC_ERR_ARG, "double CT7: type must be 1..10");
    P->ct = ct;
    P->bound = dc_get_abs_error_bound();
    P->B = bound_binary(P->bound);
    P->type = ct == 7 ? type : 1;
    P->mask20 = mask20 & 0xFFFFFu;
    const int E = (int)((mask20 >> 8) & 0x7FF);
    P->mm = std::min(std::max(P->B + E - 1023, 0), 52);
    P->mm0 = P->mm > 8 ? P->mm - 8 : 0;
    return DC_OK;
}
}  // namespace

#define DISPATCH64(CTV, KER, ...)                                      \
    switch (CTV) {                                                     \
        case 5: hipLaunchKernelGGL(KER<5>, __VA_ARGS__); break;        \
        case 6: hipLaunchKernelGGL(KER<6>, __VA_ARGS__); break;        \
        case 7: hipLaunchKernelGGL(KER<7>, __VA_ARGS__); break;        \
        default: hipLaunchKernelGGL(KER<11>, __VA_ARGS__); break;      \
    }

extern "C" size_t dc64_stream_capacity(long long n) { return (size_t)((n * 64 + 7 + 31) / 32) * 4 + 64; }

extern "C" int dc64_encode_device(int ct, const void* d_x, long long n, int type, uint32_t mask20, int start_bit,
                                  void* d_out, unsigned long long* d_total_bits) {
    hipStream_t st;
    int rc = ensure64(&st);
    if (rc) return rc;
    P64 P;
    if ((rc = make_p64(&P, ct, type, mask20))) return rc;
    if (n < 0 || start_bit < 0 || start_bit > 7) return dc_set_error(DC_ERR_ARG, "dc64_encode_device: bad n / start_bit");
    unsigned long long* tot = d_total_bits ? d_total_bits : C64.d_total;
    if (n == 0) { H64(hipMemsetAsync(tot, 0, 8, st)); if (tot != C64.d_total) H64(hipMemsetAsync(C64.d_total, 0, 8, st)); return DC_OK; }
    const long long nt = (n + ETILE - 1) / ETILE;
    if (nt > C64.enc_cap) {
        if (C64.tbits) { (void)hipFree(C64.tbits); (void)hipFree(C64.toff); }
        H64(hipMalloc((void**)&C64.tbits, (size_t)nt * 4));
        H64(hipMalloc((void**)&C64.toff, (size_t)nt * 8));
        if (C64.psum) (void)hipFree(C64.psum);
        H64(hipMalloc((void**)&C64.psum, (size_t)((nt + 1023) / 1024 + 2) * 8));
        C64.enc_cap = nt;
    }
    const double* x = (const double*)d_x;
    uint32_t* out = (uint32_t*)d_out;
    H64(hipMemsetAsync(C64.d_err, 0, 4, st));
    DISPATCH64(ct, enc_count, dim3((unsigned)nt), dim3(ETPB), 0, st, x, n, P, C64.tbits, C64.d_err);
    if (nt <= 4096) {
        hipLaunchKernelGGL(enc_scan, dim3(1), dim3(1024), 0, st, C64.tbits, nt, start_bit, C64.toff, out, tot);
    } else {
        const long long nb = (nt + 1023) / 1024;
        hipLaunchKernelGGL(enc_scan_part, dim3((unsigned)nb), dim3(1024), 0, st, C64.tbits, nt, C64.toff, C64.psum);
        hipLaunchKernelGGL(scan_top, dim3(1), dim3(1024), 0, st, C64.psum, nb);
        hipLaunchKernelGGL(enc_scan_add, dim3((unsigned)nb), dim3(1024), 0, st, nt, start_bit, C64.psum, C64.toff, out, tot);
    }
    DISPATCH64(ct, enc_write, dim3((unsigned)nt), dim3(ETPB), 0, st, x, n, P, C64.toff, out);
    DISPATCH64(ct, enc_serial, dim3(1), dim3(64), 0, st, x, n, P, start_bit, (uint8_t*)d_out, tot, C64.d_err);
    if (tot != C64.d_total) H64(hipMemcpyAsync(C64.d_total, tot, 8, hipMemcpyDeviceToDevice, st));
    H64(hipGetLastError());
    return DC_OK;
}

extern "C" int dc64_encode_result(unsigned long long* total_bits) {
    hipStream_t st;
    int rc = ensure64(&st);
    if (rc) return rc;
    H64(hipMemcpyAsync(C64.h, C64.d_total, 8, hipMemcpyDeviceToHost, st));
    H64(hipStreamSynchronize(st));
    *total_bits = C64.h[0];
    return DC_OK;
}

// decoder scratch for up to max_chunks chunks: staged words, chunk maps, composed levels, entries
namespace {
struct DecLayout {
    int nlev;                       // levels above the chunks (the last one has a single node)
    long long nnode[8];             // max nodes per level (0 = chunks)
    size_t off_w, off_map, off_lmap[8], off_ent[8], off_base[8], off_sx, off_sn, off_bad, off_list, off_psum, off_pend, off_thru, total;
};
DecLayout layout(long long max_words, long long max_chunks) {
    DecLayout Lo{};
    size_t o = 0;
    auto take = [&](size_t b) { size_t r = o; o += (b + 255) & ~(size_t)255; return r; };
    Lo.off_w = take((size_t)(max_words + 8) * 4);
    Lo.off_map = take((size_t)max_chunks * 64 * 4);
    Lo.nnode[0] = max_chunks;
    int l = 0;
    while (true) {
        Lo.off_ent[l] = take((size_t)Lo.nnode[l]);
        Lo.off_base[l] = take((size_t)Lo.nnode[l] * 8);
        if (Lo.nnode[l] <= 1 && l > 0) break;
        l++;
        Lo.nnode[l] = (Lo.nnode[l - 1] + FAN - 1) / FAN;
        Lo.off_lmap[l] = take((size_t)Lo.nnode[l] * 64 * 8);
        if (l == 7) break;
    }
    Lo.nlev = l;
    Lo.off_sx = take((size_t)max_chunks);
    Lo.off_sn = take((size_t)max_chunks * 2);
    Lo.off_bad = take((size_t)max_chunks);
    Lo.off_list = take((size_t)max_chunks * 4);
    Lo.off_psum = take((size_t)((max_chunks + 1023) / 1024 + 1) * 8);
    Lo.off_pend = take((size_t)max_chunks * 2);
    Lo.off_thru = take((size_t)max_chunks);
    Lo.total = o;
    return Lo;
}
}  // namespace

extern "C" int dc64_decode_device(int ct, const void* d_stream, long long nbytes, const unsigned long long* d_nbits,
                                  long long max_bytes, long long num, int type, uint32_t mask20, void* d_out) {
    hipStream_t st;
    int rc = ensure64(&st);
    if (rc) return rc;
    P64 P;
    if ((rc = make_p64(&P, ct, type, mask20))) return rc;
    if (num <= 0) return DC_OK;
    if (max_bytes < 0) max_bytes = nbytes;
    if (max_bytes <= 0) return dc_set_error(DC_ERR_ARG, "dc64_decode_device: empty stream for num > 0");
    const long long max_words = (max_bytes + 3) / 4 + 4;
    const long long max_chunks = (max_bytes * 8 + CB - 1) / CB;
    if (max_chunks > (1ll << 36)) return dc_set_error(DC_ERR_ARG, "stream too large");
    const DecLayout Lo = layout(max_words, max_chunks);
    C64.dbg_words = max_words;
    C64.dbg_chunks = max_chunks;
    if (Lo.total > C64.pool_cap) {
        if (C64.pool) (void)hipFree(C64.pool);
        C64.pool = nullptr; C64.pool_cap = 0;
        H64(hipMalloc(&C64.pool, Lo.total));
        C64.pool_cap = Lo.total;
    }
    char* base = (char*)C64.pool;
    uint32_t* W = (uint32_t*)(base + Lo.off_w);
    uint32_t* map = (uint32_t*)(base + Lo.off_map);
    uint16_t* pend = (uint16_t*)(base + Lo.off_pend);
    uint8_t* thru = (uint8_t*)(base + Lo.off_thru);
    double* out = (double*)d_out;
    H64(hipMemsetAsync(C64.d_err, 0, 8, st));
    hipLaunchKernelGGL(dec_plan, dim3(1), dim3(1), 0, st, C64.plan, d_nbits, (unsigned long long)nbytes * 8ull, max_chunks,
                       C64.d_err);
    hipLaunchKernelGGL(dec_stage, dim3((unsigned)std::min<long long>((max_words + 255) / 256, 4096)), dim3(256), 0, st,
                       (const uint8_t*)d_stream, C64.plan, W, max_words + 8);
    uint8_t* se = (uint8_t*)(base + Lo.off_ent[0]);
    uint8_t* sx = (uint8_t*)(base + Lo.off_sx);
    uint16_t* sn = (uint16_t*)(base + Lo.off_sn);
    uint8_t* bad = (uint8_t*)(base + Lo.off_bad);
    unsigned* list = (unsigned*)(base + Lo.off_list);
    unsigned long long* cb0 = (unsigned long long*)(base + Lo.off_base[0]);
    const unsigned g64 = (unsigned)((max_chunks + 63) / 64), g256 = (unsigned)((max_chunks + 255) / 256);
    const unsigned g1k = (unsigned)((max_chunks + 1023) / 1024);
    constexpr int ROUNDS = 4;
    H64(hipMemsetAsync(C64.ctr, 0, sizeof(unsigned) * (ROUNDS + 1), st));
    DISPATCH64(ct, dec_spec, dim3(g64), dim3(64), 0, st, W, C64.plan, P, se, sx, sn);
    for (int r = 0; r <= ROUNDS; r++) {
        hipLaunchKernelGGL(dec_links, dim3(g256), dim3(256), 0, st, C64.plan, se, sx, bad, C64.ctr + r, list);
        if (r < ROUNDS) DISPATCH64(ct, dec_relink, dim3(1024), dim3(64), 0, st, W, C64.plan, P, se, sx, sn, bad, C64.ctr + r,
                                   list);
    }
    H64(hipMemcpyAsync(C64.h + 6, C64.ctr + ROUNDS, 4, hipMemcpyDeviceToHost, st));
    H64(hipStreamSynchronize(st));
    const char* force = getenv("DC64_FORCE_MAP");                  // tests: exercise the chunk-map path
    const unsigned broken = (unsigned)C64.h[6] + ((force && *force == '1') ? 1u : 0u);
    C64.map_fallback = broken != 0;
    if (!broken) {
        unsigned long long* psum = (unsigned long long*)(base + Lo.off_psum);
        hipLaunchKernelGGL(cnt_scan_part, dim3(g1k), dim3(1024), 0, st, C64.plan, sn, cb0, psum);
        hipLaunchKernelGGL(cnt_scan_top, dim3(1), dim3(1024), 0, st, C64.plan, psum);
        hipLaunchKernelGGL(cnt_scan_add, dim3(g1k), dim3(1024), 0, st, C64.plan, psum, cb0);
    } else {
    DISPATCH64(ct, dec_map, dim3((unsigned)((max_chunks + 63) / 64)), dim3(64), 0, st, W, C64.plan, P, map, max_chunks);
    // compose upwards: level l nodes cover FAN^l chunks
    long long div = 1;
    for (int l = 1; l <= Lo.nlev; l++) {
        unsigned long long* lm = (unsigned long long*)(base + Lo.off_lmap[l]);
        if (l == 1)
            hipLaunchKernelGGL(dec_compose<uint32_t>, dim3((unsigned)Lo.nnode[l]), dim3(64), 0, st, map, Lo.nnode[0],
                               C64.plan, div, lm);
        else
            hipLaunchKernelGGL(dec_compose<unsigned long long>, dim3((unsigned)Lo.nnode[l]), dim3(64), 0, st,
                               (const unsigned long long*)(base + Lo.off_lmap[l - 1]), Lo.nnode[l - 1], C64.plan, div, lm);
        div *= FAN;
    }
    // descend from the root (level nlev, one node: entry 0, token 0)
    for (int l = Lo.nlev; l >= 1; l--) {
        div /= FAN;                                           // FAN^(l-1): chunks per child node
        uint8_t* pent = (uint8_t*)(base + Lo.off_ent[l]);
        unsigned long long* pbase = (unsigned long long*)(base + Lo.off_base[l]);
        uint8_t* cent = (uint8_t*)(base + Lo.off_ent[l - 1]);
        unsigned long long* cbase = (unsigned long long*)(base + Lo.off_base[l - 1]);
        const unsigned g = (unsigned)((Lo.nnode[l] + 63) / 64);
        if (l == 1)
            hipLaunchKernelGGL(dec_descend<uint32_t>, dim3(g), dim3(64), 0, st, map, C64.plan, div, pent, pbase, cent,
                               cbase, Lo.nnode[l], l == Lo.nlev ? 1 : 0, max_chunks);
        else
            hipLaunchKernelGGL(dec_descend<unsigned long long>, dim3(g), dim3(64), 0, st,
                               (const unsigned long long*)(base + Lo.off_lmap[l - 1]), C64.plan, div, pent, pbase, cent,
                               cbase, Lo.nnode[l], l == Lo.nlev ? 1 : 0, max_chunks);
    }
    }
    const uint8_t* cent = (const uint8_t*)(base + Lo.off_ent[0]);
    const unsigned long long* cbase = (const unsigned long long*)(base + Lo.off_base[0]);
    const unsigned gc = (unsigned)((max_chunks + 255) / 256);
    DISPATCH64(ct, dec_chunks, dim3((unsigned)((max_chunks + 63) / 64)), dim3(64), 0, st, W, C64.plan, P, cent, cbase, out, num, pend, thru, C64.d_err);
    DISPATCH64(ct, dec_fix, dim3(gc), dim3(256), 0, st, W, C64.plan, P, cent, cbase, out, pend, thru, C64.d_err);
    DISPATCH64(ct, dec_fix_serial, dim3(1), dim3(64), 0, st, W, C64.plan, P, cent, cbase, out, pend, thru, C64.d_err);
    H64(hipMemsetAsync(C64.d_total + 1, 0xFF, 8, st));
    DISPATCH64(ct, dec_exact, dim3(1), dim3(64), 0, st, W, C64.plan, P, out, num, C64.d_err, C64.d_total + 1);
    H64(hipGetLastError());
    C64.dec_pending = 1;
    C64.dec_ct = ct;
    C64.dec_num = num;
    return DC_OK;
}

// wait for the last decode; DC_ERR_STREAM if the stream held fewer than num tokens
extern "C" int dc64_decode_finish(void) {
    hipStream_t st;
    int rc = ensure64(&st);
    if (rc) return rc;
    if (!C64.dec_pending) return DC_OK;
    C64.dec_pending = 0;
    H64(hipMemcpyAsync(C64.h + 1, C64.d_err, 4, hipMemcpyDeviceToHost, st));
    H64(hipMemcpyAsync(C64.h + 2, C64.d_total + 1, 8, hipMemcpyDeviceToHost, st));
    H64(hipStreamSynchronize(st));
    const unsigned err = (unsigned)C64.h[1];
    if ((err & ERR_SERIAL) && C64.h[2] != ~0ull && (long long)C64.h[2] < C64.dec_num)
        return dc_set_error(DC_ERR_STREAM, "double decode: stream holds fewer tokens than num");
    return DC_OK;
}

// debug: the last decode's chunk records (entry, exit, count, first token) -> host arrays
extern "C" long long dc64_debug_chunks(uint8_t* e, uint8_t* x, uint16_t* n, unsigned long long* b, long long cap) {
    hipStream_t st;
    if (ensure64(&st)) return -1;
    Plan64 pl;
    if (hipMemcpy(&pl, C64.plan, sizeof pl, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    const long long nc = std::min(pl.nchunks, cap);
    const DecLayout Lo = layout(C64.dbg_words, C64.dbg_chunks);
    char* base = (char*)C64.pool;
    (void)hipMemcpy(e, base + Lo.off_ent[0], nc, hipMemcpyDeviceToHost);
    (void)hipMemcpy(x, base + Lo.off_sx, nc, hipMemcpyDeviceToHost);
    (void)hipMemcpy(n, base + Lo.off_sn, nc * 2, hipMemcpyDeviceToHost);
    (void)hipMemcpy(b, base + Lo.off_base[0], nc * 8, hipMemcpyDeviceToHost);
    return nc;
}

extern "C" int dc64_debug_ctr(unsigned* out) {
    return hipMemcpy(out, C64.ctr, 5 * sizeof(unsigned), hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}

// bit 0: the exact serial decoder ran; bit 1: speculative entries failed, the chunk-map path ran
extern "C" unsigned dc64_last_decode_flags(void) {
    return (C64.h ? ((unsigned)C64.h[1] & ERR_SERIAL) : 0u) | (C64.map_fallback ? 2u : 0u);
}

extern "C" int dc64_to_small_device(const void* d_x, long long n, void* d_out, double* min_out) {
    hipStream_t st;
    int rc = ensure64(&st);
    if (rc) return rc;
    if (n <= 0) return dc_set_error(DC_ERR_ARG, "dc64_to_small_device: n must be > 0");
    const double* x = (const double*)d_x;
    const int np = (int)std::min<long long>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(min_part, dim3(np), dim3(256), 0, st, x, n, C64.pv, C64.pi);
    hipLaunchKernelGGL(min_final, dim3(1), dim3(64), 0, st, x, C64.pv, C64.pi, np, C64.d_f);
    hipLaunchKernelGGL(sub_min, dim3((unsigned)std::min<long long>((n + 255) / 256, 8192)), dim3(256), 0, st, x, n,
                       C64.d_f, (double*)d_out);
    H64(hipGetLastError());
    if (min_out) {
        H64(hipMemcpyAsync(C64.h + 3, C64.d_f, 8, hipMemcpyDeviceToHost, st));
        H64(hipStreamSynchronize(st));
        memcpy(min_out, C64.h + 3, 8);
    }
    return DC_OK;
}

extern "C" int dc_launch_med64(const double* x, long long n, void* scratch, double* d_mean, int* d_type, int wide,
                               hipStream_t st);
extern "C" unsigned* dc_med_flag_ptr(void* scratch, long long n, int is_double);
extern "C" long long dc_med_scratch_bytes64(long long n);

// med_dataset_double (:3564-3590): the exact left-to-right double sum by the binade-transducer kernels of
// dc_aux.hip (every CU; the binade crossings one lane at a time)
extern "C" int dc64_med_device(const void* d_x, long long n, double* mean_out, int* type_out) {
    hipStream_t st;
    int rc = ensure64(&st);
    if (rc) return rc;
    if (n <= 0) return dc_set_error(DC_ERR_ARG, "dc64_med_device: n must be > 0");
    const size_t need = (size_t)dc_med_scratch_bytes64(n);
    if (C64.med_cap < need) {
        if (C64.med_scr) H64(hipFree(C64.med_scr));
        C64.med_scr = nullptr;
        C64.med_cap = 0;
        H64(hipMalloc(&C64.med_scr, need + need / 8));
        C64.med_cap = need + need / 8;
    }
    for (int wide = 0; wide < 2; wide++) {                // the narrow binade window, then the wide one if it missed
        if (dc_launch_med64((const double*)d_x, n, C64.med_scr, C64.d_f + 1, C64.d_i, wide, st))
            return dc_set_error(DC_ERR_HIP, "dc64_med_device: launch failed");
        // flag, then mean, type (MedScratch.res): one copy
        H64(hipMemcpyAsync(C64.h + 4, dc_med_flag_ptr(C64.med_scr, n, 1), 3 * 8, hipMemcpyDeviceToHost, st));
        H64(hipStreamSynchronize(st));
        if (!(uint32_t)C64.h[4] || wide) break;
    }
    if (mean_out) memcpy(mean_out, C64.h + 5, 8);
    if (type_out) *type_out = (int)(uint32_t)C64.h[6];
    return DC_OK;
}
