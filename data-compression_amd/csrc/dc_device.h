// dc_device.h -- device-side building blocks shared by the gfx950 kernels.
//
// Token grammar (reference impl/dataCompression.c):
//   '100' zero, '101'/'110'/'111' predicted (:3390-3437), raw = top 9+m bits of the pattern
//   (compress_bitwise_float :3479-3520), CT7 masked tokens (compress_bitwise_float_mask :2143-2284),
//   CT11 verbatim 32 bits (:602-605).  Bits are MSB-first in the byte stream (add_bit_to_bytes :5456).
// All float arithmetic uses explicit round-to-nearest intrinsics so no FMA contraction can change a
// predictor (the reference is built by gcc for x86-64 SSE, where it cannot contract).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "dc_shared.h"

namespace dc {

// decoder geometry: a chunk is the unit one lane parses; a group (tile) is one workgroup's chunks
// (a second build of the decoder objects uses 256-bit chunks for small streams: Makefile SMALLDEFS)
#ifndef DC_CHUNK_BITS
#define DC_CHUNK_BITS 1024
#endif
constexpr int CHUNK_BITS = DC_CHUNK_BITS;
constexpr int GROUP = 256;



__device__ __forceinline__ int mbits(int B, uint32_t E) {
    int m = B + (int)E - 127;
    return m > 23 ? 23 : (m < 0 ? 0 : m);
}

// ------------------------------------------------------------------------------------------------
// Encoder: token for one element.  b1..b3 are the ORIGINAL previous inputs (encoder history).
template <int CT>
__device__ __forceinline__ void make_token(float x, float b1, float b2, float b3, bool predict,
                                           const Params& P, uint32_t& val, int& len) {
    const uint32_t u = __float_as_uint(x);
    if (CT != 6) {
        if (fabsf(x) <= P.thr_lt) { val = 4u; len = 3; return; }              // '100'
        if (predict) {
            const float p1 = b1;
            const float p2 = __fsub_rn(__fmul_rn(2.0f, b1), b2);
            const float p3 = __fadd_rn(__fsub_rn(__fmul_rn(3.0f, b1), __fmul_rn(3.0f, b2)), b3);
            const float d1 = fabsf(__fsub_rn(p1, x));
            const float d2 = fabsf(__fsub_rn(p2, x));
            const float d3 = fabsf(__fsub_rn(p3, x));
            float dmin = d1; uint32_t code = 5u;
            if (d2 < dmin) { dmin = d2; code = 6u; }
            if (d3 < dmin) { dmin = d3; code = 7u; }
            if (dmin <= P.thr_le) { val = code; len = 3; return; }
        }
    }
    if (CT == 11) { val = u; len = 32; return; }
    const int m = mbits(P.B, (u >> 23) & 0xFFu);
    const uint32_t top = u >> (23 - m);                                       // 9+m bits
    if (CT == 7 && (u >> 23) == (P.mask17 >> 8)) {
        const uint32_t head = ((1u << P.type) - 1u) << 1;
        if (((u >> 15) & 0xFFu) == (P.mask17 & 0xFFu)) {                      // flag 0
            const int tl = m > 8 ? m - 8 : 0;
            val = (head << tl) | (top & ((1u << tl) - 1u));
            len = P.type + 2 + tl;
        } else {                                                              // flag 1
            val = ((head | 1u) << m) | (top & ((1u << m) - 1u));
            len = P.type + 2 + m;
        }
        return;
    }
    val = top; len = 9 + m;
}

// Branch-free form of make_token (selects only; same tokens).  For a CT7 masked token the exponent
// equals the mask's, so its mantissa bit count is the uniform P.mm and its value is a bit-select of
// the raw top bits with uniform constants.  The predicted code is the first strict minimum of
// (d1, d2, d3); "some prediction within threshold" is min(d1, d2, d3) <= thr_le with a NaN d1
// never predicting (token_len_enc below has the argument).
template <int CT>
__device__ __forceinline__ void make_token_bf(float x, float b1, float b2, float b3, bool predict, const Params& P,
                                              uint32_t& val, int& len) {
    const uint32_t u = __float_as_uint(x);
    int l = CT == 11 ? 32 : min(max((int)((u >> 23) & 0xFFu) + P.rawadd, 9), 32);   // 9 + m
    uint32_t v = CT == 11 ? u : (u >> (32 - l));                                     // top 9 + m bits
    if (CT == 7) {
        const bool msk = (u >> 23) == (P.mask17 >> 8);
        const bool f1 = ((u >> 15) & 0xFFu) != (P.mask17 & 0xFFu);
        const uint32_t vm = f1 ? ((v & P.em1) | P.eh1) : ((v & P.em0) | P.eh0);
        l = msk ? P.lm0 + (f1 ? P.dlm : 0) : l;
        v = msk ? vm : v;
    }
    if (CT != 6) {
        const float p2 = __fsub_rn(__fmul_rn(2.0f, b1), b2);
        const float p3 = __fadd_rn(__fsub_rn(__fmul_rn(3.0f, b1), __fmul_rn(3.0f, b2)), b3);
        const float d1 = fabsf(__fsub_rn(b1, x));
        const float d2 = fabsf(__fsub_rn(p2, x));
        const float d3 = fabsf(__fsub_rn(p3, x));
        const float d12 = fminf(d1, d2);
        const bool c2 = d2 < d1, c3 = d3 < d12;
        const uint32_t code = c3 ? 7u : (c2 ? 6u : 5u);
        const bool pr = predict && d1 == d1 && fminf(d12, d3) <= P.thr_le;
        const bool z = fabsf(x) <= P.thr_lt;
        const bool s3 = pr || z;
        v = s3 ? (z ? 4u : code) : v;
        l = s3 ? 3 : l;
    }
    val = v;
    len = l;
}

// ------------------------------------------------------------------------------------------------
// Encoder token table (per workgroup, LDS, 1 KB): a raw token's length and bit extraction depend only on
// the float's top 9 bits (sign + exponent), so tab[u >> 23] = sh | len << 8 gives v = u >> sh (the top
// len = 9 + m bits) and len (for CT7's masked exponent len = lm1, the flag-1 length; sh stays 32 - (9 + mm)).
// A CT7 masked token is v ^ K1 (flag 1) or v ^ K0 with length lm0 (flag 0: (u >> 15) == mask17).  The same
// tokens as make_token / make_token_bf with ~10 fewer VALU per float.
template <int CT>
__device__ __forceinline__ void build_enc_tab(uint16_t* tab, const Params& P, int tid, int nthr) {
    for (int i = tid; i < 512; i += nthr) {
        const int l9 = min(max((i & 0xFF) + P.rawadd, 9), 32);   // the bits v keeps: 9 + m
        const int len = (CT == 7 && (uint32_t)i == (P.mask17 >> 8)) ? P.lm1 : l9;
        tab[i] = (uint16_t)((uint32_t)(32 - l9) | ((uint32_t)len << 8));
    }
}

// a token from the table; b1..b3 the ORIGINAL previous inputs.  The predicted code ('101'/'110'/'111') is
// chosen under a wave-uniform branch, when some lane predicts (rare in ordinary data).
template <int CT>
__device__ __forceinline__ void make_token_t(float x, float b1, float b2, float b3, bool predict, const Params& P,
                                             const uint16_t* tab, uint32_t& val, int& len) {
    const uint32_t u = __float_as_uint(x);
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
        const float p2 = __fsub_rn(__fmul_rn(2.0f, b1), b2);
        const float p3 = __fadd_rn(__fsub_rn(__fmul_rn(3.0f, b1), __fmul_rn(3.0f, b2)), b3);
        const float d1 = fabsf(__fsub_rn(b1, x));
        const float d2 = fabsf(__fsub_rn(p2, x));
        const float d3 = fabsf(__fsub_rn(p3, x));
        const bool pr = predict && d1 == d1 && fminf(fminf(d1, d2), d3) <= P.thr_le;
        const bool z = fabsf(x) <= P.thr_lt;
        if (__builtin_expect(__any(pr), 0)) {
            const float d12 = fminf(d1, d2);
            const uint32_t code = d3 < d12 ? 7u : (d2 < d1 ? 6u : 5u);
            v = pr ? code : v;
        }
        v = z ? 4u : v;
        l = (pr || z) ? 3 : l;
    }
    val = v;
    len = l;
}

// the length only (count pass)
template <int CT>
__device__ __forceinline__ int token_len_t(float x, float b1, float b2, float b3, bool predict, const Params& P,
                                           const uint16_t* tab) {
    const uint32_t u = __float_as_uint(x);
    int l;
    if (CT == 11) {
        l = 32;
    } else {
        l = (int)((uint32_t)tab[u >> 23] >> 8);
        if (CT == 7) l = (u >> 15) == P.mask17 ? P.lm0 : l;
    }
    if (CT != 6) {
        const float p2 = __fsub_rn(__fmul_rn(2.0f, b1), b2);
        const float p3 = __fadd_rn(__fsub_rn(__fmul_rn(3.0f, b1), __fmul_rn(3.0f, b2)), b3);
        const float d1 = fabsf(__fsub_rn(b1, x));
        const float dmin = fminf(fminf(d1, fabsf(__fsub_rn(p2, x))), fabsf(__fsub_rn(p3, x)));
        const bool pr = predict && d1 == d1 && dmin <= P.thr_le;
        l = (pr || fabsf(x) <= P.thr_lt) ? 3 : l;
    }
    return l;
}

// Encoder: token LENGTH only (count pass).  Same decision as make_token_bf: the predicted code is
// the first strict minimum of (d1, d2, d3), so "some prediction within threshold" is
// min(d1, d2, d3) <= thr_le, where a NaN d1 keeps dmin = NaN (never predicts) and NaN d2 / d3 are
// skipped -- exactly IEEE minNum's treatment of the second and third operands.
template <int CT>
__device__ __forceinline__ int token_len_enc(float x, float b1, float b2, float b3, bool predict, const Params& P) {
    const uint32_t u = __float_as_uint(x);
    int l = CT == 11 ? 32 : min(max((int)((u >> 23) & 0xFFu) + P.rawadd, 9), 32);
    if (CT == 7) {
        const bool msk = (u >> 23) == (P.mask17 >> 8);
        const bool f1 = ((u >> 15) & 0xFFu) != (P.mask17 & 0xFFu);
        l = msk ? P.lm0 + (f1 ? P.dlm : 0) : l;
    }
    if (CT != 6) {
        const float p2 = __fsub_rn(__fmul_rn(2.0f, b1), b2);
        const float p3 = __fadd_rn(__fsub_rn(__fmul_rn(3.0f, b1), __fmul_rn(3.0f, b2)), b3);
        const float d1 = fabsf(__fsub_rn(b1, x));
        const float dmin = fminf(fminf(d1, fabsf(__fsub_rn(p2, x))), fabsf(__fsub_rn(p3, x)));
        const bool pr = predict && d1 == d1 && dmin <= P.thr_le;
        l = (pr || fabsf(x) <= P.thr_lt) ? 3 : l;
    }
    return l;
}

// ------------------------------------------------------------------------------------------------
// Decoder: token length from the next 32 stream bits (MSB-aligned).  At most 10 bits decide it.
template <int CT>
__device__ __forceinline__ int token_len(uint32_t t, const Params& P) {
    if (CT == 6) return 9 + mbits(P.B, (t >> 23) & 0xFFu);
    if (t >> 31) return 3;
    if (CT == 11) return 32;
    if (CT == 7) {
        const uint32_t ones = (1u << P.type) - 1u;
        if (((t >> (31 - P.type)) & ones) == ones)
            return P.type + 2 + (((t >> (30 - P.type)) & 1u) ? P.mm : P.mm0);
    }
    return 9 + mbits(P.B, (t >> 23) & 0xFFu);
}

// Value of a non-predicted token (zero / raw / masked / verbatim) from its MSB-aligned bits.
// Predicted codes return code 1..3 in *code (101 -> 1, 110 -> 2, 111 -> 3), 0 otherwise.
template <int CT>
__device__ __forceinline__ uint32_t token_pattern(uint32_t t, int len, const Params& P, int* code) {
    *code = 0;
    if (CT != 6 && (t >> 31)) {                                               // 3-bit code
        const uint32_t c = (t >> 29) & 3u;
        *code = (int)c;
        return 0u;                                                            // '100' -> 0.0f
    }
    if (CT == 11) return t;                                                   // verbatim
    if (CT == 7) {
        const uint32_t ones = (1u << P.type) - 1u;
        if (((t >> (31 - P.type)) & ones) == ones) {
            const int hl = P.type + 2;
            const uint32_t rest = t << hl;                                    // bits after the head
            if (((t >> (30 - P.type)) & 1u) == 0u) {                          // flag 0 (:1947-1961)
                const int tl = P.mm0;
                uint32_t u = P.mask17 << 15;
                if (tl > 0) u |= (rest >> (32 - tl)) << (15 - tl);
                if (tl < 15) u |= 1u << (14 - tl);
                return u;
            } else {                                                          // flag 1 (:1963-2010)
                const int tl = P.mm;
                uint32_t u = (P.mask17 >> 8) << 23;
                if (tl > 0) u |= (rest >> (32 - tl)) << (23 - tl);
                if (tl < 23) u |= 1u << (22 - tl);
                return u;
            }
        }
    }
    // raw: top len bits + midpoint bit (decompress_bitwise_float :3166-3184)
    if (len >= 32) return t;
    return (t & ~(0xFFFFFFFFu >> len)) | (1u << (31 - len));
}


// Branch-free token length from the next 32 stream bits, with the uniform constants of Params:
// c3 tokens (leading 1) are 3 bits; CT7 masked tokens ('0' + type ones) type+2+{mm0|mm}; raw tokens
// 9 + clamp(B + E - 127, 0, 23) = clamp(E + B - 118, 9, 32); CT11 verbatim 32.
template <int CT>
__device__ __forceinline__ int token_len_bf(uint32_t t, const Params& P) {
    const int E = (int)((t >> 23) & 0xFFu);
    int len = min(max(E + P.rawadd, 9), 32);
    if (CT == 11) len = 32;
    if (CT == 7) {
        const bool msk = (t & P.hm) == P.hm;
        const int lm = (int)__umul24(__builtin_amdgcn_ubfe(t, (uint32_t)P.fsh, 1u), (uint32_t)P.dlm) + P.lm0;
        len = msk ? lm : len;
    }
    if (CT != 6) len = ((int)t < 0) ? 3 : len;
    return len;
}

// Branch-free value pattern of a non-predicted token and its predictor code (0 = none/'100',
// 1..3 = 101/110/111).  Raw: top len bits + midpoint bit (decompress_bitwise_float :3166-3184),
// y = 0xFFFFFFFF >> len (0 for len 32); CT7 masked (:1939-2010) from the precomputed c/k constants.
template <int CT>
__device__ __forceinline__ uint32_t token_pattern_bf(uint32_t t, int len, const Params& P, int* code) {
    const bool c3 = (CT != 6) && ((int)t < 0);
    *code = c3 ? (int)__builtin_amdgcn_ubfe(t, 29u, 2u) : 0;
    uint32_t u;
    if (CT == 11) {
        u = t;
    } else {
        const uint32_t y = 0x7FFFFFFFu >> (uint32_t)(len - 1);         // 0xFFFFFFFF >> len, len in [3, 32]
        u = (t & ~y) | (y & ~(y >> 1));
        if (CT == 7) {                                                // bit selects, no divergent branch
            const uint32_t u0 = P.c0 | ((t >> P.s0) & P.k0);
            const uint32_t u1 = P.c1 | ((t >> P.s1) & P.k1);
            const uint32_t mf = (uint32_t)__builtin_amdgcn_sbfe((int)t, (uint32_t)P.fsh, 1u);   // flag: all ones
            const uint32_t mm = (t & P.hm) == P.hm ? 0xFFFFFFFFu : 0u;
            const uint32_t um = (u1 & mf) | (u0 & ~mf);
            u = (um & mm) | (u & ~mm);
        }
    }
    return c3 ? 0u : u;
}

// ------------------------------------------------------------------------------------------------
// Token tables.  Everything a token's length and (non-predicted) value pattern depend on lies in its
// first 9 bits: the c3 bit, the 8 exponent bits, and for CT7 (type <= 7, enforced by the host) the
// type head ones and the flag bit, which end at bit 30 - type >= 23.  Per-call LDS tables indexed by
// t >> 23 therefore replace the selects of token_len_bf / token_pattern_bf:
//   meta[t >> 23]          = sh | len << 8          (len 3..32; sh = the masked-token shift, 0 for raw)
//   kv[(t >> 23) & 255]    = {keep, add}: pattern = ((t >> sh) & keep) | add for every non-c3 token
// (a c3 token's pattern is 0 / a prediction, selected by the caller; CT6 has no c3 tokens and its
// sign bit passes through `keep`, so bit 31 is not needed to index kv).
struct TokLut {
    uint16_t meta[512];
    uint2 kv[256];
};

template <int CT>
__device__ __forceinline__ void build_lut_len(uint8_t* tl, const Params& P, int tid, int nthr) {
    for (int i = tid; i < 512; i += nthr) tl[i] = (uint8_t)token_len_bf<CT>((uint32_t)i << 23, P);
}

template <int CT>
__device__ __forceinline__ void build_lut_meta(uint16_t* meta, const Params& P, int tid, int nthr) {
    for (int i = tid; i < 512; i += nthr) {
        const uint32_t t = (uint32_t)i << 23;
        const int len = token_len_bf<CT>(t, P);
        int sh = 0;
        if (CT == 7 && (int)t >= 0 && (t & P.hm) == P.hm) sh = ((t >> P.fsh) & 1u) ? P.s1 : P.s0;
        meta[i] = (uint16_t)(sh | (len << 8));
    }
}

template <int CT>
__device__ __forceinline__ void build_lut(TokLut& T, const Params& P, int tid, int nthr) {
    build_lut_meta<CT>(T.meta, P, tid, nthr);
    for (int i = tid; i < 256; i += nthr) {
        const uint32_t t = (uint32_t)i << 23;                  // bit 31 clear: never a c3 token
        uint32_t keep, add;
        if (CT == 11) {
            keep = 0xFFFFFFFFu; add = 0u;
        } else {
            const int len = token_len_bf<6>(t, P);             // raw length 9 + m(E)
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

__device__ __forceinline__ uint32_t lut_pattern(const TokLut& T, uint32_t t, uint32_t meta) {
    const uint2 kv = T.kv[(t >> 23) & 255u];
    return ((t >> (meta & 31u)) & kv.x) | kv.y;
}

// NaN results follow x86 SSE (the reference's host): the first NaN operand in evaluation order,
// quieted; a NaN made from non-NaN operands (inf - inf) is the x86 default NaN 0xFFC00000.  Only
// streams decoded outside the codec's domain ever reach this (an encoder never predicts with NaNs).
__device__ __noinline__ float x86_nan(float b1, float b2, float b3, bool use3) {
    const uint32_t q = 0x00400000u;
    if (b1 != b1) return __uint_as_float(__float_as_uint(b1) | q);
    if (b2 != b2) return __uint_as_float(__float_as_uint(b2) | q);
    if (use3 && b3 != b3) return __uint_as_float(__float_as_uint(b3) | q);
    return __uint_as_float(0xFFC00000u);
}
__device__ __forceinline__ float predict2(float b1, float b2) {
    const float v = __fsub_rn(__fmul_rn(2.0f, b1), b2);
    return v != v ? x86_nan(b1, b2, 0.0f, false) : v;
}
__device__ __forceinline__ float predict3(float b1, float b2, float b3) {
    const float v = __fadd_rn(__fsub_rn(__fmul_rn(3.0f, b1), __fmul_rn(3.0f, b2)), b3);
    return v != v ? x86_nan(b1, b2, b3, true) : v;
}
__device__ __forceinline__ float predict_value(int code, float b1, float b2, float b3) {
    if (code == 1) return b1;
    if (code == 2) return predict2(b1, b2);
    return predict3(b1, b2, b3);
}

// ------------------------------------------------------------------------------------------------
// Per-lane MSB-first bit reader over a byte stream held as big-endian 32-bit words.
// Runs of 3-bit codes ('1xx': zero / predicted tokens of CT 5, 7, 11).  A walk that needs only token
// boundaries and counts (no values) steps a whole run at once: of the next ten tokens in the 32-bit
// window t (t's bit 31 must be 1) the leading 3-bit ones, capped so that a reader at pos stops on the
// first boundary >= tgt (tgt > pos) -- so exits, merges and first-word masks stay exact.  Period-3
// streams (constant input: all '100'; Himeno planes: '101' runs) take a tenth of the steps.
__device__ __forceinline__ int run3(uint32_t t, long long pos, long long tgt) {
    const uint32_t y = ~t & 0x92492490u;                        // first bits of tokens 0..9
    const int k = y ? (int)((__clz(y) * 11u) >> 5) : 10;        // clz(y) = 3j -> j
    const long long lim = (tgt - pos + 2) / 3;
    return lim < k ? (int)lim : k;
}

__device__ __forceinline__ int run3i(uint32_t t, int pos, int tgt) {  // LDS positions (int)
    const uint32_t y = ~t & 0x92492490u;
    const int k = y ? (int)((__clz(y) * 11u) >> 5) : 10;
    return min(k, (tgt - pos + 2) / 3);
}

// boundary walks in runs mode, a token of length L not starting with '1': when the 32-bit window repeats
// with period 3 (a constant input read out of phase: '001001...' parses as 9-bit raw tokens forever) and
// 3 | L, the next tokens are copies of this one -- step every copy whose first 9 bits (which fix its
// length) lie in the window, counting only tokens that start before tgt
__device__ __forceinline__ int run_per3(uint32_t t, int L, int pos, int tgt) {
    if (((t ^ (t << 3)) & 0xFFFFFFF8u) || L % 3 != 0 || L > 16) return 1;
    return min(min(1 + 23 / L, 32 / L), (tgt - pos - 1) / L + 1);    // a reader step is at most 32 bits
}

// decoders in runs mode step a run of IDENTICAL '100' (value 0) or '101' (value b1) codes at once: every
// token of it has the same value and the history after it is that value repeated.  Returns the tokens of
// the run at the reader (1 for any other token), at most kmax, counting only tokens that start before tgt.
__device__ __forceinline__ int run_same(uint32_t t, int pos, int tgt, int kmax) {
    const uint32_t hi = t >> 29;
    if (hi != 4u && hi != 5u) return 1;
    const uint32_t rep = hi == 4u ? 0x92492492u : 0xB6DB6DB6u;   // '100' / '101' repeated ten times
    const int k = (int)((__clz((t ^ rep) | 3u) * 11u) >> 5);     // equal leading 3-bit groups (clz <= 30)
    return max(1, min(min(k, kmax), (tgt - pos + 2) / 3));
}

// runs mode of a stream: below 6 bits per value it is mostly 3-bit codes (constant input: 3.0; Himeno
// planes ~3.1; random data ~20), and the walks that find boundaries step whole runs and skip the
// merge shortcut (period-3 paths in different phases never merge).  CT6 has no 3-bit codes.
// ------------------------------------------------------------------------------------------------
// Fused CRC-32 (zlib, reflected polynomial 0xEDB88320) over 16 KiB stream blocks (DC_CRCF_BLK).  CRC is linear
// over GF(2): the raw CRC (init 0, no final xor) of a block is the XOR of its pieces' raw CRCs, each shifted by
// x^(8 * bytes after it in the block), so pieces computed by different workgroups (encoder tiles, decoder jobs)
// combine with an atomic XOR.  ctab (DC_CRCF_WORDS words, dc_crcf_tables): [CRCF_NIB] eight 16-entry nibble
// tables (the byte table's entry of nibble j alone), [CRCF_KQ] kq[i] = x^(256 i) mod P (a shift by i 32-byte
// units), [CRCF_X2N] x^(2^k) mod P, k < 40.
constexpr int CRCF_NIB = 0, CRCF_KQ = 128, CRCF_X2N = 640;
constexpr uint32_t CRCF_POLY = 0xEDB88320u, CRCF_ONE = 0x80000000u;
__host__ __device__ inline long long crcf_nblk(long long nbytes) { return (nbytes + DC_CRCF_BLK - 1) / DC_CRCF_BLK; }
__device__ __forceinline__ uint32_t crcf_word(uint32_t r, uint32_t w, const uint32_t* nib) {   // 4 bytes, LE
    const uint32_t c = r ^ w;
    return (nib[c & 15u] ^ nib[16 + ((c >> 4) & 15u)]) ^ (nib[32 + ((c >> 8) & 15u)] ^ nib[48 + ((c >> 12) & 15u)]) ^
           ((nib[64 + ((c >> 16) & 15u)] ^ nib[80 + ((c >> 20) & 15u)]) ^ (nib[96 + ((c >> 24) & 15u)] ^ nib[112 + (c >> 28)]));
}
__device__ __forceinline__ uint32_t crcf_mult(uint32_t a, uint32_t b) {                       // a b mod P
    uint32_t p = 0;
#pragma unroll 8
    for (int i = 31; i >= 0; i--) {
        p ^= ((a >> i) & 1u) ? b : 0u;
        b = (b >> 1) ^ ((b & 1u) ? CRCF_POLY : 0u);
    }
    return p;
}

__device__ __forceinline__ int runs_mode(int ct, unsigned long long nbits, long long num) {
    return ct != 6 && num > 0 && nbits < 6ull * (unsigned long long)num;
}

struct BitReader {
    const uint32_t* w;        // stream viewed as 32-bit words (4-byte aligned)
    const uint8_t* b;
    long long nbytes;
    long long nwfull;         // words fully inside the stream
    uint64_t buf;             // next bits, MSB-aligned
    int nbuf;
    long long wi;             // next word to load
    long long pos;            // stream bit position of buf's MSB

    __device__ __forceinline__ uint32_t load_word(long long i) const {
        if (i < nwfull) return __builtin_bswap32(w[i]);
        uint32_t v = 0;
        for (int k = 0; k < 4; k++) {
            const long long bi = 4 * i + k;
            v = (v << 8) | (bi < nbytes ? (uint32_t)b[bi] : 0u);
        }
        return v;
    }
    __device__ __forceinline__ void refill() {
        buf |= (uint64_t)load_word(wi++) << (32 - nbuf);
        nbuf += 32;
    }
    __device__ __forceinline__ void init(const uint8_t* stream, long long nbytes_, long long p) {
        b = stream; w = reinterpret_cast<const uint32_t*>(stream);
        nbytes = nbytes_; nwfull = nbytes_ >> 2;
        wi = p >> 5; buf = 0; nbuf = 0;
        refill(); refill();
        const int sk = (int)(p & 31);
        buf <<= sk; nbuf -= sk;
        if (nbuf < 32) refill();
        pos = p;
    }
    __device__ __forceinline__ uint32_t peek() const { return (uint32_t)(buf >> 32); }
    __device__ __forceinline__ void skip(int k) {
        buf <<= k; nbuf -= k; pos += k;
        if (nbuf < 32) refill();
    }
};

// Wave-wide inclusive prefix sum without LDS: Hillis-Steele inside each 16-lane row (DPP row_shr 1, 2, 4,
// 8), then row_bcast:15 (lane 15 of rows 0 / 2 into rows 1 / 3) and row_bcast:31 (lane 31 into rows 2, 3)
// -- the GFX9-family DPP scan.  (__shfl_up / __shfl_xor lower to ds_bpermute: one LDS round trip per step.)
// Every lane of the wave must be active.
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);   // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);   // row_bcast:31
    return v;
}
// the wave's total (every lane)
__device__ __forceinline__ uint32_t wave_total(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_incl(v), 63);
}

// a - b as the reference's x86 build computes it (SSE subss): a NaN operand propagates quieted, the first one
// when both are, and an invalid result (inf - inf) is the default NaN 0xFFC00000 -- the GPU's fsub returns
// 0x7FC00000 in every case
__device__ __forceinline__ float sub_x86(float a, float b) {
    if (__builtin_expect(a != a, 0)) return __uint_as_float(__float_as_uint(a) | 0x00400000u);
    if (__builtin_expect(b != b, 0)) return __uint_as_float(__float_as_uint(b) | 0x00400000u);
    const float r = __fsub_rn(a, b);
    return r != r ? __uint_as_float(0xFFC00000u) : r;
}
// the same for a FINITE b (the fused pre-passes subtract a finite minimum; their host falls back otherwise): the
// result is NaN only when a is, and then it is a quieted
__device__ __forceinline__ float sub_fin(float a, float b) {
    const float r = __fsub_rn(a, b);
    return a != a ? __uint_as_float(__float_as_uint(a) | 0x00400000u) : r;
}
__device__ __forceinline__ double sub_fin(double a, double b) { return __dsub_rn(a, b); }   // (float path only)

__device__ __forceinline__ uint64_t ld_relaxed(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_relaxed(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// a Himeno halo plane's element (a, b) in the [mi][mj][mk] array: the plane ijk = 1/2/3 at index v, in the order of
// transform_3d_array_to_1d_array (impl/dataCompression.c:3741-3775)
__device__ __forceinline__ long long plane_index(long long a, long long b, int ijk, int v, int mj, int mk) {
    long long i, j, k;
    if (ijk == 1) { i = v; j = a; k = b; }
    else if (ijk == 2) { i = a; j = v; k = b; }
    else { i = a; j = b; k = v; }
    return (i * mj + j) * mk + k;
}

}  // namespace dc
