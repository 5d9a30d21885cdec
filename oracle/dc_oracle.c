/*
 * dc_oracle.c -- CPU restatement of the reference float codecs.  TEST INFRASTRUCTURE ONLY
 * (see dc_oracle.h).  Build: oracle/Makefile (gcc -O2 -ffp-contract=off, no -march, so every
 * float operation rounds exactly like the reference built with gcc -O3 on x86-64 SSE).
 *
 * The reference works on '0'/'1' char strings (floattostr :5244, add_bit_to_bytes :5456);
 * this restatement works on the 32-bit pattern directly.  Citations: impl/dataCompression.c.
 */
#include "dc_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* ------------------------------------------------------------------ bound helpers */
int orc_bound_binary(double bound) {            /* to_absErrorBound_binary :5512-5522 */
    for (int n = 0; n < 100; n++)
        if (bound >= pow(2, -n)) return n;
    return 100;
}

float orc_thr_lt(double bound) {
    float f = (float)bound;
    while ((double)f >= bound) f = nextafterf(f, 0.0f);
    while ((double)nextafterf(f, INFINITY) < bound) f = nextafterf(f, INFINITY);
    return f;
}

float orc_thr_le(double bound) {
    float f = (float)bound;
    while ((double)f > bound) f = nextafterf(f, 0.0f);
    while ((double)nextafterf(f, INFINITY) <= bound) f = nextafterf(f, INFINITY);
    return f;
}

/* mantissa bits kept: compress_bitwise_float :3485-3505 (exponent from the pattern, clamp 0..23) */
static inline int mbits_e(int B, int E) {
    int m = B + E - 127;
    return m > 23 ? 23 : (m < 0 ? 0 : m);
}
static inline int mbits(int B, uint32_t u) { return mbits_e(B, (int)((u >> 23) & 0xFF)); }

/* ------------------------------------------------------------------ pre-passes */
float orc_to_small(const float* data, long n, float* out) {   /* toSmallDataset_float :3543 */
    float mn = data[0];
    for (long i = 1; i < n; i++) if (data[i] < mn) mn = data[i];
    for (long i = 0; i < n; i++) out[i] = data[i] - mn;
    return mn;
}

float orc_med(const float* data, long n, int* type) {         /* med_dataset_float :3593 */
    float total = 0, mx = data[0];
    for (long i = 0; i < n; i++) {
        total += data[i];
        if (data[i] > mx) mx = data[i];
    }
    int add = 0;
    for (int i = 7; i > 0; i--) {
        add += (int)pow(2, i);
        if (mx < pow(2, add - 127)) { *type = 8 - i; break; }
    }
    return total / n;
}

uint32_t orc_mask17(float mean) { return f2u(mean) >> 15; }  /* strncpy(mask, floattostr(mean), 17) */

/* ------------------------------------------------------------------ bit writer */
/* add_bit_to_bytes :5456-5489 semantics: MSB-first; pos = 8 at a byte boundary, otherwise the
 * 1-based index of the next free bit in the last byte.  Bits are set/cleared exactly. */
typedef struct { unsigned char* buf; long bytes; int pos; } bw_t;

static void bw_begin(bw_t* w, unsigned char** bits, int* bytes, int* pos, long max_new_bits) {
    long need = *bytes + (max_new_bits + 7) / 8 + 8;
    w->buf = (unsigned char*)realloc(*bits, need > 0 ? need : 1);
    if (!w->buf) { fprintf(stderr, "oracle: out of memory\n"); exit(1); }
    w->bytes = *bytes;
    w->pos = *pos;
}

static inline void bw_put(bw_t* w, uint32_t v, int n) {
    for (int i = n - 1; i >= 0; i--) {
        int bit = (v >> i) & 1;
        if (w->pos == 8) { w->buf[w->bytes++] = 0; }
        unsigned char* p = &w->buf[w->bytes - 1];
        if (bit) *p |= (unsigned char)(1u << (w->pos - 1));
        else     *p &= (unsigned char)~(1u << (w->pos - 1));
        w->pos--;
        if (w->pos == 0) w->pos = 8;
    }
}

static void bw_end(bw_t* w, unsigned char** bits, int* bytes, int* pos) {
    unsigned char* b = (unsigned char*)realloc(w->buf, w->bytes > 0 ? w->bytes : 1);
    *bits = b ? b : w->buf;
    *bytes = (int)w->bytes;
    *pos = w->pos;
}

/* ------------------------------------------------------------------ encoders */
/* raw token (compress_bitwise_float :3479-3520): top 9+m bits of the pattern */
static inline void put_raw(bw_t* w, uint32_t u, int B) {
    int m = mbits(B, u);
    bw_put(w, u >> (23 - m), 9 + m);
}

/* compress_bitwise_float_mask :2143-2284 */
static inline void put_raw_mask(bw_t* w, uint32_t u, int B, int type, uint32_t mask17) {
    int m = mbits(B, u);
    if ((u >> 23) == (mask17 >> 8)) {                       /* sign+exponent equal the mask :2172-2180 */
        uint32_t head = ((1u << type) - 1u) << 1;           /* '0' + '1'*type (+ flag) */
        if (((u >> 15) & 0xFFu) == (mask17 & 0xFFu)) {     /* mantissa bits 1..8 equal :2199-2206 */
            bw_put(w, head, type + 2);                      /* flag 0 :2211-2220 */
            if (m > 8) bw_put(w, (u >> (23 - m)) & ((1u << (m - 8)) - 1u), m - 8);
        } else {
            bw_put(w, head | 1u, type + 2);                 /* flag 1 :2225-2265 */
            if (m > 0) bw_put(w, (u >> (23 - m)) & ((1u << m) - 1u), m);
        }
    } else {
        bw_put(w, u >> (23 - m), 9 + m);                    /* :2279-2282 */
    }
}

void orc_compress(int ct, const float* data, long num, double bound, int type, uint32_t mask17,
                  unsigned char** bits, int* bytes, int* pos) {
    const int B = orc_bound_binary(bound);
    bw_t w;
    bw_begin(&w, bits, bytes, pos, num * 32);
    /* sentinel history exactly as :2032/:2041-2067 (before_value* = -1 means empty) */
    float b1 = -1, b2 = -1, b3 = -1;
    for (long n = 0; n < num; n++) {
        float x = data[n];
        uint32_t u = f2u(x);
        if (ct == 6) { put_raw(&w, u, B); continue; }       /* myCompress_bitwise_np :2645-2654 */
        int code = 0;                                        /* 0 none, 5 '101', 6 '110', 7 '111' */
        int zero;
        if (b3 == -1 || b2 == -1 || b1 == -1) {
            zero = fabs(x) < bound;
            if (b3 == -1) b3 = x;
            else if (b2 == -1) b2 = x;
            else if (b1 == -1) b1 = x;
        } else {
            float p1 = b1;                                   /* :3362-3384 */
            float p2 = 2 * b1 - b2;
            float p3 = 3 * b1 - 3 * b2 + b3;
            float d1 = fabs(p1 - x), d2 = fabs(p2 - x), d3 = fabs(p3 - x);
            float dmin = d1; int t = 5;
            if (d2 < dmin) { dmin = d2; t = 6; }
            if (d3 < dmin) { dmin = d3; t = 7; }
            b3 = b2; b2 = b1; b1 = x;
            zero = fabs(x) < bound;
            if (!zero && dmin <= bound) code = t;
        }
        if (zero) bw_put(&w, 4u, 3);                         /* '100' */
        else if (code) bw_put(&w, (uint32_t)code, 3);        /* '101' '110' '111' */
        else if (ct == 11) bw_put(&w, u, 32);                /* verbatim :602-605 */
        else if (ct == 7) put_raw_mask(&w, u, B, type, mask17);
        else put_raw(&w, u, B);
    }
    bw_end(&w, bits, bytes, pos);
}

/* ------------------------------------------------------------------ decoders (shared) */
static inline int get_bit(const unsigned char* s, long p) { return (s[p >> 3] >> (7 - (p & 7))) & 1; }

static inline uint32_t get_bits(const unsigned char* s, long nbits_total, long p, int n) {
    uint32_t v = 0;
    for (int i = 0; i < n; i++) v = (v << 1) | (uint32_t)((p + i) < nbits_total ? get_bit(s, p + i) : 0);
    return v;
}

/* history update exactly as :1872-1889 (sentinel fill, then shift) */
static inline void hist_push(float* b1, float* b2, float* b3, float v) {
    if (*b3 == -1) *b3 = v;
    else if (*b2 == -1) *b2 = v;
    else if (*b1 == -1) *b1 = v;
    else { *b3 = *b2; *b2 = *b1; *b1 = v; }
}

static inline float decode_code(int c2, float b1, float b2, float b3) {   /* :3143-3158 */
    if (c2 == 0) return 0.0f;
    if (c2 == 1) return b1;
    if (c2 == 2) return 2 * b1 - b2;
    return 3 * b1 - 3 * b2 + b3;
}

/* raw pattern reconstruction with midpoint bit (decompress_bitwise_float :3166-3184) */
static inline uint32_t raw_pattern(uint32_t tok, int nb) {
    if (nb >= 32) return tok;
    return (tok << (32 - nb)) | (1u << (31 - nb));
}

/* masked reconstruction (decompress_bitwise_float_mask :1939-2010) */
static inline uint32_t mask_pattern(uint32_t mask17, int flag, uint32_t tail, int tl) {
    uint32_t u;
    if (!flag) {
        u = mask17 << 15;
        if (tl > 0) u |= tail << (15 - tl);
        if (17 + tl < 32) u |= 1u << (14 - tl);
    } else {
        u = (mask17 >> 8) << 23;
        if (tl > 0) u |= tail << (23 - tl);
        if (9 + tl < 32) u |= 1u << (22 - tl);
    }
    return u;
}

long orc_decompress_spec(int ct, const unsigned char* s, long bytes, long num, double bound,
                         int type, uint32_t mask17, float* out) {
    const int B = orc_bound_binary(bound);
    const long nbits = bytes * 8;
    const int mm = mbits_e(B, (int)((mask17 >> 8) & 0xFF));
    float b1 = -1, b2 = -1, b3 = -1;
    long p = 0, n = 0;
    while (n < num && p < nbits) {
        float v;
        int b0 = get_bit(s, p);
        if (ct != 6 && b0 == 1) {                           /* 3-bit code */
            if (p + 3 > nbits) break;
            v = decode_code((int)get_bits(s, nbits, p + 1, 2), b1, b2, b3);
            p += 3;
        } else if (ct == 11) {                              /* verbatim 32 bits */
            if (p + 32 > nbits) break;
            v = u2f(get_bits(s, nbits, p, 32));
            p += 32;
        } else if (ct == 7 && get_bits(s, nbits, p + 1, type) == (1u << type) - 1u) {
            int flag = (int)get_bits(s, nbits, p + 1 + type, 1);
            int tl = flag ? mm : (mm > 8 ? mm - 8 : 0);
            if (p + type + 2 + tl > nbits) break;
            uint32_t tail = tl ? get_bits(s, nbits, p + type + 2, tl) : 0;
            v = u2f(mask_pattern(mask17, flag, tail, tl));
            p += type + 2 + tl;
        } else {                                            /* raw 9+m bits */
            if (p + 9 > nbits) break;
            int m = mbits_e(B, (int)get_bits(s, nbits, p + 1, 8));
            if (p + 9 + m > nbits) break;
            v = u2f(raw_pattern(get_bits(s, nbits, p, 9 + m), 9 + m));
            p += 9 + m;
        }
        out[n++] = v;
        hist_push(&b1, &b2, &b3, v);
    }
    return n;
}

/* ------------------------------------------------------------------ faithful reference decoders */
typedef struct {
    uint64_t acc; int nb;
    float b1, b2, b3;
    long ndec, num; float* out;
} cref_t;

static inline int tok_bit(const cref_t* c, int i) { return (int)((c->acc >> (c->nb - 1 - i)) & 1); }

/* decompress_bitwise_float_mask :1900-2027 on the accumulated bits */
static float cref_value_mask(const cref_t* c, int type, uint32_t mask17) {
    int nb = c->nb;
    uint32_t tok = (uint32_t)c->acc;
    if (nb == 3 && tok_bit(c, 0) == 1)
        return decode_code((int)(tok & 3), c->b1, c->b2, c->b3);
    if (nb == 32) return u2f(tok);
    int masked = 1;
    for (int i = 1; i < type + 1; i++) if (tok_bit(c, i) != 1) { masked = 0; break; }
    if (masked) {
        int flag = tok_bit(c, type + 1);
        int tl = nb - (type + 2);
        uint32_t tail = tl > 0 ? (uint32_t)(c->acc & ((1ull << tl) - 1)) : 0;
        return u2f(mask_pattern(mask17, flag, tail, tl));
    }
    return u2f(raw_pattern(tok, nb));
}

/* decompress_bitwise_float :3137-3186 */
static float cref_value_bw(const cref_t* c, int* err) {
    uint32_t tok = (uint32_t)c->acc;
    if (c->nb == 3) {
        if (tok_bit(c, 0) == 1) return decode_code((int)(tok & 3), c->b1, c->b2, c->b3);
        *err = 1; return 0;                                  /* "Error start bit of 3 bits is 0" exit */
    }
    return u2f(raw_pattern(tok, c->nb));
}

static inline void cref_emit(cref_t* c, float v) {
    c->ndec++;
    if (c->ndec <= c->num) c->out[c->ndec - 1] = v;
    hist_push(&c->b1, &c->b2, &c->b3, v);
    c->acc = 0; c->nb = 0;
}

long orc_decompress_cref(int ct, const unsigned char* s, long bytes, long num, double bound,
                         int type, uint32_t mask17, float* out, int* stuck) {
    const int B = orc_bound_binary(bound);
    cref_t c = {0, 0, -1, -1, -1, 0, num, out};
    int offset = 0, pending = 0, err = 0;
    *stuck = 0;
    for (long i = 0; i < bytes && !err; i++) {
        for (int j = 7; j >= 0; j--) {
            int bit = (s[i] >> j) & 1;
            if (ct == 11) {                                  /* myDecompress_bitwise_op :710-795 */
                if (offset == 0) offset = bit == 0 ? 32 : 3;
                c.acc = (c.acc << 1) | (uint64_t)bit; c.nb++;
                offset--;
                if (offset == 0) cref_emit(&c, cref_value_bw(&c, &err));
                continue;
            }
            if (ct == 5 || ct == 6) {                        /* :2934-3133 / :2470-2607 */
                if (offset == 0) {
                    if (c.nb == 0) {
                        if (bit == 1 && ct == 6) { err = 2; break; }   /* "Error leading bit 1" */
                        offset = bit == 0 ? 9 : 3;
                    } else {
                        int m = mbits_e(B, (int)((c.acc >> (c.nb - 9)) & 0xFF));
                        offset = m;
                        if (m == 0) {
                            cref_emit(&c, ct == 6 ? u2f(raw_pattern((uint32_t)c.acc, c.nb)) : cref_value_bw(&c, &err));
                            if (bit == 1 && ct == 6) { err = 2; break; }
                            offset = bit == 0 ? 9 : 3;
                        }
                    }
                }
                c.acc = (c.acc << 1) | (uint64_t)bit; c.nb++;
                offset--;
                if (offset == 0 && c.nb != 9)
                    cref_emit(&c, ct == 6 ? u2f(raw_pattern((uint32_t)c.acc, c.nb)) : cref_value_bw(&c, &err));
                continue;
            }
            /* ct == 7: myDecompress_bitwise_mask :1716-1896 */
            if (offset == 0) {
                if (c.nb == 0) {
                    if (bit == 0) { pending = 1; offset = 1 + type; }
                    else offset = 3;
                } else if (pending) {
                    pending = 0;
                    int masked = 1;
                    for (int n = 1; n < type + 1; n++) if (tok_bit(&c, n) != 1) { masked = 0; break; }
                    offset = masked ? 1 : 8 - type;
                } else {
                    int E;
                    if (c.nb == 1 + 8) E = (int)((c.acc >> (c.nb - 9)) & 0xFF);
                    else if (c.nb == 1 + type + 1) E = (int)((mask17 >> 8) & 0xFF);
                    else { err = 3; break; }                 /* "bits_num error" exit */
                    int m = mbits_e(B, E);
                    offset = m;
                    if (offset > 0) {
                        if (c.nb == 1 + type + 1 && tok_bit(&c, c.nb - 1) == 0) offset -= 8;
                    } else {
                        cref_emit(&c, cref_value_mask(&c, type, mask17));
                        pending = 0;
                        if (bit == 0) { pending = 1; offset = 1 + type; }
                        else offset = 3;
                    }
                }
            }
            c.acc = (c.acc << 1) | (uint64_t)bit; c.nb++;
            offset--;
            if (offset < 0 && !pending) { *stuck = 1; goto done; }   /* Q1: never reaches 0 again */
            if (offset == 0 && c.nb != 1 + 8 && c.nb != 1 + type + 1 && !pending) {
                cref_emit(&c, cref_value_mask(&c, type, mask17));
                pending = 0;
            }
            if (c.nb > 60) { *stuck = 1; goto done; }
        }
    }
done:
    if (err) *stuck = 1 + err;
    return c.ndec < num ? c.ndec : num;
}

/* ------------------------------------------------------------------ CT1 byte-wise */
int orc_bytewise_compress(const float* data, int num, double bound, float* raw, char* codes, int* pos1) {
    float b1 = -1, b2 = -1, b3 = -1, b4 = -1;               /* :3982 */
    int nf = 0, nc = 0;
    for (int n = 0; n < num; n++) {
        float x = data[n];
        if (b4 == -1 || b3 == -1 || b2 == -1 || b1 == -1) { /* :3998-4030 */
            raw[nf++] = x;
            if (b4 == -1) b4 = x;
            else if (b3 == -1) b3 = x;
            else if (b2 == -1) b2 = x;
            else if (b1 == -1) b1 = x;
            continue;
        }
        float p1 = b1;                                       /* :4033-4063 */
        float p2 = 2 * b1 - b2;
        float p3 = 3 * b1 - 3 * b2 + b3;
        float p4 = 4 * b1 - 6 * b2 + 4 * b3 - b4;
        float d1 = fabs(p1 - x), d2 = fabs(p2 - x), d3 = fabs(p3 - x), d4 = fabs(p4 - x);
        float dmin = d1; char t = 'a';
        if (d2 < dmin) { dmin = d2; t = 'b'; }
        if (d3 < dmin) { dmin = d3; t = 'c'; }
        if (d4 < dmin) { dmin = d4; t = 'd'; }
        b4 = b3; b3 = b2; b2 = b1; b1 = x;
        if (dmin <= bound) { codes[nc] = t; nc++; pos1[nc - 1] = nf + nc; }
        else raw[nf++] = x;
    }
    return nf;
}

void orc_bytewise_decompress(const float* raw, const char* codes, const int* pos1, int ncodes,
                             int num, float* out) {                /* myDecompress :3943-3977 */
    int fp = 0, cp = 0;
    for (int i = 0; i < num; i++) {
        if (cp < ncodes && pos1[cp] - 1 == i) {
            char t = codes[cp];
            if (t == 'a') out[i] = out[i - 1];
            else if (t == 'b') out[i] = 2 * out[i - 1] - out[i - 2];
            else if (t == 'c') out[i] = 3 * out[i - 1] - 3 * out[i - 2] + out[i - 3];
            else if (t == 'd') out[i] = 4 * out[i - 1] - 6 * out[i - 2] + 4 * out[i - 3] - out[i - 4];
            cp++;
        } else {
            out[i] = raw[fp++];
        }
    }
}

/* ------------------------------------------------------------------ CRC32 (zlib) */
static uint32_t crc_tab[256];
static int crc_init = 0;
uint32_t orc_crc32_update(uint32_t crc, const unsigned char* p, long n) {
    if (!crc_init) {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
            crc_tab[i] = c;
        }
        crc_init = 1;
    }
    crc = ~crc;
    for (long i = 0; i < n; i++) crc = crc_tab[(crc ^ p[i]) & 0xFF] ^ (crc >> 8);
    return ~crc;
}
uint32_t orc_crc32(const unsigned char* p, long n) { return orc_crc32_update(0, p, n); }

/* ------------------------------------------------------------------ Hamming SECDED */
int orc_hm_length(long k) {                                  /* hmLength :5581-5592 */
    int r = 0;
    while (((1L << r) - 1) - r - k < 0) r++;
    return r;
}

/* Hamming position j of every data bit (powers of two skipped), :5549-5562.
 * check bit i = parity of the data bits whose position has bit i set  ==  bit i of the XOR of
 * the positions of all set data bits. */
static uint64_t ham_syndrome(const unsigned char* bits, long bytes, long* ones) {
    uint64_t syn = 0; long cnt = 0;
    long j = 1, nextpow = 1;
    for (long d = 0; d < bytes * 8; d++) {
        while (j == nextpow) { j++; nextpow <<= 1; }
        if (get_bit(bits, d)) { syn ^= (uint64_t)j; cnt++; }
        j++;
    }
    *ones = cnt;
    return syn;
}

void orc_hamming_encode(const unsigned char* bits, long bytes, int* r, char* c) {
    *r = orc_hm_length(bytes * 8);                           /* hamming_encode :5740-5748 */
    long ones;
    uint64_t syn = ham_syndrome(bits, bytes, &ones);
    long sum = ones;
    for (int i = 0; i < *r; i++) { c[i] = ((syn >> i) & 1) ? '1' : '0'; sum += (syn >> i) & 1; }
    c[*r] = (char)('0' + (sum % 2));                         /* :5567-5577 */
}

int orc_hamming_decode(unsigned char* bits, char* c, long bytes, int r, long* err_pos) {
    long ones;                                               /* hamming_decode :5750-5778 */
    uint64_t syn = ham_syndrome(bits, bytes, &ones);
    long pos = 0, sum = ones;
    for (int i = 0; i < r; i++) {
        int ci = c[i] - '0';
        int vi = (int)((syn >> i) & 1) != ci;                /* hamming_verify_bit :5803 */
        pos += (long)vi << i;
        sum += ci;
    }
    int vr = (int)(sum % 2) != (c[r] - '0');                 /* :5818 */
    int type = 0;                                            /* error_info :5631-5654 */
    if (pos > 0 && !vr) type = 1;
    else if (pos == 0 && vr) type = 2;
    else if (pos > 0 && vr) type = 3;
    if (err_pos) *err_pos = pos;
    if (type == 2) c[r] = c[r] == '0' ? '1' : '0';
    if (type == 3) {                                         /* hamming_rectify_bit :5822-5855 */
        long k = bytes * 8;
        if (pos <= r + k) {
            if ((pos & (pos - 1)) == 0) {
                int ci = 0; while ((1L << ci) != pos) ci++;
                c[ci] = c[ci] == '0' ? '1' : '0';
            } else {
                long npow = 0; while ((1L << npow) < pos) npow++;   /* powers of two below pos */
                long d = pos - 1 - npow;
                bits[d >> 3] ^= (unsigned char)(1u << (7 - (d & 7)));
            }
        }
    }
    return type;
}

int orc_block_size(int data_bytes, double ber) {             /* block_size :5868-5879 */
    uint64_t b = (uint64_t)(1 / ber);
    uint64_t by = b / 8;
    int bs = data_bytes;
    if ((uint64_t)bs > by) bs = (int)by;
    return bs;
}

/* ------------------------------------------------------------------ synthetic inputs */
void orc_gen_u10(float* out, long n, uint64_t seed, long offset) {
    for (long i = 0; i < n; i++) {
        uint64_t z = 0x9E3779B97F4A7C15ull * (uint64_t)(offset + i + 1) + seed;
        z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
        z ^= z >> 27; z *= 0x94D049BB133111EBull;
        z ^= z >> 31;
        out[i] = (float)(z >> 40) * 0x1p-24f * 10.0f;
    }
}

void orc_gen_himeno_plane(float* out, int imax, int jmax) {   /* initmt himenoBMTxps.c:239, it=0 */
    for (int i = 0; i < imax; i++)
        for (int j = 0; j < jmax; j++)
            out[(long)i * jmax + j] = (float)(i * i) / (float)((imax - 1) * (imax - 1));
}
