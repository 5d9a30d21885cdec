/*
 * dc_oracle64.c -- CPU restatement of the reference DOUBLE bit-wise codecs.  TEST INFRASTRUCTURE
 * ONLY (see dc_oracle.h).  Built with -ffp-contract=off like dc_oracle.c so every double operation
 * rounds exactly like the reference built with gcc -O3 on x86-64 SSE2.
 *
 * The reference works on 64-char '0'/'1' strings (doubletostr :5256, add_bit_to_bytes :5456); this
 * restatement works on the 64-bit pattern.  Citations: impl/dataCompression.c.
 */
#include "dc_oracle.h"
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static inline uint64_t d2u(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
static inline double u2d(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }

/* mantissa bits kept: compress_bitwise_double :3452-3468 (exponent from the pattern, clamp 0..52) */
int orc64_mbits(int B, int E) {
    int m = B + E - 1023;
    return m > 52 ? 52 : (m < 0 ? 0 : m);
}
static inline int mbits64(int B, uint64_t u) { return orc64_mbits(B, (int)((u >> 52) & 0x7FF)); }

/* ------------------------------------------------------------------ pre-passes */
double orc64_to_small(const double* data, long n, double* out) {   /* toSmallDataset_double :3522-3541 */
    double mn = data[0];
    for (long i = 1; i < n; i++) if (data[i] < mn) mn = data[i];
    for (long i = 0; i < n; i++) out[i] = data[i] - mn;
    return mn;
}

double orc64_med(const double* data, long n, int* type) {          /* med_dataset_double :3564-3590 */
    double total = 0, mx = data[0];
    for (long i = 0; i < n; i++) {
        total += data[i];
        if (data[i] > mx) mx = data[i];
    }
    int add = 0;
    for (int i = 10; i > 0; i--) {
        add += (int)pow(2, i);
        if (mx < pow(2, add - 1023)) { *type = 11 - i; break; }
    }
    return total / n;
}

/* first 20 chars of doubletostr(mean) (mask[1+11+8]) as the top 20 bits of the pattern */
uint32_t orc64_mask20(double mean) { return (uint32_t)(d2u(mean) >> 44); }

/* ------------------------------------------------------------------ bit writer (:5456-5489) */
typedef struct { unsigned char* buf; long bytes; int pos; } bw_t;

static void bw_begin(bw_t* w, unsigned char** bits, int* bytes, int* pos, long max_new_bits) {
    long need = *bytes + (max_new_bits + 7) / 8 + 8;
    w->buf = (unsigned char*)realloc(*bits, need > 0 ? need : 1);
    if (!w->buf) { fprintf(stderr, "oracle: out of memory\n"); exit(1); }
    w->bytes = *bytes;
    w->pos = *pos;
}

static inline void bw_put(bw_t* w, uint64_t v, int n) {            /* n <= 64, MSB first */
    for (int i = n - 1; i >= 0; i--) {
        int bit = (int)((v >> i) & 1);
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

static inline uint64_t low_bits(uint64_t v, int n) { return n >= 64 ? v : (v & ((1ull << n) - 1ull)); }

/* raw token (compress_bitwise_double :3446-3477): top 12+m bits of the pattern */
static inline void put_raw(bw_t* w, uint64_t u, int B) {
    int m = mbits64(B, u);
    bw_put(w, u >> (52 - m), 12 + m);
}

/* compress_bitwise_double_mask :1493-1588 */
static inline void put_raw_mask(bw_t* w, uint64_t u, int B, int type, uint32_t mask20) {
    int m = mbits64(B, u);
    if ((u >> 52) == (uint64_t)(mask20 >> 8)) {              /* sign+exponent equal the mask :1523-1531 */
        uint64_t head = ((1ull << type) - 1ull) << 1;         /* '0' + '1'*type (+ flag) */
        if (((u >> 44) & 0xFFu) == (mask20 & 0xFFu)) {        /* mantissa bits 1..8 equal :1538-1545 */
            bw_put(w, head, type + 2);                        /* flag 0 :1547-1559 */
            if (m > 8) bw_put(w, low_bits(u >> (52 - m), m - 8), m - 8);
        } else {
            bw_put(w, head | 1u, type + 2);                   /* flag 1 :1561-1574 */
            if (m > 0) bw_put(w, low_bits(u >> (52 - m), m), m);
        }
    } else {
        bw_put(w, u >> (52 - m), 12 + m);                     /* :1582-1586 */
    }
}

/* myCompress_bitwise_double :3189 (ct 5), _np :2633 (6), _mask :1590 (7), _op :355 (11) */
void orc64_compress(int ct, const double* data, long num, double bound, int type, uint32_t mask20,
                    unsigned char** bits, int* bytes, int* pos) {
    const int B = orc_bound_binary(bound);
    bw_t w;
    bw_begin(&w, bits, bytes, pos, num * 64);
    double b1 = -1, b2 = -1, b3 = -1;                        /* sentinel history :3191, :3206-3227 */
    for (long n = 0; n < num; n++) {
        double x = data[n];
        uint64_t u = d2u(x);
        if (ct == 6) { put_raw(&w, u, B); continue; }
        int code = 0, zero;
        if (b3 == -1 || b2 == -1 || b1 == -1) {
            zero = fabs(x) < bound;
            if (b3 == -1) b3 = x;
            else if (b2 == -1) b2 = x;
            else if (b1 == -1) b1 = x;
        } else {
            double p1 = b1;                                   /* :3231-3255 */
            double p2 = 2 * b1 - b2;
            double p3 = 3 * b1 - 3 * b2 + b3;
            double d1 = fabs(p1 - x), d2 = fabs(p2 - x), d3 = fabs(p3 - x);
            double dmin = d1; int t = 5;
            if (d2 < dmin) { dmin = d2; t = 6; }
            if (d3 < dmin) { dmin = d3; t = 7; }
            b3 = b2; b2 = b1; b1 = x;
            zero = fabs(x) < bound;
            if (!zero && dmin <= bound) code = t;
        }
        if (zero) bw_put(&w, 4u, 3);                          /* '100' */
        else if (code) bw_put(&w, (uint64_t)code, 3);
        else if (ct == 11) bw_put(&w, u, 64);                 /* verbatim :377-382 */
        else if (ct == 7) put_raw_mask(&w, u, B, type, mask20);
        else put_raw(&w, u, B);
    }
    bw_end(&w, bits, bytes, pos);
}

/* ------------------------------------------------------------------ grammar decoder */
static inline int get_bit(const unsigned char* s, long p) { return (s[p >> 3] >> (7 - (p & 7))) & 1; }
static inline uint64_t get_bits(const unsigned char* s, long nbits, long p, int n) {
    uint64_t v = 0;
    for (int i = 0; i < n; i++) v = (v << 1) | (uint64_t)((p + i) < nbits ? get_bit(s, p + i) : 0);
    return v;
}

static inline void hist_push(double* b1, double* b2, double* b3, double v) {   /* :2722-2740 */
    if (*b3 == -1) *b3 = v;
    else if (*b2 == -1) *b2 = v;
    else if (*b1 == -1) *b1 = v;
    else { *b3 = *b2; *b2 = *b1; *b1 = v; }
}

static inline double decode_code(int c2, double b1, double b2, double b3) {   /* :2873-2893 */
    if (c2 == 0) return 0.0;
    if (c2 == 1) return b1;
    if (c2 == 2) return 2 * b1 - b2;
    return 3 * b1 - 3 * b2 + b3;
}

/* raw pattern with the midpoint bit (decompress_bitwise_double :2895-2918) */
static inline uint64_t raw_pattern(uint64_t tok, int nb) {
    if (nb >= 64) return tok;
    return (tok << (64 - nb)) | (1ull << (63 - nb));
}

/* masked reconstruction (decompress_bitwise_double_mask :1424-1484) */
static inline uint64_t mask_pattern(uint32_t mask20, int flag, uint64_t tail, int tl) {
    uint64_t u;
    if (!flag) {
        u = (uint64_t)mask20 << 44;
        if (tl > 0) u |= tail << (44 - tl);
        if (20 + tl < 64) u |= 1ull << (43 - tl);
    } else {
        u = (uint64_t)(mask20 >> 8) << 52;
        if (tl > 0) u |= tail << (52 - tl);
        if (12 + tl < 64) u |= 1ull << (51 - tl);
    }
    return u;
}

long orc64_decompress_spec(int ct, const unsigned char* s, long bytes, long num, double bound,
                           int type, uint32_t mask20, double* out) {
    const int B = orc_bound_binary(bound);
    const long nbits = bytes * 8;
    const int mm = orc64_mbits(B, (int)((mask20 >> 8) & 0x7FF));
    double b1 = -1, b2 = -1, b3 = -1;
    long p = 0, n = 0;
    while (n < num && p < nbits) {
        double v;
        int b0 = get_bit(s, p);
        if (ct != 6 && b0 == 1) {
            if (p + 3 > nbits) break;
            v = decode_code((int)get_bits(s, nbits, p + 1, 2), b1, b2, b3);
            p += 3;
        } else if (ct == 11) {
            if (p + 64 > nbits) break;
            v = u2d(get_bits(s, nbits, p, 64));
            p += 64;
        } else if (ct == 7 && get_bits(s, nbits, p + 1, type) == (1ull << type) - 1ull) {
            int flag = (int)get_bits(s, nbits, p + 1 + type, 1);
            int tl = flag ? mm : (mm > 8 ? mm - 8 : 0);
            if (p + type + 2 + tl > nbits) break;
            uint64_t tail = tl ? get_bits(s, nbits, p + type + 2, tl) : 0;
            v = u2d(mask_pattern(mask20, flag, tail, tl));
            p += type + 2 + tl;
        } else {
            if (p + 12 > nbits) break;
            int m = orc64_mbits(B, (int)get_bits(s, nbits, p + 1, 11));
            if (p + 12 + m > nbits) break;
            v = u2d(raw_pattern(get_bits(s, nbits, p, 12 + m), 12 + m));
            p += 12 + m;
        }
        out[n++] = v;
        hist_push(&b1, &b2, &b3, v);
    }
    return n;
}

/* synthetic double input: the U10 generator's 53-bit variant (z >> 11) * 2^-53 * 10 */
void orc64_gen_u10(double* out, long n, uint64_t seed, long offset) {
    for (long i = 0; i < n; i++) {
        uint64_t z = 0x9E3779B97F4A7C15ull * (uint64_t)(offset + i + 1) + seed;
        z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
        z ^= z >> 27; z *= 0x94D049BB133111EBull;
        z ^= z >> 31;
        out[i] = (double)(z >> 11) * 0x1p-53 * 10.0;
    }
}

/* Test helper: the true token boundaries of a double stream cut into chunks of cb bits -- for every
 * chunk the entry offset of its first token, the tokens starting in it and its exit into the next. */
long orc64_chunk_records(int ct, const unsigned char* s, long bytes, long num, double bound, int type,
                         uint32_t mask20, long cb, unsigned char* ent, unsigned char* ex, unsigned short* cnt) {
    const int B = orc_bound_binary(bound);
    const long nbits = bytes * 8;
    const int mm = orc64_mbits(B, (int)((mask20 >> 8) & 0x7FF));
    const long nc = (nbits + cb - 1) / cb;
    for (long c = 0; c < nc; c++) { ent[c] = 0; ex[c] = 0; cnt[c] = 0; }
    long p = 0, n = 0;
    int started = -1;
    while (n < num && p < nbits) {
        int len;
        if (ct != 6 && get_bit(s, p)) len = 3;
        else if (ct == 11) len = 64;
        else if (ct == 7 && get_bits(s, nbits, p + 1, type) == (1ull << type) - 1ull)
            len = type + 2 + (get_bits(s, nbits, p + 1 + type, 1) ? mm : (mm > 8 ? mm - 8 : 0));
        else len = 12 + orc64_mbits(B, (int)get_bits(s, nbits, p + 1, 11));
        if (p + len > nbits) break;
        const long c = p / cb;
        if (c != started) { ent[c] = (unsigned char)(p - c * cb); started = (int)c; }
        cnt[c]++;
        if ((p + len) / cb != c && c + 1 < nc) ex[c] = (unsigned char)(p + len - (c + 1) * cb);
        p += len;
        n++;
    }
    return nc;
}

/* ------------------------------------------------------------------ CT1 byte-wise for doubles */
int orc64_bytewise_compress(const double* data, int num, double bound, double* raw, char* codes, int* pos1) {
    double b1 = -1, b2 = -1, b3 = -1, b4 = -1;              /* myCompress_double :3815-3941 */
    int nf = 0, nc = 0;
    for (int n = 0; n < num; n++) {
        double x = data[n];
        if (b4 == -1 || b3 == -1 || b2 == -1 || b1 == -1) {
            raw[nf++] = x;
            if (b4 == -1) b4 = x;
            else if (b3 == -1) b3 = x;
            else if (b2 == -1) b2 = x;
            else if (b1 == -1) b1 = x;
            continue;
        }
        double p1 = b1, p2 = 2 * b1 - b2, p3 = 3 * b1 - 3 * b2 + b3, p4 = 4 * b1 - 6 * b2 + 4 * b3 - b4;
        double d1 = fabs(p1 - x), d2 = fabs(p2 - x), d3 = fabs(p3 - x), d4 = fabs(p4 - x);
        double dmin = d1; char t = 'a';
        if (d2 < dmin) { dmin = d2; t = 'b'; }
        if (d3 < dmin) { dmin = d3; t = 'c'; }
        if (d4 < dmin) { dmin = d4; t = 'd'; }
        b4 = b3; b3 = b2; b2 = b1; b1 = x;
        if (dmin <= bound) { codes[nc] = t; nc++; pos1[nc - 1] = nf + nc; }
        else raw[nf++] = x;
    }
    return nf;
}

void orc64_bytewise_decompress(const double* raw, const char* codes, const int* pos1, int ncodes, int num,
                               double* out) {                /* myDecompress_double :3778-3813 */
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
