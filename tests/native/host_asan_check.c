/* Host-side C of libdcamd under AddressSanitizer + UBSan (`make -C data-compression_amd asan`).
 *
 * Exercises the host helpers that run without a GPU -- the single-token codecs and the add_bit_to_bytes
 * stream growth they share with the serial codecs (impl/dataCompression.c:3479-3520, 2143-2284,
 * 3137-3186, 5456-5489), the character-level Hamming SECDED (:5544-5868), cast_bits_to_char, getDoubleBin
 * and the binary readers -- with round-trip checks, so that an out-of-bounds access, a use after free
 * or undefined arithmetic in them aborts the run.  No HIP call is made (the library is linked whole). */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dataCompression.h"

static int fails = 0;
#define CHECK(c, ...)                                  \
    do {                                               \
        if (!(c)) {                                    \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);              \
            fputc('\n', stderr);                       \
            fails++;                                   \
        }                                              \
    } while (0)

/* the stream's bits [from, from + n) as a '0'/'1' string */
static void bits_of(const unsigned char* s, int from, int n, char* out) {
    for (int i = 0; i < n; i++) out[i] = ((s[(from + i) >> 3] >> (7 - ((from + i) & 7))) & 1) ? '1' : '0';
    out[n] = 0;
}

/* bits in a stream after add_bit_to_bytes (pos counts down: the next bit's position, 8 = a new byte) */
static int total_bits(int bytes, int pos) { return bytes * 8 - (pos % 8); }

static unsigned rng = 12345u;
static unsigned nextu(void) { rng = rng * 1664525u + 1013904223u; return rng; }

static void tokens_float(void) {
    /* raw tokens: compress_bitwise_float appends 9 + m bits; the decoder's value is within the bound */
    unsigned char* s = NULL;
    int bytes = 0, pos = 8;
    float xs[4096];
    int start[4096], len[4096];
    for (int i = 0; i < 4096; i++) {
        xs[i] = (float)(nextu() % 1000000) * 1e-5f + 0.01f;
        start[i] = total_bits(bytes, pos);
        compress_bitwise_float(xs[i], &s, &bytes, &pos);
        len[i] = total_bits(bytes, pos) - start[i];
        CHECK(len[i] >= 9 && len[i] <= 32, "token length %d", len[i]);
    }
    char bits[64];
    for (int i = 0; i < 4096; i++) {
        bits_of(s, start[i], len[i], bits);
        const float v = decompress_bitwise_float(bits, len[i], 0.f, 0.f, 0.f);
        CHECK(fabs((double)v - (double)xs[i]) <= absErrBound * 1.0000001, "float %d: %g vs %g", i, v, xs[i]);
        const float w = decompress_bitwise_float_np(bits, len[i]);
        CHECK(w == v, "np %d", i);
    }
    free(s);
}

static void tokens_double(void) {
    unsigned char* s = NULL;
    int bytes = 0, pos = 8;
    for (int i = 0; i < 2048; i++) {
        const double x = (double)(nextu() % 1000000) * 1e-5 + 0.01;
        const int st = total_bits(bytes, pos);
        compress_bitwise_double(x, &s, &bytes, &pos);
        const int n = total_bits(bytes, pos) - st;
        CHECK(n >= 12 && n <= 64, "double token length %d", n);
        char bits[80];
        bits_of(s, st, n, bits);
        const double v = decompress_bitwise_double(bits, n, 0.0, 0.0, 0.0);
        CHECK(fabs(v - x) <= absErrBound * 1.0000001, "double %d: %g vs %g", i, v, x);
    }
    free(s);
    /* getDoubleBin (:5232) writes bit VALUES (0/1, not chars): the low 32 bits of the pattern, twice */
    char bin[64];
    const double d = 1.0 + 0x1.23456789p-40;
    unsigned long long u;
    memcpy(&u, &d, 8);
    getDoubleBin(d, bin);
    for (int i = 0; i < 64; i++)
        CHECK(bin[i] == (char)(((unsigned)u >> (31 - (i & 31))) & 1u), "getDoubleBin %d", i);
}

static void hamming_chars(void) {
    /* k data chars, r check chars (+ overall parity): every single-bit error is located and repaired */
    enum { K = 57, R = 6 };
    char data[K + 1], orig[K + 1], c[R + 2], v[R + 2];
    for (int i = 0; i < K; i++) data[i] = (nextu() & 1) ? '1' : '0';
    data[K] = 0;
    memcpy(orig, data, sizeof data);
    memset(c, 0, sizeof c);
    hamming_code(data, c, K, R);
    for (int e = 0; e < K; e++) {
        memcpy(data, orig, sizeof data);
        data[e] = data[e] == '1' ? '0' : '1';
        memset(v, 0, sizeof v);
        hamming_verify(data, c, K, R, v);
        int ebp = 0;
        const int kind = error_info(v, R, &ebp);
        CHECK(kind != 0, "error %d not detected", e);
        hamming_rectify(data, c, K, R, ebp);
        CHECK(memcmp(data, orig, K) == 0, "error %d not repaired (kind %d, pos %d)", e, kind, ebp);
    }
}

static void hamming_bits(void) {
    enum { BYTES = 32, R = 9 };
    unsigned char bits[BYTES], orig[BYTES];
    char data[BYTES * 8 + 1], c[R + 2], v[R + 2];
    for (int i = 0; i < BYTES; i++) bits[i] = (unsigned char)nextu();
    memcpy(orig, bits, sizeof bits);
    cast_bits_to_char(bits, data, BYTES);
    data[BYTES * 8] = 0;
    for (int i = 0; i < BYTES * 8; i++)
        CHECK(data[i] == (((bits[i >> 3] >> (7 - (i & 7))) & 1) ? '1' : '0'), "cast_bits_to_char %d", i);
    memset(c, 0, sizeof c);
    hamming_code(data, c, BYTES * 8, R);
    for (int e = 0; e < BYTES * 8; e += 7) {
        memcpy(bits, orig, sizeof bits);
        bits[e >> 3] ^= (unsigned char)(0x80u >> (e & 7));
        memset(v, 0, sizeof v);
        hamming_verify_bit(bits, c, BYTES, R, v);
        int ebp = 0;
        (void)error_info(v, R, &ebp);
        hamming_rectify_bit(bits, c, BYTES, R, ebp);
        CHECK(memcmp(bits, orig, BYTES) == 0, "bit error %d not repaired", e);
    }
}

static void readers(void) {
    const char* path = "/tmp/dc_asan_check.bin";
    float f[1000];
    for (int i = 0; i < 1000; i++) f[i] = (float)i * 0.5f;
    FILE* fp = fopen(path, "wb");
    CHECK(fp != NULL, "tmp file");
    if (!fp) return;
    fwrite(f, sizeof(float), 1000, fp);
    fclose(fp);
    float* g = readfrombinary_float(path, 1000);
    CHECK(g != NULL && memcmp(f, g, sizeof f) == 0, "readfrombinary_float");
    free(g);
    remove(path);
}

int main(void) {
    tokens_float();
    tokens_double();
    hamming_chars();
    hamming_bits();
    readers();
    if (fails) {
        fprintf(stderr, "%d check(s) failed\n", fails);
        return 1;
    }
    printf("host_asan_check: ok\n");
    return 0;
}
