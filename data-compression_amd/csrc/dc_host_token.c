/*
 * dc_host_token.c -- the reference's single-token and bit-string helpers (impl/dataCompression.h:64-156):
 * the per-element encode / decode functions its serial codecs are built from, the character-level
 * Hamming SECDED routines, and the binary readers.  These are scalar host functions in the reference
 * (one call per element, strings of '0'/'1' characters), so they stay scalar host C here: the GPU
 * codecs (dc_encode.hip, dc_decode_fast.hip, dc_f64.hip) never call them.  Every function states the
 * reference lines it follows; the token grammar is SURVEY.md 8.0.
 *
 * Differences from the reference, all on inputs the reference handles by crashing or exiting:
 *  - decoders never realloc the caller's string (the reference reallocs `bits` to 32/64 chars and
 *    leaves the caller holding a possibly moved pointer, :2616, :3175);
 *  - a midpoint bit that would land past the last pattern bit (masked flag-0 tokens with m = 23, or
 *    m = 52 for doubles) is dropped instead of written one byte past a malloc'd buffer (:1954, :1404);
 *  - the invalid-input exits (:3158 "Error start bit of 3 bits is 0", :2273 "error error") print the
 *    reference's message, set dc_last_error() and return 0 / append nothing instead of exit()ing.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/dataCompression.h"
#include "../../include/dc_gpu.h"

int dc_set_error(int code, const char* msg);      /* dc_host.c: sets dc_last_error() */

/* ---- shared pieces --------------------------------------------------------------------------- */
static int bound_bits(void) {                       /* absErrorBound_binary, lazily cached (:21-22) */
    if (absErrorBound_binary == -100) absErrorBound_binary = to_absErrorBound_binary(absErrBound);
    return absErrorBound_binary;
}

static int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

static void append_bits(unsigned char** data_bits, int* bytes, int* pos, uint64_t v, int n) {
    for (int i = n - 1; i >= 0; i--) add_bit_to_bytes(data_bits, bytes, pos, (int)((v >> i) & 1u));
}

static void append_ones(unsigned char** data_bits, int* bytes, int* pos, int n) {
    for (int i = 0; i < n; i++) add_bit_to_bytes(data_bits, bytes, pos, 1);
}

/* bits[i] of a '0'/'1' string as an integer, MSB first */
static uint64_t str_bits(const char* s, int from, int to) {
    uint64_t v = 0;
    for (int i = from; i < to; i++) v = (v << 1) | (uint64_t)(s[i] == '1');
    return v;
}

/* ---- float ----------------------------------------------------------------------------------- */
/* compress_bitwise_float (:3479-3520): append the raw token, the top 1+8+m bits of the pattern */
void compress_bitwise_float(float real_value, unsigned char** data_bits, int* bytes, int* pos) {
    uint32_t u;
    memcpy(&u, &real_value, 4);
    const int m = clampi(bound_bits() + (int)((u >> 23) & 0xFFu) - 127, 0, 23);
    append_bits(data_bits, bytes, pos, u >> (23 - m), 9 + m);
}

/* compress_bitwise_float_mask (:2143-2284): sign + exponent equal to mask[0..8] -> '0' + type ones +
 * flag ('0' when pattern bits 9..16 equal mask[9..16]: then pattern bits 17..8+m follow, else bits
 * 9..8+m); otherwise the raw token */
void compress_bitwise_float_mask(float real_value, unsigned char** data_bits, int* bytes, int* pos, int type,
                                 char mask[1 + 8 + 8]) {
    uint32_t u;
    memcpy(&u, &real_value, 4);
    const int m = clampi(bound_bits() + (int)((u >> 23) & 0xFFu) - 127, 0, 23);
    const uint32_t mk = (uint32_t)str_bits(mask, 0, 17);
    if ((u >> 23) != (mk >> 8)) {
        append_bits(data_bits, bytes, pos, u >> (23 - m), 9 + m);
        return;
    }
    add_bit_to_bytes(data_bits, bytes, pos, 0);
    append_ones(data_bits, bytes, pos, type);
    if (((u >> 15) & 0xFFu) == (mk & 0xFFu)) {          /* flag 0: pattern bits [17, 9+m) */
        add_bit_to_bytes(data_bits, bytes, pos, 0);
        if (m > 8) append_bits(data_bits, bytes, pos, (u >> (23 - m)) & ((1u << (m - 8)) - 1u), m - 8);
    } else {                                            /* flag 1: pattern bits [9, 9+m) */
        add_bit_to_bytes(data_bits, bytes, pos, 1);
        if (m > 0) append_bits(data_bits, bytes, pos, (u >> (23 - m)) & ((1u << m) - 1u), m);
    }
}

/* pattern bits + a midpoint '1' right after them (when it fits), then zeros (:2616-2628) */
static uint64_t with_midpoint(uint64_t prefix, int nbits, int width) {
    uint64_t v = nbits >= width ? prefix : prefix << (width - nbits);
    if (nbits < width) v |= 1ull << (width - 1 - nbits);
    return v;
}

/* masked token (:1936-2010, :1430-1484): the mask's first `full` (flag 0) or `part` (flag 1) chars, the
 * token's chars after the flag, a midpoint '1', zeros -- assembled as the reference does in a char
 * buffer and read back as `width` bits (chars it writes past `width` are never read back) */
static uint64_t masked_pattern(const char* bits, int bits_num, int type, const char* mask, int full, int part,
                               int width) {
    char b[256];
    const int h = bits[type + 1] == '0' ? full : part;
    int i = 0;
    for (; i < full; i++) b[i] = mask[i];              /* the reference copies all 1+E+8 mask chars */
    i = h;
    for (int j = type + 2; j < bits_num && i < 250; j++) b[i++] = bits[j];
    b[i++] = '1';
    for (; i < width; i++) b[i] = '0';
    return str_bits(b, 0, width);
}

static float f_of(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static double d_of(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }

/* decompress_bitwise_float_np (:2611-2630) */
float decompress_bitwise_float_np(char* bits, int bits_num) {
    if (bits_num >= 32) return f_of((uint32_t)str_bits(bits, 0, 32));
    return f_of((uint32_t)with_midpoint(str_bits(bits, 0, bits_num), bits_num, 32));
}

/* decompress_bitwise_float (:3137-3186): a 3-bit string is a code (zero / the three predictors on the
 * caller's history, float arithmetic as the reference's float expressions), else raw + midpoint */
float decompress_bitwise_float(char* bits, int bits_num, float before_value1, float before_value2,
                               float before_value3) {
    if (bits_num == 3) {
        if (bits[0] != '1') {
            printf("Error start bit of 3 bits is 0\n");
            dc_set_error(DC_ERR_STREAM, "decompress_bitwise_float: a 3-bit token must start with 1 (:3158)");
            return 0.0f;
        }
        const int c = (bits[1] == '1') * 2 + (bits[2] == '1');
        if (c == 0) return 0.0f;
        if (c == 1) return before_value1;
        if (c == 2) return 2 * before_value1 - before_value2;
        return 3 * before_value1 - 3 * before_value2 + before_value3;
    }
    return decompress_bitwise_float_np(bits, bits_num);
}

/* decompress_bitwise_float_mask (:1900-2027) */
float decompress_bitwise_float_mask(char* bits, int bits_num, float before_value1, float before_value2,
                                    float before_value3, int type, char mask[1 + 8 + 8]) {
    if (bits_num == 3 && bits[0] == '1') {
        const int c = (bits[1] == '1') * 2 + (bits[2] == '1');
        if (c == 0) return 0.0f;
        if (c == 1) return before_value1;
        if (c == 2) return 2 * before_value1 - before_value2;
        return 3 * before_value1 - 3 * before_value2 + before_value3;
    }
    if (bits_num == 32) return f_of((uint32_t)str_bits(bits, 0, 32));
    int masked = 1;
    for (int n = 1; n < type + 1; n++)
        if (bits[n] != '1') { masked = 0; break; }
    if (!masked) return decompress_bitwise_float_np(bits, bits_num);
    return f_of((uint32_t)masked_pattern(bits, bits_num, type, mask, 17, 9, 32));
}

/* ---- double (the same grammar on 1+11+52 bits, :1396-1560, :2438-2457, :2871-2920, :3446-3477) --- */
void compress_bitwise_double(double real_value, unsigned char** data_bits, int* bytes, int* pos) {
    uint64_t u;
    memcpy(&u, &real_value, 8);
    const int m = clampi(bound_bits() + (int)((u >> 52) & 0x7FFu) - 1023, 0, 52);
    append_bits(data_bits, bytes, pos, u >> (52 - m), 12 + m);
}

void compress_bitwise_double_mask(double real_value, unsigned char** data_bits, int* bytes, int* pos, int type,
                                  char mask[1 + 11 + 8]) {
    uint64_t u;
    memcpy(&u, &real_value, 8);
    const int m = clampi(bound_bits() + (int)((u >> 52) & 0x7FFu) - 1023, 0, 52);
    const uint64_t mk = str_bits(mask, 0, 20);
    if ((u >> 52) != (mk >> 8)) {
        append_bits(data_bits, bytes, pos, u >> (52 - m), 12 + m);
        return;
    }
    add_bit_to_bytes(data_bits, bytes, pos, 0);
    append_ones(data_bits, bytes, pos, type);
    if (((u >> 44) & 0xFFu) == (mk & 0xFFu)) {
        add_bit_to_bytes(data_bits, bytes, pos, 0);
        if (m > 8) append_bits(data_bits, bytes, pos, (u >> (52 - m)) & ((1ull << (m - 8)) - 1ull), m - 8);
    } else {
        add_bit_to_bytes(data_bits, bytes, pos, 1);
        if (m > 0) append_bits(data_bits, bytes, pos, (u >> (52 - m)) & ((1ull << m) - 1ull), m);
    }
}

double decompress_bitwise_double_np(char* bits, int bits_num) {
    if (bits_num >= 64) return d_of(str_bits(bits, 0, 64));
    return d_of(with_midpoint(str_bits(bits, 0, bits_num), bits_num, 64));
}

double decompress_bitwise_double(char* bits, int bits_num, double before_value1, double before_value2,
                                 double before_value3) {
    if (bits_num == 3) {
        if (bits[0] != '1') {
            printf("Error start bit of 3 bits is 0\n");
            dc_set_error(DC_ERR_STREAM, "decompress_bitwise_double: a 3-bit token must start with 1 (:2892)");
            return 0.0;
        }
        const int c = (bits[1] == '1') * 2 + (bits[2] == '1');
        if (c == 0) return 0.0;
        if (c == 1) return before_value1;
        if (c == 2) return 2 * before_value1 - before_value2;
        return 3 * before_value1 - 3 * before_value2 + before_value3;
    }
    return decompress_bitwise_double_np(bits, bits_num);
}

double decompress_bitwise_double_mask(char* bits, int bits_num, double before_value1, double before_value2,
                                      double before_value3, int type, char mask[1 + 11 + 8]) {
    if (bits_num == 3 && bits[0] == '1') {
        const int c = (bits[1] == '1') * 2 + (bits[2] == '1');
        if (c == 0) return 0.0;
        if (c == 1) return before_value1;
        if (c == 2) return 2 * before_value1 - before_value2;
        return 3 * before_value1 - 3 * before_value2 + before_value3;
    }
    if (bits_num == 64) return d_of(str_bits(bits, 0, 64));
    int masked = 1;
    for (int n = 1; n < type + 1; n++)
        if (bits[n] != '1') { masked = 0; break; }
    if (!masked) return decompress_bitwise_double_np(bits, bits_num);
    return d_of(masked_pattern(bits, bits_num, type, mask, 20, 12, 64));
}

/* :5232-5242 (digits 0/1, not chars).  The reference reads the double through an int* and tests
 * (*f) & (1 << (63-i)); as it compiles on x86-64 (shift counts taken mod 32) the 64 digits are the low
 * 32-bit word twice, which the ratio estimators (c:5024, :5110, :5180) then read. */
void getDoubleBin(double num, char bin[]) {
    uint64_t c;
    memcpy(&c, &num, 8);
    const uint32_t lo = (uint32_t)c;
    for (int i = 0; i < 64; i++) bin[i] = (char)((lo >> (31 - (i & 31))) & 1u);
}

/* ---- character-level Hamming SECDED (:5544-5855) ----------------------------------------------
 * Hamming positions 1..r+k; powers of two hold check bits, the others the data bits in order.  Check
 * bit i covers the data bits whose position has bit i set; c[r] / v[r] is the overall parity. */
static int is_pow2(long long j) { return (j & (j - 1)) == 0; }

static void syndrome_chars(const char* data, int k, int r, int* chk) {
    for (int i = 0; i < r; i++) chk[i] = 0;
    long long j = 1;
    for (int d = 0; d < k; d++, j++) {
        while (is_pow2(j)) j++;
        if (data[d] == '1')
            for (int i = 0; i < r; i++) chk[i] ^= (int)((j >> i) & 1);
    }
}

void hamming_code(char* data, char* c, int k, int r) {                    /* :5544-5579 */
    int chk[64];
    syndrome_chars(data, k, r, chk);
    int sum = 0;
    for (int i = 0; i < r; i++) { c[i] = chk[i] ? '1' : '0'; sum += chk[i]; }
    for (int i = 0; i < k; i++) sum += data[i] - '0';
    c[r] = (char)('0' + sum % 2);
}

void hamming_verify(char* data, char* c, int k, int r, char* v) {        /* :5595-5629 */
    int chk[64];
    syndrome_chars(data, k, r, chk);
    int sum = 0;
    for (int i = 0; i < k; i++) sum += data[i] - '0';
    for (int i = 0; i < r; i++) { v[i] = chk[i] == c[i] - '0' ? '0' : '1'; sum += c[i] - '0'; }
    v[r] = sum % 2 == c[r] - '0' ? '0' : '1';
}

int error_info(char* v, int r, int* error_bit_pos) {                     /* :5631-5654 (adds to *pos) */
    for (int i = 0; i < r; i++) *error_bit_pos += (v[i] - '0') << i;
    if (*error_bit_pos > 0 && v[r] == '0') return 1;                      /* two-bit error */
    if (*error_bit_pos == 0 && v[r] == '1') return 2;                     /* parity bit */
    if (*error_bit_pos > 0 && v[r] == '1') return 3;                      /* one bit */
    return 0;
}

void hamming_print(char* data, char* c, int k, int r) {                  /* :5656-5676 */
    int dnum = 0, cnum = 0;
    for (long long j = 1; j < (long long)r + k + 1; j++) {
        if (is_pow2(j)) printf("%c", c[cnum++]);
        else printf("%c", data[dnum++]);
    }
    printf(" %c\n", c[r]);
}

/* flip Hamming position `pos` (:5678-5710 / :5822-5855): a check bit when it is a power of two, else
 * data bit pos - 1 - (number of powers of two below pos); nothing when pos is out of range */
static long long ham_data_index(long long pos, int r, long long k, int* cidx) {
    *cidx = -1;
    if (pos < 1 || pos > (long long)r + k) return -1;
    if (is_pow2(pos)) {
        int ci = 0;
        while ((1ll << ci) != pos) ci++;
        *cidx = ci;
        return -1;
    }
    long long npow = 0;
    while ((1ll << npow) < pos) npow++;
    return pos - 1 - npow;
}

void hamming_rectify(char* data, char* c, int k, int r, int error_bit_pos) {
    int ci;
    const long long d = ham_data_index(error_bit_pos, r, k, &ci);
    if (ci >= 0) c[ci] = c[ci] == '0' ? '1' : '0';
    else if (d >= 0) data[d] = data[d] == '0' ? '1' : '0';
}

void cast_bits_to_char(unsigned char* bits, char* data, int bytes) {     /* :5712-5723 */
    for (int i = 0; i < bytes; i++)
        for (int j = 0; j < 8; j++) data[i * 8 + j] = (char)(((bits[i] >> (7 - j)) & 1) + '0');
}

/* hamming_verify_bit (:5781-5820): the byte-stream form of hamming_verify; the syndrome of a long block
 * is the XOR of the positions of its 1-bits, which the GPU computes (ham_syndrome in dc_host.c) -- here
 * a host loop, since this entry takes the caller's check string and returns the verdict string */
void hamming_verify_bit(unsigned char* bits, char* c, int bytes, int r, char* v) {
    unsigned long long syn = 0;
    long long ones = 0, j = 1;
    const long long k = (long long)bytes * 8;
    for (long long d = 0; d < k; d++, j++) {
        while (is_pow2(j)) j++;
        if ((bits[d >> 3] >> (7 - (d & 7))) & 1) { syn ^= (unsigned long long)j; ones++; }
    }
    long long sum = ones;
    for (int i = 0; i < r; i++) {
        v[i] = (int)((syn >> i) & 1) == c[i] - '0' ? '0' : '1';
        sum += c[i] - '0';
    }
    v[r] = sum % 2 == c[r] - '0' ? '0' : '1';
}

void hamming_rectify_bit(unsigned char* bits, char* c, int bytes, int r, int error_bit_pos) {   /* :5822-5855 */
    int ci;
    const long long d = ham_data_index(error_bit_pos, r, (long long)bytes * 8, &ci);
    if (ci >= 0) c[ci] = c[ci] == '0' ? '1' : '0';
    else if (d >= 0) bits[d >> 3] ^= (unsigned char)(1u << (7 - (d & 7)));
}

/* ---- binary readers (:5341-5381); the reference exit(0)s when the file cannot be opened -------- */
static void* read_array(const char* file, size_t sz, int count) {
    FILE* fp = fopen(file, "rb");
    if (!fp) {
        printf("failed to open %s\n", file);
        dc_set_error(DC_ERR_ARG, "cannot open the binary file");
        return NULL;
    }
    void* arr = malloc(sz * (size_t)(count > 0 ? count : 1));
    if (arr && count > 0 && fread(arr, sz, (size_t)count, fp) != (size_t)count) { /* short file: as fread leaves it */ }
    fclose(fp);
    return arr;
}
float* readfrombinary_float(const char* file, int count) { return (float*)read_array(file, sizeof(float), count); }
double* readfrombinary_double(const char* file, int count) { return (double*)read_array(file, sizeof(double), count); }
