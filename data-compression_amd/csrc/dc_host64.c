/*
 * dc_host64.c -- the reference's DOUBLE codec ABI (impl/dataCompression.h:63-98) on the gfx950
 * kernels of dc_f64.hip: host buffers in, host malloc() buffers out, append semantics of
 * add_bit_to_bytes (:5456-5489).  No CPU codec path: every call runs on the GPU or reports an error.
 */
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dc_shared.h"
#include "../../include/dc_gpu.h"

int dc_set_error(int code, const char* msg);
void dc_abi_set_status(int rc);

/* device staging buffers of this file */
static void* g_a; static size_t g_a_cap;
static void* g_b; static size_t g_b_cap;

static int grow(void** p, size_t* cap, size_t need) {
    if (need <= *cap) return DC_OK;
    if (*p) (void)hipFree(*p);
    *p = NULL; *cap = 0;
    if (hipMalloc(p, need) != hipSuccess) return DC_ERR_HIP;
    *cap = need;
    return DC_OK;
}

static void fail(const char* fn, int rc) {
    dc_abi_set_status(rc);
    fprintf(stderr, "libdcamd: %s failed (%d): %s\n", fn, rc, dc_last_error());
}

static uint32_t mask20_from_chars(const char* mask) {
    uint32_t m = 0;
    for (int i = 0; i < 20; i++) m = (m << 1) | (uint32_t)(mask[i] == '1');
    return m;
}

static int compress64(const char* fn, int ct, const double* data, int num, unsigned char** data_bits, int* bytes,
                      int* pos, int type, uint32_t mask20) {
    int rc = dc_init(0);
    dc_abi_set_status(DC_OK);
    if (rc) { fail(fn, rc); return rc; }
    if (num <= 0) return DC_OK;
    const long long used = (long long)(*bytes) * 8 - (*pos == 8 ? 0 : *pos);
    const int sb = (int)(used & 7);
    const long long keep = used >> 3;
    const hipStream_t st = (hipStream_t)dc_get_stream();
    if ((rc = grow(&g_a, &g_a_cap, (size_t)num * 8 + 64)) || (rc = grow(&g_b, &g_b_cap, dc64_stream_capacity(num)))) {
        fail(fn, rc); return rc;
    }
    if (hipMemcpyAsync(g_a, data, (size_t)num * 8, hipMemcpyHostToDevice, st) != hipSuccess) { fail(fn, DC_ERR_HIP); return DC_ERR_HIP; }
    unsigned long long tb = 0;
    if ((rc = dc64_encode_device(ct, g_a, num, type, mask20, sb, g_b, NULL)) || (rc = dc64_encode_result(&tb))) {
        fail(fn, rc); return rc;
    }
    const long long nb_new = (long long)((sb + tb + 7) >> 3);
    const long long total = keep + nb_new;
    const unsigned char old = sb ? (unsigned char)((*data_bits)[keep] & (0xFFu << (8 - sb))) : 0;
    unsigned char* nb = (unsigned char*)realloc(*data_bits, total > 0 ? (size_t)total : 1);
    if (!nb) { fail(fn, DC_ERR_ARG); return DC_ERR_ARG; }
    *data_bits = nb;
    if (hipMemcpy(nb + keep, g_b, (size_t)nb_new, hipMemcpyDeviceToHost) != hipSuccess) { fail(fn, DC_ERR_HIP); return DC_ERR_HIP; }
    if (sb) nb[keep] |= old;
    const long long tot_bits = keep * 8 + sb + (long long)tb;
    *bytes = (int)total;
    *pos = (tot_bits & 7) ? (int)(8 - (tot_bits & 7)) : 8;
    return DC_OK;
}

static double* decompress64(const char* fn, int ct, const unsigned char* data_bits, int bytes, int num, int type,
                            uint32_t mask20) {
    /* on an error the result is all zeros and dc_abi_status() reports it */
    const size_t osz = sizeof(double) * (size_t)(num > 0 ? num : 1);
    double* out = (double*)malloc(osz);
    int rc = dc_init(0);
    dc_abi_set_status(DC_OK);
    if (!out) { fail(fn, DC_ERR_ARG); return out; }
    memset(out, 0, osz);
    if (rc) { fail(fn, rc); return out; }
    if (num <= 0 || bytes <= 0) return out;
    const hipStream_t st = (hipStream_t)dc_get_stream();
    if ((rc = grow(&g_a, &g_a_cap, (size_t)bytes + 64)) || (rc = grow(&g_b, &g_b_cap, (size_t)num * 8 + 64))) {
        fail(fn, rc); return out;
    }
    if (hipMemcpyAsync(g_a, data_bits, (size_t)bytes, hipMemcpyHostToDevice, st) != hipSuccess) { fail(fn, DC_ERR_HIP); return out; }
    if ((rc = dc64_decode_device(ct, g_a, bytes, NULL, bytes, num, type, mask20, g_b)) || (rc = dc64_decode_finish())) {
        fail(fn, rc); return out;
    }
    if (hipMemcpy(out, g_b, (size_t)num * 8, hipMemcpyDeviceToHost) != hipSuccess) { fail(fn, DC_ERR_HIP); memset(out, 0, osz); }
    return out;
}

/* myCompress_bitwise_double (:3189), _np (:2633), _op (:355), _mask (:1590) */
void myCompress_bitwise_double(double data[], int num, unsigned char** data_bits, int* bytes, int* pos) {
    compress64("myCompress_bitwise_double", 5, data, num, data_bits, bytes, pos, 0, 0);
}
void myCompress_bitwise_double_np(double data[], int num, unsigned char** data_bits, int* bytes, int* pos) {
    compress64("myCompress_bitwise_double_np", 6, data, num, data_bits, bytes, pos, 0, 0);
}
void myCompress_bitwise_double_op(double data[], int num, unsigned char** data_bits, int* bytes, int* pos) {
    compress64("myCompress_bitwise_double_op", 11, data, num, data_bits, bytes, pos, 0, 0);
}
void myCompress_bitwise_double_mask(double data[], int num, unsigned char** data_bits, int* bytes, int* pos, int type,
                                    char mask[1 + 11 + 8]) {
    compress64("myCompress_bitwise_double_mask", 7, data, num, data_bits, bytes, pos, type, mask20_from_chars(mask));
}

/* myDecompress_bitwise_double (:2656), _np (:2286), _op (:476), _mask (:1199) */
double* myDecompress_bitwise_double(unsigned char* data_bits, int bytes, int num) {
    return decompress64("myDecompress_bitwise_double", 5, data_bits, bytes, num, 0, 0);
}
double* myDecompress_bitwise_double_np(unsigned char* data_bits, int bytes, int num) {
    return decompress64("myDecompress_bitwise_double_np", 6, data_bits, bytes, num, 0, 0);
}
double* myDecompress_bitwise_double_op(unsigned char* data_bits, int bytes, int num) {
    return decompress64("myDecompress_bitwise_double_op", 11, data_bits, bytes, num, 0, 0);
}
double* myDecompress_bitwise_double_mask(unsigned char* data_bits, int bytes, int num, int type, char mask[1 + 11 + 8]) {
    return decompress64("myDecompress_bitwise_double_mask", 7, data_bits, bytes, num, type, mask20_from_chars(mask));
}

/* toSmallDataset_double (:3522-3541): min reduce + subtract on the GPU */
double toSmallDataset_double(double data[], double** data_small, int num) {
    *data_small = (double*)malloc(sizeof(double) * (size_t)(num > 0 ? num : 1));
    if (num <= 0) return 0.0;
    int rc = dc_init(0);
    double mn = 0.0;
    if (rc || (rc = grow(&g_a, &g_a_cap, (size_t)num * 8 + 64)) || (rc = grow(&g_b, &g_b_cap, (size_t)num * 8 + 64))) {
        fail("toSmallDataset_double", rc); return mn;
    }
    const hipStream_t st = (hipStream_t)dc_get_stream();
    if (hipMemcpyAsync(g_a, data, (size_t)num * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
        (rc = dc64_to_small_device(g_a, num, g_b, &mn)) ||
        hipMemcpy(*data_small, g_b, (size_t)num * 8, hipMemcpyDeviceToHost) != hipSuccess)
        fail("toSmallDataset_double", rc ? rc : DC_ERR_HIP);
    return mn;
}

/* med_dataset_double (:3564-3590): sequential double sum, max, type on the GPU */
double med_dataset_double(double* data, int num, int* type) {
    double mean = 0.0;
    int rc = dc_init(0);
    if (num <= 0) return mean;
    if (rc || (rc = grow(&g_a, &g_a_cap, (size_t)num * 8 + 64))) { fail("med_dataset_double", rc); return mean; }
    const hipStream_t st = (hipStream_t)dc_get_stream();
    if (hipMemcpyAsync(g_a, data, (size_t)num * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
        (rc = dc64_med_device(g_a, num, &mean, type)))
        fail("med_dataset_double", rc ? rc : DC_ERR_HIP);
    return mean;
}

/* ---- CT1 byte-wise codec for doubles (myCompress_double :3815-3941 / myDecompress_double :3778-3813) */
static void* c_scr; static size_t c_scr_cap;
static void* c_codes; static size_t c_codes_cap;
static void* c_pos; static size_t c_pos_cap;
static unsigned* c_err;

static int c1_setup(long long n, uint32_t** traw, unsigned long long** rawoff, uint8_t** carr) {
    const long long nt = dc_ct1_tiles(n > 0 ? n : 1);
    const size_t need = (size_t)(nt + 1) * 8 + (size_t)nt * 4 + 16 + (size_t)n + 64;
    if (grow(&c_scr, &c_scr_cap, need)) return DC_ERR_HIP;
    if (!c_err && hipMalloc((void**)&c_err, 64) != hipSuccess) return DC_ERR_HIP;
    char* p = (char*)c_scr;
    *rawoff = (unsigned long long*)p;
    *traw = (uint32_t*)(p + (size_t)(nt + 1) * 8);
    *carr = (uint8_t*)(p + (size_t)(nt + 1) * 8 + (size_t)nt * 4 + 16);
    return DC_OK;
}

/* h:122 c:3815-3941: *array_double / *array_char / *array_char_displacement realloc()ed to the raw and
 * code counts (untouched when a count is 0, as the reference); returns the raw count */
int myCompress_double(double data[], double** array_double, char** array_char, int** array_char_displacement, int num) {
    const char* fn = "myCompress_double";
    int rc = dc_init(0);
    if (rc) { fail(fn, rc); return 0; }
    if (num <= 0) return 0;
    const size_t n = (size_t)num;
    const hipStream_t st = (hipStream_t)dc_get_stream();
    uint32_t* traw; unsigned long long* rawoff; uint8_t* carr;
    if ((rc = grow(&g_a, &g_a_cap, n * 8 + 64)) || (rc = grow(&g_b, &g_b_cap, n * 8 + 64)) ||
        (rc = grow(&c_codes, &c_codes_cap, n + 64)) || (rc = grow(&c_pos, &c_pos_cap, n * 4 + 64)) ||
        (rc = c1_setup(num, &traw, &rawoff, &carr))) { fail(fn, rc); return 0; }
    unsigned long long h[2] = {0, 0};
    const long long nt = dc_ct1_tiles(num);
    if (hipMemcpyAsync(g_a, data, n * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemsetAsync(c_err, 0, 4, st) != hipSuccess ||
        dc_launch_ct1_encode64((const double*)g_a, num, dc_get_abs_error_bound(), traw, rawoff, (double*)g_b,
                               (char*)c_codes, (int*)c_pos, c_err, st) ||
        hipMemcpyAsync(&h[0], rawoff + nt, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(&h[1], c_err, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) { fail(fn, DC_ERR_HIP); return 0; }
    if (h[1] & 1u) { fail(fn, dc_set_error(DC_ERR_INPUT, "input contains -1.0 (the reference's history sentinel)")); return 0; }
    const long long nraw = (long long)h[0], nc = num - nraw;
    if (nraw > 0) {
        double* a = (double*)realloc(*array_double, sizeof(double) * (size_t)nraw);
        if (!a) { fail(fn, DC_ERR_ARG); return 0; }
        *array_double = a;
        if (hipMemcpy(a, g_b, sizeof(double) * (size_t)nraw, hipMemcpyDeviceToHost) != hipSuccess) { fail(fn, DC_ERR_HIP); return 0; }
    }
    if (nc > 0) {
        char* c = (char*)realloc(*array_char, (size_t)nc);
        int* p = (int*)realloc(*array_char_displacement, sizeof(int) * (size_t)nc);
        if (!c || !p) { fail(fn, DC_ERR_ARG); return 0; }
        *array_char = c;
        *array_char_displacement = p;
        if (hipMemcpy(c, c_codes, (size_t)nc, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(p, c_pos, sizeof(int) * (size_t)nc, hipMemcpyDeviceToHost) != hipSuccess) { fail(fn, DC_ERR_HIP); return 0; }
    }
    return (int)nraw;
}

/* h:123 c:3778-3813; the code count is taken as in myDecompress (dc_host.c): entries while they increase
 * and stay within [1, num] */
double* myDecompress_double(double array_double[], char array_char[], int array_char_displacement[], int num) {
    const char* fn = "myDecompress_double";
    double* out = (double*)malloc(sizeof(double) * (size_t)(num > 0 ? num : 1));
    int rc = dc_init(0);
    if (rc) { fail(fn, rc); return out; }
    if (num <= 0) return out;
    long long nc = 0;
    if (array_char_displacement) {
        int prev = 0;
        while (nc < num && array_char_displacement[nc] > prev && array_char_displacement[nc] <= num) {
            prev = array_char_displacement[nc];
            nc++;
        }
    }
    const long long nraw = num - nc;
    const size_t n = (size_t)num;
    const hipStream_t st = (hipStream_t)dc_get_stream();
    uint32_t* traw; unsigned long long* rawoff; uint8_t* carr;
    if ((rc = grow(&g_a, &g_a_cap, n * 8 + 64)) || (rc = grow(&g_b, &g_b_cap, n * 8 + 64)) ||
        (rc = grow(&c_codes, &c_codes_cap, n + 64)) || (rc = grow(&c_pos, &c_pos_cap, n * 4 + 64)) ||
        (rc = c1_setup(num, &traw, &rawoff, &carr))) { fail(fn, rc); return out; }
    unsigned h = 0;
    if ((nraw > 0 && hipMemcpyAsync(g_a, array_double, sizeof(double) * (size_t)nraw, hipMemcpyHostToDevice, st) != hipSuccess) ||
        (nc > 0 && hipMemcpyAsync(c_codes, array_char, (size_t)nc, hipMemcpyHostToDevice, st) != hipSuccess) ||
        (nc > 0 && hipMemcpyAsync(c_pos, array_char_displacement, sizeof(int) * (size_t)nc, hipMemcpyHostToDevice, st) != hipSuccess) ||
        hipMemsetAsync(c_err, 0, 4, st) != hipSuccess ||
        dc_launch_ct1_decode64((const double*)g_a, nraw, (const char*)c_codes, (const int*)c_pos, nc, num, carr, traw,
                               rawoff, (double*)g_b, c_err, st) ||
        hipMemcpyAsync(&h, c_err, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) { fail(fn, DC_ERR_HIP); return out; }
    if (h & 4u) fail(fn, dc_set_error(DC_ERR_STREAM, "ct1 codes out of range or raw array too short"));
    if (hipMemcpy(out, g_b, sizeof(double) * n, hipMemcpyDeviceToHost) != hipSuccess) fail(fn, DC_ERR_HIP);
    return out;
}

/* ---- double file helpers of the k-means / mm / lu link closure */
void writetobinary_double(const char* file, double* data, int count) {          /* :5307-5322 */
    FILE* fp = fopen(file, "wb");
    if (!fp) { printf("failed to open %s\n", file); return; }
    fwrite(data, sizeof(double), (size_t)(count > 0 ? count : 0), fp);
    fclose(fp);
    printf("saved %s\n", file);
}

double* readfrombinary_writetotxt_double(const char* binaryfile, const char* txtfile, int count) {   /* :5434-5454 */
    FILE* fp = fopen(binaryfile, "rb");
    if (!fp) { dc_set_error(DC_ERR_ARG, "cannot open the binary file"); return NULL; }
    double* arr = (double*)malloc(sizeof(double) * (size_t)(count > 0 ? count : 1));
    size_t got = arr ? fread(arr, sizeof(double), (size_t)(count > 0 ? count : 0), fp) : 0;
    fclose(fp);
    (void)got;
    fp = fopen(txtfile, "w");
    if (!fp) { dc_set_error(DC_ERR_ARG, "cannot open the text file"); return arr; }
    for (int i = 0; i < count; i++) fprintf(fp, "%lf\n", arr[i]);
    fclose(fp);
    return arr;
}
