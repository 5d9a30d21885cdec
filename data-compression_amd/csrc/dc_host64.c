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

#include "../../include/dc_gpu.h"

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

static void fail(const char* fn, int rc) { fprintf(stderr, "libdcamd: %s failed (%d): %s\n", fn, rc, dc_last_error()); }

static uint32_t mask20_from_chars(const char* mask) {
    uint32_t m = 0;
    for (int i = 0; i < 20; i++) m = (m << 1) | (uint32_t)(mask[i] == '1');
    return m;
}

static int compress64(const char* fn, int ct, const double* data, int num, unsigned char** data_bits, int* bytes,
                      int* pos, int type, uint32_t mask20) {
    int rc = dc_init(0);
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
    double* out = (double*)malloc(sizeof(double) * (size_t)(num > 0 ? num : 1));
    int rc = dc_init(0);
    if (rc) { fail(fn, rc); return out; }
    if (num <= 0 || bytes <= 0) return out;
    const hipStream_t st = (hipStream_t)dc_get_stream();
    if ((rc = grow(&g_a, &g_a_cap, (size_t)bytes + 64)) || (rc = grow(&g_b, &g_b_cap, (size_t)num * 8 + 64))) {
        fail(fn, rc); return out;
    }
    if (hipMemcpyAsync(g_a, data_bits, (size_t)bytes, hipMemcpyHostToDevice, st) != hipSuccess) { fail(fn, DC_ERR_HIP); return out; }
    if ((rc = dc64_decode_device(ct, g_a, bytes, NULL, bytes, num, type, mask20, g_b)) || (rc = dc64_decode_finish()))
        fail(fn, rc);
    if (hipMemcpy(out, g_b, (size_t)num * 8, hipMemcpyDeviceToHost) != hipSuccess) fail(fn, DC_ERR_HIP);
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
