/*
 * dataCompression.h -- drop-in C ABI of libdcamd for the float bit-wise codec path of
 * smallcat9603/data-compression (impl/dataCompression.h / impl/dataCompression.c).
 *
 * Every declaration below has the reference's name, argument order, argument meaning and ownership
 * rules; the line numbers cite the reference declaration (impl/dataCompression.h) and definition
 * (impl/dataCompression.c) it replaces.  The compute runs on an MI355X (gfx950) behind these
 * host-pointer entry points; the device-pointer API is in dc_gpu.h.
 *
 * Ownership (as in the reference): *data_bits is realloc()ed by the callee (pass NULL, bytes = 0,
 * pos = 8 for a new stream; a non-empty stream is appended to); returned float* / *data_small /
 * hamming check strings are malloc()ed host memory owned by the caller.
 * Errors: the reference printf()s and exit()s on malformed streams (c:2503, :1775, :3162); this
 * library prints the reason to stderr (also dc_last_error(), dc_gpu.h) and returns instead: a failed
 * compress leaves *data_bits / *bytes / *pos untouched, a failed decompress returns its malloc()ed
 * buffer with unspecified contents.  There is no CPU fallback: a missing gfx950 device is such an
 * error.
 * absErrorBound: the reference bakes the bound in at compile time (#define absErrorBound, :3).  The
 * library is built with -DDC_ABS_ERROR_BOUND=<value> (default 1e-6, the reference header's value) and
 * exports the reference's globals absErrBound / absErrorBound_binary (impl/dataCompression.c:21-22);
 * dc_set_abs_error_bound() (dc_gpu.h) changes it at run time.
 */
#ifndef DC_DATACOMPRESSION_H
#define DC_DATACOMPRESSION_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- application configuration macros of the reference header (impl/dataCompression.h:4-41): the
 *      apps (pingpong.c, himenoBMTxps.c) read them; each can be overridden with -D.  absErrorBound
 *      must equal the bound libdcamd was built with (make BOUND=...). ------------------------------ */
#ifndef BER
#define BER 1e-6
#endif
#ifndef absErrorBound
#define absErrorBound 0.000001
#endif
#ifndef byte_or_bit
#define byte_or_bit 2
#endif
#ifndef filename
#define filename "dataset/testfloat_8_8_128"
#endif
#ifndef suffix
#define suffix ".txt"
#endif
#ifndef output_suffix
#define output_suffix "_output_"
#endif
#ifndef clusters
#define clusters 100
#endif
#define bin_suffix ".dat"
#define sz_suffix ".sz"
#define zs_suffix ".zs"
#define out_suffix ".out"
#define sz_comp_cmd_prefix "./sz -z -f -c sz.config -M ABS -A "
#define sz_comp_cmd_prefix_double "./sz -z -d -c sz.config -M ABS -A "
#define sz_comp_cmd_suffix1 " -i "
#define sz_comp_cmd_suffix2 ".dat -1 "
#define sz_decomp_cmd_prefix "./sz -x -f -s "
#define sz_decomp_cmd_prefix_double "./sz -x -d -s "
#define sz_decomp_cmd_suffix ".dat.zs -1 "

extern double absErrBound;            /* impl/dataCompression.c:21 */
extern int absErrorBound_binary;      /* impl/dataCompression.c:22 */

/* ---- CT5: zero / 3-predictor / raw tokens ------------------------------------------------------ */
/* h:90  c:3310-3444 */
void myCompress_bitwise(float data[], int num, unsigned char** data_bits, int* bytes, int* pos);
/* h:86  c:2922-3135 */
float* myDecompress_bitwise(unsigned char* data_bits, int bytes, int num);

/* ---- CT6: raw tokens only (no prediction) ------------------------------------------------------ */
/* h:77  c:2645-2654 */
void myCompress_bitwise_np(float data[], int num, unsigned char** data_bits, int* bytes, int* pos);
/* h:74  c:2459-2609 */
float* myDecompress_bitwise_np(unsigned char* data_bits, int bytes, int num);

/* ---- CT11: 3-bit codes or verbatim 32-bit floats ----------------------------------------------- */
/* h:81  c:577-696 */
void myCompress_bitwise_op(float data[], int num, unsigned char** data_bits, int* bytes, int* pos);
/* h:82  c:698-797 */
float* myDecompress_bitwise_op(unsigned char* data_bits, int bytes, int num);

/* ---- CT7 (and the CT9 payload): bitmask-based tokens; mask = 17 '0'/'1' chars (sign, exponent,
 *      8 mantissa bits of the dataset mean), type from med_dataset_float ------------------------- */
/* h:70  c:2030-2141 */
void myCompress_bitwise_mask(float data[], int num, unsigned char** data_bits, int* bytes, int* pos, int type,
                             char mask[1 + 8 + 8]);
/* h:67  c:1703-1898 */
float* myDecompress_bitwise_mask(unsigned char* data_bits, int bytes, int num, int type, char mask[1 + 8 + 8]);

/* ---- CT1: byte-wise 4-predictor split into raw floats + ('a'..'d', 1-based position) codes ----- */
/* h:120 c:3980-4118: *array_float, *array_char, *array_char_displacement realloc()ed; returns the raw count */
int myCompress(float data[], float** array_float, char** array_char, int** array_char_displacement, int num);
/* h:121 c:3943-3977 */
float* myDecompress(float array_float[], char array_char[], int array_char_displacement[], int num);

/* ---- double bit-wise codecs (k-means / mm / lu payloads), same shapes as the float ones --------- */
/* h:89  c:3189-3308 */
void myCompress_bitwise_double(double data[], int num, unsigned char** data_bits, int* bytes, int* pos);
/* h:76  c:2633-2643 */
void myCompress_bitwise_double_np(double data[], int num, unsigned char** data_bits, int* bytes, int* pos);
/* h:79  c:355-475 */
void myCompress_bitwise_double_op(double data[], int num, unsigned char** data_bits, int* bytes, int* pos);
/* h:66  c:1590-1701: mask = the first 1+11+8 chars of doubletostr(mean) */
void myCompress_bitwise_double_mask(double data[], int num, unsigned char** data_bits, int* bytes, int* pos, int type,
                                    char mask[1 + 11 + 8]);
/* h:84  c:2656-2869 */
double* myDecompress_bitwise_double(unsigned char* data_bits, int bytes, int num);
/* h:72  c:2286-2457 */
double* myDecompress_bitwise_double_np(unsigned char* data_bits, int bytes, int num);
/* h:80  c:476-575 */
double* myDecompress_bitwise_double_op(unsigned char* data_bits, int bytes, int num);
/* h:63  c:1199-1394 */
double* myDecompress_bitwise_double_mask(unsigned char* data_bits, int bytes, int num, int type, char mask[1 + 11 + 8]);
/* h:95  c:3522-3541 */
double toSmallDataset_double(double data[], double** data_small, int num);
/* h:98  c:3564-3590: left-to-right double mean; *type from the maximum */
double med_dataset_double(double* data, int num, int* type);

/* h:122 c:3815-3941: CT1 byte-wise for doubles */
int myCompress_double(double data[], double** array_double, char** array_char, int** array_char_displacement, int num);
/* h:123 c:3778-3813 */
double* myDecompress_double(double array_double[], char array_char[], int array_char_displacement[], int num);
/* h:130 c:5307 */
void writetobinary_double(const char* file, double* data, int count);
/* h:136 c:5434: count doubles from binaryfile, also written to txtfile as "%lf\n" */
double* readfrombinary_writetotxt_double(const char* binaryfile, const char* txtfile, int count);

/* ---- pre-passes ---------------------------------------------------------------------------------- */
/* h:96  c:3543-3562: *data_small = data - min (new malloc array), returns min */
float toSmallDataset_float(float data[], float** data_small, int num);
/* h:99  c:3593-3620: left-to-right float mean; *type from the maximum */
float med_dataset_float(float* data, int num, int* type);

/* ---- integrity (CT8/CT9: CRC-32, CT10: Hamming SECDED per block) --------------------------------- */
/* h:143 c:5524-5534 (zlib crc32) */
uint32_t do_crc32(unsigned char* data_bits, int bytes);
/* h:146 c:5581 */
int hmLength(int k);
/* h:153 c:5740-5748: *c = r+1 '0'/'1' chars (check bits + overall parity) */
void hamming_encode(unsigned char* bits, char** c, int bytes, int* r);
/* h:154 c:5750-5779: 0 ok, 1 two-bit error (resend), 2 parity-bit flip, 3 single bit corrected */
int hamming_decode(unsigned char* bits, char* c, int bytes, int r);
/* h:158 c:5868 */
int block_size(int data_bytes);
/* h:157 c:5858 */
void bit_flip(unsigned char* bits, int bytes);
/* h:144 c:5536 */
uint64_t get_random_int(uint64_t from, uint64_t to);

/* ---- helpers the callers link against ------------------------------------------------------------ */
/* h:141 c:5512 */
int to_absErrorBound_binary(double absErrBound);
/* h:117 c:5220 */
void getFloatBin(float f, char bin[]);
/* h:125 c:5244 */
void floattostr(float* f, char* str);
/* h:126 c:5256 */
void doubletostr(double* d, char* str);
/* h:127 c:5267 */
float strtofloat(char* str);
/* h:128 c:5279 */
double strtodbl(char* str);
/* h:138 c:5456 */
void add_bit_to_bytes(unsigned char** data_bits, int* bytes, int* pos, int flag);
/* h:139 c:5492 */
void bit_set(unsigned char* p_data, unsigned char position, int flag);

/* ---- Himeno halo plane extraction and binary file helpers (link closure of pingpong/himenoBMTxps) -
 * The 3-D array extent comes from the app's param.h (MIMAX/MJMAX/MKMAX, impl/param.h:7-9), which the
 * reference compiles into dataCompression.c together with the app; libdcamd is built with the same
 * values (make ... PARAM="-DMIMAX=.. -DMJMAX=.. -DMKMAX=..", default the reference param.h 129/129/131).
 * dc_transform_3d_array_to_1d_array takes the extent explicitly for callers with another param.h. */
#ifndef MIMAX
#define MIMAX 129
#endif
#ifndef MJMAX
#define MJMAX 129
#endif
#ifndef MKMAX
#define MKMAX 131
#endif
/* h:124 c:3741-3775: plane ijk (1: i=v, 2: j=v, 3: k=v) of data as a new malloc()ed array, row-major */
float* transform_3d_array_to_1d_array(float data[MIMAX][MJMAX][MKMAX], int ijk, int v, int imax, int jmax, int kmax);
float* dc_transform_3d_array_to_1d_array(const float* data, int mi, int mj, int mk, int ijk, int v, int imax,
                                         int jmax, int kmax);
/* ---- single-token helpers the serial codecs are built from (host, dc_host_token.c) ---------------
 * compress_*: append one element's raw (or CT7 masked) token to the caller's stream (add_bit_to_bytes
 * semantics); decompress_*: value of one token given as a '0'/'1' string of bits_num chars, with the
 * caller's history for the 3-bit codes.  The caller's string is never realloc()ed. */
/* h:93  c:3479-3520 */
void compress_bitwise_float(float real_value, unsigned char** data_bits, int* bytes, int* pos);
/* h:69  c:2143-2284 */
void compress_bitwise_float_mask(float real_value, unsigned char** data_bits, int* bytes, int* pos, int type,
                                 char mask[1 + 8 + 8]);
/* h:87  c:3137-3186 */
float decompress_bitwise_float(char* bits, int bits_num, float before_value1, float before_value2, float before_value3);
/* h:75  c:2611-2630 */
float decompress_bitwise_float_np(char* bits, int bits_num);
/* h:68  c:1900-2027 */
float decompress_bitwise_float_mask(char* bits, int bits_num, float before_value1, float before_value2,
                                    float before_value3, int type, char mask[1 + 8 + 8]);
/* h:92  c:3446-3477 */
void compress_bitwise_double(double real_value, unsigned char** data_bits, int* bytes, int* pos);
/* h:65  c:1493-1588 */
void compress_bitwise_double_mask(double real_value, unsigned char** data_bits, int* bytes, int* pos, int type,
                                  char mask[1 + 11 + 8]);
/* h:85  c:2871-2920 */
double decompress_bitwise_double(char* bits, int bits_num, double before_value1, double before_value2,
                                 double before_value3);
/* h:73  c:2438-2457 */
double decompress_bitwise_double_np(char* bits, int bits_num);
/* h:64  c:1396-1491 */
double decompress_bitwise_double_mask(char* bits, int bits_num, double before_value1, double before_value2,
                                      double before_value3, int type, char mask[1 + 11 + 8]);
/* h:118 c:5232 */
void getDoubleBin(double num, char bin[]);

/* ---- character-level Hamming SECDED (k data chars, r check chars + overall parity) ---------------- */
/* h:147 c:5544 */
void hamming_code(char* data, char* c, int k, int r);
/* h:148 c:5595: v[i] = '1' where check bit i disagrees, v[r] the overall parity verdict */
void hamming_verify(char* data, char* c, int k, int r, char* v);
/* h:149 c:5631: *error_bit_pos += the syndrome (not initialised, as the reference); 0..3 as hamming_decode */
int error_info(char* v, int r, int* error_bit_pos);
/* h:150 c:5656 */
void hamming_print(char* data, char* c, int k, int r);
/* h:151 c:5678 */
void hamming_rectify(char* data, char* c, int k, int r, int error_bit_pos);
/* h:152 c:5712: 8 '0'/'1' chars per byte, MSB first */
void cast_bits_to_char(unsigned char* bits, char* data, int bytes);
/* h:155 c:5781 */
void hamming_verify_bit(unsigned char* bits, char* c, int bytes, int r, char* v);
/* h:156 c:5822 */
void hamming_rectify_bit(unsigned char* bits, char* c, int bytes, int r, int error_bit_pos);

/* ---- CT2 / CT3 compression-ratio estimators (GPU reductions, dc_ratio.hip): compressed / original bits
 *      of the bit-wise raw tokens, the SZ-style prediction estimate and the lossless residual estimates -- */
/* h:100 c:3702 */
float calCompressRatio_bitwise_float(float data[], int num);
/* h:101 c:3662 */
float calCompressRatio_bitwise_double(double data[], int num);
/* h:102 c:3622: the floats as doubles */
float calCompressRatio_bitwise_double2(float data[], int num);
/* h:103 c:4636 */
float calcCompressionRatio_sz_float(float data[], int num);
/* h:104 c:4928 */
float calcCompressionRatio_sz_double(double data[], int num);
/* h:105 c:4772 */
float calcCompressionRatio_nolossy_performance_float(float data[], int num);
/* h:106 c:5064 */
float calcCompressionRatio_nolossy_performance_double(double data[], int num);
/* h:107 c:4841 */
float calcCompressionRatio_nolossy_area_float(float data[], int num);
/* h:108 c:5133 */
float calcCompressionRatio_nolossy_area_double(double data[], int num);
/* h:109-112 c:4121-4635: the same on plane ijk = v of a Himeno array (transform_3d_array_to_1d_array order) */
float calcCompressionRatio_himeno_ij_ik_jk(float data[MIMAX][MJMAX][MKMAX], int ijk, int v, int imax, int jmax, int kmax);
float calcCompressionRatio_himeno_sz(float data[MIMAX][MJMAX][MKMAX], int ijk, int v, int imax, int jmax, int kmax);
float calcCompressionRatio_himeno_nolossy_performance(float data[MIMAX][MJMAX][MKMAX], int ijk, int v, int imax, int jmax,
                                                       int kmax);
float calcCompressionRatio_himeno_nolossy_area(float data[MIMAX][MJMAX][MKMAX], int ijk, int v, int imax, int jmax, int kmax);

/* h:132 c:5341 (NULL instead of exit(0) when the file cannot be opened) */
float* readfrombinary_float(const char* file, int count);
/* h:133 c:5362 */
double* readfrombinary_double(const char* file, int count);

/* h:129 c:5290 */
void writetobinary_float(const char* file, float* data, int count);
/* h:131 c:5324 */
void writetobinary_char(const char* file, unsigned char* data, int count);
/* h:134 c:5383: whole file, *bytes_sz = its size */
unsigned char* readfrombinary_char(const char* file, int* bytes_sz);
/* h:135 c:5412: count floats from binaryfile, also written to txtfile as "%f\n" */
float* readfrombinary_writetotxt_float(const char* binaryfile, const char* txtfile, int count);

#ifdef __cplusplus
}
#endif
/* the MPI wrappers of libdcamd_mpi.so (the reference header declares them after mpi.h, h:43-61) */
#if defined(MPI_VERSION)
#include "dc_mpi.h"
#endif
#endif
