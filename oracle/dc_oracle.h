/*
 * dc_oracle.h -- CPU restatement of the reference float codecs (TEST INFRASTRUCTURE ONLY).
 *
 * This header and dc_oracle.c are the parity oracle for the MI355X build.  They are
 * linked/loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
 * always as the checker, never as the thing measured or shipped.  The product library
 * (data-compression_amd/) never includes or links this code.
 *
 * Every function restates an algorithm of the reference
 * (smallcat9603/data-compression, impl/dataCompression.c) and cites the lines it follows.
 * Parity is pinned by the reference's own committed KATs (impl/dataset/testfloat_8_8_128.txt.bc,
 * tools/float_eq_*.txt.bc) and by golden vectors produced by the compiled reference
 * (oracle/build_ref.sh -> oracle/_ref/, fixtures in tests/golden/, generator tests/golden/make_golden.py).
 */
#ifndef DC_ORACLE_H
#define DC_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* to_absErrorBound_binary (dataCompression.c:5512-5522): smallest n>=0 with bound >= 2^-n. */
int orc_bound_binary(double bound);
/* largest float f with (double)f < bound  -- the `fabs(x) < absErrorBound` test (:2044) */
float orc_thr_lt(double bound);
/* largest float f with (double)f <= bound -- the `diff_min <= absErrorBound` test (:2106) */
float orc_thr_le(double bound);

/* toSmallDataset_float (:3543-3562): out[i] = data[i]-min, returns min. */
float orc_to_small(const float* data, long n, float* out);
/* med_dataset_float (:3593-3620): sequential float sum / (float)n, type from max. */
float orc_med(const float* data, long n, int* type);
/* first 17 chars of floattostr(mean) (pingpong.c:202-206) as the top 17 bits of the pattern */
uint32_t orc_mask17(float mean);

/*
 * Bit-wise encoders.  ct = 5 (myCompress_bitwise :3310), 6 (myCompress_bitwise_np :2645),
 * 7 (myCompress_bitwise_mask :2030), 11 (myCompress_bitwise_op :577).
 * Append semantics identical to add_bit_to_bytes (:5456): bits is realloc'ed, bytes and pos updated.
 * type/mask17 are only used by ct 7.
 */
void orc_compress(int ct, const float* data, long num, double bound, int type, uint32_t mask17,
                  unsigned char** bits, int* bytes, int* pos);

/* Token grammar decoder (spec of SURVEY 8.0).  Decodes min(num, tokens present) elements
 * into out, returns the number decoded. */
long orc_decompress_spec(int ct, const unsigned char* bits, long bytes, long num, double bound,
                         int type, uint32_t mask17, float* out);

/* Faithful restatement of the reference decoder state machines (myDecompress_bitwise :2922,
 * myDecompress_bitwise_np :2459, myDecompress_bitwise_mask :1703, myDecompress_bitwise_op :698),
 * including their quirks.  Writes only the elements the reference writes; returns
 * decompressed_num (capped at num), sets *stuck if the machine stopped emitting (Q1). */
long orc_decompress_cref(int ct, const unsigned char* bits, long bytes, long num, double bound,
                         int type, uint32_t mask17, float* out, int* stuck);

/* CT1 byte-wise codec: myCompress (:3980-4118) / myDecompress (:3943-3977).
 * raw must hold num floats, codes/pos num entries.  Returns array_float_len. */
int orc_bytewise_compress(const float* data, int num, double bound, float* raw, char* codes, int* pos1);
void orc_bytewise_decompress(const float* raw, const char* codes, const int* pos1, int ncodes,
                             int num, float* out);

/* do_crc32 (:5524-5534) == zlib crc32 == CRC-32/ISO-HDLC. */
uint32_t orc_crc32(const unsigned char* p, long n);
uint32_t orc_crc32_update(uint32_t crc, const unsigned char* p, long n);

/* Hamming SECDED (:5544-5855). hmLength, hamming_encode (c has r+1 chars '0'/'1'),
 * hamming_decode (returns error type 0..3, corrects in place like the reference). */
int orc_hm_length(long k);
void orc_hamming_encode(const unsigned char* bits, long bytes, int* r, char* c);
int orc_hamming_decode(unsigned char* bits, char* c, long bytes, int r, long* err_pos);
/* block_size (:5868-5879) for a given BER */
int orc_block_size(int data_bytes, double ber);

/* ---- double codecs (dc_oracle64.c): myCompress_bitwise_double :3189 (ct 5), _np :2633 (6),
 * _mask :1590 (7), _op :355 (11); grammar decoder of myDecompress_bitwise_double :2656 / _np :2286 /
 * _mask :1199 / _op :476.  mask20 = the top 20 bits of the mean's pattern (char mask[1+11+8]). */
int orc64_mbits(int B, int E);
double orc64_to_small(const double* data, long n, double* out);   /* toSmallDataset_double :3522 */
double orc64_med(const double* data, long n, int* type);          /* med_dataset_double :3564 */
uint32_t orc64_mask20(double mean);
void orc64_compress(int ct, const double* data, long num, double bound, int type, uint32_t mask20,
                    unsigned char** bits, int* bytes, int* pos);
long orc64_decompress_spec(int ct, const unsigned char* bits, long bytes, long num, double bound,
                           int type, uint32_t mask20, double* out);
void orc64_gen_u10(double* out, long n, uint64_t seed, long offset);
int orc64_bytewise_compress(const double* data, int num, double bound, double* raw, char* codes, int* pos1);
void orc64_bytewise_decompress(const double* raw, const char* codes, const int* pos1, int ncodes, int num, double* out);
long orc64_chunk_records(int ct, const unsigned char* s, long bytes, long num, double bound, int type,
                         uint32_t mask20, long cb, unsigned char* ent, unsigned char* ex, unsigned short* cnt);

/* Synthetic inputs: U10 counter-based splitmix64, HIMENO-L plane. */
void orc_gen_u10(float* out, long n, uint64_t seed, long offset);
void orc_gen_himeno_plane(float* out, int imax, int jmax);

#ifdef __cplusplus
}
#endif
#endif
