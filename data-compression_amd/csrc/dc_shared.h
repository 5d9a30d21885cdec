/* dc_shared.h -- plain-C structs and launcher prototypes shared by the C host layer (dc_host.c)
 * and the HIP kernels (dc_encode.hip, dc_decode.hip).  No torch or HIP C++ types. */
#ifndef DC_SHARED_H
#define DC_SHARED_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
namespace dc {
#endif

typedef struct Params {  /* per-call codec parameters, computed on the host */
    int ct;              /* 5, 6, 7, 11 */
    int B;               /* to_absErrorBound_binary(bound), impl/dataCompression.c:5512 */
    float thr_lt;        /* largest float f with (double)f <  bound  (zero test, :2044) */
    float thr_le;        /* largest float f with (double)f <= bound  (predictor test, :2106) */
    int type;            /* CT7 leading-ones count (med_dataset_float :3605-3614) */
    uint32_t mask17;     /* CT7 mask: top 17 bits of the mean's pattern (pingpong.c:202-206) */
    int mm;              /* m(mask exponent) */
    int mm0;             /* max(mm - 8, 0) */
    /* derived decode constants (token length / value without branches, dc_device.h) */
    int rawadd;          /* B - 118: raw length = clamp(E + rawadd, 9, 32) */
    uint32_t hm;         /* CT7: the type leading-one bits after the first bit of a masked token */
    int fsh;             /* CT7: shift of the masked token's flag bit (30 - type) */
    int lm0, dlm;        /* CT7: masked length flag 0 = lm0, flag 1 = lm0 + dlm */
    int rs;              /* CT7: type + 2 (head length) */
    uint32_t c0, k0;     /* CT7 flag 0 value = c0 | ((t << rs) >> 17 & k0) */
    uint32_t c1, k1;     /* CT7 flag 1 value = c1 | ((t << rs) >> 9 & k1) */
    int s0, s1;          /* CT7: the same as c0 | ((t >> s0) & k0), c1 | ((t >> s1) & k1): 17 - rs, 9 - rs */
    uint32_t em0, eh0;   /* CT7 encoder, flag 0 token = (v & em0) | eh0 (v = top 9+mm bits of the float) */
    uint32_t em1, eh1;   /* CT7 encoder, flag 1 token = (v & em1) | eh1 */
    /* CT7 encoder, as XOR constants on v = the top 9+mm bits of a masked float (whose top 9 bits are the
       mask's): flag 1 token = v ^ K1 (length lm1), flag 0 token = v ^ K0 (length lm0) */
    uint32_t K0, K1;
    int lm1;
    /* (dc_encode_sub_device) encode x - submin instead of x, the subtraction as the reference's x86 build makes it
       (toSmallDataset_float); the single-pass encoder only, submin finite */
    int sub;
    float submin;
    const float* subp;   /* (device) the minimum, when set: read by the kernel instead of submin (the halo path) */
} Params;

typedef struct Plan {    /* device-resident sizes of the stream being decoded */
    unsigned long long nbits;
    long long nbytes;
    long long nchunks;
    long long ngroups;
    int runs;            /* mostly 3-bit codes (< 6 bits per value, CT 5/7/11): boundary walks step whole runs */
} Plan;

typedef struct DecBufs { /* decoder metadata, sized for the maximum chunk count */
    Plan* plan;
    uint8_t* p_exit;
    uint16_t* p_cnt;
    uint32_t* p_mask;
    uint32_t* map;       /* [chunk][32]  exit<<26 | count for entries in known[] */
    uint32_t* known;     /* [chunk] entries with a valid map[] word (besides P's own positions) */
    uint32_t* exitmask;  /* [chunk][2] exits of all known entries, by closure-round parity */
    uint32_t* fullmap;   /* [group][32]  exit<<26 | count */
    uint64_t* gran;      /* [group][33]  look-back granules (32 map entries + inclusive) */
    uint64_t* hist;      /* [group][6]   decoder-history look-back granules (3 aggregate + 3 final) */
    uint32_t* cmeta;     /* [chunk] standard count | std exit<<10 | extra entries<<16 | ok<<20 */
    uint32_t* tmap;      /* [group][4]  tile record: P_0 mask, n_0 | x_0<<16 | tile exit<<24, rest count */
    uint32_t* tentry;    /* [group] true entry of the tile's first chunk | its token count << 8 */
    unsigned long long* tbase;   /* [group] first token index of the tile */
    uint8_t* entry;
    unsigned long long* tokoff;
    uint16_t* pend;
    uint16_t* done;
    unsigned* err;       /* 8 unknown entry, 16 spin timeout, 32 pending left, 64 closure overflow */
    unsigned* ctr;       /* [0,1] resolve ticket/exit, [2,3] parse, [4,5] decode */
    unsigned long long* dbg;   /* optional phase stamps (s_memrealtime) [tile][16], NULL = off */
    int shard;           /* 0: the stream starts the data; 1: a shard, the three values before it come
                            later (dc_decode_shard_fix); 2: a shard with those values in hin */
    const float* hin;    /* [3] b1, b2, b3 before the shard (device), shard == 2 */
} DecBufs;

/* segment decoder (dc_decode3.hip): 256-bit chunks; a parse lane walks a segment of `seg` chunks
 * after a 1024-bit pre-walk and records every chunk's entry offset and token count */
typedef struct Dec3Bufs {
    uint16_t* rec;                 /* [chunk] entry (bits 0..4) | tokens << 8 */
    uint32_t* rel;                 /* [decode job = 64 chunks] first token, relative to its parse job */
    uint32_t* ptot;                /* [parse job = 64 segments] tokens */
    uint64_t* pexit;               /* [parse job] epoch << 32 | its last lane's exit (main walk) */
    uint64_t* hist;                /* [decode job][3] the job's last three values, epoch-tagged granules */
    unsigned* err;                 /* the DecBufs status word; 512 = this path declined the stream */
    int seg;                       /* chunks per parse segment: 4, 8 or 16 (dc_decode3_seg); the pre-walk is
                                      1024 bits whatever seg */
    long long max_chunks;          /* this stream's chunk capacity (<= the rec pool's) */
    long long capw;                /* readable words of the stream buffer (a multiple of 4, >= 4) */
    int shard;                     /* 1: the stream is a shard of a longer one (dc_decode_shard3_device):
                                      predictions among its first tokens read the three values before
                                      it, which come later -- decoded as pending, fixed by
                                      dc_decode_shard3_fix; 2: the first such shard (no values before it:
                                      a prediction among its first three tokens declines, as for a
                                      whole stream) */
    uint32_t* spend;               /* [0] tokens of the shard's first chunk that wait for those values */
    uint64_t* ftag;                /* [fused job = 4 parse jobs] epoch << 32 | tokens (fused3_kernel) */
    uint32_t* frel;                /* fused3d_kernel: rel by fused job, (4 SEG + 31) & ~31 words each (no
                                      128-B line shared by two fused jobs: they are handed to other CUs) */
    uint32_t* fsub;                /* fused3d_kernel: [fused job] 16-B granule {epoch, tokens before its parse
                                      jobs 1, 2, 3} */
    unsigned* fq;                  /* fused3d_kernel: 8 decode-job queue heads + a done counter, 128 B apart
                                      (zero between launches: the launch's last wave resets them) */
} Dec3Bufs;

#ifdef __cplusplus
}  /* namespace dc */
extern "C" {
#define DC_NS dc::
#else
#define DC_NS
#endif

typedef struct ihipStream_t* dc_hip_stream;

int dc_launch_encode(const float* x, long long n, long long idx0, const DC_NS Params* P, uint32_t* out,
                     uint64_t* desc, unsigned* flag, uint32_t epoch, int start_bit,
                     unsigned long long* total_bits, unsigned long long* total_bits2, unsigned* err,
                     unsigned long long* dbg, int mode, const uint32_t* crc_tab, uint32_t* crc_blk,
                     dc_hip_stream stream);
int dc_encode_mode(void);
int dc_encode_crc_fused_last(void);      /* 1: the last encode launch computed the fused CRC pieces */
int dc_set_encode_help(int on);
unsigned dc_encode_epoch_limit(void);
long long dc_encode_group_count(long long n);
long long dc_encode_tile_count(long long n);
long long dc_encode_desc_words(long long n);
int dc_launch_encode_bits(const float* x, long long n, long long idx0, const DC_NS Params* P, uint64_t* desc,
                          unsigned long long* total_bits, unsigned* err, dc_hip_stream stream);

int dc_launch_decode(const uint8_t* s, const unsigned long long* dev_nbits, unsigned long long host_nbits,
                     long long max_chunks, const DC_NS Params* P, const DC_NS DecBufs* D, float* out,
                     long long num, uint32_t epoch, int rounds, int fix_iters, dc_hip_stream st);
int dc_launch_resolve(long long max_chunks, const DC_NS DecBufs* D, uint32_t epoch, dc_hip_stream st);
int dc_launch_decode_fast_resolved(const uint8_t* s, long long max_chunks, const DC_NS Params* P,
                                   const DC_NS DecBufs* D, float* out, long long num, uint32_t epoch, dc_hip_stream st);
int dc_launch_decode_more(const uint8_t* s, long long max_chunks, const DC_NS Params* P,
                          const DC_NS DecBufs* D, float* out, long long num, uint32_t epoch,
                          int fix_iters, dc_hip_stream st);
int dc_launch_decode_fast(const uint8_t* s, const unsigned long long* dev_nbits, unsigned long long host_nbits,
                          long long max_chunks, const DC_NS Params* P, const DC_NS DecBufs* D, float* out,
                          long long num, uint32_t epoch, dc_hip_stream st);
int dc_launch_decode_serial(const uint8_t* s, const DC_NS Params* P, const DC_NS DecBufs* D, float* out,
                            long long num, dc_hip_stream st);
/* dense = 1: the decode3 instantiation with a 2080-value job buffer (streams of < ~16 bits per value);
   the single-launch parse + decode (fused3_kernel) instead of parse3 + decode3 when it is switched on
   (dc_set_fused3) and the stream qualifies (dc_decode3_last_fused() then says so) */
int dc_launch_decode3(const uint8_t* s, const unsigned long long* dev_nbits, unsigned long long host_nbits,
                      const DC_NS Params* P, const DC_NS Dec3Bufs* D3, float* out, long long num, uint32_t epoch,
                      int dense, dc_hip_stream st);
int dc_decode3_last_fused(void);
int dc_maps_seg(int seg);
void dc_set_encode_mirror(void* dst);
int dc_launch_crc32_pair(const uint8_t* a, const uint8_t* b, long long nbytes, const uint32_t* d_tab,
                         const uint32_t* d_x2n, uint32_t* d_parts, uint32_t* d_out_a, uint32_t* d_out_b,
                         dc_hip_stream st);
void dc_decode3_clear_fused(void);
/* the chunks of the last fused decode of a stream of this capacity: the next launch's segment length */
void dc_decode3_size_hint(long long max_chunks, long long nchunks);
int dc_launch_merge_shards(const uint8_t* g, long long P, int world, const unsigned long long* counts, uint8_t* out,
                           long long out_bytes, unsigned long long* total_out, unsigned* err, long long max_bytes,
                           dc_hip_stream st);
int dc_launch_occupy(double us, int blocks, int lds, unsigned* sink, dc_hip_stream st);
int dc_launch_extract_shard(const uint8_t* g, long long g_bytes, const unsigned long long* counts, int rank, uint8_t* d,
                            long long d_bytes, unsigned long long* nbits_out, unsigned* err, dc_hip_stream st);
int dc_launch_shard3_fix(const uint8_t* s, const DC_NS Params* P, const DC_NS Dec3Bufs* D3, const float* hin,
                         float* out, long long num, dc_hip_stream st);
int dc_launch_decode_tiny(const uint8_t* s, long long capb, const unsigned long long* dev_nbits,
                          unsigned long long host_nbits, const DC_NS Params* P, float* out, long long num, unsigned* err,
                          dc_hip_stream st);
long long dc_tiny_max_values(void);
int dc_launch_decode_runs(const uint8_t* s, const unsigned long long* dev_nbits, unsigned long long host_nbits,
                          long long max_chunks, const DC_NS Params* P, uint8_t* maps, unsigned* err, float* out,
                          long long num, dc_hip_stream st);
int dc_launch_decode_runs_scatter(const uint8_t* s, const unsigned long long* dev_nbits, unsigned long long host_nbits,
                                  long long max_chunks, const DC_NS Params* P, uint8_t* maps, unsigned* err, long long num,
                                  float* p, const float* d_min, int mj, int mk, int ijk, int v, int B, dc_hip_stream st);
long long dc_decode_runs_max_chunks(void);
/* the maps parse of streams whose token paths merge slowly (dc_decode_maps.hip): fills D3's rec / rel / ptot
   as parse3 would, for dc_launch_decode3_values; scratch: dc_maps_scratch_bytes(max_chunks) bytes */
long long dc_maps_scratch_bytes(long long max_chunks);
int dc_launch_maps_parse(const uint8_t* s, const unsigned long long* dev_nbits, unsigned long long host_nbits,
                         const DC_NS Params* P, const DC_NS Dec3Bufs* D3, long long num, void* scratch,
                         dc_hip_stream st);
int dc_launch_decode3_values(const uint8_t* s, const unsigned long long* dev_nbits, unsigned long long host_nbits,
                             const DC_NS Params* P, const DC_NS Dec3Bufs* D3, float* out, long long num, uint32_t epoch,
                             int dense, dc_hip_stream st);
size_t dc_decode_runs_scratch_bytes(void);
int dc_decode3_seg(long long max_chunks, int B, int ct);
long long dc_ct1_tiles(long long n);
int dc_launch_ct1_encode(const float* x, long long n, float thr_le, uint32_t* traw, unsigned long long* rawoff,
                         float* raw, char* codes, int* pos1, unsigned* err, dc_hip_stream st);
int dc_launch_ct1_decode(const float* raw, long long nraw, const char* codes, const int* pos1, long long ncodes,
                         long long num, uint8_t* carr, uint32_t* traw, unsigned long long* rawoff, float* out,
                         unsigned* err, dc_hip_stream st);
int dc_launch_ct1_encode64(const double* x, long long n, double bound, uint32_t* traw, unsigned long long* rawoff,
                           double* raw, char* codes, int* pos1, unsigned* err, dc_hip_stream st);
int dc_launch_ct1_decode64(const double* raw, long long nraw, const char* codes, const int* pos1, long long ncodes,
                           long long num, uint8_t* carr, uint32_t* traw, unsigned long long* rawoff, double* out,
                           unsigned* err, dc_hip_stream st);
int dc_launch_find_sentinel(const float* out, long long num, unsigned* err, dc_hip_stream st);
int dc_launch_fixup_serial(const uint8_t* s, const DC_NS Params* P, const DC_NS DecBufs* D, float* out,
                           long long num, dc_hip_stream st);
long long dc_decode_chunk_bits(void);
void dc_mark_phase(int k, dc_hip_stream st);
void dc_mark_next_set(void);
int dc_timing_enable(int nsets);
int dc_timing_read(int set, float* ms);
int dc_timing_read_all(int set, float* ms);
void dc_timing_finish(int on);
long long dc_decode_group(void);
/* the same decoder built with 256-bit chunks (Makefile SMALLDEFS renames its symbols with _s) */
int dc_launch_decode_s(const uint8_t* s, const unsigned long long* dev_nbits, unsigned long long host_nbits,
                       long long max_chunks, const DC_NS Params* P, const DC_NS DecBufs* D, float* out,
                       long long num, uint32_t epoch, int rounds, int fix_iters, dc_hip_stream st);
int dc_launch_resolve_s(long long max_chunks, const DC_NS DecBufs* D, uint32_t epoch, dc_hip_stream st);
int dc_launch_decode_fast_resolved_s(const uint8_t* s, long long max_chunks, const DC_NS Params* P,
                                     const DC_NS DecBufs* D, float* out, long long num, uint32_t epoch, dc_hip_stream st);
int dc_launch_decode_more_s(const uint8_t* s, long long max_chunks, const DC_NS Params* P,
                            const DC_NS DecBufs* D, float* out, long long num, uint32_t epoch,
                            int fix_iters, dc_hip_stream st);
int dc_launch_decode_fast_s(const uint8_t* s, const unsigned long long* dev_nbits, unsigned long long host_nbits,
                            long long max_chunks, const DC_NS Params* P, const DC_NS DecBufs* D, float* out,
                            long long num, uint32_t epoch, dc_hip_stream st);
int dc_launch_decode_serial_s(const uint8_t* s, const DC_NS Params* P, const DC_NS DecBufs* D, float* out,
                              long long num, dc_hip_stream st);
int dc_launch_find_sentinel_s(const float* out, long long num, unsigned* err, dc_hip_stream st);
int dc_launch_fixup_serial_s(const uint8_t* s, const DC_NS Params* P, const DC_NS DecBufs* D, float* out,
                             long long num, dc_hip_stream st);
long long dc_decode_chunk_bits_s(void);
long long dc_decode_group_s(void);

int dc_launch_to_small(const float* x, long long n, float* y, float* part_v, long long* part_i, float* d_min,
                       dc_hip_stream st);
#define DC_MIN_PARTS 2048                /* toSmallDataset: per-workgroup minima combined by min_final */
int dc_launch_med(const float* x, long long n, float s_init, void* scratch, float* d_mean, int* d_type, float* d_sum,
                  float* d_max, dc_hip_stream st);
int dc_launch_med_sub(const float* x, long long n, void* scratch, float* d_min, float* pv, long long* pi, float* d_mean,
                      int* d_type, int wide, hipStream_t st);
/* (clr64[0..n64) and clr32[0..n32) zeroed on the way, NULL / 0: none; cnt: a zeroed counter of this stream's own, the
   minimum finished by the gather's last workgroup, NULL: a second launch) */
int dc_launch_plane_gather_min(const float* p, int mj, int mk, int ijk, int v, int A, int B, float* out, float* part_v,
                               long long* part_i, float* d_min, uint64_t* clr64, int n64, uint32_t* clr32, int n32,
                               unsigned* cnt, dc_hip_stream st);
int dc_encode_plain(void);
int dc_launch_sub_ptr(const float* x, long long n, const float* d_min, float* y, dc_hip_stream st);
int dc_launch_sub_value(const float* x, long long n, float m, float* y, hipStream_t st);
int dc_launch_med_wide(const float* x, long long n, float s_init, void* scratch, float* d_mean, int* d_type,
                       float* d_sum, float* d_max, int fresh, dc_hip_stream st);
unsigned* dc_med_flag_ptr(void* scratch, long long n, int is_double);
int dc_launch_med_shard(const float* x, long long n, double s_est, int trans, void* scratch, long long** d_rec,
                        dc_hip_stream st);
int dc_med_shard_binades(void);
int dc_launch_ratio(int is_double, int mode, const void* x, long long n, int B, double thr_le, unsigned long long* d_sum,
                    unsigned* d_flag, uint8_t* sizes, dc_hip_stream st);
int dc_launch_ratio_area(const uint8_t* sizes, long long n, unsigned long long* d_out, dc_hip_stream st);
int dc_launch_ratio_serial(int is_double, int mode, const void* x, long long n, int B, double thr_le,
                           unsigned long long* d_out, dc_hip_stream st);
long long dc_med_scratch_bytes(long long n);
long long dc_crc_parts(long long nbytes);
int dc_crc_run_bytes(void);
int dc_launch_crc32(const uint8_t* s, long long nbytes, const uint32_t* d_tab, const uint32_t* d_x2n,
                    uint32_t* d_parts, uint32_t init, uint32_t* d_out, dc_hip_stream st);
int dc_launch_crc32_copy(const uint8_t* src, uint8_t* dst, long long nbytes, const uint32_t* d_tab,
                         const uint32_t* d_x2n, uint32_t* d_parts, uint32_t* d_out, dc_hip_stream st);
int dc_launch_crc32_resend(const uint8_t* src, uint8_t* dst, long long nbytes, const uint32_t* d_tab,
                           const uint32_t* d_x2n, uint32_t* d_parts, uint32_t* crc2, unsigned* count, dc_hip_stream st);
int dc_launch_bit_shift_copy(const uint8_t* s, long long sbytes, unsigned long long start_bit, unsigned long long nbits,
                             uint8_t* d, long long nout, dc_hip_stream st);
int dc_launch_shard_fix(const uint8_t* s, const DC_NS Params* P, const DC_NS DecBufs* D, float* out, long long num,
                        long long nchunks, const float* hin, dc_hip_stream st);
int dc_launch_shard_fix_s(const uint8_t* s, const DC_NS Params* P, const DC_NS DecBufs* D, float* out, long long num,
                          long long nchunks, const float* hin, dc_hip_stream st);
int dc_launch_plane_gather(const float* p, int mj, int mk, int ijk, int v, int A, int B, float* out, dc_hip_stream st);
int dc_launch_plane_scatter(const float* x, const float* d_min, float* p, int mj, int mk, int ijk, int v, int A, int B,
                            dc_hip_stream st);
int dc_launch_hash_words(const void* p, long long nbytes, unsigned long long* d_out, dc_hip_stream st);
int dc_launch_stream_copy(const void* src, void* dst, long long bytes, int variant, dc_hip_stream st);
/* fused CRC-32 (zlib) over 16 KiB stream blocks: per-block raw CRCs (XOR-accumulated by the producers, or by
   dc_launch_crcf_blocks from a byte range, optionally copying it: the CT9 resend), then one combine launch
   (crc_out = zlib CRC of the first nbytes / *d_nbits bits' bytes; blk zeroed for the next use; with ref: a
   mismatch increments *count).  gate (optional, two CRCs): the blocks launch runs only when they differ. */
#define DC_CRCF_BLK 16384
#define DC_CRCF_WORDS 680
long long dc_crcf_blocks(long long nbytes);
int dc_crcf_tables(uint32_t* h_tab);        /* the DC_CRCF_WORDS table words (nibble tables, shifts, x^2^k) */
int dc_launch_crcf_blocks(const uint8_t* src, uint8_t* dst, long long nbytes, const uint32_t* d_ctab, uint32_t* blk,
                          const uint32_t* gate, unsigned* gate_count, dc_hip_stream st);
int dc_launch_crcf_final(uint32_t* blk, long long max_bytes, long long nbytes, const unsigned long long* d_nbits,
                         const uint32_t* d_ctab, uint32_t* crc_out, const uint32_t* ref, unsigned* count,
                         const uint32_t* gate, dc_hip_stream st);
int dc_launch_flip_bits(uint8_t* s, unsigned long long nbits, long long count, unsigned long long seed,
                        dc_hip_stream st);
int dc_launch_crc_resend(const uint32_t* crc, const uint8_t* src, uint8_t* dst, long long nbytes, int copy,
                         unsigned* count, dc_hip_stream st);
int dc_launch_ham_syndrome(const uint8_t* s, long long nbytes, unsigned long long* d_syn_ones, dc_hip_stream st);

#ifdef __cplusplus
}
#endif
#endif
