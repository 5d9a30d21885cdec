/*
 * dc_gpu.h -- device-pointer extension API of libdcamd (MI355X / gfx950).
 *
 * The reference ABI (dataCompression.h) takes host buffers; these entry points take device
 * buffers that are already resident in HBM, so a caller (bench.py, a GPU-resident solver, the
 * multi-GPU all-gather path) can run the codec without PCIe copies.  Plain C, no HIP/torch types:
 * device pointers are void*, the HIP stream is the library's per-process stream (dc_get_stream).
 *
 * Every function returns 0 on success or a negative DC_ERR_* code; dc_last_error() explains.
 */
#ifndef DC_GPU_H
#define DC_GPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    DC_OK = 0,
    DC_ERR_HIP = -1,          /* HIP runtime error (message in dc_last_error) */
    DC_ERR_ARG = -2,          /* bad argument */
    DC_ERR_INPUT = -3,        /* input outside the codec's domain (e.g. -1.0f sentinel value) */
    DC_ERR_STREAM = -4,       /* stream could not be decoded (corrupt / truncated / unsupported) */
    DC_ERR_NOGPU = -5         /* no usable gfx950 device */
};

/* ---- library state ---------------------------------------------------------------------- */
int dc_init(int device);                       /* optional; first call of any entry point inits dev 0 */
const char* dc_last_error(void);
void* dc_get_stream(void);                     /* hipStream_t all library work is ordered on */
int dc_synchronize(void);
/* Encoder launches of dc_encode_device go to this hipStream_t (NULL: dc_get_stream()); each such encode
 * first waits for the work already queued on dc_get_stream().  The caller orders a later decode of the
 * stream (on dc_get_stream()) after the encode with its own event.  Internal callers (the host ABI, the
 * halo path, the MPI wrappers) always encode on dc_get_stream(). */
int dc_set_encode_stream(void* stream);
void dc_set_abs_error_bound(double bound);     /* runtime absErrorBound (default: header macro) */
double dc_get_abs_error_bound(void);

/* ---- device-pointer codec (asynchronous on dc_get_stream()) ----------------------------- */
/* Bytes an encode of n floats may write (stream bytes + word padding). */
size_t dc_stream_capacity(long long n);

/* Encode n floats at d_x (device).  idx0 = global index of d_x[0] within the logical array; when
 * idx0 > 0 the three floats d_x[-3..-1] must be readable (predictor halo for a shard).
 * start_bit (0..7): number of already-used high bits in the first output byte (append mode /
 * shard stitching); those bits are written as zero.  d_out must hold dc_stream_capacity(n) bytes.
 * *d_total_bits (device, may be NULL) receives start_bit + bits written. */
int dc_encode_device(int ct, const void* d_x, long long n, long long idx0, int type, uint32_t mask17,
                     int start_bit, void* d_out, unsigned long long* d_total_bits);
/* Stream bits an encode of these n floats would produce, without writing a stream (count + scan
 * kernels only; synchronous).  The multi-GPU path uses it to place shards before encoding them. */
int dc_encode_bits_device(int ct, const void* d_x, long long n, long long idx0, int type, uint32_t mask17,
                          unsigned long long* bits_out);
/* Wait for the last encode and return start_bit + bits written (host value). */
int dc_encode_result(unsigned long long* total_bits);
/* the encoder's error word, read as is (bit 0: a -1.0f input; 2: an offset outside the stream; 4: a
   single-pass look-back timed out -- dc_encode_result then re-encodes wait-free when that encode is the
   only one issued since the word was last checked, and reports an error otherwise); synchronous */
int dc_encode_status(unsigned* status_out);
/* clear that word (after dc_encode_result reported a timeout among several outstanding encodes) */
int dc_encode_clear_status(void);
/* encoder variant of the last encode: 1 single pass, 2 count + pack, 3 count + scan + pack */
int dc_encode_mode(void);
/* encodes re-run wait-free after a look-back timeout (process lifetime) */
int dc_encode_retries(void);

/* Decode num floats from a device stream of nbytes bytes (nbytes < 0: take the length in bits
 * from *d_nbits, device memory, e.g. the d_total_bits of a preceding dc_encode_device).
 * max_bytes bounds the stream size (buffer capacity).  Asynchronous: call dc_decode_finish(). */
int dc_decode_device(int ct, const void* d_stream, long long nbytes, const unsigned long long* d_nbits,
                     long long max_bytes, long long num, int type, uint32_t mask17, void* d_out);
/* Wait, check the decoder's status words and complete rare slow paths (extra closure rounds,
 * serial prediction chains) of the LAST decode.  Returns DC_OK or DC_ERR_STREAM.  Several decodes may
 * be queued before one finish; if any of them left the fast path the status words say so, only the last
 * one can be completed, and finish returns DC_ERR_STREAM ("an earlier decode was not completed"). */
int dc_decode_finish(void);
/* Wait and return the fast path's status word OR-ed over every decode since the last finish, without
 * running any slow path (0: every queued decode completed on the fast path).  For benchmarks. */
int dc_decode_status(unsigned* status_out);
/* Status of the last reference-ABI call (myCompress_* / myDecompress_* / the MPI wrappers): DC_OK or
 * the DC_ERR_* code it failed with (the ABI signatures have no error return). */
int dc_abi_status(void);

/* Shards of one global stream (multi-GPU decode): decode num values from the
 * tokens at bits [start_bit, start_bit + nbits) of d_stream (stream_bytes long; start_bit must be a
 * token boundary -- the shard offsets of the encode).  d_hin = the three values before the shard
 * (b1 = x[-1], b2 = x[-2], b3 = x[-3], device floats), or NULL when they are not known yet: values
 * that depend on them are then left for dc_decode_shard_fix (after dc_decode_finish).  Shards that
 * need the exact slow paths report DC_ERR_STREAM (decode the whole stream instead). */
int dc_decode_shard_device(int ct, const void* d_stream, long long stream_bytes, unsigned long long start_bit,
                           unsigned long long nbits, long long num, int type, uint32_t mask17, const float* d_hin,
                           void* d_out);
int dc_decode_shard_fix(const float* d_hin);

/* The device-side multi-GPU step (nothing is read back on the host):
 * dc_merge_shards_device: world shards, each encoded at start bit 0 (dc_encode_device with its global
 *   idx0) and all-gathered into slots of slot_bytes (a multiple of 4, >= each shard's bytes + 8), with
 *   their all-gathered bit counts (device u64[world]) -> the single global stream, byte-identical to one
 *   encode of the whole array, in d_out (out_bytes of room, 4-byte aligned) and its bit count in d_total.
 *   Problems set a sticky status word read by dc_merge_status (1: a shard longer than its slot, 2: the
 *   stream longer than the output).
 * dc_decode_shard3_device: decode one such shard (its own encoded buffer, bit count on the device) with
 *   the segment decoder; predictions among its first tokens wait for the previous shard's last three
 *   values: dc_decode_shard3_fix(d_hin) decodes them once they are on the device (b1 = x[-1], b2, b3).
 *   has_history 0 marks the first shard (nothing before it): a prediction among its first three tokens
 *   then declines it, as for a whole stream.
 *   A shard the segment decoder declines sets dc_decode_status (decode it with dc_decode_shard_device). */
int dc_merge_shards_device(const void* d_gathered, long long slot_bytes, int world, const unsigned long long* d_counts,
                           void* d_out, long long out_bytes, unsigned long long* d_total);
int dc_merge_status(unsigned* status_out, int reset);
/* dc_extract_shard_device: the receiver's side of the all-gather -- shard `rank` cut out of the merged global
 *   stream d_global (g_bytes of buffer; d_counts the shards' bit counts, as given to the merge) to bit 0 of
 *   d_out (out_bytes of room, 4-byte aligned), its bit count to *d_nbits: the bytes that arrived, ready for
 *   dc_decode_shard3_device.  A shard that does not fit sets dc_merge_status bit 4 (nothing written). */
int dc_extract_shard_device(const void* d_global, long long g_bytes, const unsigned long long* d_counts, int rank,
                            void* d_out, long long out_bytes, unsigned long long* d_nbits);
int dc_decode_shard3_device(int ct, const void* d_stream, const unsigned long long* d_nbits, long long max_bytes,
                            long long num, int type, uint32_t mask17, void* d_out, int has_history);
int dc_decode_shard3_fix(const float* d_hin);
int dc_decode_status_clear(void);           /* clear the decoder status word (after a declined shard) */

/* Himeno halo planes on device-resident p[mi][mj][mk] (the fused form of transform_3d_array_to_1d_array +
 * toSmallDataset_float + compress, impl/himenoBMTxps.c:483-706): encode the plane ijk (1: i = v,
 * 2: j = v, 3: k = v) of extent imax x jmax x kmax; *d_min (device) gets the plane minimum.  CT7 with
 * type <= 0 derives type / mask from the plane (med_dataset_float, synchronous) and returns them in
 * *type_out / *mask17_out.  Decode: stream -> plane values + *d_min written back into p's plane. */
int dc_halo_encode_device(int ct, const void* d_p, int mi, int mj, int mk, int ijk, int v, int imax, int jmax,
                          int kmax, int type, uint32_t mask17, void* d_stream, unsigned long long* d_bits,
                          float* d_min, int* type_out, uint32_t* mask17_out);
int dc_halo_decode_device(int ct, const void* d_stream, long long nbytes, const unsigned long long* d_bits, int type,
                          uint32_t mask17, const float* d_min, void* d_p, int mi, int mj, int mk, int ijk, int v,
                          int imax, int jmax, int kmax);
/* 1: dc_halo_decode_device returns without a host read (the plane is complete on the library stream if
 * dc_decode_status() reads 0 after the caller's steps; else decode it again with this off).  Returns the
 * previous setting. */
int dc_set_halo_async(int on);
/* 1: dc_halo_encode_device takes the separate passes (gather, toSmallDataset's three launches, a copy of the
 * minimum, encode) instead of the fused ones (gather with the minimum's partials, min_final, an encode that subtracts
 * the minimum while loading); the same stream and minimum.  Returns the previous setting. */
int dc_set_halo_unfused(int on);
/* Two planes of one array encoded at once (each on its own stream with its own scratch; the fused path only --
 * otherwise one after the other): streams, bit counts and minima as two dc_halo_encode_device calls. */
int dc_halo_encode2_device(int ct, const void* d_p, int mi, int mj, int mk, int ijk, int v0, int v1, int imax, int jmax,
                           int kmax, int type, uint32_t mask17, void* s0, void* s1, unsigned long long* bits0,
                           unsigned long long* bits1, float* dmin0, float* dmin1);
/* Two planes of one array decoded at once (each on its own stream; asynchronous, dc_set_halo_async(1) required,
 * else the planes go one after the other): the two z-neighbour planes of a Himeno step.  A plane the small-stream
 * decoder declines sets dc_decode_status(); decode it again with dc_halo_decode_device. */
int dc_halo_decode2_device(int ct, const void* s0, const void* s1, const unsigned long long* bits0,
                           const unsigned long long* bits1, int type, uint32_t mask17, const float* dmin0,
                           const float* dmin1, void* d_p, int mi, int mj, int mk, int ijk, int v0, int v1, int imax,
                           int jmax, int kmax);
/* HIP graphs (no reference counterpart: the launch-bound Himeno halo step of impl/himenoBMTxps.c:644-690 replayed with
 * one launch).  dc_capture_begin .. dc_capture_end record the library calls in between into a graph; dc_graph_launch
 * replays it on the library stream, reading the same device buffers (rewrite the data in place between replays).
 * Recordable: the encoders (dc_encode_device, dc_halo_encode_device, dc_halo_encode2_device) and async halo decodes
 * on the small-stream decoder (dc_set_halo_async(1)); any other decode fails and then dc_capture_end fails.  Run the
 * step once uncaptured first (buffers are sized on first use).  Read dc_encode_status / dc_decode_status after
 * replays: a replay has no host-side fallback. */
int dc_capture_begin(void);
int dc_capture_end(void** graph_out);
int dc_graph_launch(void* graph);
int dc_graph_destroy(void* graph);

/* Pre-passes on device data: toSmallDataset_float and med_dataset_float (exact). */
int dc_to_small_device(const void* d_x, long long n, void* d_out, float* min_out);
int dc_med_device(const void* d_x, long long n, float* mean_out, int* type_out);
/* The two pre-passes fused, for the bitmask chain of impl/pingpong.c:148-209 (toSmallDataset_float, then
 * med_dataset_float of data_small): min_out = toSmallDataset_float's minimum of x, mean_out / type_out =
 * med_dataset_float of x - min, without writing x - min (one read of x for the minimum and the chunk statistics,
 * one for the transducers).  Synchronous.  Replaces dc_to_small_device + dc_med_device on the same data. */
int dc_prep_device(const void* d_x, long long n, float* min_out, float* mean_out, int* type_out);
/* dc_encode_device (idx0 = 0, start_bit = 0) of x - min, the subtraction made while loading x (the reference's x86
 * subtraction, as toSmallDataset_float): the stream myCompress_bitwise* makes from data_small
 * (impl/dataCompression.c:3543-3562 then :2030-2284), with no data_small array.  Asynchronous. */
int dc_encode_sub_device(int ct, const void* d_x, long long n, float min, int type, uint32_t mask17, void* d_out,
                         unsigned long long* d_total_bits);
/* 1 when the last dc_med_device / dc_med_sum_device needed the wide binade window: the narrow window tried
   first, [E_est - 1, E_est + 1] around the double estimate of the running sum, missed more than 16 chunks
   (DC_MED_WIDE=1 in the environment goes to the wide window at once) */
int dc_med_last_wide(void);
/* Multi-GPU med_dataset_float over contiguous shards: the exact left-to-right float sum of x[0..n)
 * continued from s_init (0 on the first shard, else the sum the previous shard returned) and the max of
 * x; the global mean is sum / (float)n_total and the type dc_type_from_max(global max).  Synchronous. */
int dc_med_sum_device(const void* d_x, long long n, float s_init, float* sum_out, float* max_out);
/* The exscan form of the same (every rank in parallel, no chain of passes): a shard's double sum, its max
 * (NaNs never win; the global max folds the first shard's x[0] with every shard's max, strict >) and x[0],
 * and its whole-shard transducer for the dc_med_shard_binades() binades E = *e_lo + w of the window its
 * running sum is estimated to enter at s_est (the double sums of the earlier shards): a sum k * 2^(E-150)
 * entering with k in [2^23, 2^24) leaves as (k + units[2w + (k & 1)]) * 2^(E-150) when flags[w] & 4 is 0 and
 * that stays below 2^24; flags[w] & 1 / & 2 are the end parities from start parity 0 / 1.  Synchronous. */
int dc_med_shard_stats(const void* d_x, long long n, double* sum_out, float* max_out, float* first_out);
int dc_med_shard_trans(const void* d_x, long long n, double s_est, int* e_lo, long long* units, unsigned char* flags);
int dc_med_shard_binades(void);
int dc_type_from_max(float mx);
/* zlib-compatible CRC-32 of a device byte range. */
int dc_crc32_device(const void* d_s, long long nbytes, uint32_t* crc_out);
/* The same, asynchronous on the library stream, result to device memory d_crc (one uint32). */
int dc_crc32_device_async(const void* d_s, long long nbytes, uint32_t* d_crc);
/* A 64-bit hash of a device byte range: the sum over its 32-bit little-endian words w_i (bytes past nbytes
 * zero) of splitmix64(i << 32 | w_i) mod 2^64 (bench.py's self-check against hashes of the oracle's
 * output, tests/golden/make_bench_hashes.py).  Synchronous. */
int dc_hash_device(const void* d_buf, long long nbytes, unsigned long long* hash_out);
/* The achievable HBM rate of this GPU: a hand-written streaming copy (16-byte buffer loads and stores,
 * 4 or 8 in flight per lane, default or nontemporal policy: 4 variants) of `bytes` (a multiple of 16,
 * < 2 GiB) from d_src to d_dst, `reps` launches per variant timed with HIP events on the library stream;
 * *gbs_out = the best variant's (read + written bytes) / average launch time, in GB/s; *variant_out its
 * index.  Synchronous. */
int dc_copy_rate_device(const void* d_src, void* d_dst, long long bytes, int reps, double* gbs_out, int* variant_out);
/* The single-pass encoder's tiles wait for lower tiles.  With one process per GPU that is safe (dispatch is in
 * order per XCD).  Where several processes run look-back kernels on one GPU, a predecessor can stay undispatched
 * behind their waiting waves: on = 1 selects the helping instantiation, whose waiting tiles (and scanner) compute
 * a late predecessor's count and tail themselves (also DC_ENC_HELP=1).  Returns the previous setting. */
int dc_set_encode_help(int on);
/* Co-residency tests: `blocks` workgroups of 256 threads with `lds` bytes of LDS each that stay resident for `us`
 * microseconds on `stream` (NULL: a stream of the library's own, not the codec's), so that the codec can be
 * run while other work holds CU slots.  Asynchronous. */
int dc_occupy_device(void* stream, double us, int blocks, int lds);
/* The CT9 flow without CRC passes of its own (fused CRC-32 over 16 KiB blocks; each a zlib crc32 of the stream
 * bytes, written to device memory, asynchronous on the library stream):
 * dc_encode_crc_device: dc_encode_device at start bit 0 (d_total_bits required) plus the stream's CRC into
 *   *d_crc, computed by the encoder's tiles from the words they store, and one combine launch;
 * dc_crc32_stream_device: a stream's CRC by one pass (16-byte aligned, readable to nbytes rounded up to 16);
 * dc_crc_resend_crc_device: the receiver's check with the resend (d_crc2[0] sender's CRC, d_crc2[1] receiver's):
 *   on a mismatch d_src is copied over d_dst (d_count[0] += 1) and the copy's CRC, computed as it is written,
 *   replaces d_crc2[1]; a mismatch left after that increments d_count[1]. */
int dc_encode_crc_device(int ct, const void* d_x, long long n, long long idx0, int type, uint32_t mask17, void* d_out,
                         unsigned long long* d_total_bits, uint32_t* d_crc);
int dc_crc32_stream_device(const void* d_s, long long nbytes, uint32_t* d_crc);
/* CT9 send without a copy pass (replaces the reference's MPI send of the compressed buffer,
 * impl/pingpong.c:260-289): the encode of dc_encode_device (start bit 0) with its stream words also written
 * into the receiver's buffer d_mirror (4-byte aligned, the stream's capacity); the sender keeps d_out for a
 * resend.  Then dc_crc32_pair_device gives the sender's CRC of d_out and the receiver's of d_mirror (after any
 * channel damage) in one pass over both (16-byte aligned buffers, device results). */
int dc_encode_send_device(int ct, const void* d_x, long long n, long long idx0, int type, uint32_t mask17,
                          void* d_out, void* d_mirror, unsigned long long* d_total_bits);
int dc_crc32_pair_device(const void* d_a, const void* d_b, long long nbytes, uint32_t* d_crc_a, uint32_t* d_crc_b);
/* CT9 send: d_src copied to d_dst (the channel) and the zlib CRC-32 of the bytes sent into *d_crc (device), in one
   pass (16-byte aligned, < 2 GiB) */
int dc_crc32_copy_device(const void* d_src, void* d_dst, long long nbytes, uint32_t* d_crc);
int dc_crc_resend_crc_device(uint32_t* d_crc2, const void* d_src, void* d_dst, long long nbytes, unsigned* d_count);
/* BER fault injection (CT8/CT9 flow): flip `count` bits of the stream at positions
 * splitmix64(seed + i) mod nbits (MSB-first in each byte, as bit_flip).  The stream buffer must be
 * 4-byte aligned and padded to whole words.  Asynchronous. */
int dc_flip_bits_device(void* d_s, unsigned long long nbits, long long count, unsigned long long seed);
/* CT9 receiver check on the device, on the library stream (no host round trip): d_crc2[0] = sender's CRC-32,
   d_crc2[1] = receiver's.  copy = 1: on a mismatch d_src (nbytes) is copied over d_dst (the resend) and
   d_count[0] incremented; copy = 0: a mismatch increments d_count[1].  16-byte aligned streams. */
int dc_crc_resend_device(const uint32_t* d_crc2, const void* d_src, void* d_dst, long long nbytes, int copy,
                         unsigned* d_count);

/* CT1 byte-wise codec on device buffers: d_raw (n floats), d_codes (n chars), d_pos1 (n ints) must
 * hold the worst case; *nraw_out = raw count (codes = n - raw).  Synchronous. */
int dc_ct1_encode_device(const void* d_x, long long n, void* d_raw, void* d_codes, void* d_pos1, long long* nraw_out);
int dc_ct1_decode_device(const void* d_raw, long long nraw, const void* d_codes, const void* d_pos1, long long ncodes,
                         long long num, void* d_out);

/* ---- double codecs (CT 5/6/7/11 of myCompress_bitwise_double*, impl/dataCompression.c:355-3308) ---
 * mask20 = the top 20 bits of the mean's pattern (char mask[1+11+8]).  d_out of the encoder needs
 * dc64_stream_capacity(n) bytes, 4-byte aligned; start_bit 0..7 leaves that many zero bits first
 * (the host ABI ORs the bits of a partially filled last byte there).  Asynchronous on the library
 * stream; *d_total_bits (device, optional) receives the bit count. */
size_t dc64_stream_capacity(long long n);
int dc64_encode_device(int ct, const void* d_x, long long n, int type, uint32_t mask20, int start_bit, void* d_out,
                       unsigned long long* d_total_bits);
int dc64_encode_result(unsigned long long* total_bits);                   /* sync + bits of the last encode */
/* Decode num doubles from a device stream of nbytes bytes (or *d_nbits bits when d_nbits is given;
 * max_bytes bounds the scratch).  Asynchronous; dc64_decode_finish() waits and reports a short stream. */
int dc64_decode_device(int ct, const void* d_stream, long long nbytes, const unsigned long long* d_nbits,
                       long long max_bytes, long long num, int type, uint32_t mask20, void* d_out);
int dc64_decode_finish(void);
unsigned dc64_last_decode_flags(void);            /* after finish: 1 = the exact serial decoder ran */
int dc64_to_small_device(const void* d_x, long long n, void* d_out, double* min_out);   /* synchronous */
int dc64_med_device(const void* d_x, long long n, double* mean_out, int* type_out);     /* synchronous */

/* Decoder/encoder geometry (for tests and bench). */
long long dc_decode_chunk_bits_value(void);                 /* chunk bits of the last decode's build */
/* Streams of at most this capacity (bytes) decode with the 256-bit-chunk build of the decoder, larger
 * ones with the 1024-bit build (< 0: the default, 1 MiB; 0: never).  Returns the previous value. */
long long dc_set_small_chunk_max_bytes(long long max_bytes);
/* Streams of at least this capacity (bytes) decode with the segment decoder (dc_decode3.hip), which
 * hands streams it cannot take to the chunk-map decoder (< -1: the default, 16 KiB + 1; -1: never;
 * 0: every stream).  Returns the previous value. */
long long dc_set_decode3_min_bytes(long long min_bytes);
/* The segment decoder's parse segment length in 256-bit chunks: 4, 8 or 16 forces one, 0 chooses by the
 * stream's capacity and bound (dc_decode3.hip dc_decode3_seg).  Returns the previous setting. */
int dc_set_decode3_seg(int seg);
/* Experiments: 1 decodes 16-chunk-segment streams with the single-launch parse + decode (fused3_kernel,
 * DESIGN section 4b), 0 with parse3 + decode3 (the default; DC_FUSED3=1 sets it at start).  Returns the
 * previous setting. */
int dc_set_fused3(int on);
/* The last fused launch's per-job stamps when DC_FUSED3_STAMPS is set (4 per fused job: start, parse end,
 * prefix known, decode end; s_memrealtime, 100 MHz): the number of jobs copied, 0 when none were recorded. */
long long dc_fused3_stamps(unsigned long long* out, long long max_jobs);
/* The segment length (chunks) of the last fused launch: 16, 20, 24, 32 or 64 (0: none yet). */
int dc_fused3_last_seg(void);
/* 1 if the last segment-decoder launch was the fused one. */
int dc_decode3_last_fused(void);
/* 1 if the last decode's values came from the segment decoder (after dc_decode_finish). */
int dc_last_decode_was_v3(void);
/* 1: the last finished decode's values came from the segment decoder after the maps parse (a stream whose
 * parse paths merge slowly: noisy ramps, smooth data at small bounds, CT11 without 3-bit codes) */
int dc_last_decode_used_maps(void);
/* tests: 1 = parse every segment decode by maps (returns the previous setting) */
int dc_set_decode3_maps(int on);   /* (-1: also forget the parameters remembered for the maps parse / dense buffer) */
/* Streams of at most this capacity (bytes) decode with the small-stream decoder (dc_decode_runs.hip: chunk
 * entry maps composed by a scan, one workgroup), unless dc_set_decode3_min_bytes(0) forces the segment
 * decoder; Himeno halo planes take it whatever their capacity (< -1: the default, 16 KiB + 256: 2^12 floats; -1:
 * never).  Returns the previous value. */
long long dc_set_runs_max_bytes(long long max_bytes);
/* 1 if the last decode's values came from the small-stream decoder (after dc_decode_finish). */
int dc_last_decode_was_runs(void);
/* 1 when the last finished decode stayed on the one-workgroup decoder of small streams (at most 2^14 values, 2^19
 * bits: dc_decode_tiny.hip).  Opt-in: dc_set_decode_tiny(1) (or DC_TINY=1); it returns the previous setting. */
int dc_last_decode_was_tiny(void);
int dc_last_decode_launched_tiny(void);
int dc_set_decode_tiny(int on);
int dc_last_decode_launched_runs(void);     /* 1: the last dc_decode_device launched it (it may decline) */
/* 1: the last dc_decode_device launched the segment decoder (its values may still come from the chunk-map
 * decoder if it declined the stream: dc_last_decode_was_v3 after dc_decode_finish tells) */
int dc_last_decode_launched_v3(void);

#ifdef __cplusplus
}
#endif
#endif
