/*
 * dc_host.c -- host side of libdcamd: the reference's C ABI (impl/dataCompression.h) on top of
 * the gfx950 kernels, plus the device-pointer API of include/dc_gpu.h.
 *
 * Plain C.  The only bridge to HIP C++ is the extern "C" launcher set in dc_shared.h; everything
 * else here is HIP runtime C API (memory, copies, stream) and host bookkeeping: realloc/append
 * semantics of *data_bits, malloc'ed results owned by the caller, char-string masks.
 * No hot-path work runs on the CPU: if the GPU is unusable the entry points report an error
 * (dc_last_error) instead of computing anything.
 */
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dc_shared.h"
#include "../../include/dc_gpu.h"

#ifndef DC_ABS_ERROR_BOUND
#define DC_ABS_ERROR_BOUND 0.000001      /* impl/dataCompression.h:5 default */
#endif

/* globals of the reference (impl/dataCompression.c:21-22) */
double absErrBound = DC_ABS_ERROR_BOUND;
int absErrorBound_binary = -100;

/* ------------------------------------------------------------------------------------------ */
typedef struct {
    int inited, device;
    hipStream_t st;
    hipStream_t enc_st;              /* encoder stream (dc_set_encode_stream), NULL = st */
    hipEvent_t ev_enc;               /* orders an encode on enc_st after the work queued on st */
    hipEvent_t ev_lib;               /* orders an internal encode on st after the work queued on enc_st */
    hipStream_t last_enc_st;         /* stream of the last encode (dc_encode_result waits on it) */
    int abi_rc;                      /* status of the last reference-ABI call (dc_abi_status) */
    /* encoder */
    uint64_t* enc_desc;
    long long enc_desc_cap;
    unsigned long long* enc_dbg;   /* DC_DEBUG_STAMPS: [tile][8] encoder phase stamps */
    unsigned long long* d_total;
    unsigned* d_enc_err;
    unsigned* d_enc_flag;            /* the pack kernel's scan-published flag (encode epoch) */
    uint32_t enc_epoch;
    struct {                         /* the last encode's launch, re-run wait-free after a look-back timeout */
        const float* x; long long n, idx0; Params P; uint32_t* out; int start_bit;
        unsigned long long* tot; hipStream_t st; int valid;
        uint32_t* crc;               /* dc_encode_crc_device's CRC output (recomputed after a retry) */
        void* mirror;                /* dc_encode_send_device's receiver buffer (written again by a retry) */
    } last_enc;
    int enc_retries;                 /* encodes re-run wait-free (dc_encode_retries) */
    int enc_outstanding;             /* single-pass encodes issued since the error word was last checked clean
                                        or cleared: a timeout is retried only when it is the only one */
    /* decoder */
    DecBufs D;
    void* dec_pool;
    long long dec_cap_chunks;
    uint32_t dec_epoch;
    int dec_small;                   /* the current decode runs the 256-bit-chunk decoder build */
    int dec_pending;
    int dec_queued;                  /* decodes issued since the last finish */
    Params dec_P;
    const uint8_t* dec_s;
    long long dec_max_chunks;
    float* dec_out;
    long long dec_num;
    unsigned long long dec_nbits;
    int dec_runs;                 /* the last decode's stream is in runs mode (Plan.runs) */
    int dec_shard;                   /* shard mode of the pending decode (DecBufs.shard) */
    Dec3Bufs D3;                     /* segment decoder (dc_decode3.hip) */
    void* dec3_pool;
    long long dec3_cap;              /* 256-bit chunks the pool holds */
    int dec3_used;                   /* the pending decode ran the segment decoder */
    int dec3_last;                   /* the last finished decode's values came from it */
    int dec3_launched;               /* the last dc_decode_device launched it (it may decline later) */
    int dec3_dense;                  /* ... with the dense job buffer (dc_launch_decode3's `dense`) */
    int dense_key;                   /* ct * 256 + bound exponent of the last stream found dense (+1; 0: none):
                                        later decodes with the same parameters start with the dense buffer */
    int dec3_maps;                   /* the pending segment decode parsed by entry -> exit maps */
    int maps_key;                    /* as dense_key, for streams whose parse paths did not meet */
    int dec3_fusedl;                 /* the pending segment decode's launch was the fused one */
    void* maps_scr; size_t maps_scr_cap;
    int halo_async;                  /* dc_halo_decode_device without dc_decode_finish (dc_set_halo_async) */
    int runs_used;                   /* the pending decode ran the small-stream decoder (dc_decode_runs.hip) */
    int runs_last;                   /* the last finished decode's values came from it */
    uint8_t* runs_maps;              /* its chunk maps */
    const uint8_t* sh3_s;            /* the last dc_decode_shard3_device call (for its fix) */
    Params sh3_P;
    Dec3Bufs sh3_D3;
    float* sh3_out;
    long long sh3_num;
    int sh3_ok;
    const unsigned long long* dec_dnbits;   /* the pending decode's device bit count (or NULL) */
    unsigned long long dec_hnbits;          /* ... or its host bit count */
    const float* dec_hin;            /* its incoming values (shard mode 2) */
    int shard_deferred;              /* 1: tile-0 prefixes wait for dc_decode_shard_fix, 2: later tiles too */
    void* shard_buf; size_t shard_cap;
    void* halo_a; size_t halo_a_cap;
    void* halo_b; size_t halo_b_cap;
    /* pinned host scratch */
    unsigned long long* h_scratch;   /* [0] total bits [1] err [2..] misc */
    /* staging for the host-pointer ABI */
    void* d_a; size_t d_a_cap;
    void* d_b; size_t d_b_cap;
    /* aux */
    float* part_v; long long* part_i;
    float* d_f;                      /* [0] min [1] mean */
    void* prep_part; size_t prep_part_cap;  /* dc_prep_device: the chunks' partial minima (float) and first zeros (i64) */
    void* sub_buf; size_t sub_buf_cap;      /* x - min written out: dc_prep_device / dc_encode_sub_device fallbacks */
    const float* enc_sub;                   /* encode_on: the minimum to subtract while loading (NULL: none) */
    const float* enc_subp;                  /* encode_on: the same on the device (the halo path; NULL: none) */
    hipStream_t st2;                        /* dc_halo_decode2_device: the second plane's stream */
    hipEvent_t ev_h0, ev_h1;                /* its fork and join with the library stream */
    void* halo_a2; size_t halo_a2_cap;      /* the second plane's values (decode2) / gathered floats (encode2) */
    float* part_v2; long long* part_i2;     /* encode2: the second plane's minimum partials */
    uint64_t* enc_desc2; long long enc_desc2_cap;   /* encode2: the second encode's tile states */
    unsigned* d_enc_flag2;                  /* encode2: its flags */
    uint32_t enc_epoch2;                    /* encode2: its epoch */
    uint8_t* runs_maps2;                    /* the second plane's small-stream decoder scratch */
    int halo_unfused;                       /* 1: the halo encode's separate passes (dc_set_halo_unfused, A/B) */
    int capturing;                          /* between dc_capture_begin and dc_capture_end */
    int enc_precleared;                     /* (capture) the next encode's tile states were zeroed by min_final */
    unsigned* gcnt;                         /* the halo gathers' last-workgroup counters (one per halo stream) */
    int capture_bad;                        /* a call inside the capture that a replay cannot repeat */
    char capture_why[160];
    int tiny_used, tiny_last;               /* the pending decode went to / the last finished one stayed on the
                                               one-workgroup decoder (dc_decode_tiny.hip) */
    int tiny_key;                           /* ct * 256 + B + 1 of parameters whose small stream it declined */
    long long dec_max_bytes;                /* the pending decode's readable stream bytes */
    void* med_scr; size_t med_scr_cap;  /* exact mean: chunk transducers (dc_med_scratch_bytes) */
    int med_wide;                        /* the last exact mean needed the wide binade window */
    int* d_i;                        /* [0] type */
    uint32_t* d_crctab; uint32_t* d_x2n; uint32_t* d_crcparts; long long crcparts_cap; uint32_t* d_crc;
    uint32_t* d_crcf;                /* the fused CRC's tables (dc_crcf_tables) */
    uint32_t* crcf_blk[3];           /* 16 KiB block accumulators: the encoder's, a stream's, the resend's */
    long long crcf_cap[3];
    unsigned long long* d_ham;
    unsigned long long* d_ratio;     /* ratio estimators: [0] bits [1] -1.0 flag */
    /* CT1 byte-wise codec */
    void* c1_scr; size_t c1_scr_cap;
    void* c1_in; size_t c1_in_cap;
    void* c1_codes; size_t c1_codes_cap;
    void* c1_pos; size_t c1_pos_cap;
    void* c1_out; size_t c1_out_cap;
    char msg[512];
} dc_ctx;

static dc_ctx G;

static int seterr(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(G.msg, sizeof G.msg, fmt, ap);
    va_end(ap);
    return code;
}

#define HIPCHK(call)                                                                              \
    do {                                                                                          \
        hipError_t e_ = (call);                                                                   \
        if (e_ != hipSuccess) return seterr(DC_ERR_HIP, "%s: %s", #call, hipGetErrorString(e_)); \
    } while (0)

const char* dc_last_error(void) { return G.msg; }
#define ENC_ST (G.enc_st ? G.enc_st : G.st)
/* the decoder build of the current decode: 1024-bit chunks, or 256-bit chunks (symbols with _s) */
#define DV(fn) (G.dec_small ? fn##_s : fn)
static long long g_small_max = -2;
static long long small_chunk_max_bytes(void) {   /* DC_SMALL_CHUNK_MAX_BYTES overrides (0: never) */
    if (g_small_max == -2) {
        const char* e = getenv("DC_SMALL_CHUNK_MAX_BYTES");
        g_small_max = (e && *e) ? atoll(e) : (1ll << 20);
    }
    return g_small_max;
}
/* streams of at most this capacity decode with the 256-bit-chunk build (< 0: the default, 1 MiB);
 * returns the previous value */
long long dc_set_small_chunk_max_bytes(long long v) {
    const long long old = small_chunk_max_bytes();
    g_small_max = v < 0 ? (1ll << 20) : v;
    return old;
}
static int ensure_init(void);
/* encoder launches go to this HIP stream (NULL: the library stream), so a caller can overlap the
 * encode of one buffer with the decode of another; the caller orders dependent work with events */
int dc_set_encode_stream(void* stream) {
    int rc = ensure_init();
    if (rc) return rc;
    G.enc_st = (hipStream_t)stream;
    if (G.enc_st == G.st) G.enc_st = NULL;
    return DC_OK;
}
int dc_abi_status(void) { return G.abi_rc; }
void dc_abi_set_status(int rc) { G.abi_rc = rc; }      /* the double ABI (dc_host64.c) reports through it too */
int dc_set_error(int code, const char* msg) { return seterr(code, "%s", msg); }
void* dc_get_stream(void) { return (void*)G.st; }
void dc_set_abs_error_bound(double bound) { absErrBound = bound; absErrorBound_binary = -100; }
double dc_get_abs_error_bound(void) { return absErrBound; }
long long dc_decode_chunk_bits_value(void) { return DV(dc_decode_chunk_bits)(); }   /* of the last decode */

/* diagnostic: copy the decoder phase stamps ([tile][16] s_memrealtime, 100 MHz) to the host */
int dc_debug_stamps(unsigned long long* host, long long n) {
    if (!G.D.dbg) return DC_ERR_ARG;
    if (n > 4096 * 16) n = 4096 * 16;
    HIPCHK(hipStreamSynchronize(G.st));
    HIPCHK(hipMemcpy(host, G.D.dbg, (size_t)n * 8, hipMemcpyDeviceToHost));
    return DC_OK;
}

int dc_debug_enc_stamps(unsigned long long* host, long long n) {
    if (!G.enc_dbg) return DC_ERR_ARG;
    if (n > 16384 * 8) n = 16384 * 8;
    HIPCHK(hipStreamSynchronize(G.st));
    HIPCHK(hipMemcpy(host, G.enc_dbg, (size_t)n * 8, hipMemcpyDeviceToHost));
    return DC_OK;
}

/* carry-less a*b mod P (reflected CRC-32) and x^(8n) mod P, as zlib's crc32_combine */
static uint32_t h_multmodp(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (int i = 0; i < 32; i++) {
        if (a & m) p ^= b;
        m >>= 1;
        b = (b & 1u) ? (b >> 1) ^ 0xEDB88320u : b >> 1;
    }
    return p;
}
static uint32_t h_xpow8n(unsigned long long n, const uint32_t* x2n) {
    uint32_t p = 1u << 31;                          /* x^0 */
    int k = 3;
    while (n) {
        if (n & 1) p = h_multmodp(x2n[k & 31], p);
        n >>= 1;
        k++;
    }
    return p;
}

int dc_init(int device) {
    if (G.inited) return DC_OK;
    {   /* run-time override of the compile-time bound, so an unchanged app binary can run at another
         * bound (the reference recompiles after impl/set-parameter.sh edits the header) */
        const char* eb = getenv("DC_ABS_ERROR_BOUND");
        if (eb && *eb && atof(eb) > 0.0) dc_set_abs_error_bound(atof(eb));
    }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return seterr(DC_ERR_NOGPU, "no HIP device visible");
    if (device < 0 || device >= n) return seterr(DC_ERR_ARG, "device %d out of range", device);
    HIPCHK(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return seterr(DC_ERR_NOGPU, "device %d is %s, libdcamd is built for gfx950", device, prop.gcnArchName);
    G.device = device;
    HIPCHK(hipStreamCreateWithFlags(&G.st, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&G.ev_enc, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&G.ev_lib, hipEventDisableTiming));
    HIPCHK(hipHostMalloc((void**)&G.h_scratch, 64 * sizeof(unsigned long long), 0));
    HIPCHK(hipMalloc((void**)&G.d_total, 64));
    HIPCHK(hipMalloc((void**)&G.d_enc_err, 64));
    HIPCHK(hipMemset(G.d_enc_err, 0, 64));
    /* a flag per 2048 tiles (up to 2^33 floats) + the single pass's tile ticket (word 1088) */
    HIPCHK(hipMalloc((void**)&G.d_enc_flag, 8192));
    HIPCHK(hipMemset(G.d_enc_flag, 0, 8192));
    G.enc_epoch = 0;
    HIPCHK(hipMalloc((void**)&G.part_v, DC_MIN_PARTS * sizeof(float)));
    HIPCHK(hipMalloc((void**)&G.part_i, DC_MIN_PARTS * sizeof(long long)));
    HIPCHK(hipMalloc((void**)&G.d_f, 64));
    HIPCHK(hipMalloc((void**)&G.d_i, 64));
    HIPCHK(hipMalloc((void**)&G.d_crc, 64));
    HIPCHK(hipMalloc((void**)&G.d_ham, 64));
    /* CRC tables: zlib's byte table T0, slicing tables T1..T3 (a byte followed by k zero bytes),
     * x^(2^k) mod P (reflected) and kpow[j] = x^(8 * run * j) mod P for the block combine */
    uint32_t tab[4 * 256 + 256], x2n[32];
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        tab[i] = c;
    }
    for (int k = 1; k < 4; k++)
        for (int i = 0; i < 256; i++) tab[k * 256 + i] = (tab[(k - 1) * 256 + i] >> 8) ^ tab[tab[(k - 1) * 256 + i] & 0xFFu];
    uint32_t p = 1u << 30;                          /* x^1 */
    x2n[0] = p;
    for (int k = 1; k < 32; k++) x2n[k] = p = h_multmodp(p, p);
    {
        const unsigned long long run = (unsigned long long)dc_crc_run_bytes();
        for (int j = 0; j < 256; j++) tab[1024 + j] = h_xpow8n(run * (unsigned long long)j, x2n);
    }
    {
        uint32_t ct[DC_CRCF_WORDS];
        dc_crcf_tables(ct);
        HIPCHK(hipMalloc((void**)&G.d_crcf, sizeof ct));
        HIPCHK(hipMemcpy(G.d_crcf, ct, sizeof ct, hipMemcpyHostToDevice));
    }
    HIPCHK(hipMalloc((void**)&G.d_crctab, sizeof tab));
    HIPCHK(hipMalloc((void**)&G.d_x2n, sizeof x2n));
    HIPCHK(hipMemcpy(G.d_crctab, tab, sizeof tab, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(G.d_x2n, x2n, sizeof x2n, hipMemcpyHostToDevice));
    G.dec_epoch = 1;
    G.inited = 1;
    return DC_OK;
}

static int ensure_init(void) { return G.inited ? DC_OK : dc_init(0); }

int dc_synchronize(void) {
    int rc = ensure_init();
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(G.st));
    if (G.enc_st) HIPCHK(hipStreamSynchronize(G.enc_st));
    return DC_OK;
}

static int grow(void** p, size_t* cap, size_t need) {
    if (*cap >= need) return DC_OK;
    if (*p) HIPCHK(hipFree(*p));
    *p = NULL;
    size_t n = need + need / 8 + 4096;
    HIPCHK(hipMalloc(p, n));
    *cap = n;
    return DC_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* codec parameters (bound-derived thresholds computed exactly as the reference's double compares) */
static int bound_binary(double bound) {                     /* to_absErrorBound_binary :5512 */
    for (int n = 0; n < 100; n++)
        if (bound >= pow(2, -n)) return n;
    return 100;
}

static float thr_lt(double bound) {
    float f = (float)bound;
    while ((double)f >= bound) f = nextafterf(f, 0.0f);
    while ((double)nextafterf(f, INFINITY) < bound) f = nextafterf(f, INFINITY);
    return f;
}

static float thr_le(double bound) {
    float f = (float)bound;
    while ((double)f > bound) f = nextafterf(f, 0.0f);
    while ((double)nextafterf(f, INFINITY) <= bound) f = nextafterf(f, INFINITY);
    return f;
}

static void make_params(Params* P, int ct, int type, uint32_t mask17) {
    memset(P, 0, sizeof *P);                         /* (P->sub = 0: dc_encode_sub_device sets it) */
    P->ct = ct;
    P->B = bound_binary(absErrBound);
    P->thr_lt = thr_lt(absErrBound);
    P->thr_le = thr_le(absErrBound);
    P->type = type;
    P->mask17 = mask17 & 0x1FFFFu;
    int m = P->B + (int)((P->mask17 >> 8) & 0xFF) - 127;
    P->mm = m > 23 ? 23 : (m < 0 ? 0 : m);
    P->mm0 = P->mm > 8 ? P->mm - 8 : 0;
    P->rawadd = P->B - 118;
    P->hm = type > 0 ? (((1u << type) - 1u) << (31 - type)) : 0u;
    P->fsh = 30 - type;
    P->rs = type + 2;
    P->s0 = 17 - P->rs;
    P->s1 = 9 - P->rs;
    P->lm0 = type + 2 + P->mm0;
    P->dlm = P->mm - P->mm0;
    const int tl0 = P->mm0, tl1 = P->mm;
    P->c0 = (P->mask17 << 15) | (tl0 < 15 ? 1u << (14 - tl0) : 0u);
    P->k0 = tl0 > 0 ? (((1u << tl0) - 1u) << (15 - tl0)) : 0u;
    P->c1 = ((P->mask17 >> 8) << 23) | (tl1 < 23 ? 1u << (22 - tl1) : 0u);
    P->k1 = tl1 > 0 ? (((1u << tl1) - 1u) << (23 - tl1)) : 0u;
    {   /* masked token = head ones(type), flag, then the low tl bits of the raw top bits */
        const uint32_t head = type > 0 ? ((1u << type) - 1u) << 1 : 0u;
        P->em0 = (1u << tl0) - 1u;
        P->eh0 = head << tl0;
        P->em1 = tl1 >= 32 ? 0xFFFFFFFFu : (1u << tl1) - 1u;
        P->eh1 = (head | 1u) << tl1;
        /* v of a masked float with flag 0 (mantissa top 8 bits = the mask's) and zero bits below them:
           the mask's 17 bits cut to 9 + mm bits; its low tl0 bits are the token's tail bits */
        const uint32_t v0 = (P->mask17 << 15) >> (23 - tl1);
        P->K0 = v0 ^ P->eh0;
        P->K1 = ((P->mask17 >> 8) << tl1) ^ P->eh1;
        P->lm1 = P->lm0 + P->dlm;
    }
}

static int valid_ct(int ct) { return ct == 5 || ct == 6 || ct == 7 || ct == 11; }

size_t dc_stream_capacity(long long n) { return (size_t)((n * 32 + 7 + 31) / 32) * 4 + 64; }

/* ------------------------------------------------------------------------------------------ */
static int encode_on(hipStream_t st, int ct, const void* d_x, long long n, long long idx0, int type, uint32_t mask17,
                     int start_bit, void* d_out, unsigned long long* d_total_bits, uint32_t* crc_blk);

/* public entry: on the encode stream (dc_set_encode_stream) after the work queued on the library stream */
int dc_encode_device(int ct, const void* d_x, long long n, long long idx0, int type, uint32_t mask17,
                     int start_bit, void* d_out, unsigned long long* d_total_bits) {
    int rc = ensure_init();
    if (rc) return rc;
    if (G.enc_st) {
        HIPCHK(hipEventRecord(G.ev_enc, G.st));
        HIPCHK(hipStreamWaitEvent(G.enc_st, G.ev_enc, 0));
    }
    return encode_on(ENC_ST, ct, d_x, n, idx0, type, mask17, start_bit, d_out, d_total_bits, NULL);
}

/* internal callers (host ABI, halo path): always on the library stream */
static int encode_lib(int ct, const void* d_x, long long n, long long idx0, int type, uint32_t mask17, int start_bit,
                      void* d_out, unsigned long long* d_total_bits) {
    if (G.enc_st) {                       /* the encoder scratch is shared with encodes on the encode stream */
        HIPCHK(hipEventRecord(G.ev_lib, G.enc_st));
        HIPCHK(hipStreamWaitEvent(G.st, G.ev_lib, 0));
    }
    return encode_on(G.st, ct, d_x, n, idx0, type, mask17, start_bit, d_out, d_total_bits, NULL);
}

/* the fused CRC's block accumulators of slot k, for streams of up to max_bytes (zeroed when grown; each combine
   launch zeroes the blocks it reads) */
static uint32_t* crcf_slot(int k, long long max_bytes) {
    const long long nb = dc_crcf_blocks(max_bytes) + 4;
    if (nb > G.crcf_cap[k]) {
        if (G.crcf_blk[k] && hipFree(G.crcf_blk[k]) != hipSuccess) return NULL;
        G.crcf_blk[k] = NULL;
        if (hipMalloc((void**)&G.crcf_blk[k], (size_t)nb * 4) != hipSuccess) return NULL;
        if (hipMemset(G.crcf_blk[k], 0, (size_t)nb * 4) != hipSuccess) return NULL;
        G.crcf_cap[k] = nb;
    }
    return G.crcf_blk[k];
}

/* CT9 sender: dc_encode_device at start bit 0, plus the zlib CRC-32 of the stream bytes into d_crc (device, one
   uint32): the encoder's tiles XOR the raw CRCs of the words they store into 16 KiB block accumulators and one
   combine launch follows -- no pass over the stream (dc_encode_result re-encodes wait-free after a look-back
   timeout and then computes the CRC by a pass) */
int dc_encode_crc_device(int ct, const void* d_x, long long n, long long idx0, int type, uint32_t mask17, void* d_out,
                         unsigned long long* d_total_bits, uint32_t* d_crc) {
    int rc = ensure_init();
    if (rc) return rc;
    if (!d_crc || !d_total_bits) return seterr(DC_ERR_ARG, "encode crc: need d_total_bits and d_crc");
    if (G.enc_st) {
        HIPCHK(hipEventRecord(G.ev_enc, G.st));
        HIPCHK(hipStreamWaitEvent(G.enc_st, G.ev_enc, 0));
    }
    const long long cap = (long long)dc_stream_capacity(n);
    uint32_t* blk = crcf_slot(0, cap);
    if (!blk) return seterr(DC_ERR_HIP, "crc block allocation failed");
    if ((rc = encode_on(ENC_ST, ct, d_x, n, idx0, type, mask17, 0, d_out, d_total_bits, n > 0 ? blk : NULL))) return rc;
    G.last_enc.crc = d_crc;
    if (n > 0 && !dc_encode_crc_fused_last()) {  /* (a multi-pass or chained look-back variant: a pass of its own) */
        unsigned long long bits = 0;
        HIPCHK(hipMemcpyAsync(&bits, d_total_bits, 8, hipMemcpyDeviceToHost, ENC_ST));
        HIPCHK(hipStreamSynchronize(ENC_ST));
        if (dc_launch_crcf_blocks((const uint8_t*)d_out, NULL, (long long)((bits + 7) / 8), G.d_crcf, blk, NULL, NULL, ENC_ST))
            return seterr(DC_ERR_HIP, "crc launch failed");
    }
    if (dc_launch_crcf_final(blk, cap, n > 0 ? -1 : 0, n > 0 ? d_total_bits : NULL, G.d_crcf, d_crc, NULL, NULL, NULL,
                             ENC_ST))
        return seterr(DC_ERR_HIP, "crc launch failed");
    return DC_OK;
}

/* dc_launch_encode, and for an encode of x - min (P->sub) that the chosen variant cannot subtract while loading
   (dc_launch_encode returns -3: the three-launch retry, the CRC / send / helping instantiations), x - min written
   into sub_buf first and encoded from there */
static int launch_enc(const float* x, long long n, long long idx0, const Params* P, uint32_t* out, uint64_t* desc,
                      unsigned* flag, uint32_t epoch, int start_bit, unsigned long long* tb, unsigned long long* tb2,
                      unsigned* err, unsigned long long* dbg, int mode, const uint32_t* ctab, uint32_t* cblk,
                      hipStream_t st) {
    const int r = dc_launch_encode(x, n, idx0, P, out, desc, flag, epoch, start_bit, tb, tb2, err, dbg, mode, ctab, cblk, st);
    if (r != -3) return r;
    if (grow(&G.sub_buf, &G.sub_buf_cap, (size_t)n * 4 + 64)) return -1;
    if (P->subp ? dc_launch_sub_ptr(x, n, P->subp, (float*)G.sub_buf, st)
                : dc_launch_sub_value(x, n, P->submin, (float*)G.sub_buf, st))
        return -1;
    Params Q = *P;
    Q.sub = 0;
    return dc_launch_encode((const float*)G.sub_buf, n, idx0, &Q, out, desc, flag, epoch, start_bit, tb, tb2, err, dbg,
                            mode, ctab, cblk, st);
}

static int encode_on(hipStream_t st, int ct, const void* d_x, long long n, long long idx0, int type, uint32_t mask17,
                     int start_bit, void* d_out, unsigned long long* d_total_bits, uint32_t* crc_blk) {
    if (!valid_ct(ct)) return seterr(DC_ERR_ARG, "unsupported CT %d", ct);
    if (start_bit < 0 || start_bit > 7 || n < 0) return seterr(DC_ERR_ARG, "bad start_bit/n");
    if (n > (1ll << 33)) return seterr(DC_ERR_ARG, "n above 2^33 floats");
    if (ct == 7 && (type < 1 || type > 7)) return seterr(DC_ERR_ARG, "CT7 type %d outside 1..7", type);
    if (((uintptr_t)d_x & 15u) || ((uintptr_t)d_out & 3u)) return seterr(DC_ERR_ARG, "misaligned device buffer");
    Params P;
    make_params(&P, ct, type, mask17);
    if (G.enc_subp) {                                /* the halo path: the minimum on the device */
        if (idx0) return seterr(DC_ERR_ARG, "encode of x - min: idx0 must be 0");
        P.sub = 1;
        P.subp = G.enc_subp;
    } else if (G.enc_sub) {                          /* dc_encode_sub_device */
        if (idx0) return seterr(DC_ERR_ARG, "encode of x - min: idx0 must be 0");
        P.sub = 1;
        P.submin = *G.enc_sub;
        if (!isfinite(P.submin)) {                   /* (the kernels' subtraction assumes a finite minimum) */
            if (n > 0 && (grow(&G.sub_buf, &G.sub_buf_cap, (size_t)n * 4 + 64) ||
                          dc_launch_sub_value((const float*)d_x, n, P.submin, (float*)G.sub_buf, st)))
                return seterr(DC_ERR_HIP, "x - min launch failed");
            d_x = G.sub_buf;
            P.sub = 0;
        }
    }
    if (dc_encode_desc_words(n) + 8 > G.enc_desc_cap) {
        if (G.enc_desc) HIPCHK(hipFree(G.enc_desc));
        long long cap = dc_encode_desc_words(n) + 1024;
        HIPCHK(hipMalloc((void**)&G.enc_desc, cap * sizeof(uint64_t)));
        HIPCHK(hipMemsetAsync(G.enc_desc, 0, cap * sizeof(uint64_t), st));
        G.enc_desc_cap = cap;
    }
    unsigned long long* tot = d_total_bits ? d_total_bits : G.d_total;
    G.last_enc_st = st;
    if (n == 0) {
        unsigned long long v = (unsigned long long)start_bit;
        HIPCHK(hipMemcpyAsync(tot, &v, sizeof v, hipMemcpyHostToDevice, st));
        if (tot != G.d_total) HIPCHK(hipMemcpyAsync(G.d_total, &v, sizeof v, hipMemcpyHostToDevice, st));
        return DC_OK;
    }
    if (getenv("DC_DEBUG_STAMPS") && !G.enc_dbg) {
        HIPCHK(hipMalloc((void**)&G.enc_dbg, 16384 * 8 * 8));
        HIPCHK(hipMemset(G.enc_dbg, 0, 16384 * 8 * 8));
    }
    /* the kernel writes the total to both (no copy node per encode).  Epochs tag the tile states and flags:
       when they wrap, every old tag is cleared (a state of an old encode must never read as published) */
    if (G.capturing) {
        /* a graph replays the same epoch each time: the tile states this encode reads are cleared in the graph
           (by the halo path's min_final launch, or here) */
        if (!G.enc_precleared) {
            HIPCHK(hipMemsetAsync(G.enc_desc, 0, (size_t)(dc_encode_desc_words(n) + 8) * sizeof(uint64_t), st));
            HIPCHK(hipMemsetAsync(G.d_enc_flag, 0, 4096, st));
        }
        G.enc_epoch = 1;
    } else if (++G.enc_epoch >= dc_encode_epoch_limit() || G.enc_epoch == 1) {
        HIPCHK(hipMemsetAsync(G.enc_desc, 0, (size_t)G.enc_desc_cap * sizeof(uint64_t), st));
        HIPCHK(hipMemsetAsync(G.d_enc_flag, 0, 4096, st));
        G.enc_epoch = 1;
    }
    if (launch_enc((const float*)d_x, n, idx0, &P, (uint32_t*)d_out, G.enc_desc, G.d_enc_flag, G.enc_epoch,
                         start_bit, tot, tot != G.d_total ? G.d_total : NULL, G.d_enc_err, G.enc_dbg, 0,
                         crc_blk ? G.d_crcf : NULL, crc_blk, st))
        return seterr(DC_ERR_HIP, "encode launch failed: %s", hipGetErrorString(hipGetLastError()));
    G.last_enc.x = (const float*)d_x; G.last_enc.n = n; G.last_enc.idx0 = idx0; G.last_enc.P = P;
    G.last_enc.out = (uint32_t*)d_out; G.last_enc.start_bit = start_bit; G.last_enc.tot = tot; G.last_enc.st = st;
    G.last_enc.valid = 1;
    G.last_enc.crc = NULL;
    G.last_enc.mirror = NULL;
    G.enc_outstanding++;
    return DC_OK;
}

/* CT9 send: the encode, its stream words written into the receiver's buffer d_mirror as well (the channel) --
   the sender keeps d_out for a resend; the CRCs come after (dc_crc32_pair_device) */
int dc_encode_send_device(int ct, const void* d_x, long long n, long long idx0, int type, uint32_t mask17,
                          void* d_out, void* d_mirror, unsigned long long* d_total_bits) {
    int rc = ensure_init();
    if (rc) return rc;
    if (!d_mirror || ((uintptr_t)d_mirror & 3u)) return seterr(DC_ERR_ARG, "send: the receiver's buffer must be 4-byte aligned");
    if (G.enc_st) {
        HIPCHK(hipEventRecord(G.ev_enc, G.st));
        HIPCHK(hipStreamWaitEvent(G.enc_st, G.ev_enc, 0));
    }
    dc_set_encode_mirror(d_mirror);
    rc = encode_on(ENC_ST, ct, d_x, n, idx0, type, mask17, 0, d_out, d_total_bits, NULL);
    dc_set_encode_mirror(NULL);
    if (!rc) G.last_enc.mirror = d_mirror;
    return rc;
}

/* bits an encode of these n floats would produce (no stream written); synchronous */
int dc_encode_bits_device(int ct, const void* d_x, long long n, long long idx0, int type, uint32_t mask17,
                          unsigned long long* bits_out) {
    int rc = ensure_init();
    if (rc) return rc;
    if (!valid_ct(ct)) return seterr(DC_ERR_ARG, "unsupported CT %d", ct);
    if (n < 0) return seterr(DC_ERR_ARG, "n < 0");
    if (ct == 7 && (type < 1 || type > 7)) return seterr(DC_ERR_ARG, "CT7 type %d outside 1..7", type);
    if ((uintptr_t)d_x & 15u) return seterr(DC_ERR_ARG, "misaligned device buffer");
    if (n == 0) { *bits_out = 0; return DC_OK; }
    Params P;
    make_params(&P, ct, type, mask17);
    if (G.enc_st) {
        HIPCHK(hipEventRecord(G.ev_enc, G.st));
        HIPCHK(hipStreamWaitEvent(G.enc_st, G.ev_enc, 0));
    }
    if (dc_encode_desc_words(n) + 8 > G.enc_desc_cap) {
        if (G.enc_desc) HIPCHK(hipFree(G.enc_desc));
        const long long cap = dc_encode_desc_words(n) + 1024;
        HIPCHK(hipMalloc((void**)&G.enc_desc, cap * sizeof(uint64_t)));
        G.enc_desc_cap = cap;
    }
    /* (its own error word: the single-pass encodes' word keeps what they left) */
    HIPCHK(hipMemsetAsync(G.d_enc_err + 8, 0, 4, ENC_ST));
    if (dc_launch_encode_bits((const float*)d_x, n, idx0, &P, G.enc_desc, G.d_total, G.d_enc_err + 8, ENC_ST))
        return seterr(DC_ERR_HIP, "encode launch failed");
    HIPCHK(hipMemcpyAsync(&G.h_scratch[0], G.d_total, 8, hipMemcpyDeviceToHost, ENC_ST));
    HIPCHK(hipMemcpyAsync(&G.h_scratch[1], G.d_enc_err + 8, 4, hipMemcpyDeviceToHost, ENC_ST));
    HIPCHK(hipStreamSynchronize(ENC_ST));
    if (G.h_scratch[1] & 1u) return seterr(DC_ERR_INPUT, "input contains -1.0f (the reference's history sentinel)");
    *bits_out = G.h_scratch[0];
    return DC_OK;
}

/* after an encode error that is reported, not repaired: the fused CRC's slot-0 block accumulators may hold
   pieces of tiles past the bits the combine read (it zeroes only those), so clear the whole slot; the
   receiver's buffer and CRC of that encode are forgotten (a later retry must not write into them) */
static int enc_forget_failed(hipStream_t st) {
    if (G.crcf_blk[0] && G.crcf_cap[0] > 0) HIPCHK(hipMemsetAsync(G.crcf_blk[0], 0, (size_t)G.crcf_cap[0] * 4, st));
    G.last_enc.mirror = NULL;
    G.last_enc.crc = NULL;
    G.last_enc.valid = 0;
    return DC_OK;
}

/* re-run the last encode with no wait between workgroups (count, scan launch, pack) */
static int encode_retry(hipStream_t st) {
    HIPCHK(hipMemsetAsync(G.d_enc_err, 0, 4, st));
    if (++G.enc_epoch >= dc_encode_epoch_limit()) {
        HIPCHK(hipMemsetAsync(G.enc_desc, 0, (size_t)G.enc_desc_cap * sizeof(uint64_t), st));
        HIPCHK(hipMemsetAsync(G.d_enc_flag, 0, 4096, st));
        G.enc_epoch = 1;
    }
    unsigned long long* tot = G.last_enc.tot;
    dc_set_encode_mirror(G.last_enc.mirror);
    const int lrc = launch_enc(G.last_enc.x, G.last_enc.n, G.last_enc.idx0, &G.last_enc.P, G.last_enc.out,
                                     G.enc_desc, G.d_enc_flag, G.enc_epoch, G.last_enc.start_bit, tot,
                                     tot != G.d_total ? G.d_total : NULL, G.d_enc_err, NULL, 3, NULL, NULL, st);
    dc_set_encode_mirror(NULL);
    if (lrc) return seterr(DC_ERR_HIP, "encode launch failed: %s", hipGetErrorString(hipGetLastError()));
    G.enc_retries++;
    G.enc_outstanding = 1;
    return DC_OK;
}
int dc_encode_retries(void) { return G.enc_retries; }

/* the encoder's error word as the kernels left it (synchronous; nothing cleared, nothing re-run): bit 0 the
   -1.0f sentinel in the input, 2 a tile offset outside the stream, 4 a look-back / flag wait timed out */
int dc_encode_status(unsigned* status_out) {
    int rc = ensure_init();
    if (rc) return rc;
    hipStream_t st = G.last_enc_st ? G.last_enc_st : G.st;
    HIPCHK(hipMemcpyAsync(&G.h_scratch[1], G.d_enc_err, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    *status_out = (unsigned)(G.h_scratch[1] & 0xFFFFFFFFu);
    return DC_OK;
}

int dc_encode_result(unsigned long long* total_bits) {
    int rc = ensure_init();
    if (rc) return rc;
    hipStream_t st = G.last_enc_st ? G.last_enc_st : G.st;
    HIPCHK(hipMemcpyAsync(&G.h_scratch[0], G.d_total, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&G.h_scratch[1], G.d_enc_err, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    unsigned err = (unsigned)(G.h_scratch[1] & 0xFFFFFFFFu);
    if ((err & 4u) && G.enc_outstanding > 1) {
        /* the error word is OR-ed over every encode since it was last checked: the one that timed out may be
           an earlier one, whose stream a later launch has already consumed -- re-running the last encode
           would not repair it, so report it and leave the word set (dc_encode_clear_status clears it) */
        if ((rc = enc_forget_failed(st))) return rc;
        return seterr(DC_ERR_HIP, "a look-back wait timed out in one of the %d encodes issued since the encoder's "
                                  "error word was last checked (err=%u): their streams may lack tiles",
                      G.enc_outstanding, err);
    }
    if ((err & 4u) && !(err & 1u) && G.last_enc.valid) {
        /* a single-pass tile waited past its bound for a predecessor (a workgroup not resident: another
           process on the GPU) and stored nothing: encode again with the wait-free three-launch variant */
        const int ok = encode_retry(st);
        if (ok) return ok;
        HIPCHK(hipMemcpyAsync(&G.h_scratch[0], G.d_total, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(&G.h_scratch[1], G.d_enc_err, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        err = (unsigned)(G.h_scratch[1] & 0xFFFFFFFFu);
        if (!err && G.last_enc.crc) {             /* the retried stream's CRC, by a pass of its own */
            const long long nb = (long long)((G.h_scratch[0] + 7) / 8);
            uint32_t* blk = crcf_slot(0, nb);
            if (!blk || dc_launch_crcf_blocks((const uint8_t*)G.last_enc.out, NULL, nb, G.d_crcf, blk, NULL, NULL, st) ||
                dc_launch_crcf_final(blk, nb, nb, NULL, G.d_crcf, G.last_enc.crc, NULL, NULL, NULL, st))
                return seterr(DC_ERR_HIP, "crc launch failed");
        }
    }
    if (err) {
        HIPCHK(hipMemsetAsync(G.d_enc_err, 0, 4, st));
        G.enc_outstanding = 0;
        if ((rc = enc_forget_failed(st))) return rc;
        if (err & 1u)
            return seterr(DC_ERR_INPUT, "input contains -1.0f, the reference encoder's empty-history sentinel "
                                        "(impl/dataCompression.c:2032); CT5/7/11 inputs must be >= 0 (toSmallDataset_float)");
        return seterr(DC_ERR_HIP, "encoder tile offsets inconsistent, nothing stored (err=%u)", err);
    }
    G.enc_outstanding = 0;                       /* every encode so far checked clean */
    if (total_bits) *total_bits = G.h_scratch[0];
    return DC_OK;
}

/* clear the single-pass encoder's error word (after dc_encode_result reported a timeout among several
   outstanding encodes) */
int dc_encode_clear_status(void) {
    int rc = ensure_init();
    if (rc) return rc;
    hipStream_t st = G.last_enc_st ? G.last_enc_st : G.st;
    HIPCHK(hipMemsetAsync(G.d_enc_err, 0, 4, st));
    G.enc_outstanding = 0;
    return enc_forget_failed(st);
}

/* ------------------------------------------------------------------------------------------ */
static int dec_ensure(long long max_chunks) {
    if (max_chunks <= G.dec_cap_chunks) return DC_OK;
    if (G.dec_pool) HIPCHK(hipFree(G.dec_pool));
    G.dec_pool = NULL;
    long long C = max_chunks + 4096;
    long long GR = (C + dc_decode_group() - 1) / dc_decode_group() + 1;
    size_t off = 0, sz[20];
    sz[0] = 256;                          /* plan */
    sz[1] = (size_t)C;                    /* p_exit */
    sz[2] = (size_t)C * 2;                /* p_cnt */
    sz[3] = (size_t)C * 4;                /* p_mask */
    sz[4] = (size_t)C * 32 * 4;           /* map */
    sz[5] = (size_t)GR * 32 * 4;          /* fullmap */
    sz[6] = (size_t)GR * 34 * 8;          /* gran */
    sz[7] = (size_t)C;                    /* entry */
    sz[8] = (size_t)C * 8;                /* tokoff */
    sz[9] = (size_t)C * 2;                /* pend */
    sz[10] = (size_t)C * 2;               /* done */
    sz[11] = 64;                          /* err */
    sz[12] = 64;                          /* ctr */
    sz[13] = (size_t)C * 4;               /* known */
    sz[14] = (size_t)C * 8;               /* exitmask */
    sz[15] = (size_t)GR * 6 * 8;          /* hist */
    sz[16] = (size_t)C * 4;               /* cmeta */
    sz[17] = (size_t)GR * 32 * 4;         /* tmap */
    sz[18] = (size_t)GR * 4;              /* tentry */
    sz[19] = (size_t)GR * 8;              /* tbase */
    size_t tot = 0;
    for (int i = 0; i < 20; i++) tot += (sz[i] + 255) & ~(size_t)255;
    HIPCHK(hipMalloc(&G.dec_pool, tot));
    HIPCHK(hipMemsetAsync(G.dec_pool, 0, tot, G.st));
    char* b = (char*)G.dec_pool;
    void* ptr[20];
    for (int i = 0; i < 20; i++) { ptr[i] = b + off; off += (sz[i] + 255) & ~(size_t)255; }
    G.D.plan = (Plan*)ptr[0];
    G.D.p_exit = (uint8_t*)ptr[1];
    G.D.p_cnt = (uint16_t*)ptr[2];
    G.D.p_mask = (uint32_t*)ptr[3];
    G.D.map = (uint32_t*)ptr[4];
    G.D.known = (uint32_t*)ptr[13];
    G.D.exitmask = (uint32_t*)ptr[14];
    G.D.hist = (uint64_t*)ptr[15];
    G.D.cmeta = (uint32_t*)ptr[16];
    G.D.tmap = (uint32_t*)ptr[17];
    G.D.tentry = (uint32_t*)ptr[18];
    G.D.tbase = (unsigned long long*)ptr[19];
    G.D.fullmap = (uint32_t*)ptr[5];
    G.D.gran = (uint64_t*)ptr[6];
    G.D.entry = (uint8_t*)ptr[7];
    G.D.tokoff = (unsigned long long*)ptr[8];
    G.D.pend = (uint16_t*)ptr[9];
    G.D.done = (uint16_t*)ptr[10];
    G.D.err = (unsigned*)ptr[11];
    G.D.ctr = (unsigned*)ptr[12];
    G.dec_cap_chunks = C;
    G.dec_epoch = 1;
    G.D.dbg = NULL;
    if (getenv("DC_DEBUG_STAMPS")) {
        HIPCHK(hipMalloc((void**)&G.D.dbg, 4096 * 16 * 8));
        HIPCHK(hipMemset(G.D.dbg, 0, 4096 * 16 * 8));
    }
    return DC_OK;
}

/* next decoder epoch; look-back flags carry 22 epoch bits, so on a wrap the flag arrays are cleared
 * (a stale flag of an old epoch must never read as published) */
static int dec_next_epoch(void) {
    if (++G.dec_epoch >= (1u << 22)) {
        const long long GR = (G.dec_cap_chunks + dc_decode_group() - 1) / dc_decode_group() + 1;
        HIPCHK(hipMemsetAsync(G.D.gran, 0, (size_t)GR * 34 * 8, G.st));
        HIPCHK(hipMemsetAsync(G.D.hist, 0, (size_t)GR * 6 * 8, G.st));
        if (G.dec3_pool) {
            HIPCHK(hipMemsetAsync(G.D3.pexit, 0, (size_t)(G.dec3_cap + 4096) / 256 * 8 + 64 * 8, G.st));
            HIPCHK(hipMemsetAsync(G.D3.hist, 0, (size_t)((G.dec3_cap + 4096) / 64 + 64) * 3 * 8, G.st));
            HIPCHK(hipMemsetAsync(G.D3.ftag, 0, (size_t)((G.dec3_cap + 4096) / 256 + 64) * 8, G.st));
            HIPCHK(hipMemsetAsync(G.D3.fsub, 0, (size_t)((G.dec3_cap + 4096) / 256 + 64) * 16, G.st));
        }
        G.dec_epoch = 1;
    }
    return DC_OK;
}

/* segment decoder buffers for streams of up to max_chunks 256-bit chunks */
static int dec3_ensure(long long max_chunks, int B, int ct) {
    const int seg = dc_decode3_seg(max_chunks, B, ct);
    /* the kernels size their grids from D3.max_chunks: this stream's capacity, not the pool's (a small
       stream after a large one would otherwise launch thousands of idle workgroups) */
    if (max_chunks <= G.dec3_cap && seg == G.D3.seg) { G.D3.max_chunks = max_chunks; return DC_OK; }
    if (max_chunks > G.dec3_cap) {
        if (G.dec3_pool) HIPCHK(hipFree(G.dec3_pool));
        G.dec3_pool = NULL;
        G.sh3_ok = 0;                         /* a pending shard fix would read the freed spend/rec */
        const long long C = max_chunks + 4096;
        const long long DJ = C / 64 + 64, PJ = C / (64 * 4) + 64;
        size_t sz[10], off = 0, tot = 0;
        sz[0] = (size_t)C * 2;                /* rec */
        sz[1] = (size_t)DJ * 4;               /* rel */
        sz[2] = (size_t)PJ * 4;               /* ptot */
        sz[3] = (size_t)PJ * 8;               /* pexit */
        sz[4] = (size_t)DJ * 3 * 8;           /* hist */
        sz[5] = 256;                          /* spend */
        sz[6] = (size_t)PJ * 8;               /* ftag */
        sz[7] = (size_t)DJ * 4 * 2 + 4096;    /* frel (fused jobs of >= 16-chunk segments: < 1.5x rel) */
        sz[8] = (size_t)PJ * 16;              /* fsub */
        sz[9] = 4096;                         /* fq */
        for (int i = 0; i < 10; i++) tot += (sz[i] + 255) & ~(size_t)255;
        HIPCHK(hipMalloc(&G.dec3_pool, tot));
        HIPCHK(hipMemsetAsync(G.dec3_pool, 0, tot, G.st));
        char* b = (char*)G.dec3_pool;
        void* ptr[10];
        for (int i = 0; i < 10; i++) { ptr[i] = b + off; off += (sz[i] + 255) & ~(size_t)255; }
        G.D3.rec = (uint16_t*)ptr[0];
        G.D3.rel = (uint32_t*)ptr[1];
        G.D3.ptot = (uint32_t*)ptr[2];
        G.D3.pexit = (uint64_t*)ptr[3];
        G.D3.hist = (uint64_t*)ptr[4];
        G.D3.spend = (uint32_t*)ptr[5];
        G.D3.ftag = (uint64_t*)ptr[6];
        G.D3.frel = (uint32_t*)ptr[7];
        G.D3.fsub = (uint32_t*)ptr[8];
        G.D3.fq = (unsigned*)ptr[9];
        G.dec3_cap = max_chunks;
    }
    G.D3.max_chunks = max_chunks;
    G.D3.seg = seg;
    return DC_OK;
}

/* streams of at least this capacity use the segment decoder (DC_DEC3_MIN_BYTES; DC_DEC3=0 disables it):
   16 KiB -- from 2^12 floats on (r03: 1 MiB; 4-chunk segments made small streams one short walk) */
#define DEC3_MIN_DEFAULT ((16ll << 10) + 1)
static long long g_dec3_min = -2;
static long long dec3_min_bytes(void) {
    if (g_dec3_min == -2) {
        const char* d = getenv("DC_DEC3");
        const char* e = getenv("DC_DEC3_MIN_BYTES");
        g_dec3_min = (d && *d == '0') ? -1 : ((e && *e) ? atoll(e) : DEC3_MIN_DEFAULT);
    }
    return g_dec3_min;
}
/* DC_TINY=1 (or dc_set_decode_tiny(1)): small streams on the one-workgroup decoder -- opt-in: measured at parity
   with the segment decoder at 2^14 (one CU's VALU issue bounds it) */
static int g_tiny_on = -1;
static int tiny_on(void) {
    if (g_tiny_on < 0) g_tiny_on = (getenv("DC_TINY") && *getenv("DC_TINY") == '1') ? 1 : 0;
    return g_tiny_on;
}
int dc_set_decode_tiny(int on) {
    const int old = tiny_on();
    g_tiny_on = on ? 1 : 0;
    return old;
}
int dc_last_decode_was_tiny(void) { return G.tiny_last; }
/* < -1: the default; -1 disables the segment decoder; returns the previous value */
int dc_last_decode_was_v3(void) { return G.dec3_last; }
int dc_last_decode_used_maps(void) { return G.dec3_last && G.dec3_maps; }
int dc_last_decode_was_runs(void) { return G.runs_last; }
int dc_set_halo_unfused(int on) {
    const int old = G.halo_unfused;
    G.halo_unfused = on ? 1 : 0;
    return old;
}
int dc_set_halo_async(int on) {
    const int old = G.halo_async;
    G.halo_async = on ? 1 : 0;
    /* leaving async mode: the caller has read the status of its planes itself (dc_decode_status), so the queued
       count of those decodes must not make the next decode's dc_decode_finish report them as never completed */
    if (old && !G.halo_async) {
        G.dec_queued = 0;
        G.dec_pending = 0;
    }
    return old;
}
int dc_last_decode_launched_runs(void) { return G.runs_used; }
int dc_last_decode_launched_tiny(void) { return G.tiny_used; }
/* streams of at most this capacity (bytes) use the small-stream decoder (dc_decode_runs.hip), unless the
   segment decoder is forced (dc_set_decode3_min_bytes(0)); halo planes use it up to its chunk limit */
static long long g_runs_max = -2;
static long long runs_max_bytes(void) {
    if (g_runs_max == -2) {
        const char* e = getenv("DC_RUNS_MAX_BYTES");
        g_runs_max = (e && *e) ? atoll(e) : (16ll << 10) + 256;
    }
    return g_runs_max;
}
long long dc_set_runs_max_bytes(long long v) {
    const long long old = runs_max_bytes();
    g_runs_max = v < -1 ? (16ll << 10) + 256 : v;
    return old;
}
int dc_last_decode_launched_v3(void) { return G.dec3_launched; }
long long dc_set_decode3_min_bytes(long long v) {
    const long long old = dec3_min_bytes();
    g_dec3_min = v < -1 ? DEC3_MIN_DEFAULT : v;
    return old;
}

#define DEC_ROUNDS 3
#define DEC_FIX_ITERS 3

/* tests: every segment decode parsed by maps (DC_DEC3_MAPS=1 or dc_set_decode3_maps(1)) */
static int g_maps_force = -1;
static int maps_forced(void) {
    if (g_maps_force < 0) g_maps_force = (getenv("DC_DEC3_MAPS") && *getenv("DC_DEC3_MAPS") == '1') ? 1 : 0;
    return g_maps_force;
}
int dc_set_decode3_maps(int on) {
    const int old = maps_forced();
    g_maps_force = on ? 1 : 0;
    if (on < 0) { G.maps_key = 0; G.dense_key = 0; G.tiny_key = 0; g_maps_force = 0; }   /* tests: forget the remembered streams */
    return old;
}
/* the segment decoder's launch for the pending decode: parse3 + decode3, or the maps parse + decode3
   (G.dec3_maps), with the job buffer G.dec3_dense picks */
static int dec3_launch(const uint8_t* s, const Params* P, float* out, long long num) {
    if (G.dec3_maps) {
        const size_t need = (size_t)dc_maps_scratch_bytes(G.D3.max_chunks);
        if (grow(&G.maps_scr, &G.maps_scr_cap, need)) return DC_ERR_HIP;
        if (dc_launch_maps_parse(s, G.dec_dnbits, G.dec_hnbits, P, &G.D3, num, G.maps_scr, G.st) ||
            dc_launch_decode3_values(s, G.dec_dnbits, G.dec_hnbits, P, &G.D3, out, num, G.dec_epoch, G.dec3_dense, G.st))
            return seterr(DC_ERR_HIP, "decode launch failed: %s", hipGetErrorString(hipGetLastError()));
        return DC_OK;
    }
    if (dc_launch_decode3(s, G.dec_dnbits, G.dec_hnbits, P, &G.D3, out, num, G.dec_epoch, G.dec3_dense, G.st))
        return seterr(DC_ERR_HIP, "decode launch failed: %s", hipGetErrorString(hipGetLastError()));
    G.dec3_fusedl = dc_decode3_last_fused();
    return DC_OK;
}

/* the segment decoder for the pending decode's stream (also after the one-workgroup decoder declined it) */
static int seg_decode_launch(const uint8_t* d_stream, long long nbytes, long long max_bytes, const Params* P,
                             float* d_out, long long num) {
    int rc;
    const int ct = P->ct;
    if ((rc = dec3_ensure((max_bytes * 8 + 255) / 256 + 1, P->B, ct))) return rc;
    G.D3.err = G.D.err;
    G.D3.capw = max_bytes / 16 * 4;
    /* a decode job holds 64 chunks (16384 bits): streams of fewer than ~16 bits per value overflow the
       1040-value job buffer, so a stream known to be that dense (its length given, or the last stream of
       these parameters was) takes the 2080-value instantiation */
    G.dec3_dense = (nbytes >= 0 && nbytes * 8 < 18 * num && (ct == 6 || nbytes * 8 >= 6 * num)) ||
                   G.dense_key == ct * 256 + P->B + 1;                   /* (not runs mode: < 6 bits per value) */
    /* a stream of these parameters whose parse paths did not meet last time: the maps parse at once */
    G.dec3_maps = G.maps_key == ct * 256 + P->B + 1 || maps_forced();
    return dec3_launch(d_stream, P, d_out, num);
}

/* halo: a Himeno halo plane (dc_halo_decode_device): the small-stream decoder up to its chunk limit */
static int decode_device_h(int ct, const void* d_stream, long long nbytes, const unsigned long long* d_nbits,
                           long long max_bytes, long long num, int type, uint32_t mask17, void* d_out, int halo);
int dc_decode_device(int ct, const void* d_stream, long long nbytes, const unsigned long long* d_nbits,
                     long long max_bytes, long long num, int type, uint32_t mask17, void* d_out) {
    return decode_device_h(ct, d_stream, nbytes, d_nbits, max_bytes, num, type, mask17, d_out, 0);
}
static int decode_device_h(int ct, const void* d_stream, long long nbytes, const unsigned long long* d_nbits,
                           long long max_bytes, long long num, int type, uint32_t mask17, void* d_out, int halo) {
    int rc = ensure_init();
    if (rc) return rc;
    if (!valid_ct(ct)) return seterr(DC_ERR_ARG, "unsupported CT %d", ct);
    if (ct == 7 && (type < 1 || type > 7)) return seterr(DC_ERR_ARG, "CT7 type %d outside 1..7", type);
    if ((uintptr_t)d_stream & 3u) return seterr(DC_ERR_ARG, "stream must be 4-byte aligned");
    if (nbytes < 0 && !d_nbits) return seterr(DC_ERR_ARG, "need nbytes or d_nbits");
    if (max_bytes < nbytes) max_bytes = nbytes;
    dc_decode3_clear_fused();             /* (set again by a fused segment-decoder launch) */
    G.dec3_fusedl = 0;
    /* small streams (a Himeno halo plane: 25 KB) decode with 256-bit chunks: 4x more lanes, 4x shorter walks */
    G.dec_small = max_bytes <= small_chunk_max_bytes();
    long long cb = DV(dc_decode_chunk_bits)();
    long long max_chunks = (max_bytes * 8 + cb - 1) / cb;
    if (max_chunks < 1) max_chunks = 1;
    rc = dec_ensure(max_chunks);
    if (rc) return rc;
    if ((rc = dec_next_epoch())) return rc;
    Params P;
    make_params(&P, ct, type, mask17);
    const long long m3 = dec3_min_bytes();
    /* the segment decoder reads whole 16-byte groups through a buffer resource (32-bit byte range): every
       stream byte must lie in one inside max_bytes, and max_bytes and the output below 2 GiB */
    const long long need16 = nbytes >= 0 ? (nbytes + 15) / 16 * 16 : 0;
    const long long mc256 = (max_bytes * 8 + 255) / 256 + 1;
    /* -1 in either knob (DC_DEC3=0 / dc_set_decode3_min_bytes(-1), dc_set_runs_max_bytes(-1)) keeps every
       stream, halo planes included, off the small-stream decoder; 0 forces the segment decoder */
    const long long rmax = runs_max_bytes();
    G.runs_used = !G.D.shard && num >= 1 && mc256 <= dc_decode_runs_max_chunks() + 8 && m3 > 0 && rmax >= 0 &&
                  (halo || max_bytes <= rmax);
    G.dec3_used = !halo && !G.runs_used && m3 >= 0 && max_bytes >= m3 && max_bytes >= 16 && max_bytes >= need16 && max_bytes < (1ll << 31) && num < (1ll << 29) && !G.D.shard &&
                  !((uintptr_t)d_stream & 15u) && !((uintptr_t)d_out & 15u);
    /* (r06) streams of at most 2^14 values whose bits fit 2^19: the one-workgroup decoder (dc_decode_tiny.hip),
       after the small-stream decoder's range, when enabled (DC_TINY=1 / dc_set_decode_tiny(1)) */
    G.tiny_used = 0;
    G.dec_max_bytes = max_bytes;
    if (G.dec3_used && tiny_on() && num <= dc_tiny_max_values() && !((uintptr_t)d_out & 15u) &&
        G.tiny_key != ct * 256 + P.B + 1) {
        G.tiny_used = 1;
        G.dec3_used = 0;
    }
    G.dec3_launched = G.dec3_used;
    /* inside a capture only the small-stream decoder of an async halo plane: the other decoders tag their flags
       with a host epoch a replay would repeat, and a synchronous halo decode reads the status on the host */
    if (G.capturing && !(halo && G.halo_async && G.runs_used)) {
        G.capture_bad = 1;
        snprintf(G.capture_why, sizeof G.capture_why, "a decode other than an async halo plane's small-stream decode");
        return seterr(DC_ERR_ARG, "decode not capturable (only async halo planes on the small-stream decoder)");
    }
    G.dec_dnbits = nbytes >= 0 ? NULL : d_nbits;
    G.dec_hnbits = nbytes >= 0 ? (unsigned long long)nbytes * 8ull : 0ull;
    if (G.tiny_used) {
        if (dc_launch_decode_tiny((const uint8_t*)d_stream, max_bytes, G.dec_dnbits, G.dec_hnbits, &P, (float*)d_out,
                                  num, G.D.err, G.st))
            return seterr(DC_ERR_HIP, "decode launch failed: %s", hipGetErrorString(hipGetLastError()));
        G.dec3_used = 1;                  /* (a first decoder that may decline: dc_decode_finish falls back) */
    } else if (G.runs_used) {
        if (!G.runs_maps) HIPCHK(hipMalloc((void**)&G.runs_maps, dc_decode_runs_scratch_bytes()));
        if (dc_launch_decode_runs((const uint8_t*)d_stream, G.dec_dnbits, G.dec_hnbits, mc256, &P, G.runs_maps, G.D.err,
                                  (float*)d_out, num, G.st))
            return seterr(DC_ERR_HIP, "decode launch failed: %s", hipGetErrorString(hipGetLastError()));
        G.dec3_used = 1;                  /* (a first decoder that may decline: dc_decode_finish falls back) */
    } else if (G.dec3_used) {
        if ((rc = seg_decode_launch((const uint8_t*)d_stream, nbytes, max_bytes, &P, (float*)d_out, num))) return rc;
    } else if (DV(dc_launch_decode_fast)((const uint8_t*)d_stream, G.dec_dnbits, G.dec_hnbits, max_chunks, &P, &G.D,
                                         (float*)d_out, num, G.dec_epoch, G.st))
        return seterr(DC_ERR_HIP, "decode launch failed: %s", hipGetErrorString(hipGetLastError()));
    G.dec_pending = 1;
    G.dec_queued++;
    G.dec_shard = G.D.shard;
    G.dec_P = P;
    G.dec_s = (const uint8_t*)d_stream;
    G.dec_max_chunks = max_chunks;
    G.dec_out = (float*)d_out;
    G.dec_num = num;
    return DC_OK;
}

/* ---- a shard of a longer stream through the segment decoder (the multi-GPU step):
   the shard was encoded at start bit 0 with its global index (its first predictions read the previous
   shard's last values), its bit count is on the device.  Nothing is read back: predictions among its
   first tokens are decoded as pending and fixed by dc_decode_shard3_fix once the previous shard's last
   three values are here; a stream the segment decoder declines sets the status word (dc_decode_status),
   and the caller decodes the shard again on the chunk-map path (dc_decode_shard_device). */
int dc_decode_shard3_device(int ct, const void* d_stream, const unsigned long long* d_nbits, long long max_bytes,
                            long long num, int type, uint32_t mask17, void* d_out, int has_history) {
    int rc = ensure_init();
    if (rc) return rc;
    if (!valid_ct(ct)) return seterr(DC_ERR_ARG, "unsupported CT %d", ct);
    if (ct == 7 && (type < 1 || type > 7)) return seterr(DC_ERR_ARG, "CT7 type %d outside 1..7", type);
    if (!d_nbits || num < 3) return seterr(DC_ERR_ARG, "need the device bit count and num >= 3");
    if (((uintptr_t)d_stream & 15u) || ((uintptr_t)d_out & 15u) || max_bytes < 16 || max_bytes >= (1ll << 31) ||
        num >= (1ll << 29))
        return seterr(DC_ERR_ARG, "shard outside the segment decoder's limits (16-byte aligned, < 2 GiB)");
    if ((rc = dec_ensure((max_bytes * 8 + 1023) / 1024 + 1))) return rc;
    if ((rc = dec_next_epoch())) return rc;
    Params P;
    make_params(&P, ct, type, mask17);
    if ((rc = dec3_ensure((max_bytes * 8 + 255) / 256 + 1, P.B, ct))) return rc;
    G.D3.err = G.D.err;
    G.D3.capw = max_bytes / 16 * 4;
    G.D3.shard = has_history ? 1 : 2;            /* 2: the first shard, no values before it */
    const int lrc = dc_launch_decode3((const uint8_t*)d_stream, d_nbits, 0ull, &P, &G.D3, (float*)d_out, num,
                                      G.dec_epoch, 0, G.st);
    G.D3.shard = 0;
    if (lrc) return seterr(DC_ERR_HIP, "shard decode launch failed: %s", hipGetErrorString(hipGetLastError()));
    G.sh3_s = (const uint8_t*)d_stream;
    G.sh3_P = P;
    G.sh3_D3 = G.D3;
    G.sh3_out = (float*)d_out;
    G.sh3_num = num;
    G.sh3_ok = 1;
    return DC_OK;
}

/* the all-gathered shards (world slots of slot_bytes, each a shard encoded at start bit 0) and their
   all-gathered bit counts (device) -> the single global stream in d_out (out_bytes of room) and its bit
   count in d_total; no host read (the status word: dc_merge_status) */
int dc_merge_shards_device(const void* d_gathered, long long slot_bytes, int world, const unsigned long long* d_counts,
                           void* d_out, long long out_bytes, unsigned long long* d_total) {
    int rc = ensure_init();
    if (rc) return rc;
    if (!d_gathered || !d_counts || !d_out || !d_total || world < 1 || slot_bytes < 16 || (slot_bytes & 3) ||
        ((uintptr_t)d_gathered & 3u) || ((uintptr_t)d_out & 3u))
        return seterr(DC_ERR_ARG, "merge: bad buffers (4-byte aligned, slot a multiple of 4 bytes)");
    if (dc_launch_merge_shards((const uint8_t*)d_gathered, slot_bytes, world, d_counts, (uint8_t*)d_out, out_bytes,
                               d_total, G.d_enc_err + 4, out_bytes, G.st))
        return seterr(DC_ERR_HIP, "merge launch failed");
    return DC_OK;
}

/* the receiver's side: shard `rank` of the merged global stream d_global (g_bytes of buffer, the shards' bit
   counts d_counts as merged) to bit 0 of d_out (out_bytes of room), its bit count to d_nbits; no host read.
   A shard that does not fit sets bit 4 of dc_merge_status */
int dc_extract_shard_device(const void* d_global, long long g_bytes, const unsigned long long* d_counts, int rank,
                            void* d_out, long long out_bytes, unsigned long long* d_nbits) {
    int rc = ensure_init();
    if (rc) return rc;
    if (!d_global || !d_counts || !d_out || !d_nbits || rank < 0 || ((uintptr_t)d_global & 3u) || ((uintptr_t)d_out & 3u))
        return seterr(DC_ERR_ARG, "extract: bad buffers (4-byte aligned)");
    if (dc_launch_extract_shard((const uint8_t*)d_global, g_bytes, d_counts, rank, (uint8_t*)d_out, out_bytes, d_nbits,
                                G.d_enc_err + 4, G.st))
        return seterr(DC_ERR_HIP, "extract launch failed");
    return DC_OK;
}

/* 1: a shard longer than its slot, 2: the global stream longer than the output, 4: an extracted shard that did
   not fit (sticky; reset = 1 clears) */
int dc_merge_status(unsigned* status_out, int reset) {
    int rc = ensure_init();
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(&G.h_scratch[3], G.d_enc_err + 4, 4, hipMemcpyDeviceToHost, G.st));
    HIPCHK(hipStreamSynchronize(G.st));
    *status_out = (unsigned)(G.h_scratch[3] & 0xFFFFFFFFu);
    if (reset) HIPCHK(hipMemsetAsync(G.d_enc_err + 4, 0, 4, G.st));
    return DC_OK;
}

/* d_hin: the previous shard's last three values, last first (device, 3 floats) */
int dc_decode_shard3_fix(const float* d_hin) {
    int rc = ensure_init();
    if (rc) return rc;
    if (!G.sh3_ok) return seterr(DC_ERR_ARG, "no shard decode to fix");
    if (dc_launch_shard3_fix(G.sh3_s, &G.sh3_P, &G.sh3_D3, d_hin, G.sh3_out, G.sh3_num, G.st))
        return seterr(DC_ERR_HIP, "shard fix launch failed");
    return DC_OK;
}

static int read_dec_err(unsigned* err) {
    HIPCHK(hipMemcpyAsync(&G.h_scratch[2], G.D.err, 4, hipMemcpyDeviceToHost, G.st));
    HIPCHK(hipMemcpyAsync(&G.h_scratch[12], G.D.plan, sizeof(Plan), hipMemcpyDeviceToHost, G.st));
    /* a fused segment decode of a stream whose length is on the device: the length, for the next launch's
       segment length (dc_decode3_size_hint; the launch itself reads nothing back) */
    const int hint = G.dec3_fusedl && G.dec_dnbits != NULL;
    if (hint) HIPCHK(hipMemcpyAsync(&G.h_scratch[4], G.dec_dnbits, 8, hipMemcpyDeviceToHost, G.st));
    HIPCHK(hipStreamSynchronize(G.st));
    if (hint) dc_decode3_size_hint(G.D3.max_chunks, (long long)((G.h_scratch[4] + 255) / 256));
    *err = (unsigned)(G.h_scratch[2] & 0xFFFFFFFFu);
    const Plan* pl = (const Plan*)&G.h_scratch[12];
    G.dec_nbits = pl->nbits;
    G.dec_runs = pl->runs;
    return DC_OK;
}

int dc_decode_status(unsigned* status_out) {
    int rc = ensure_init();
    if (rc) return rc;
    unsigned err = 0;
    if ((rc = read_dec_err(&err))) return rc;
    if (status_out) *status_out = err;
    return DC_OK;
}

/* clear the decoder's status word (after a dc_decode_shard3_device that declined, before the caller
   decodes the shard again on the other path) */
int dc_decode_status_clear(void) {
    int rc = ensure_init();
    if (rc) return rc;
    if (!G.D.err) return DC_OK;                  /* (no decode yet) */
    HIPCHK(hipMemsetAsync(G.D.err, 0, 4, G.st));
    G.dec_pending = 0;
    G.dec_queued = 0;
    return DC_OK;
}

static int decode_finish_body(void);
/* the slow paths' launches are timed into the current step's event set (dc_timing_read_all) */
int dc_decode_finish(void) {
    dc_timing_finish(1);
    const int rc = decode_finish_body();
    dc_timing_finish(0);
    return rc;
}

static int decode_finish_body(void) {
    int rc = ensure_init();
    if (rc) return rc;
    unsigned err = 0;
    rc = read_dec_err(&err);
    if (rc) return rc;
    const int queued = G.dec_queued;
    int fast_values = 0;                   /* the values came from the fast decode (sentinel checked there) */
    G.dec_queued = 0;
    G.shard_deferred = 0;
    if (err && queued > 1 && !G.dec_shard) {
        /* the status words are OR-ed over every decode since the last finish: only the last one's
         * arguments are kept, so an earlier decode that left the fast path cannot be completed */
        G.dec_pending = 0;
        HIPCHK(hipMemsetAsync(G.D.err, 0, 4, G.st));
        return seterr(DC_ERR_STREAM, "decoder status 0x%x over %d queued decodes: an earlier decode left the fast "
                                     "path and was not completed (call dc_decode_finish after each decode)", err, queued);
    }
    /* the one-workgroup decoder declined (link or pending chains past its rounds, e.g. CT11's slowly
       resynchronising 32-bit tokens): the segment decoder, and for these parameters from the start next time;
       a stream it declines for the sentinel or its length goes on below like any declined segment decode */
    if ((err & 512u) && G.dec_pending && G.tiny_used && !(err & (4096u | 16384u))) {
        if (getenv("DC_DEBUG_ERR")) fprintf(stderr, "[dcamd] one-workgroup decoder declined (status 0x%x)\n", err);
        HIPCHK(hipMemsetAsync(G.D.err, 0, 4, G.st));
        if ((rc = dec_next_epoch())) return rc;
        G.tiny_key = G.dec_P.ct * 256 + G.dec_P.B + 1;
        G.tiny_used = 0;
        if ((rc = seg_decode_launch(G.dec_s, G.dec_hnbits ? (long long)(G.dec_hnbits / 8) : -1, G.dec_max_bytes,
                                    &G.dec_P, G.dec_out, G.dec_num)))
            return rc;
        rc = read_dec_err(&err);
        if (rc) return rc;
    }
    /* segment-decoder declines it recovers from itself: a job denser than the 1040-value buffer (the 2080-value
       instantiation) and parse paths that did not meet (the maps parse); each is remembered per (CT, bound),
       so later decodes of such streams start with it */
    for (int r = 0; r < 2; r++) {
        if (!((err & 512u) && G.dec_pending && G.dec3_used && !G.runs_used && !G.tiny_used && !G.dec_shard)) break;
        if (err & (1024u | 4096u | 16384u | 65536u)) break;       /* runs mode, short, sentinel, shard: other paths */
        const int want_maps = G.dec3_maps || (err & 2048u) != 0;
        const int want_dense = G.dec3_dense || (err & 8192u) != 0;
        if (want_maps == G.dec3_maps && want_dense == G.dec3_dense) break;
        if (getenv("DC_DEBUG_ERR"))
            fprintf(stderr, "[dcamd] segment decoder declined (status 0x%x): again with%s%s\n", err,
                    want_maps ? " the maps parse" : "", want_dense ? " the dense job buffer" : "");
        HIPCHK(hipMemsetAsync(G.D.err, 0, 4, G.st));
        if ((rc = dec_next_epoch())) return rc;
        if (want_dense) G.dense_key = G.dec_P.ct * 256 + G.dec_P.B + 1;
        if (want_maps) G.maps_key = G.dec_P.ct * 256 + G.dec_P.B + 1;
        G.dec3_dense = want_dense;
        G.dec3_maps = want_maps;
        if ((rc = dec3_launch(G.dec_s, &G.dec_P, G.dec_out, G.dec_num))) return rc;
        rc = read_dec_err(&err);
        if (rc) return rc;
    }
    G.tiny_last = G.tiny_used && !(err & 512u);
    G.dec3_last = G.dec3_used && !G.runs_used && !G.tiny_used && !(err & 512u);
    G.runs_last = G.dec3_used && G.runs_used && !(err & 512u);
    if ((err & 512u) && G.dec_pending && G.dec3_used) {
        /* the segment decoder declined the stream (runs mode, an unconverged repair, a dense job, the
         * history sentinel): decode it again with the chunk-map decoder, then its slow paths below */
        if (getenv("DC_DEBUG_ERR")) fprintf(stderr, "[dcamd] segment decoder declined (status 0x%x)\n", err);
        HIPCHK(hipMemsetAsync(G.D.err, 0, 4, G.st));
        G.dec3_used = 0;
        if ((rc = dec_next_epoch())) return rc;
        if (DV(dc_launch_decode_fast)(G.dec_s, G.dec_dnbits, G.dec_hnbits, G.dec_max_chunks, &G.dec_P, &G.D, G.dec_out,
                                      G.dec_num, G.dec_epoch, G.st))
            return seterr(DC_ERR_HIP, "decode launch failed");
        rc = read_dec_err(&err);
        if (rc) return rc;
    }
    if (G.dec_shard == 1 && (err & (256u | 32u))) {  /* shard prefixes waiting for their incoming values */
        G.shard_deferred = (err & 32u) ? 2 : 1;
        err &= ~(256u | 32u);
        HIPCHK(hipMemsetAsync(G.D.err, 0, 4, G.st));
    }
    if (!err) { G.dec_pending = 0; return DC_OK; }
    if (getenv("DC_DEBUG_ERR")) fprintf(stderr, "[dcamd] fast decode status 0x%x\n", err);
    if (G.dec_shard && (err & (8u | 64u | 128u | 16u))) {
        /* a shard outside the fast path (e.g. a locally periodic stream): exact sequential decode of the
         * shard from its incoming values -- now, or in dc_decode_shard_fix when they come later */
        HIPCHK(hipMemsetAsync(G.D.err, 0, 4, G.st));
        G.dec_pending = 0;
        if (G.dec_shard == 1) { G.shard_deferred = 3; return DC_OK; }
        DecBufs D = G.D;
        D.shard = 2;
        D.hin = G.dec_hin;
        if (DV(dc_launch_decode_serial)(G.dec_s, &G.dec_P, &D, G.dec_out, G.dec_num, G.st))
            return seterr(DC_ERR_HIP, "decode launch failed");
        HIPCHK(hipStreamSynchronize(G.st));
        return DC_OK;
    }
    if ((err & (8u | 64u)) && !(err & (16u | 128u)) && G.dec_pending) {
        /* outside the fast path's assumptions: exact multi-kernel path (closure rounds, then
         * complete entry maps for every chunk if an entry is still unresolved) */
        HIPCHK(hipMemsetAsync(G.D.err, 0, 4, G.st));
        if ((rc = dec_next_epoch())) return rc;
        if (G.dec_runs) {
            /* runs mode: the parse left every chunk map its tiles reach -- compose them, then the fast
             * decode kernel (which checks the history sentinel itself) from the resolved entries */
            dc_mark_phase(12, G.st);
            if (DV(dc_launch_resolve)(G.dec_max_chunks, &G.D, G.dec_epoch, G.st))
                return seterr(DC_ERR_HIP, "decode launch failed");
            dc_mark_phase(13, G.st);
            dc_mark_phase(14, G.st);
            if (DV(dc_launch_decode_fast_resolved)(G.dec_s, G.dec_max_chunks, &G.dec_P, &G.D, G.dec_out, G.dec_num,
                                               G.dec_epoch, G.st))
                return seterr(DC_ERR_HIP, "decode launch failed");
            dc_mark_phase(15, G.st);
            fast_values = 1;
        } else if (DV(dc_launch_decode)(G.dec_s, NULL, G.dec_nbits, G.dec_max_chunks, &G.dec_P, &G.D, G.dec_out, G.dec_num,
                                    G.dec_epoch, DEC_ROUNDS, DEC_FIX_ITERS, G.st))
            return seterr(DC_ERR_HIP, "decode launch failed");
        rc = read_dec_err(&err);
        if (rc) return rc;
        if ((err & 8u) && !(err & 16u)) {
            fast_values = 0;
            HIPCHK(hipMemsetAsync(G.D.err, 0, 4, G.st));
            if ((rc = dec_next_epoch())) return rc;
            if (DV(dc_launch_decode_more)(G.dec_s, G.dec_max_chunks, &G.dec_P, &G.D, G.dec_out, G.dec_num, G.dec_epoch,
                                      DEC_FIX_ITERS, G.st))
                return seterr(DC_ERR_HIP, "decode launch failed");
            rc = read_dec_err(&err);
            if (rc) return rc;
        }
    }
    if ((err & 32u) && !(err & (8u | 16u | 128u)) && G.dec_pending) {
        fast_values = 0;
        HIPCHK(hipMemsetAsync(G.D.err, 0, 4, G.st));
        if (G.dec_shard == 2) {                      /* a shard with known incoming values */
            if (DV(dc_launch_shard_fix)(G.dec_s, &G.dec_P, &G.D, G.dec_out, G.dec_num, G.dec_max_chunks, G.dec_hin, G.st))
                return seterr(DC_ERR_HIP, "decode launch failed");
        } else if (DV(dc_launch_fixup_serial)(G.dec_s, &G.dec_P, &G.D, G.dec_out, G.dec_num, G.st))
            return seterr(DC_ERR_HIP, "decode launch failed");
        rc = read_dec_err(&err);
        if (rc) return rc;
    }
    if (!err && G.dec_pending && !fast_values) {   /* a slow path wrote values: check for the history sentinel */
        if (DV(dc_launch_find_sentinel)(G.dec_out, G.dec_num, G.D.err, G.st))
            return seterr(DC_ERR_HIP, "decode launch failed");
        rc = read_dec_err(&err);
        if (rc) return rc;
    }
    if ((err & 128u) && !(err & 16u) && G.dec_pending) {
        /* -1.0f history sentinel in the stream: exact sequential decode (reference semantics) */
        HIPCHK(hipMemsetAsync(G.D.err, 0, 4, G.st));
        if (DV(dc_launch_decode_serial)(G.dec_s, &G.dec_P, &G.D, G.dec_out, G.dec_num, G.st))
            return seterr(DC_ERR_HIP, "decode launch failed");
        rc = read_dec_err(&err);
        if (rc) return rc;
    }
    G.dec_pending = 0;
    HIPCHK(hipMemsetAsync(G.D.err, 0, 4, G.st));
    if (err) return seterr(DC_ERR_STREAM, "decoder status 0x%x (8: unresolved entry, 16: look-back timeout, "
                                          "32: prediction chain)", err);
    return DC_OK;
}

/* ---- shards of one global stream: decode tokens [start_bit, start_bit + nbits) ------ */
int dc_decode_shard_device(int ct, const void* d_stream, long long stream_bytes, unsigned long long start_bit,
                           unsigned long long nbits, long long num, int type, uint32_t mask17, const float* d_hin,
                           void* d_out) {
    int rc = ensure_init();
    if (rc) return rc;
    const long long nb = (long long)((nbits + 7) / 8);
    if (grow(&G.shard_buf, &G.shard_cap, (size_t)nb + 64)) return DC_ERR_HIP;
    if (dc_launch_bit_shift_copy((const uint8_t*)d_stream, stream_bytes, start_bit, nbits, (uint8_t*)G.shard_buf, nb + 8,
                                 G.st))
        return seterr(DC_ERR_HIP, "shard copy launch failed");
    G.D.shard = d_hin ? 2 : 1;
    G.D.hin = d_hin;
    rc = dc_decode_device(ct, G.shard_buf, nb, NULL, nb, num, type, mask17, d_out);
    G.dec_shard = G.D.shard;
    G.dec_hin = d_hin;
    G.D.shard = 0;
    G.D.hin = NULL;
    return rc;
}

int dc_decode_shard_fix(const float* d_hin) {
    int rc = ensure_init();
    if (rc) return rc;
    if (!G.shard_deferred) return DC_OK;
    DecBufs D = G.D;
    D.shard = 2;
    D.hin = d_hin;
    if (G.shard_deferred == 3) {                    /* exact sequential decode of the whole shard */
        if (DV(dc_launch_decode_serial)(G.dec_s, &G.dec_P, &D, G.dec_out, G.dec_num, G.st))
            return seterr(DC_ERR_HIP, "shard fix launch failed");
    } else {
        const long long nc = G.shard_deferred == 2 ? G.dec_max_chunks : dc_decode_group();
        if (DV(dc_launch_shard_fix)(G.dec_s, &G.dec_P, &D, G.dec_out, G.dec_num, nc, d_hin, G.st))
            return seterr(DC_ERR_HIP, "shard fix launch failed");
    }
    HIPCHK(hipStreamSynchronize(G.st));             /* re-runnable with other values until the next decode */
    return DC_OK;
}

/* ---- Himeno halo planes on the device (impl/himenoBMTxps.c:483-706) ------------- */
static int plane_dims(int ijk, int imax, int jmax, int kmax, int* A, int* B) {
    if (ijk == 1) { *A = jmax; *B = kmax; }
    else if (ijk == 2) { *A = imax; *B = kmax; }
    else if (ijk == 3) { *A = imax; *B = jmax; }
    else return seterr(DC_ERR_ARG, "ijk %d outside 1..3", ijk);
    return DC_OK;
}

/* (r06) the halo gathers finish the plane's minimum in their last workgroup (a counter per halo stream, zeroed once
   and reset by that workgroup); DC_HALO_MIN2=1: the separate min_final launch (A/B) */
static int halo_counters(void) {
    if (!G.gcnt) {
        HIPCHK(hipMalloc((void**)&G.gcnt, 64));
        HIPCHK(hipMemset(G.gcnt, 0, 64));
    }
    return DC_OK;
}
static unsigned* halo_cnt(int i) {
    static int two = -1;
    if (two < 0) two = getenv("DC_HALO_MIN2") && atoi(getenv("DC_HALO_MIN2")) == 1;
    return two ? NULL : G.gcnt + 4 * i;
}

int dc_halo_encode_device(int ct, const void* d_p, int mi, int mj, int mk, int ijk, int v, int imax, int jmax,
                          int kmax, int type, uint32_t mask17, void* d_stream, unsigned long long* d_bits,
                          float* d_min, int* type_out, uint32_t* mask17_out) {
    int rc = ensure_init();
    if (rc) return rc;
    int A = 0, B = 0;
    if ((rc = plane_dims(ijk, imax, jmax, kmax, &A, &B))) return rc;
    if (v < 0 || (ijk == 1 && v >= mi) || (ijk == 2 && v >= mj) || (ijk == 3 && v >= mk) || A > (ijk == 1 ? mj : mi) ||
        B > (ijk == 3 ? mj : mk))
        return seterr(DC_ERR_ARG, "plane outside the %dx%dx%d array", mi, mj, mk);
    const long long n = (long long)A * B;
    if (n <= 0) return seterr(DC_ERR_ARG, "empty plane");
    if (grow(&G.halo_a, &G.halo_a_cap, (size_t)n * 4 + 64) || grow(&G.halo_b, &G.halo_b_cap, (size_t)n * 4 + 64))
        return DC_ERR_HIP;
    if (!(ct == 7 && type <= 0) && !G.halo_unfused) {
        /* (r06) the gather computes toSmallDataset's minimum partials, min_final writes the minimum where the caller
           wants it, and the encoder subtracts it while loading (no x - min written, no copy of the minimum): three
           launches instead of six */
        float* dmin = d_min ? d_min : &G.d_f[0];
        /* recorded into a graph: min_final zeroes the encoder's tile states and flag (no memset nodes), when the
           encoder's buffer will not grow */
        const long long dw = dc_encode_desc_words(n) + 8;
        const int pre = G.capturing && G.enc_desc && dw <= G.enc_desc_cap && dw < (1 << 30);
        if ((rc = halo_counters())) return rc;
        if (dc_launch_plane_gather_min((const float*)d_p, mj, mk, ijk, v, A, B, (float*)G.halo_a, G.part_v, G.part_i,
                                       dmin, pre ? (uint64_t*)G.enc_desc : NULL, pre ? (int)dw : 0,
                                       pre ? (uint32_t*)G.d_enc_flag : NULL, pre ? 1024 : 0, halo_cnt(0), G.st))
            return seterr(DC_ERR_HIP, "plane gather launch failed");
        G.enc_precleared = pre;
        if (type_out) *type_out = type;
        if (mask17_out) *mask17_out = mask17;
        if (G.enc_st) {
            HIPCHK(hipEventRecord(G.ev_lib, G.enc_st));
            HIPCHK(hipStreamWaitEvent(G.st, G.ev_lib, 0));
        }
        G.enc_subp = dmin;
        rc = encode_on(G.st, ct, G.halo_a, n, 0, type, mask17, 0, d_stream, d_bits, NULL);
        G.enc_subp = NULL;
        G.enc_precleared = 0;
        return rc;
    }
    if (dc_launch_plane_gather((const float*)d_p, mj, mk, ijk, v, A, B, (float*)G.halo_a, G.st))
        return seterr(DC_ERR_HIP, "plane gather launch failed");
    if (dc_launch_to_small((const float*)G.halo_a, n, (float*)G.halo_b, G.part_v, G.part_i, &G.d_f[0], G.st))
        return seterr(DC_ERR_HIP, "to_small launch failed");
    if (d_min) HIPCHK(hipMemcpyAsync(d_min, &G.d_f[0], 4, hipMemcpyDeviceToDevice, G.st));
    if (ct == 7 && type <= 0) {                     /* mask of this plane, as himenoBMTxps.c:483-500 */
        float mean;
        if ((rc = dc_med_device(G.halo_b, n, &mean, &type))) return rc;
        uint32_t u;
        memcpy(&u, &mean, 4);
        mask17 = u >> 15;
    }
    if (type_out) *type_out = type;
    if (mask17_out) *mask17_out = mask17;
    return encode_lib(ct, G.halo_b, n, 0, type, mask17, 0, d_stream, d_bits);
}

int dc_halo_decode_device(int ct, const void* d_stream, long long nbytes, const unsigned long long* d_bits, int type,
                          uint32_t mask17, const float* d_min, void* d_p, int mi, int mj, int mk, int ijk, int v,
                          int imax, int jmax, int kmax) {
    int rc = ensure_init();
    if (rc) return rc;
    int A = 0, B = 0;
    if ((rc = plane_dims(ijk, imax, jmax, kmax, &A, &B))) return rc;
    (void)mi;
    const long long n = (long long)A * B;
    if (grow(&G.halo_a, &G.halo_a_cap, (size_t)n * 4 + 64)) return DC_ERR_HIP;
    const long long cap = nbytes >= 0 ? nbytes : (long long)dc_stream_capacity(n);
    /* a plane is a runs-mode stream (copy runs), which the segment decoder declines: straight to the
       chunk-map decoder */
    if ((rc = decode_device_h(ct, d_stream, nbytes, d_bits, cap, n, type, mask17, G.halo_a, 1))) return rc;
    /* async (dc_set_halo_async): no host read here -- the caller reads dc_decode_status() after its steps
       and decodes a plane again synchronously if it is not 0 */
    if (!G.halo_async && (rc = dc_decode_finish())) return rc;
    if (dc_launch_plane_scatter((const float*)G.halo_a, d_min, (float*)d_p, mj, mk, ijk, v, A, B, G.st))
        return seterr(DC_ERR_HIP, "plane scatter launch failed");
    return DC_OK;
}

/* (r06) Two halo planes of one array encoded at once (impl/himenoBMTxps.c:644-690: a rank compresses its two z-halo
   planes every iteration): plane v0 as dc_halo_encode_device on the library stream, plane v1 on a second stream with
   its own gathered floats, minimum partials and encoder scratch -- each encode of 65,536 floats is a few small
   launches, so the two overlap.  The fused path only (not CT7 with type <= 0, which needs the mean); otherwise, or
   when the encoder runs a non-default variant, the planes go one after the other. */
static int halo_streams(void) {
    if (!G.st2) {
        HIPCHK(hipStreamCreateWithFlags(&G.st2, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&G.ev_h0, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&G.ev_h1, hipEventDisableTiming));
    }
    return DC_OK;
}
int dc_halo_encode2_device(int ct, const void* d_p, int mi, int mj, int mk, int ijk, int v0, int v1, int imax, int jmax,
                           int kmax, int type, uint32_t mask17, void* s0, void* s1, unsigned long long* bits0,
                           unsigned long long* bits1, float* dmin0, float* dmin1) {
    int rc = ensure_init();
    if (rc) return rc;
    int A = 0, B = 0;
    if ((rc = plane_dims(ijk, imax, jmax, kmax, &A, &B))) return rc;
    const long long n = (long long)A * B;
    if (!valid_ct(ct) || (ct == 7 && type <= 0) || G.halo_unfused || !dc_encode_plain() || !bits1 || !dmin1 || n <= 0 ||
        v1 < 0 || (ijk == 1 && v1 >= mi) || (ijk == 2 && v1 >= mj) || (ijk == 3 && v1 >= mk) ||
        ((uintptr_t)s1 & 3u) || A > (ijk == 1 ? mj : mi) || B > (ijk == 3 ? mj : mk)) {
        if ((rc = dc_halo_encode_device(ct, d_p, mi, mj, mk, ijk, v0, imax, jmax, kmax, type, mask17, s0, bits0, dmin0,
                                        NULL, NULL)))
            return rc;
        return dc_halo_encode_device(ct, d_p, mi, mj, mk, ijk, v1, imax, jmax, kmax, type, mask17, s1, bits1, dmin1,
                                     NULL, NULL);
    }
    if ((rc = halo_streams()) || (rc = halo_counters())) return rc;
    if (grow(&G.halo_a2, &G.halo_a2_cap, (size_t)n * 4 + 64)) return DC_ERR_HIP;
    if (!G.part_v2) {
        HIPCHK(hipMalloc((void**)&G.part_v2, DC_MIN_PARTS * sizeof(float)));
        HIPCHK(hipMalloc((void**)&G.part_i2, DC_MIN_PARTS * sizeof(long long)));
        HIPCHK(hipMalloc((void**)&G.d_enc_flag2, 8192));
        HIPCHK(hipMemset(G.d_enc_flag2, 0, 8192));
    }
    if (dc_encode_desc_words(n) + 8 > G.enc_desc2_cap) {
        if (G.enc_desc2) HIPCHK(hipFree(G.enc_desc2));
        const long long cap = dc_encode_desc_words(n) + 1024;
        HIPCHK(hipMalloc((void**)&G.enc_desc2, cap * sizeof(uint64_t)));
        HIPCHK(hipMemset(G.enc_desc2, 0, cap * sizeof(uint64_t)));
        G.enc_desc2_cap = cap;
        G.enc_epoch2 = 0;
    }
    HIPCHK(hipEventRecord(G.ev_h0, G.st));                            /* the second stream after the library's */
    HIPCHK(hipStreamWaitEvent(G.st2, G.ev_h0, 0));
    if ((rc = dc_halo_encode_device(ct, d_p, mi, mj, mk, ijk, v0, imax, jmax, kmax, type, mask17, s0, bits0, dmin0, NULL,
                                    NULL)))
        return rc;
    const long long dw = dc_encode_desc_words(n) + 8;     /* (capacity ensured above) */
    const int pre = G.capturing && dw < (1 << 30);
    if (dc_launch_plane_gather_min((const float*)d_p, mj, mk, ijk, v1, A, B, (float*)G.halo_a2, G.part_v2, G.part_i2,
                                   dmin1, pre ? (uint64_t*)G.enc_desc2 : NULL, pre ? (int)dw : 0,
                                   pre ? (uint32_t*)G.d_enc_flag2 : NULL, pre ? 1024 : 0, halo_cnt(1), G.st2))
        return seterr(DC_ERR_HIP, "plane gather launch failed");
    Params P;
    make_params(&P, ct, type, mask17);
    P.sub = 1;
    P.subp = dmin1;
    if (G.capturing) {                          /* (as encode_on: min_final cleared what this encode reads) */
        if (!pre) {
            HIPCHK(hipMemsetAsync(G.enc_desc2, 0, (size_t)dw * sizeof(uint64_t), G.st2));
            HIPCHK(hipMemsetAsync(G.d_enc_flag2, 0, 4096, G.st2));
        }
        G.enc_epoch2 = 1;
    } else if (++G.enc_epoch2 >= dc_encode_epoch_limit() || G.enc_epoch2 == 1) {
        HIPCHK(hipMemsetAsync(G.enc_desc2, 0, (size_t)G.enc_desc2_cap * sizeof(uint64_t), G.st2));
        HIPCHK(hipMemsetAsync(G.d_enc_flag2, 0, 4096, G.st2));
        G.enc_epoch2 = 1;
    }
    if (dc_launch_encode((const float*)G.halo_a2, n, 0, &P, (uint32_t*)s1, G.enc_desc2, G.d_enc_flag2, G.enc_epoch2, 0,
                         bits1, NULL, G.d_enc_err, NULL, 0, NULL, NULL, G.st2))
        return seterr(DC_ERR_HIP, "encode launch failed: %s", hipGetErrorString(hipGetLastError()));
    G.enc_outstanding++;                             /* (a timeout in either encode is reported, not re-run) */
    HIPCHK(hipEventRecord(G.ev_h1, G.st2));                           /* the library stream after both */
    HIPCHK(hipStreamWaitEvent(G.st, G.ev_h1, 0));
    return DC_OK;
}

/* (r06) Two halo planes of one array (the two z-neighbours' planes of a Himeno step, impl/himenoBMTxps.c:696-706)
   decoded at once: each plane's small-stream decode and scatter on its own stream -- the decoders are one-
   workgroup scans, so two of them overlap on the GPU.  Asynchronous, as dc_halo_decode_device under
   dc_set_halo_async(1): a stream the small-stream decoder declines sets the status word (dc_decode_status) and the
   caller decodes that plane again with dc_halo_decode_device.  Planes it cannot take go one after the other. */
int dc_halo_decode2_device(int ct, const void* s0, const void* s1, const unsigned long long* bits0,
                           const unsigned long long* bits1, int type, uint32_t mask17, const float* dmin0,
                           const float* dmin1, void* d_p, int mi, int mj, int mk, int ijk, int v0, int v1, int imax,
                           int jmax, int kmax) {
    int rc = ensure_init();
    if (rc) return rc;
    if (!valid_ct(ct)) return seterr(DC_ERR_ARG, "unsupported CT %d", ct);
    if (ct == 7 && (type < 1 || type > 7)) return seterr(DC_ERR_ARG, "CT7 type %d outside 1..7", type);
    int A = 0, B = 0;
    if ((rc = plane_dims(ijk, imax, jmax, kmax, &A, &B))) return rc;
    const long long n = (long long)A * B;
    const long long cap = (long long)dc_stream_capacity(n);
    const long long mc256 = (cap * 8 + 255) / 256 + 1;
    if (!bits0 || !bits1 || ((uintptr_t)s0 & 3u) || ((uintptr_t)s1 & 3u) || mc256 > dc_decode_runs_max_chunks() + 8 ||
        runs_max_bytes() < 0 || dec3_min_bytes() <= 0 || !G.halo_async) {
        if ((rc = dc_halo_decode_device(ct, s0, -1, bits0, type, mask17, dmin0, d_p, mi, mj, mk, ijk, v0, imax, jmax,
                                        kmax)))
            return rc;
        return dc_halo_decode_device(ct, s1, -1, bits1, type, mask17, dmin1, d_p, mi, mj, mk, ijk, v1, imax, jmax, kmax);
    }
    if ((rc = halo_streams())) return rc;
    if (grow(&G.halo_a, &G.halo_a_cap, (size_t)n * 4 + 64) || grow(&G.halo_a2, &G.halo_a2_cap, (size_t)n * 4 + 64))
        return DC_ERR_HIP;
    if (!G.runs_maps) HIPCHK(hipMalloc((void**)&G.runs_maps, dc_decode_runs_scratch_bytes()));
    if (!G.runs_maps2) HIPCHK(hipMalloc((void**)&G.runs_maps2, dc_decode_runs_scratch_bytes()));
    if ((rc = dec_ensure((cap * 8 + 1023) / 1024 + 1))) return rc;     /* (the status word) */
    Params P;
    make_params(&P, ct, type, mask17);
    HIPCHK(hipEventRecord(G.ev_h0, G.st));                            /* the second stream after the library's */
    HIPCHK(hipStreamWaitEvent(G.st2, G.ev_h0, 0));
    static int scat = -1;                      /* DC_HALO_SCATTER=1: the values kernel scatters (measured slower) */
    if (scat < 0) scat = getenv("DC_HALO_SCATTER") && atoi(getenv("DC_HALO_SCATTER")) == 1;
    if (scat && !G.halo_unfused) {
        /* (r06) each plane decoded straight into the array (the values kernel adds the minimum and scatters): one
           launch less, but its lanes each write a block's values with the plane's stride, 20.9 us against 10.6 for
           the values and 4.5 for the coalesced scatter pass (rocprof, CT5 halo planes) */
        if (dc_launch_decode_runs_scatter((const uint8_t*)s0, bits0, 0ull, mc256, &P, G.runs_maps, G.D.err, n,
                                          (float*)d_p, dmin0, mj, mk, ijk, v0, B, G.st) ||
            dc_launch_decode_runs_scatter((const uint8_t*)s1, bits1, 0ull, mc256, &P, G.runs_maps2, G.D.err, n,
                                          (float*)d_p, dmin1, mj, mk, ijk, v1, B, G.st2))
            return seterr(DC_ERR_HIP, "halo decode launch failed: %s", hipGetErrorString(hipGetLastError()));
    } else if (dc_launch_decode_runs((const uint8_t*)s0, bits0, 0ull, mc256, &P, G.runs_maps, G.D.err,
                                     (float*)G.halo_a, n, G.st) ||
               dc_launch_plane_scatter((const float*)G.halo_a, dmin0, (float*)d_p, mj, mk, ijk, v0, A, B, G.st) ||
               dc_launch_decode_runs((const uint8_t*)s1, bits1, 0ull, mc256, &P, G.runs_maps2, G.D.err,
                                     (float*)G.halo_a2, n, G.st2) ||
               dc_launch_plane_scatter((const float*)G.halo_a2, dmin1, (float*)d_p, mj, mk, ijk, v1, A, B, G.st2))
        return seterr(DC_ERR_HIP, "halo decode launch failed: %s", hipGetErrorString(hipGetLastError()));
    HIPCHK(hipEventRecord(G.ev_h1, G.st2));                           /* the library stream after both */
    HIPCHK(hipStreamWaitEvent(G.st, G.ev_h1, 0));
    return DC_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* (r06) HIP graphs.  A Himeno halo step is ~14 small launches (per plane: gather + minimum, min_final, the encoder;
   the small-stream decoder's three kernels and the scatter) whose GPU work is a few microseconds each, so a step
   issued call by call is bound by the host's launch rate.  dc_capture_begin .. dc_capture_end records the library
   calls in between (the library stream and the second halo stream, forked and joined by events) into a graph;
   dc_graph_launch replays it with one launch.  A replay reads the same device pointers (the caller rewrites the
   data in place between replays) and repeats the same work: encodes clear the tile states they read inside the
   graph, and only decodes with no host epoch or host read (async halo planes on the small-stream decoder) may be
   recorded -- any other call fails and makes dc_capture_end fail. */
int dc_capture_begin(void) {
    int rc = ensure_init();
    if (rc) return rc;
    if (G.capturing) return seterr(DC_ERR_ARG, "a capture is already open");
    if ((rc = halo_streams())) return rc;
    HIPCHK(hipStreamBeginCapture(G.st, hipStreamCaptureModeRelaxed));
    G.capturing = 1;
    G.capture_bad = 0;
    G.capture_why[0] = 0;
    return DC_OK;
}

int dc_capture_end(void** graph_out) {
    int rc = ensure_init();
    if (rc) return rc;
    if (!G.capturing) return seterr(DC_ERR_ARG, "no capture open");
    if (graph_out) *graph_out = NULL;
    hipGraph_t g = NULL;
    const hipError_t e = hipStreamEndCapture(G.st, &g);
    G.capturing = 0;
    /* replays tag tile states with epoch 1: the next direct encodes start a fresh epoch cycle (a full clear) */
    G.enc_epoch = 0;
    G.enc_epoch2 = 0;
    if (e != hipSuccess || !g) {
        (void)hipGetLastError();
        return seterr(DC_ERR_HIP, "stream capture failed: %s", hipGetErrorString(e));
    }
    if (G.capture_bad) {
        hipGraphDestroy(g);
        G.capture_bad = 0;
        return seterr(DC_ERR_ARG, "capture discarded: %s was called inside it", G.capture_why);
    }
    hipGraphExec_t ex = NULL;
    const hipError_t ei = hipGraphInstantiate(&ex, g, NULL, NULL, 0);
    hipGraphDestroy(g);
    if (ei != hipSuccess) return seterr(DC_ERR_HIP, "graph instantiate failed: %s", hipGetErrorString(ei));
    if (graph_out) *graph_out = (void*)ex;
    else hipGraphExecDestroy(ex);
    return DC_OK;
}

int dc_graph_launch(void* graph) {
    int rc = ensure_init();
    if (rc) return rc;
    if (!graph) return seterr(DC_ERR_ARG, "null graph");
    if (G.capturing) return seterr(DC_ERR_ARG, "graph launch inside a capture");
    HIPCHK(hipGraphLaunch((hipGraphExec_t)graph, G.st));
    return DC_OK;
}

int dc_graph_destroy(void* graph) {
    if (graph) HIPCHK(hipGraphExecDestroy((hipGraphExec_t)graph));
    return DC_OK;
}

/* ------------------------------------------------------------------------------------------ */
int dc_to_small_device(const void* d_x, long long n, void* d_out, float* min_out) {
    int rc = ensure_init();
    if (rc) return rc;
    if (n <= 0) return seterr(DC_ERR_ARG, "empty input");
    if (dc_launch_to_small((const float*)d_x, n, (float*)d_out, G.part_v, G.part_i, &G.d_f[0], G.st))
        return seterr(DC_ERR_HIP, "to_small launch failed");
    if (min_out) {
        float h;
        HIPCHK(hipMemcpyAsync(&h, &G.d_f[0], 4, hipMemcpyDeviceToHost, G.st));
        HIPCHK(hipStreamSynchronize(G.st));
        *min_out = h;
    }
    return DC_OK;
}



/* DC_MED_WIDE=1: the exact mean goes straight to the wide binade window (tests compare both windows) */
static int med_force_wide(void) {
    const char* e = getenv("DC_MED_WIDE");
    return e && *e == '1';
}

/* 1 when the last exact mean ran the wide binade window (the narrow one missed; dc_aux.hip) */
int dc_med_last_wide(void) { return G.med_wide; }

/* (DC_MED_PROF builds) the compose kernel's section counters of the last dc_med_device on n floats */
int dc_med_prof_read(long long n, long long* out16) {
    int rc = ensure_init();
    if (rc) return rc;
    if (!G.med_scr || n <= 0) return seterr(DC_ERR_ARG, "no med scratch");
    const long long nch = (n + 2047) / 2048;
    const long long off = ((nch * (8 + 4 + 4 + 6 * 2 * 4 + 6 + 1) + 7) & ~7ll) + 32 * 8;
    HIPCHK(hipMemcpy(out16, (char*)G.med_scr + off, 16 * 8, hipMemcpyDeviceToHost));
    return DC_OK;
}

int dc_med_device(const void* d_x, long long n, float* mean_out, int* type_out) {
    int rc = ensure_init();
    if (rc) return rc;
    if (n <= 0) return seterr(DC_ERR_ARG, "empty input");
    if (grow(&G.med_scr, &G.med_scr_cap, (size_t)dc_med_scratch_bytes(n))) return DC_ERR_HIP;
    float m;
    int t;
    unsigned fl = 0;
    const int forced = med_force_wide();
    for (int wide = forced; wide < 2; wide++) {       /* the narrow window, then the wide one if it missed */
        if (wide ? dc_launch_med_wide((const float*)d_x, n, 0.0f, G.med_scr, &G.d_f[1], &G.d_i[0], NULL, NULL, forced, G.st)
                 : dc_launch_med((const float*)d_x, n, 0.0f, G.med_scr, &G.d_f[1], &G.d_i[0], NULL, NULL, G.st))
            return seterr(DC_ERR_HIP, "med launch failed");
        /* flag, then mean, type, sum, max (dc_aux.hip MedScratch.res): one copy */
        long long r[5];
        HIPCHK(hipMemcpyAsync(r, dc_med_flag_ptr(G.med_scr, n, 0), sizeof r, hipMemcpyDeviceToHost, G.st));
        HIPCHK(hipStreamSynchronize(G.st));
        fl = (unsigned)r[0];
        { const uint32_t b = (uint32_t)r[1]; memcpy(&m, &b, 4); }
        t = (int)r[2];
        G.med_wide = wide;
        if (!fl || wide) break;
    }
    if (mean_out) *mean_out = m;
    if (type_out) *type_out = t;
    return DC_OK;
}

/* The reference's pre-passes for the bitmask codecs (impl/pingpong.c:148-206: min = toSmallDataset_float(data,
 * &data_small); medium = med_dataset_float(data_small, &type)) on device data, fused: one read of x for
 * the minimum and the chunk statistics, the exact mean of x - min from x itself; x - min is never written.  With
 * dc_encode_sub_device the whole chain (min, mean, mask, encode of data_small) reads x three times and writes
 * only the stream.  A non-finite minimum (NaN or infinite data[0] / data) takes the separate passes.  Synchronous. */
int dc_prep_device(const void* d_x, long long n, float* min_out, float* mean_out, int* type_out) {
    int rc = ensure_init();
    if (rc) return rc;
    if (n <= 0) return seterr(DC_ERR_ARG, "empty input");
    if (((uintptr_t)d_x & 15u)) return seterr(DC_ERR_ARG, "misaligned device buffer");
    const long long nch = (n + 2047) / 2048;
    if (grow(&G.med_scr, &G.med_scr_cap, (size_t)dc_med_scratch_bytes(n)) ||
        grow(&G.prep_part, &G.prep_part_cap, (size_t)nch * 12 + 64))
        return DC_ERR_HIP;
    float* pv = (float*)G.prep_part;
    long long* pi = (long long*)((char*)G.prep_part + (((size_t)nch * 4 + 15) & ~(size_t)15));
    float mn = 0.0f, m = 0.0f;
    int t = 0;
    const int forced = med_force_wide();
    for (int wide = forced; wide < 2; wide++) {     /* the narrow window, then the wide one if it missed */
        if (dc_launch_med_sub((const float*)d_x, n, G.med_scr, &G.d_f[0], pv, pi, &G.d_f[1], &G.d_i[0],
                              wide && forced ? 2 : wide, G.st))
            return seterr(DC_ERR_HIP, "prep launch failed");
        long long r[6];                              /* flag, mean, type, sum, max, minimum not finite */
        HIPCHK(hipMemcpyAsync(r, dc_med_flag_ptr(G.med_scr, n, 0), sizeof r, hipMemcpyDeviceToHost, G.st));
        HIPCHK(hipMemcpyAsync(&mn, &G.d_f[0], 4, hipMemcpyDeviceToHost, G.st));
        HIPCHK(hipStreamSynchronize(G.st));
        if (r[5]) {                                  /* the separate passes: x - min written out */
            if (grow(&G.sub_buf, &G.sub_buf_cap, (size_t)n * 4 + 64)) return DC_ERR_HIP;
            if ((rc = dc_to_small_device(d_x, n, G.sub_buf, &mn)) || (rc = dc_med_device(G.sub_buf, n, &m, &t))) return rc;
            break;
        }
        { const uint32_t b = (uint32_t)r[1]; memcpy(&m, &b, 4); }
        t = (int)r[2];
        G.med_wide = wide;
        if (!(unsigned)r[0]) break;
    }
    if (min_out) *min_out = mn;
    if (mean_out) *mean_out = m;
    if (type_out) *type_out = t;
    return DC_OK;
}

/* dc_encode_device of x - min (the minimum dc_prep_device returned), x - min computed while loading: the stream is
 * the one dc_encode_device makes from toSmallDataset_float's array.  Asynchronous, as dc_encode_device. */
int dc_encode_sub_device(int ct, const void* d_x, long long n, float min, int type, uint32_t mask17, void* d_out,
                         unsigned long long* d_total_bits) {
    int rc = ensure_init();
    if (rc) return rc;
    if (G.enc_st) {
        HIPCHK(hipEventRecord(G.ev_enc, G.st));
        HIPCHK(hipStreamWaitEvent(G.enc_st, G.ev_enc, 0));
    }
    G.enc_sub = &min;
    rc = encode_on(ENC_ST, ct, d_x, n, 0, type, mask17, 0, d_out, d_total_bits, NULL);
    G.enc_sub = NULL;
    return rc;
}

/* multi-GPU med_dataset_float: the exact running float sum of x[0..n) continued from s_init (the sum
 * the previous shards ended with) and the max of x; synchronous */
int dc_med_sum_device(const void* d_x, long long n, float s_init, float* sum_out, float* max_out) {
    int rc = ensure_init();
    if (rc) return rc;
    if (n <= 0) return seterr(DC_ERR_ARG, "empty input");
    if (grow(&G.med_scr, &G.med_scr_cap, (size_t)dc_med_scratch_bytes(n))) return DC_ERR_HIP;
    float h[2];
    unsigned fl = 0;
    const int forced = med_force_wide();
    for (int wide = forced; wide < 2; wide++) {
        if (wide ? dc_launch_med_wide((const float*)d_x, n, s_init, G.med_scr, &G.d_f[1], &G.d_i[0], &G.d_f[2], &G.d_f[3],
                                      forced, G.st)
                 : dc_launch_med((const float*)d_x, n, s_init, G.med_scr, &G.d_f[1], &G.d_i[0], &G.d_f[2], &G.d_f[3], G.st))
            return seterr(DC_ERR_HIP, "med launch failed");
        long long r[5];
        HIPCHK(hipMemcpyAsync(r, dc_med_flag_ptr(G.med_scr, n, 0), sizeof r, hipMemcpyDeviceToHost, G.st));
        HIPCHK(hipStreamSynchronize(G.st));
        fl = (unsigned)r[0];
        { const uint32_t b = (uint32_t)r[3]; memcpy(&h[0], &b, 4); }
        { const uint32_t b = (uint32_t)r[4]; memcpy(&h[1], &b, 4); }
        G.med_wide = wide;
        if (!fl || wide) break;
    }
    if (sum_out) *sum_out = h[0];
    if (max_out) *max_out = h[1];
    return DC_OK;
}

/* multi-GPU med_dataset_float, the exscan form (dcamd.global_med): a shard's double sum and max (stats), or
 * its whole-shard transducer for the MW binades [*e_lo, *e_lo + MW) of the window its running sum is
 * estimated to enter at s_est: units[2w + p] units of 2^(E-150) added from start parity p, flags[w] end
 * parity from 0 | end parity from 1 << 1 | 4 when the shard is no transducer for that binade; synchronous */
static int med_shard(const void* d_x, long long n, double s_est, int trans, long long* h) {
    int rc = ensure_init();
    if (rc) return rc;
    if (n <= 0) return seterr(DC_ERR_ARG, "empty input");
    if (grow(&G.med_scr, &G.med_scr_cap, (size_t)dc_med_scratch_bytes(n))) return DC_ERR_HIP;
    long long* d_rec = NULL;
    if (dc_launch_med_shard((const float*)d_x, n, s_est, trans, G.med_scr, &d_rec, G.st))
        return seterr(DC_ERR_HIP, "med shard launch failed");
    HIPCHK(hipMemcpyAsync(h, d_rec, 21 * 8, hipMemcpyDeviceToHost, G.st));
    HIPCHK(hipStreamSynchronize(G.st));
    return DC_OK;
}

int dc_med_shard_stats(const void* d_x, long long n, double* sum_out, float* max_out, float* first_out) {
    long long h[21];
    int rc = med_shard(d_x, n, 0.0, 0, h);
    if (rc) return rc;
    if (sum_out) memcpy(sum_out, &h[0], 8);
    if (max_out) { const uint32_t b = (uint32_t)h[1]; memcpy(max_out, &b, 4); }
    if (first_out) { const uint32_t b = (uint32_t)h[2]; memcpy(first_out, &b, 4); }
    return DC_OK;
}

int dc_med_shard_trans(const void* d_x, long long n, double s_est, int* e_lo, long long* units, unsigned char* flags) {
    long long h[21];
    const int mw = dc_med_shard_binades();
    int rc = med_shard(d_x, n, s_est, 1, h);
    if (rc) return rc;
    if (e_lo) *e_lo = (int)h[2];
    for (int w = 0; w < mw; w++) {
        if (units) { units[2 * w] = h[3 + 2 * w]; units[2 * w + 1] = h[4 + 2 * w]; }
        if (flags) flags[w] = (unsigned char)h[15 + w];
    }
    return DC_OK;
}

/* type of med_dataset_float from a (global) max (impl/dataCompression.c:3605-3614) */
int dc_type_from_max(float mx) {
    int add = 0;
    for (int i = 7; i > 0; i--) {
        add += 1 << i;
        if ((double)mx < ldexp(1.0, add - 127)) return 8 - i;
    }
    return 0;
}

int dc_flip_bits_device(void* d_s, unsigned long long nbits, long long count, unsigned long long seed) {
    int rc = ensure_init();
    if (rc) return rc;
    if ((uintptr_t)d_s & 3u) return seterr(DC_ERR_ARG, "stream must be 4-byte aligned");
    if (dc_launch_flip_bits((uint8_t*)d_s, nbits, count, seed, G.st)) return seterr(DC_ERR_HIP, "flip launch failed");
    return DC_OK;
}

static int crc_into(const void* d_s, long long nbytes, uint32_t* d_out);

int dc_crc_resend_device(const uint32_t* d_crc2, const void* d_src, void* d_dst, long long nbytes, int copy,
                         unsigned* d_count) {
    int rc = ensure_init();
    if (rc) return rc;
    if (nbytes < 0) return seterr(DC_ERR_ARG, "nbytes < 0");
    if (copy && (((uintptr_t)d_src | (uintptr_t)d_dst) & 15u)) return seterr(DC_ERR_ARG, "streams must be 16-byte aligned");
    if (dc_launch_crc_resend(d_crc2, (const uint8_t*)d_src, (uint8_t*)d_dst, nbytes, copy, d_count, G.st))
        return seterr(DC_ERR_HIP, "resend launch failed");
    return DC_OK;
}

/* CT9 checks after dc_encode_send_device: the sender's CRC of a and the receiver's CRC of b (nbytes each, device
   results) in one pass over both */
int dc_crc32_pair_device(const void* d_a, const void* d_b, long long nbytes, uint32_t* d_crc_a, uint32_t* d_crc_b) {
    int rc = ensure_init();
    if (rc) return rc;
    if (nbytes < 0 || nbytes > 0x7FFFFF00ll - 64 || (((uintptr_t)d_a | (uintptr_t)d_b) & 15u))
        return seterr(DC_ERR_ARG, "crc pair: 16-byte aligned streams below 2 GiB");
    if (nbytes == 0) {
        if ((rc = crc_into(d_a, 0, d_crc_a))) return rc;
        return crc_into(d_b, 0, d_crc_b);
    }
    const long long parts = 2 * dc_crc_parts(nbytes) + 1;
    if (parts > G.crcparts_cap) {
        if (G.d_crcparts) HIPCHK(hipFree(G.d_crcparts));
        HIPCHK(hipMalloc((void**)&G.d_crcparts, parts * 4 + 1024));
        G.crcparts_cap = parts;
    }
    if (dc_launch_crc32_pair((const uint8_t*)d_a, (const uint8_t*)d_b, nbytes, G.d_crctab, G.d_x2n, G.d_crcparts,
                             d_crc_a, d_crc_b, G.st))
        return seterr(DC_ERR_HIP, "crc pair launch failed");
    return DC_OK;
}

/* CT9 send: the stream copied to the receiver's buffer (the channel) with the CRC of the bytes sent computed in
   the same pass (*d_crc, device) */
int dc_crc32_copy_device(const void* d_src, void* d_dst, long long nbytes, uint32_t* d_crc) {
    int rc = ensure_init();
    if (rc) return rc;
    if (nbytes < 0 || nbytes > 0x7FFFFF00ll - 64 || (((uintptr_t)d_src | (uintptr_t)d_dst) & 15u))
        return seterr(DC_ERR_ARG, "crc copy: 16-byte aligned streams below 2 GiB");
    if (nbytes == 0) return crc_into(d_src, 0, d_crc);
    const long long parts = dc_crc_parts(nbytes) + 1;
    if (parts > G.crcparts_cap) {
        if (G.d_crcparts) HIPCHK(hipFree(G.d_crcparts));
        HIPCHK(hipMalloc((void**)&G.d_crcparts, parts * 4 + 1024));
        G.crcparts_cap = parts;
    }
    if (dc_launch_crc32_copy((const uint8_t*)d_src, (uint8_t*)d_dst, nbytes, G.d_crctab, G.d_x2n, G.d_crcparts, d_crc,
                             G.st))
        return seterr(DC_ERR_HIP, "crc copy launch failed");
    return DC_OK;
}

int dc_crc32_device_async(const void* d_s, long long nbytes, uint32_t* d_crc) {
    int rc = ensure_init();
    if (rc) return rc;
    return crc_into(d_s, nbytes, d_crc);
}

int dc_crc32_device(const void* d_s, long long nbytes, uint32_t* crc_out) {
    int rc = ensure_init();
    if (rc) return rc;
    if ((rc = crc_into(d_s, nbytes, G.d_crc))) return rc;
    if (crc_out) {
        uint32_t h;
        HIPCHK(hipMemcpyAsync(&h, G.d_crc, 4, hipMemcpyDeviceToHost, G.st));
        HIPCHK(hipStreamSynchronize(G.st));
        *crc_out = h;
    }
    return DC_OK;
}

int dc_hash_device(const void* d_buf, long long nbytes, unsigned long long* hash_out) {
    int rc = ensure_init();
    if (rc) return rc;
    if (nbytes < 0 || ((uintptr_t)d_buf & 3u)) return seterr(DC_ERR_ARG, "hash: nbytes < 0 or buffer not 4-byte aligned");
    if (dc_launch_hash_words(d_buf, nbytes, (unsigned long long*)G.d_crc + 1, G.st))
        return seterr(DC_ERR_HIP, "hash launch failed");
    unsigned long long h = 0;
    HIPCHK(hipMemcpyAsync(&h, (unsigned long long*)G.d_crc + 1, 8, hipMemcpyDeviceToHost, G.st));
    HIPCHK(hipStreamSynchronize(G.st));
    if (hash_out) *hash_out = h;
    return DC_OK;
}

/* co-residency tests: `blocks` workgroups (256 threads, lds bytes of LDS each) resident for `us` microseconds on
   `stream` (NULL: a stream of the library's own, not the codec's) -- asynchronous */
int dc_occupy_device(void* stream, double us, int blocks, int lds) {
    int rc = ensure_init();
    if (rc) return rc;
    static hipStream_t own = NULL;
    if (!stream) {
        if (!own) HIPCHK(hipStreamCreateWithFlags(&own, hipStreamNonBlocking));
        stream = own;
    }
    if (dc_launch_occupy(us, blocks, lds, G.d_enc_err + 12, (hipStream_t)stream))   /* (a word nothing reads) */
        return seterr(DC_ERR_ARG, "occupy: blocks >= 1, 0 <= us <= 1e6, lds <= 160 KiB");
    return DC_OK;
}

int dc_copy_rate_device(const void* d_src, void* d_dst, long long bytes, int reps, double* gbs_out, int* variant_out) {
    int rc = ensure_init();
    if (rc) return rc;
    if (bytes < 16 || (bytes & 15) || bytes > 0x7FFFFF00ll || reps < 1 || (((uintptr_t)d_src | (uintptr_t)d_dst) & 15u))
        return seterr(DC_ERR_ARG, "copy rate: 16-byte aligned buffers, bytes a multiple of 16 below 2 GiB");
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    double best = 0.0;
    int bv = 0;
    for (int v = 0; v < 4; v++) {
        for (int w = 0; w < 2; w++)                  /* warm-up */
            if (dc_launch_stream_copy(d_src, d_dst, bytes, v, G.st)) return seterr(DC_ERR_HIP, "copy launch failed");
        HIPCHK(hipEventRecord(e0, G.st));
        for (int r = 0; r < reps; r++)
            if (dc_launch_stream_copy(d_src, d_dst, bytes, v, G.st)) return seterr(DC_ERR_HIP, "copy launch failed");
        HIPCHK(hipEventRecord(e1, G.st));
        HIPCHK(hipEventSynchronize(e1));
        float ms = 0.0f;
        HIPCHK(hipEventElapsedTime(&ms, e0, e1));
        const double gbs = ms > 0.0f ? 2.0 * (double)bytes * reps / (ms * 1e-3) / 1e9 : 0.0;
        if (gbs > best) { best = gbs; bv = v; }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (gbs_out) *gbs_out = best;
    if (variant_out) *variant_out = bv;
    return DC_OK;
}

/* the fused-CRC forms (dc_gpu.h): a stream's CRC by the 16 KiB block kernel + one combine; the CT9 resend with
   the receiver's CRC of the copy computed as it is written */
int dc_crc32_stream_device(const void* d_s, long long nbytes, uint32_t* d_crc) {
    int rc = ensure_init();
    if (rc) return rc;
    if (nbytes < 0 || nbytes > 0x7FFFFF00ll - 64 || ((uintptr_t)d_s & 15u)) return seterr(DC_ERR_ARG, "crc: bad stream");
    uint32_t* blk = crcf_slot(1, nbytes);
    if (!blk) return seterr(DC_ERR_HIP, "crc block allocation failed");
    if (dc_launch_crcf_blocks((const uint8_t*)d_s, NULL, nbytes, G.d_crcf, blk, NULL, NULL, G.st) ||
        dc_launch_crcf_final(blk, nbytes, nbytes, NULL, G.d_crcf, d_crc, NULL, NULL, NULL, G.st))
        return seterr(DC_ERR_HIP, "crc launch failed");
    return DC_OK;
}

int dc_crc_resend_crc_device(uint32_t* d_crc2, const void* d_src, void* d_dst, long long nbytes, unsigned* d_count) {
    int rc = ensure_init();
    if (rc) return rc;
    if (nbytes < 0 || nbytes > 0x7FFFFF00ll - 64 || (((uintptr_t)d_src | (uintptr_t)d_dst) & 15u))
        return seterr(DC_ERR_ARG, "resend: 16-byte aligned streams below 2 GiB");
    if (nbytes == 0) return DC_OK;
    /* the 32 KiB-block CRC with the copy in its loads and a gated combine (the 16 KiB-block form with the
       encoder's fused layout measured 102 us per 163 MB, this one ~70) */
    const long long parts = dc_crc_parts(nbytes) + 1;
    if (parts > G.crcparts_cap) {
        if (G.d_crcparts) HIPCHK(hipFree(G.d_crcparts));
        HIPCHK(hipMalloc((void**)&G.d_crcparts, parts * 4 + 1024));
        G.crcparts_cap = parts;
    }
    if (dc_launch_crc32_resend((const uint8_t*)d_src, (uint8_t*)d_dst, nbytes, G.d_crctab, G.d_x2n, G.d_crcparts,
                               d_crc2, d_count, G.st))
        return seterr(DC_ERR_HIP, "resend launch failed");
    return DC_OK;
}

static int crc_into(const void* d_s, long long nbytes, uint32_t* d_out) {
    long long parts = dc_crc_parts(nbytes) + 1;
    if (parts > G.crcparts_cap) {
        if (G.d_crcparts) HIPCHK(hipFree(G.d_crcparts));
        HIPCHK(hipMalloc((void**)&G.d_crcparts, parts * 4 + 1024));
        G.crcparts_cap = parts;
    }
    if (dc_launch_crc32((const uint8_t*)d_s, nbytes, G.d_crctab, G.d_x2n, G.d_crcparts, 0u, d_out, G.st))
        return seterr(DC_ERR_HIP, "crc launch failed");
    return DC_OK;
}

/* ============================================================================================
 * Reference ABI (impl/dataCompression.h).  Host buffers in, host malloc'ed buffers out.
 * ========================================================================================== */
static uint32_t mask_from_chars(const char* mask) {
    uint32_t m = 0;
    for (int i = 0; i < 17; i++) m = (m << 1) | (uint32_t)(mask[i] == '1');
    return m;
}

static void abi_fail(const char* fn, int rc) {
    G.abi_rc = rc;
    fprintf(stderr, "libdcamd: %s failed (%d): %s\n", fn, rc, G.msg);
}

/* add_bit_to_bytes-compatible append of a GPU-encoded stream (:5456-5489 semantics) */
static int abi_compress(const char* fn, int ct, const float* data, int num, unsigned char** data_bits, int* bytes,
                        int* pos, int type, uint32_t mask17) {
    int rc = ensure_init();
    G.abi_rc = DC_OK;
    if (rc) { abi_fail(fn, rc); return rc; }
    if (num <= 0) return DC_OK;
    const long long used = (long long)(*bytes) * 8 - (*pos == 8 ? 0 : *pos);
    const int sb = (int)(used & 7);
    const long long keep = used >> 3;
    if ((rc = grow(&G.d_a, &G.d_a_cap, (size_t)num * 4 + 64)) || (rc = grow(&G.d_b, &G.d_b_cap, dc_stream_capacity(num)))) {
        abi_fail(fn, rc); return rc;
    }
    if (hipMemcpyAsync(G.d_a, data, (size_t)num * 4, hipMemcpyHostToDevice, G.st) != hipSuccess) {
        rc = seterr(DC_ERR_HIP, "H2D copy failed"); abi_fail(fn, rc); return rc;
    }
    unsigned long long tb = 0;
    if ((rc = encode_lib(ct, G.d_a, num, 0, type, mask17, sb, G.d_b, NULL)) || (rc = dc_encode_result(&tb))) {
        abi_fail(fn, rc); return rc;
    }
    const long long nb_new = (long long)((tb + 7) >> 3);
    const long long total = keep + nb_new;
    const unsigned char old = sb ? (unsigned char)((*data_bits)[keep] & (0xFFu << (8 - sb))) : 0;
    unsigned char* nb = (unsigned char*)realloc(*data_bits, total > 0 ? (size_t)total : 1);
    if (!nb) { rc = seterr(DC_ERR_ARG, "realloc of %lld bytes failed", total); abi_fail(fn, rc); return rc; }
    *data_bits = nb;
    if (hipMemcpy(nb + keep, G.d_b, (size_t)nb_new, hipMemcpyDeviceToHost) != hipSuccess) {
        rc = seterr(DC_ERR_HIP, "D2H copy failed"); abi_fail(fn, rc); return rc;
    }
    if (sb) nb[keep] |= old;
    const long long tot_bits = keep * 8 + (long long)tb;
    *bytes = (int)total;
    *pos = (tot_bits & 7) ? (int)(8 - (tot_bits & 7)) : 8;
    return DC_OK;
}

static float* abi_decompress(const char* fn, int ct, const unsigned char* data_bits, int bytes, int num, int type,
                             uint32_t mask17) {
    /* on an error the result is all zeros (never stale device data) and dc_abi_status() reports it */
    const size_t osz = sizeof(float) * (size_t)(num > 0 ? num : 1);
    float* out = (float*)malloc(osz);
    int rc = ensure_init();
    G.abi_rc = DC_OK;
    if (rc) { abi_fail(fn, rc); if (out) memset(out, 0, osz); return out; }
    if (!out) { abi_fail(fn, seterr(DC_ERR_ARG, "malloc of %zu bytes failed", osz)); return out; }
    if (num <= 0 || bytes <= 0) { memset(out, 0, osz); return out; }
    if ((rc = grow(&G.d_a, &G.d_a_cap, (size_t)bytes + 64)) || (rc = grow(&G.d_b, &G.d_b_cap, (size_t)num * 4 + 64))) {
        abi_fail(fn, rc); memset(out, 0, osz); return out;
    }
    if (hipMemcpyAsync(G.d_a, data_bits, (size_t)bytes, hipMemcpyHostToDevice, G.st) != hipSuccess) {
        abi_fail(fn, seterr(DC_ERR_HIP, "H2D copy failed")); memset(out, 0, osz); return out;
    }
    if ((rc = dc_decode_device(ct, G.d_a, bytes, NULL, bytes + 64, num, type, mask17, G.d_b)) || (rc = dc_decode_finish())) {
        abi_fail(fn, rc); memset(out, 0, osz); return out;
    }
    if (hipMemcpy(out, G.d_b, (size_t)num * 4, hipMemcpyDeviceToHost) != hipSuccess) {
        abi_fail(fn, seterr(DC_ERR_HIP, "D2H copy failed")); memset(out, 0, osz);
    }
    return out;
}

/* myCompress_bitwise (:3310), _np (:2645), _op (:577), _mask (:2030) */
void myCompress_bitwise(float data[], int num, unsigned char** data_bits, int* bytes, int* pos) {
    abi_compress("myCompress_bitwise", 5, data, num, data_bits, bytes, pos, 0, 0);
}
void myCompress_bitwise_np(float data[], int num, unsigned char** data_bits, int* bytes, int* pos) {
    abi_compress("myCompress_bitwise_np", 6, data, num, data_bits, bytes, pos, 0, 0);
}
void myCompress_bitwise_op(float data[], int num, unsigned char** data_bits, int* bytes, int* pos) {
    abi_compress("myCompress_bitwise_op", 11, data, num, data_bits, bytes, pos, 0, 0);
}
void myCompress_bitwise_mask(float data[], int num, unsigned char** data_bits, int* bytes, int* pos, int type,
                             char mask[1 + 8 + 8]) {
    abi_compress("myCompress_bitwise_mask", 7, data, num, data_bits, bytes, pos, type, mask_from_chars(mask));
}

/* myDecompress_bitwise (:2922), _np (:2459), _op (:698), _mask (:1703) */
float* myDecompress_bitwise(unsigned char* data_bits, int bytes, int num) {
    return abi_decompress("myDecompress_bitwise", 5, data_bits, bytes, num, 0, 0);
}
float* myDecompress_bitwise_np(unsigned char* data_bits, int bytes, int num) {
    return abi_decompress("myDecompress_bitwise_np", 6, data_bits, bytes, num, 0, 0);
}
float* myDecompress_bitwise_op(unsigned char* data_bits, int bytes, int num) {
    return abi_decompress("myDecompress_bitwise_op", 11, data_bits, bytes, num, 0, 0);
}
float* myDecompress_bitwise_mask(unsigned char* data_bits, int bytes, int num, int type, char mask[1 + 8 + 8]) {
    return abi_decompress("myDecompress_bitwise_mask", 7, data_bits, bytes, num, type, mask_from_chars(mask));
}

/* toSmallDataset_float (:3543-3562): *data_small = malloc'ed data - min, returns min */
float toSmallDataset_float(float data[], float** data_small, int num) {
    *data_small = (float*)malloc(sizeof(float) * (size_t)(num > 0 ? num : 1));
    int rc = ensure_init();
    if (rc || num <= 0) { if (rc) abi_fail("toSmallDataset_float", rc); return num > 0 ? data[0] : 0.0f; }
    if ((rc = grow(&G.d_a, &G.d_a_cap, (size_t)num * 4 + 64)) || (rc = grow(&G.d_b, &G.d_b_cap, (size_t)num * 4 + 64))) {
        abi_fail("toSmallDataset_float", rc); return data[0];
    }
    float mn = data[0];
    if (hipMemcpyAsync(G.d_a, data, (size_t)num * 4, hipMemcpyHostToDevice, G.st) != hipSuccess ||
        (rc = dc_to_small_device(G.d_a, num, G.d_b, &mn)) ||
        hipMemcpy(*data_small, G.d_b, (size_t)num * 4, hipMemcpyDeviceToHost) != hipSuccess)
        abi_fail("toSmallDataset_float", rc ? rc : DC_ERR_HIP);
    return mn;
}

/* med_dataset_float (:3593-3620) */
float med_dataset_float(float* data, int num, int* type) {
    int rc = ensure_init();
    if (rc || num <= 0) { if (rc) abi_fail("med_dataset_float", rc); return 0.0f; }
    if ((rc = grow(&G.d_a, &G.d_a_cap, (size_t)num * 4 + 64))) { abi_fail("med_dataset_float", rc); return 0.0f; }
    float mean = 0.0f;
    int t = *type;
    if (hipMemcpyAsync(G.d_a, data, (size_t)num * 4, hipMemcpyHostToDevice, G.st) != hipSuccess ||
        (rc = dc_med_device(G.d_a, num, &mean, &t))) {
        abi_fail("med_dataset_float", rc ? rc : DC_ERR_HIP);
        return 0.0f;
    }
    if (t) *type = t;                      /* the reference leaves *type untouched if no i matches */
    return mean;
}

/* do_crc32 (:5524-5534) */
uint32_t do_crc32(unsigned char* data_bits, int bytes) {
    int rc = ensure_init();
    if (rc) { abi_fail("do_crc32", rc); return 0; }
    if (bytes <= 0) return 0;
    uint32_t crc = 0;
    if ((rc = grow(&G.d_a, &G.d_a_cap, (size_t)bytes + 64)) ||
        hipMemcpyAsync(G.d_a, data_bits, (size_t)bytes, hipMemcpyHostToDevice, G.st) != hipSuccess ||
        (rc = dc_crc32_device(G.d_a, bytes, &crc)))
        abi_fail("do_crc32", rc ? rc : DC_ERR_HIP);
    return crc;
}

/* ---- Hamming SECDED (:5544-5855) -------------------------------------------------------- */
int hmLength(int k) {                                        /* :5581-5592 */
    int r = 0;
    while (((1LL << r) - 1) - r - (long long)k < 0) r++;
    return r;
}

static int ham_syndrome(const unsigned char* bits, int bytes, unsigned long long* syn, unsigned long long* ones) {
    int rc = ensure_init();
    if (rc) return rc;
    if ((rc = grow(&G.d_a, &G.d_a_cap, (size_t)bytes + 64))) return rc;
    HIPCHK(hipMemcpyAsync(G.d_a, bits, (size_t)bytes, hipMemcpyHostToDevice, G.st));
    if (dc_launch_ham_syndrome((const uint8_t*)G.d_a, bytes, G.d_ham, G.st)) return seterr(DC_ERR_HIP, "hamming launch");
    HIPCHK(hipMemcpyAsync(&G.h_scratch[4], G.d_ham, 16, hipMemcpyDeviceToHost, G.st));
    HIPCHK(hipStreamSynchronize(G.st));
    *syn = G.h_scratch[4];
    *ones = G.h_scratch[5];
    return DC_OK;
}

void hamming_encode(unsigned char* bits, char** c, int bytes, int* r) {   /* :5740-5748 */
    *r = hmLength(bytes * 8);
    *c = (char*)malloc((size_t)(*r + 1));
    unsigned long long syn = 0, ones = 0;
    int rc = ham_syndrome(bits, bytes, &syn, &ones);
    if (rc) { abi_fail("hamming_encode", rc); memset(*c, '0', (size_t)(*r + 1)); return; }
    unsigned long long sum = ones;
    for (int i = 0; i < *r; i++) { (*c)[i] = (char)('0' + ((syn >> i) & 1)); sum += (syn >> i) & 1; }
    (*c)[*r] = (char)('0' + (sum & 1));
}

int hamming_decode(unsigned char* bits, char* c, int bytes, int r) {       /* :5750-5778 */
    unsigned long long syn = 0, ones = 0;
    int rc = ham_syndrome(bits, bytes, &syn, &ones);
    if (rc) { abi_fail("hamming_decode", rc); return 0; }
    long long pos = 0;
    unsigned long long sum = ones;
    for (int i = 0; i < r; i++) {
        const int ci = c[i] - '0';
        pos += (long long)((int)((syn >> i) & 1) != ci) << i;     /* hamming_verify_bit :5803 */
        sum += (unsigned long long)ci;
    }
    const int vr = (int)(sum & 1) != (c[r] - '0');
    int type = 0;                                                 /* error_info :5631-5654 */
    if (pos > 0 && !vr) type = 1;
    else if (pos == 0 && vr) type = 2;
    else if (pos > 0 && vr) type = 3;
    if (type == 1) printf("two-bit error\n");
    if (type == 2) { printf("parity error\n"); c[r] = c[r] == '0' ? '1' : '0'; }
    if (type == 3) {                                              /* hamming_rectify_bit :5822 */
        printf("one bit error: pos = %lld\n", pos);
        const long long k = (long long)bytes * 8;
        if (pos <= r + k) {
            if ((pos & (pos - 1)) == 0) {
                int ci = 0;
                while ((1LL << ci) != pos) ci++;
                c[ci] = c[ci] == '0' ? '1' : '0';
            } else {
                long long npow = 0;
                while ((1LL << npow) < pos) npow++;
                const long long d = pos - 1 - npow;
                bits[d >> 3] ^= (unsigned char)(1u << (7 - (d & 7)));
            }
        }
    }
    return type;
}

/* ---- small helpers of the reference ABI ------------------------------------------------- */
int to_absErrorBound_binary(double bound) { return bound_binary(bound); }   /* :5512-5522 */

#ifndef BER
#define BER 1e-6                                                 /* impl/dataCompression.h:4 */
#endif
int block_size(int data_bytes) {                                 /* :5868-5879 */
    double ber = BER;
    uint64_t b = (uint64_t)(1 / ber);
    uint64_t by = b / 8;
    int bs = data_bytes;
    if ((uint64_t)bs > by) bs = (int)by;
    return bs;
}

void bit_flip(unsigned char* bits, int bytes) {                  /* :5858-5865, libc rand() */
    int num = rand() % (bytes * 8);
    bits[num / 8] ^= (unsigned char)(1 << (7 - num % 8));
}

uint64_t get_random_int(uint64_t from, uint64_t to) { return (uint64_t)rand() % (to - from + 1) + from; }

/* ---- Himeno plane extraction and binary file helpers (link closure of the float apps) ----------- */
#ifndef MIMAX
#define MIMAX 129                                                /* impl/param.h:7-9 */
#endif
#ifndef MJMAX
#define MJMAX 129
#endif
#ifndef MKMAX
#define MKMAX 131
#endif

/* transform_3d_array_to_1d_array (:3741-3775) for an explicit [mi][mj][mk] extent */
float* dc_transform_3d_array_to_1d_array(const float* data, int mi, int mj, int mk, int ijk, int v, int imax,
                                         int jmax, int kmax) {
    int A, B;
    if (ijk == 1) { A = jmax; B = kmax; }
    else if (ijk == 2) { A = imax; B = kmax; }
    else if (ijk == 3) { A = imax; B = jmax; }
    else { seterr(DC_ERR_ARG, "transform_3d_array_to_1d_array: ijk %d", ijk); return NULL; }
    float* o = (float*)malloc(sizeof(float) * (size_t)(A > 0 ? A : 1) * (size_t)(B > 0 ? B : 1));
    if (!o) return NULL;
    (void)mi;
    size_t n = 0;
    for (int a = 0; a < A; a++)
        for (int b = 0; b < B; b++) {
            size_t i, j, k;
            if (ijk == 1) { i = (size_t)v; j = (size_t)a; k = (size_t)b; }
            else if (ijk == 2) { i = (size_t)a; j = (size_t)v; k = (size_t)b; }
            else { i = (size_t)a; j = (size_t)b; k = (size_t)v; }
            o[n++] = data[(i * (size_t)mj + j) * (size_t)mk + k];
        }
    return o;
}

float* transform_3d_array_to_1d_array(float data[MIMAX][MJMAX][MKMAX], int ijk, int v, int imax, int jmax, int kmax) {
    return dc_transform_3d_array_to_1d_array(&data[0][0][0], MIMAX, MJMAX, MKMAX, ijk, v, imax, jmax, kmax);
}

/* :5290-5339 (the reference reports success / failure on stdout) */
static void write_binary(const char* file, const void* data, size_t sz, int count) {
    FILE* fp = fopen(file, "wb");
    if (!fp) { printf("failed to open %s\n", file); return; }
    fwrite(data, sz, (size_t)count, fp);
    fclose(fp);
    printf("saved %s\n", file);
}
void writetobinary_float(const char* file, float* data, int count) { write_binary(file, data, sizeof(float), count); }
void writetobinary_char(const char* file, unsigned char* data, int count) { write_binary(file, data, 1, count); }

/* :5383-5410: the whole file; the reference exit(0)s when it cannot be opened, this returns NULL */
unsigned char* readfrombinary_char(const char* file, int* bytes_sz) {
    FILE* fp = fopen(file, "rb");
    if (!fp) { printf("failed to open %s\n", file); seterr(DC_ERR_ARG, "cannot open %s", file); return NULL; }
    fseek(fp, 0, SEEK_END);
    long sz = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    unsigned char* arr = (unsigned char*)malloc(sz > 0 ? (size_t)sz : 1);
    size_t got = arr ? fread(arr, 1, (size_t)(sz > 0 ? sz : 0), fp) : 0;
    fclose(fp);
    *bytes_sz = (int)got;
    return arr;
}

/* :5412-5432 */
float* readfrombinary_writetotxt_float(const char* binaryfile, const char* txtfile, int count) {
    FILE* fp = fopen(binaryfile, "rb");
    if (!fp) { seterr(DC_ERR_ARG, "cannot open %s", binaryfile); return NULL; }
    float* arr = (float*)malloc(sizeof(float) * (size_t)(count > 0 ? count : 1));
    size_t got = arr ? fread(arr, sizeof(float), (size_t)(count > 0 ? count : 0), fp) : 0;
    fclose(fp);
    (void)got;
    fp = fopen(txtfile, "w");
    if (!fp) { seterr(DC_ERR_ARG, "cannot open %s", txtfile); return arr; }
    for (int i = 0; i < count; i++) fprintf(fp, "%f\n", arr[i]);
    fclose(fp);
    return arr;
}

void floattostr(float* a, char* str) {                           /* :5244-5252 */
    uint32_t c;
    memcpy(&c, a, 4);
    for (int i = 0; i < 32; i++) str[i] = (char)('0' + ((c >> (31 - i)) & 1));
    str[32] = '\0';
}

float strtofloat(char* str) {                                    /* :5267-5276 */
    uint32_t u = 0;
    for (int i = 0; i < 32; i++) u = (u << 1) + (uint32_t)(str[i] - '0');
    float f;
    memcpy(&f, &u, 4);
    return f;
}

void doubletostr(double* a, char* str) {                         /* :5256-5264 */
    uint64_t c;
    memcpy(&c, a, 8);
    for (int i = 0; i < 64; i++) str[i] = (char)('0' + ((c >> (63 - i)) & 1));
    str[64] = '\0';
}

double strtodbl(char* str) {                                     /* :5279-5288 */
    uint64_t u = 0;
    for (int i = 0; i < 64; i++) u = (u << 1) + (uint64_t)(str[i] - '0');
    double d;
    memcpy(&d, &u, 8);
    return d;
}

void getFloatBin(float num, char bin[]) {                        /* :5220-5230 (digits 0/1, not chars) */
    uint32_t c;
    memcpy(&c, &num, 4);
    for (int i = 0; i < 32; i++) bin[i] = (char)((c >> (31 - i)) & 1);
}

void bit_set(unsigned char* p_data, unsigned char position, int flag) {   /* :5492-5510 */
    if (!p_data || position > 8 || position < 1 || (flag != 0 && flag != 1)) return;
    if (flag != ((*p_data >> (position - 1)) & 1)) *p_data ^= (unsigned char)(1 << (position - 1));
}

void add_bit_to_bytes(unsigned char** data_bits, int* bytes, int* pos, int flag) {   /* :5456-5489 */
    if (*pos <= 0 || *pos >= 9) return;
    if (*pos == 8) {
        unsigned char* more = (unsigned char*)realloc(*data_bits, (size_t)(*bytes + 1));
        if (!more) { fprintf(stderr, "libdcamd: add_bit_to_bytes: realloc failed\n"); return; }
        *data_bits = more;
        (*bytes)++;
        (*data_bits)[*bytes - 1] = 0;
    }
    bit_set(&(*data_bits)[*bytes - 1], (unsigned char)*pos, flag);
    (*pos)--;
    if (*pos == 0) *pos = 8;
}

/* ============================================================================================
 * CT1 byte-wise codec: myCompress (impl/dataCompression.c:3980-4118), myDecompress (:3943-3977)
 * ========================================================================================== */
static int c1_scratch(long long n, uint32_t** traw, unsigned long long** rawoff, uint8_t** carr) {
    const long long nt = dc_ct1_tiles(n > 0 ? n : 1);
    const size_t need = (size_t)nt * 4 + 16 + (size_t)(nt + 1) * 8 + (size_t)n + 64;
    int rc = grow(&G.c1_scr, &G.c1_scr_cap, need);
    if (rc) return rc;
    char* p = (char*)G.c1_scr;
    *rawoff = (unsigned long long*)p;                    /* 8-byte aligned first */
    *traw = (uint32_t*)(p + (size_t)(nt + 1) * 8);
    *carr = (uint8_t*)(p + (size_t)(nt + 1) * 8 + (size_t)nt * 4 + 16);
    return DC_OK;
}

int dc_ct1_encode_device(const void* d_x, long long n, void* d_raw, void* d_codes, void* d_pos1, long long* nraw_out) {
    int rc = ensure_init();
    if (rc) return rc;
    if (n < 0) return seterr(DC_ERR_ARG, "n < 0");
    if (n == 0) { if (nraw_out) *nraw_out = 0; return DC_OK; }
    uint32_t* traw; unsigned long long* rawoff; uint8_t* carr;
    if ((rc = c1_scratch(n, &traw, &rawoff, &carr))) return rc;
    HIPCHK(hipMemsetAsync(G.d_enc_err + 12, 0, 4, G.st));
    if (dc_launch_ct1_encode((const float*)d_x, n, thr_le(absErrBound), traw, rawoff, (float*)d_raw, (char*)d_codes,
                             (int*)d_pos1, G.d_enc_err + 12, G.st))
        return seterr(DC_ERR_HIP, "ct1 encode launch failed");
    const long long nt = dc_ct1_tiles(n);
    HIPCHK(hipMemcpyAsync(&G.h_scratch[0], rawoff + nt, 8, hipMemcpyDeviceToHost, G.st));
    HIPCHK(hipMemcpyAsync(&G.h_scratch[1], G.d_enc_err + 12, 4, hipMemcpyDeviceToHost, G.st));
    HIPCHK(hipStreamSynchronize(G.st));
    if (G.h_scratch[1] & 1u) return seterr(DC_ERR_INPUT, "input contains -1.0f (the reference's history sentinel)");
    if (nraw_out) *nraw_out = (long long)G.h_scratch[0];
    return DC_OK;
}

int dc_ct1_decode_device(const void* d_raw, long long nraw, const void* d_codes, const void* d_pos1, long long ncodes,
                         long long num, void* d_out) {
    int rc = ensure_init();
    if (rc) return rc;
    if (num <= 0) return DC_OK;
    uint32_t* traw; unsigned long long* rawoff; uint8_t* carr;
    if ((rc = c1_scratch(num, &traw, &rawoff, &carr))) return rc;
    HIPCHK(hipMemsetAsync(G.d_enc_err + 12, 0, 4, G.st));
    if (dc_launch_ct1_decode((const float*)d_raw, nraw, (const char*)d_codes, (const int*)d_pos1, ncodes, num, carr, traw,
                             rawoff, (float*)d_out, G.d_enc_err + 12, G.st))
        return seterr(DC_ERR_HIP, "ct1 decode launch failed");
    HIPCHK(hipMemcpyAsync(&G.h_scratch[1], G.d_enc_err + 12, 4, hipMemcpyDeviceToHost, G.st));
    HIPCHK(hipStreamSynchronize(G.st));
    if (G.h_scratch[1] & 4u) return seterr(DC_ERR_STREAM, "ct1 codes out of range or raw array too short");
    return DC_OK;
}

/* h:120 c:3980-4118.  *array_float / *array_char / *array_char_displacement are realloc()ed to the
 * raw and code counts (left untouched when a count is 0, as the reference does); returns the raw count. */
int myCompress(float data[], float** array_float, char** array_char, int** array_char_displacement, int num) {
    const char* fn = "myCompress";
    int rc = ensure_init();
    if (rc) { abi_fail(fn, rc); return 0; }
    if (num <= 0) return 0;
    const size_t n = (size_t)num;
    if ((rc = grow(&G.c1_in, &G.c1_in_cap, n * 4 + 64)) || (rc = grow(&G.c1_out, &G.c1_out_cap, n * 4 + 64)) ||
        (rc = grow(&G.c1_codes, &G.c1_codes_cap, n + 64)) || (rc = grow(&G.c1_pos, &G.c1_pos_cap, n * 4 + 64))) {
        abi_fail(fn, rc); return 0;
    }
    if (hipMemcpyAsync(G.c1_in, data, n * 4, hipMemcpyHostToDevice, G.st) != hipSuccess) {
        abi_fail(fn, seterr(DC_ERR_HIP, "H2D copy failed")); return 0;
    }
    long long nraw = 0;
    if ((rc = dc_ct1_encode_device(G.c1_in, num, G.c1_out, G.c1_codes, G.c1_pos, &nraw))) { abi_fail(fn, rc); return 0; }
    const long long nc = num - nraw;
    if (nraw > 0) {
        float* a = (float*)realloc(*array_float, sizeof(float) * (size_t)nraw);
        if (!a) { abi_fail(fn, seterr(DC_ERR_ARG, "realloc failed")); return 0; }
        *array_float = a;
        if (hipMemcpy(a, G.c1_out, sizeof(float) * (size_t)nraw, hipMemcpyDeviceToHost) != hipSuccess) {
            abi_fail(fn, seterr(DC_ERR_HIP, "D2H copy failed")); return 0;
        }
    }
    if (nc > 0) {
        char* c = (char*)realloc(*array_char, (size_t)nc);
        int* p = (int*)realloc(*array_char_displacement, sizeof(int) * (size_t)nc);
        if (!c || !p) { abi_fail(fn, seterr(DC_ERR_ARG, "realloc failed")); return 0; }
        *array_char = c;
        *array_char_displacement = p;
        if (hipMemcpy(c, G.c1_codes, (size_t)nc, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(p, G.c1_pos, sizeof(int) * (size_t)nc, hipMemcpyDeviceToHost) != hipSuccess) {
            abi_fail(fn, seterr(DC_ERR_HIP, "D2H copy failed")); return 0;
        }
    }
    return (int)nraw;
}

/* h:121 c:3943-3977.  The reference does not pass the code count: it consumes displacement entries
 * while they name a later position (reading one entry past the last code).  The same rule gives the
 * count here: entries are taken while they increase and stay within [1, num]. */
float* myDecompress(float array_float[], char array_char[], int array_char_displacement[], int num) {
    const char* fn = "myDecompress";
    float* out = (float*)malloc(sizeof(float) * (size_t)(num > 0 ? num : 1));
    int rc = ensure_init();
    if (rc) { abi_fail(fn, rc); return out; }
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
    if ((rc = grow(&G.c1_in, &G.c1_in_cap, n * 4 + 64)) || (rc = grow(&G.c1_out, &G.c1_out_cap, n * 4 + 64)) ||
        (rc = grow(&G.c1_codes, &G.c1_codes_cap, n + 64)) || (rc = grow(&G.c1_pos, &G.c1_pos_cap, n * 4 + 64))) {
        abi_fail(fn, rc); return out;
    }
    if ((nraw > 0 && hipMemcpyAsync(G.c1_in, array_float, sizeof(float) * (size_t)nraw, hipMemcpyHostToDevice, G.st) != hipSuccess) ||
        (nc > 0 && hipMemcpyAsync(G.c1_codes, array_char, (size_t)nc, hipMemcpyHostToDevice, G.st) != hipSuccess) ||
        (nc > 0 && hipMemcpyAsync(G.c1_pos, array_char_displacement, sizeof(int) * (size_t)nc, hipMemcpyHostToDevice, G.st) != hipSuccess)) {
        abi_fail(fn, seterr(DC_ERR_HIP, "H2D copy failed")); return out;
    }
    if ((rc = dc_ct1_decode_device(G.c1_in, nraw, G.c1_codes, G.c1_pos, nc, num, G.c1_out))) abi_fail(fn, rc);
    if (hipMemcpy(out, G.c1_out, sizeof(float) * n, hipMemcpyDeviceToHost) != hipSuccess)
        abi_fail(fn, seterr(DC_ERR_HIP, "D2H copy failed"));
    return out;
}

/* ============================================================================================
 * CT2 / CT3 compression-ratio estimators (impl/dataCompression.c:3622-3739, :4121-5219) on the GPU
 * (dc_ratio.hip): a data-parallel pass sums every element's bits (the history is the original data);
 * an input holding -1.0 (the reference's empty-history sentinel) is re-estimated by one lane running the
 * reference loop; the area estimators pack per-element sizes greedily in one lane.  The returned float
 * is formed with the reference's own integer / float types.
 * ========================================================================================== */
static int ratio_scratch(void) {
    if (!G.d_ratio) HIPCHK(hipMalloc((void**)&G.d_ratio, 64));
    return DC_OK;
}

/* bits (or, for the area mode, 512-bit blocks) of x[0..n) (host) under estimator `mode` */
static int ratio_run(int is_double, int mode, const void* x, long long n, unsigned long long* out) {
    int rc = ensure_init();
    if (rc) return rc;
    *out = 0;
    if (n <= 0) return DC_OK;
    const size_t esz = is_double ? 8 : 4;
    if ((rc = ratio_scratch()) || (rc = grow(&G.d_a, &G.d_a_cap, (size_t)n * esz + 64))) return rc;
    if (mode == 4 && (rc = grow(&G.d_b, &G.d_b_cap, (size_t)n + 64))) return rc;
    HIPCHK(hipMemcpyAsync(G.d_a, x, (size_t)n * esz, hipMemcpyHostToDevice, G.st));
    HIPCHK(hipMemsetAsync(G.d_ratio, 0, 16, G.st));
    const double bound = absErrBound;
    const double tle = is_double ? bound : (double)thr_le(bound);
    if (dc_launch_ratio(is_double, mode, G.d_a, n, bound_binary(bound), tle, G.d_ratio, (unsigned*)(G.d_ratio + 1),
                        (uint8_t*)G.d_b, G.st))
        return seterr(DC_ERR_HIP, "ratio launch failed");
    HIPCHK(hipMemcpyAsync(&G.h_scratch[10], G.d_ratio, 16, hipMemcpyDeviceToHost, G.st));
    HIPCHK(hipStreamSynchronize(G.st));
    const int neg1 = (int)(G.h_scratch[11] & 1u);
    if (mode >= 2 && neg1) {                 /* the -1 history sentinel: the reference loop, one lane */
        if (dc_launch_ratio_serial(is_double, mode, G.d_a, n, bound_binary(bound), tle, G.d_ratio, G.st))
            return seterr(DC_ERR_HIP, "ratio launch failed");
    } else if (mode == 4) {
        if (dc_launch_ratio_area((const uint8_t*)G.d_b, n, G.d_ratio, G.st)) return seterr(DC_ERR_HIP, "ratio launch failed");
    } else {
        *out = G.h_scratch[10];
        return DC_OK;
    }
    HIPCHK(hipMemcpyAsync(&G.h_scratch[10], G.d_ratio, 8, hipMemcpyDeviceToHost, G.st));
    HIPCHK(hipStreamSynchronize(G.st));
    *out = G.h_scratch[10];
    return DC_OK;
}

/* calCompressRatio_bitwise_* (:3622-3739): int bits_after_compress (wraps as the reference's int) over
 * sizeof(T)*8*num */
static float ratio_bitwise(int is_double, int mode, const void* x, int num, const char* fn, size_t wbytes) {
    unsigned long long b = 0;
    const int rc = ratio_run(is_double, mode, x, num, &b);
    if (rc) { abi_fail(fn, rc); return 0.0f; }
    const int bits = (int)(uint32_t)b;
    return (float)bits / (wbytes * 8 * (size_t)num);
}
float calCompressRatio_bitwise_float(float data[], int num) {
    return ratio_bitwise(0, 0, data, num, "calCompressRatio_bitwise_float", sizeof(float));
}
float calCompressRatio_bitwise_double(double data[], int num) {
    return ratio_bitwise(1, 0, data, num, "calCompressRatio_bitwise_double", sizeof(double));
}
float calCompressRatio_bitwise_double2(float data[], int num) {
    return ratio_bitwise(0, 1, data, num, "calCompressRatio_bitwise_double2", sizeof(double));
}

/* sz / nolossy: long compressed_bits / long origin_bits (:4636-5219) */
static float ratio_bits(int is_double, int mode, const void* x, int num, const char* fn) {
    unsigned long long b = 0;
    const int rc = ratio_run(is_double, mode, x, num, &b);
    if (rc) { abi_fail(fn, rc); return 0.0f; }
    const long origin = (long)num * (long)(is_double ? 64 : 32);
    const long cb = mode == 4 ? (long)b * 512 : (long)b;
    return (float)cb / origin;
}
float calcCompressionRatio_sz_float(float data[], int num) { return ratio_bits(0, 2, data, num, "calcCompressionRatio_sz_float"); }
float calcCompressionRatio_sz_double(double data[], int num) { return ratio_bits(1, 2, data, num, "calcCompressionRatio_sz_double"); }
float calcCompressionRatio_nolossy_performance_float(float data[], int num) {
    return ratio_bits(0, 3, data, num, "calcCompressionRatio_nolossy_performance_float");
}
float calcCompressionRatio_nolossy_performance_double(double data[], int num) {
    return ratio_bits(1, 3, data, num, "calcCompressionRatio_nolossy_performance_double");
}
float calcCompressionRatio_nolossy_area_float(float data[], int num) {
    return ratio_bits(0, 4, data, num, "calcCompressionRatio_nolossy_area_float");
}
float calcCompressionRatio_nolossy_area_double(double data[], int num) {
    return ratio_bits(1, 4, data, num, "calcCompressionRatio_nolossy_area_double");
}

/* the Himeno variants (:4121-4635) walk plane ijk = v of p[MIMAX][MJMAX][MKMAX] in
 * transform_3d_array_to_1d_array order: the plane, then the flat estimator */
static float* himeno_plane(float data[MIMAX][MJMAX][MKMAX], int ijk, int v, int imax, int jmax, int kmax, int* n) {
    int A = 0, B = 0;
    if (plane_dims(ijk, imax, jmax, kmax, &A, &B)) return NULL;
    *n = A * B;
    return transform_3d_array_to_1d_array(data, ijk, v, imax, jmax, kmax);
}
float calcCompressionRatio_himeno_sz(float data[MIMAX][MJMAX][MKMAX], int ijk, int v, int imax, int jmax, int kmax) {
    int n = 0;
    float* p = himeno_plane(data, ijk, v, imax, jmax, kmax, &n);
    if (!p) { abi_fail("calcCompressionRatio_himeno_sz", DC_ERR_ARG); return 0.0f; }
    const float r = calcCompressionRatio_sz_float(p, n);
    free(p);
    return r;
}
float calcCompressionRatio_himeno_nolossy_performance(float data[MIMAX][MJMAX][MKMAX], int ijk, int v, int imax, int jmax,
                                                       int kmax) {
    int n = 0;
    float* p = himeno_plane(data, ijk, v, imax, jmax, kmax, &n);
    if (!p) { abi_fail("calcCompressionRatio_himeno_nolossy_performance", DC_ERR_ARG); return 0.0f; }
    const float r = calcCompressionRatio_nolossy_performance_float(p, n);
    free(p);
    return r;
}
float calcCompressionRatio_himeno_nolossy_area(float data[MIMAX][MJMAX][MKMAX], int ijk, int v, int imax, int jmax,
                                               int kmax) {
    int n = 0;
    float* p = himeno_plane(data, ijk, v, imax, jmax, kmax, &n);
    if (!p) { abi_fail("calcCompressionRatio_himeno_nolossy_area", DC_ERR_ARG); return 0.0f; }
    const float r = calcCompressionRatio_nolossy_area_float(p, n);
    free(p);
    return r;
}
/* :4121-4279: the CT1 byte-wise split of the plane (raw floats vs 2-bit codes) on the CT1 kernels */
float calcCompressionRatio_himeno_ij_ik_jk(float data[MIMAX][MJMAX][MKMAX], int ijk, int v, int imax, int jmax, int kmax) {
    const char* fn = "calcCompressionRatio_himeno_ij_ik_jk";
    int n = 0;
    float* p = himeno_plane(data, ijk, v, imax, jmax, kmax, &n);
    if (!p) { abi_fail(fn, DC_ERR_ARG); return 0.0f; }
    int rc = ensure_init();
    long long nraw = 0;
    if (!rc && n > 0) {
        if ((rc = grow(&G.c1_in, &G.c1_in_cap, (size_t)n * 4 + 64)) || (rc = grow(&G.c1_out, &G.c1_out_cap, (size_t)n * 4 + 64)) ||
            (rc = grow(&G.c1_codes, &G.c1_codes_cap, (size_t)n + 64)) ||
            (rc = grow(&G.c1_pos, &G.c1_pos_cap, (size_t)n * 4 + 64))) {
        } else if (hipMemcpyAsync(G.c1_in, p, (size_t)n * 4, hipMemcpyHostToDevice, G.st) != hipSuccess) {
            rc = seterr(DC_ERR_HIP, "H2D copy failed");
        } else {
            rc = dc_ct1_encode_device(G.c1_in, n, G.c1_out, G.c1_codes, G.c1_pos, &nraw);
        }
    }
    free(p);
    if (rc) { abi_fail(fn, rc); return 0.0f; }
    const long long nchar = n - nraw;
    return (float)((size_t)nchar * 2 + (size_t)nraw * sizeof(float) * 8) / ((size_t)(nchar + nraw) * sizeof(float) * 8);
}
