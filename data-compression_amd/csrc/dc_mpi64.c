/*
 * dc_mpi64.c -- the reference's DOUBLE MPI wrappers over libdcamd (impl/dataCompression.c:24-353,
 * :800-1197; declared in impl/dataCompression.h:43-61), built with mpicc into lib/libdcamd_mpi.so.
 * The codec work (toSmallDataset_double, med_dataset_double, the bit-wise double codecs, CRC-32,
 * Hamming) runs on the GPU behind the reference C ABI; MPI moves host bytes as in the reference.
 *
 *  MPI_Send/Recv_bitwise_double{,_np,_op}: one MPI_CHAR message [int bytes][double min][stream]; the
 *    receiver decodes count doubles and adds min back (:226-353).  As in dc_mpi.c the receiver stages
 *    the message in its own buffer (the reference receives count*8+12 bytes into buf).
 *  MPI_Send/Recv_bitwise_double{,_np,_op}_cn: the first len doubles compressed, the rest sent raw
 *    (:24-164).
 *  MPI_Bcast_bitwise_crc / _mask_crc / _crc_hamming (:800-1197): root compresses (CT5 / CT7 with the
 *    mean's mask / CT5), broadcasts bytes, min (CT7: mean, type), stream and CRC-32 (CT10: Hamming check
 *    strings per block_size() block); receivers check the CRC -- the reference simulates a failure with
 *    probability bits*BER (CT8/9) or flips floor(bits*BER) random bits and tries Hamming correction
 *    (CT10) -- the root resends to every receiver that reports 'n'; the root accumulates
 *    mean |decoded + min - x| into *gosa, receivers overwrite buffer.  BER is the reference header's
 *    macro (1e-6); DC_BER in the environment overrides it.
 */
#include <math.h>
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/dataCompression.h"
#include "../../include/dc_gpu.h"
#include "../../include/dc_mpi.h"

enum { HDR64 = (int)(sizeof(int) + sizeof(double)) };

static double ber(void) {
    const char* e = getenv("DC_BER");
    return (e && *e) ? atof(e) : 1e-6;                    /* impl/dataCompression.h:4 */
}

static int compress_ct(int ct, const double* x, int n, unsigned char** bits, int* bytes, double* mn) {
    const char* inj = getenv("DC_TEST_FAIL_COMPRESS");   /* test hook: the root's compress fails */
    if (inj && *inj == '1') return -1;
    double* small = NULL;
    *mn = toSmallDataset_double((double*)x, &small, n);
    if (!small) return -1;
    int pos = 8;
    if (ct == 5) myCompress_bitwise_double(small, n, bits, bytes, &pos);
    else if (ct == 6) myCompress_bitwise_double_np(small, n, bits, bytes, &pos);
    else myCompress_bitwise_double_op(small, n, bits, bytes, &pos);
    free(small);
    return ((n > 0 && !*bits) || dc_abi_status() != DC_OK) ? -1 : 0;
}

static double* decompress_ct(int ct, unsigned char* bits, int bytes, int n) {
    if (ct == 5) return myDecompress_bitwise_double(bits, bytes, n);
    if (ct == 6) return myDecompress_bitwise_double_np(bits, bytes, n);
    return myDecompress_bitwise_double_op(bits, bytes, n);
}

static int send64(int ct, const double* buf, int len, int dest, int tag, MPI_Comm comm) {
    unsigned char* bits = NULL;
    int bytes = 0;
    double mn = 0;
    if (compress_ct(ct, buf, len, &bits, &bytes, &mn)) return MPI_ERR_OTHER;
    unsigned char* msg = (unsigned char*)malloc((size_t)HDR64 + (size_t)bytes);
    if (!msg) { free(bits); return MPI_ERR_OTHER; }
    memcpy(msg, &bytes, sizeof(int));
    memcpy(msg + sizeof(int), &mn, sizeof(double));
    if (bytes) memcpy(msg + HDR64, bits, (size_t)bytes);
    free(bits);
    const int ret = MPI_Send(msg, HDR64 + bytes, MPI_CHAR, dest, tag, comm);
    free(msg);
    return ret;
}

static int recv64(int ct, double* buf, int len, int source, int tag, MPI_Comm comm, MPI_Status* status) {
    MPI_Status st;
    MPI_Status* sp = status == MPI_STATUS_IGNORE ? &st : status;
    int ret = MPI_Probe(source, tag, comm, sp);
    if (ret != MPI_SUCCESS) return ret;
    int mlen = 0;
    MPI_Get_count(sp, MPI_CHAR, &mlen);
    unsigned char* msg = (unsigned char*)malloc(mlen > 0 ? (size_t)mlen : 1);
    if (!msg) return MPI_ERR_OTHER;
    ret = MPI_Recv(msg, mlen, MPI_CHAR, sp->MPI_SOURCE, sp->MPI_TAG, comm, sp);
    if (ret != MPI_SUCCESS) { free(msg); return ret; }
    int bytes = 0;
    double mn = 0;
    if (mlen < HDR64) { free(msg); return MPI_ERR_TRUNCATE; }
    memcpy(&bytes, msg, sizeof(int));
    memcpy(&mn, msg + sizeof(int), sizeof(double));
    if (bytes < 0 || HDR64 + bytes > mlen) { free(msg); return MPI_ERR_TRUNCATE; }
    double* dec = decompress_ct(ct, msg + HDR64, bytes, len);
    free(msg);
    if (!dec) return MPI_ERR_OTHER;
    if (dc_abi_status() != DC_OK) { free(dec); return MPI_ERR_OTHER; }
    for (int i = 0; i < len; i++) buf[i] = dec[i] + mn;   /* :245-248 */
    free(dec);
    return ret;
}

#define DC_PAIR64(SUF, CT)                                                                                  \
    int MPI_Send_bitwise_double##SUF(const void* buf, int count, MPI_Datatype datatype, int dest, int tag,     \
                                     MPI_Comm comm) {                                                      \
        (void)datatype;                                                                                    \
        return send64(CT, (const double*)buf, count, dest, tag, comm);                                     \
    }                                                                                                      \
    int MPI_Recv_bitwise_double##SUF(void* buf, int count, MPI_Datatype datatype, int source, int tag,         \
                                     MPI_Comm comm, MPI_Status* status) {                                  \
        (void)datatype;                                                                                    \
        return recv64(CT, (double*)buf, count, source, tag, comm, status);                                 \
    }                                                                                                      \
    int MPI_Send_bitwise_double##SUF##_cn(const void* buf, int count, MPI_Datatype datatype, int dest, int tag, \
                                          MPI_Comm comm, int len) {                                        \
        int ret = send64(CT, (const double*)buf, len, dest, tag, comm);                                    \
        if (ret == MPI_SUCCESS && count > len)                                                             \
            ret = MPI_Send((const double*)buf + len, count - len, datatype, dest, tag, comm);              \
        return ret;                                                                                        \
    }                                                                                                      \
    int MPI_Recv_bitwise_double##SUF##_cn(void* buf, int count, MPI_Datatype datatype, int source, int tag,    \
                                          MPI_Comm comm, MPI_Status* status, int len) {                    \
        int ret = recv64(CT, (double*)buf, len, source, tag, comm, status);                                \
        if (ret == MPI_SUCCESS && count > len)                                                             \
            ret = MPI_Recv((double*)buf + len, count - len, datatype, source, tag, comm, status);          \
        return ret;                                                                                        \
    }

DC_PAIR64(, 5)
DC_PAIR64(_np, 6)
DC_PAIR64(_op, 11)

/* MPI_Bcast_bitwise_double (:165-224): one broadcast of count*8+12 bytes, framing [int bytes][double min]
 * [stream] (the stream never exceeds count*8 bytes: a CT5 token is at most 64 bits) */
int MPI_Bcast_bitwise_double(void* buf, int count, MPI_Datatype datatype, int root, MPI_Comm comm) {
    (void)datatype;
    int myrank = 0;
    MPI_Comm_rank(comm, &myrank);
    const size_t tot = (size_t)HDR64 + (size_t)(count > 0 ? count : 0) * sizeof(double);
    unsigned char* aux = (unsigned char*)calloc(tot > 0 ? tot : 1, 1);
    if (!aux) return MPI_ERR_OTHER;
    int fail = 0;
    if (myrank == root) {
        unsigned char* bits = NULL;
        int bytes = 0;
        double mn = 0;
        fail = compress_ct(5, (const double*)buf, count, &bits, &bytes, &mn) || (size_t)HDR64 + (size_t)bytes > tot;
        if (!fail) {
            memcpy(aux, &bytes, sizeof(int));
            memcpy(aux + sizeof(int), &mn, sizeof(double));
            if (bytes) memcpy(aux + HDR64, bits, (size_t)bytes);
        } else {
            const int bad = -1;              /* tells every receiver the root failed: it never touches buf */
            memcpy(aux, &bad, sizeof(int));
        }
        free(bits);
    }
    int ret = MPI_Bcast(aux, (int)tot, MPI_UNSIGNED_CHAR, root, comm);
    if (ret == MPI_SUCCESS && myrank != root) {
        int bytes = 0;
        double mn = 0;
        memcpy(&bytes, aux, sizeof(int));
        memcpy(&mn, aux + sizeof(int), sizeof(double));
        double* dec = (bytes >= 0 && (size_t)HDR64 + (size_t)bytes <= tot) ? decompress_ct(5, aux + HDR64, bytes, count) : NULL;
        if (!dec || dc_abi_status() != DC_OK) ret = MPI_ERR_OTHER;
        else for (int i = 0; i < count; i++) ((double*)buf)[i] = dec[i] + mn;   /* :213-216 */
        free(dec);
    }
    free(aux);
    return fail ? MPI_ERR_OTHER : ret;
}

/* ---- broadcasts with CRC-32 / Hamming (:800-1197) */
enum { BC_CRC = 0, BC_MASK = 1, BC_HAM = 2 };

static void bcast64(int mode, double* buffer, int count, int root, int rank, int procs, float* compress_ratio,
                    double* gosa, int* resend) {
    uint32_t crc = 0, crc_check = 0;
    unsigned char crc_ok = 'y';
    unsigned char* oks = NULL;
    int bytes = 0, type = 0;
    double mn = 0, medium = 0;
    unsigned char* bits = NULL;
    srand((unsigned)time(NULL));                                          /* :807 */
    if (rank == root) {
        double* small = NULL;
        mn = toSmallDataset_double(buffer, &small, count);
        int pos = 8;
        if (mode == BC_MASK) {                                            /* :985-994 */
            medium = med_dataset_double(small, count, &type);
            char arr[65];
            doubletostr(&medium, arr);
            myCompress_bitwise_double_mask(small, count, &bits, &bytes, &pos, type, arr);
        } else {
            myCompress_bitwise_double(small, count, &bits, &bytes, &pos);
        }
        free(small);
        crc = do_crc32(bits, bytes);
    }
    MPI_Bcast(&bytes, 1, MPI_INT, root, MPI_COMM_WORLD);
    MPI_Bcast(&mn, 1, MPI_DOUBLE, root, MPI_COMM_WORLD);
    *compress_ratio += bytes * 8.0 / (count * sizeof(double) * 8);
    /* CT10: Hamming check strings per block (:826-851) */
    int bs = 1, nblk = 0, last = 0;
    int* r = NULL;
    char** c = NULL;
    if (mode == BC_HAM) {
        bs = block_size(bytes);
        if (bs <= 0) bs = 1;
        nblk = bytes / bs;
        last = bytes % bs;
        if (last > 0) nblk++;
        r = (int*)calloc((size_t)(nblk > 0 ? nblk : 1), sizeof(int));
        c = (char**)calloc((size_t)(nblk > 0 ? nblk : 1), sizeof(char*));
        if (rank == root)
            for (int i = 0; i < nblk; i++)
                hamming_encode(&bits[(size_t)i * bs], &c[i], (last > 0 && i == nblk - 1) ? last : bs, &r[i]);
    }
    if (rank != root) bits = (unsigned char*)malloc(bytes > 0 ? (size_t)bytes : 1);
    MPI_Bcast(bits, bytes, MPI_UNSIGNED_CHAR, root, MPI_COMM_WORLD);
    if (mode == BC_MASK) {
        MPI_Bcast(&medium, 1, MPI_DOUBLE, root, MPI_COMM_WORLD);
        MPI_Bcast(&type, 1, MPI_INT, root, MPI_COMM_WORLD);
    }
    MPI_Bcast(&crc, 1, MPI_UNSIGNED, root, MPI_COMM_WORLD);
    if (mode == BC_HAM) {
        MPI_Bcast(r, nblk, MPI_INT, root, MPI_COMM_WORLD);
        for (int i = 0; i < nblk; i++) {
            if (rank != root) c[i] = (char*)malloc((size_t)r[i] + 1);
            MPI_Bcast(c[i], r[i] + 1, MPI_CHAR, root, MPI_COMM_WORLD);
        }
    }
    if (rank != root) {
        const double b = ber();
        if (mode == BC_HAM) {                                             /* :872-934 */
            if (b > 0) {
                const uint64_t to = (uint64_t)(1 / b);
                const int errors = (int)((uint64_t)bytes * 8 / to);
                for (int k = 0; k < errors; k++) bit_flip(bits, bytes);
            }
            crc_check = do_crc32(bits, bytes);
            crc_ok = 'y';
            if (crc != crc_check)
                for (int i = 0; i < nblk; i++)
                    if (hamming_decode(&bits[(size_t)i * bs], c[i], (last > 0 && i == nblk - 1) ? last : bs, r[i]) == 1) {
                        crc_ok = 'n';
                        break;
                    }
        } else {                                                          /* :1040-1066 */
            crc_check = do_crc32(bits, bytes);
            if (b > 0) {
                const uint64_t to = (uint64_t)(1 / b);
                if (get_random_int(0, to) < (uint64_t)bytes * 8) crc_check = 0;
            }
            crc_ok = crc == crc_check ? 'y' : 'n';
        }
    } else {
        oks = (unsigned char*)malloc((size_t)procs);
    }
    MPI_Gather(&crc_ok, 1, MPI_UNSIGNED_CHAR, oks, 1, MPI_UNSIGNED_CHAR, root, MPI_COMM_WORLD);
    if (rank == root) {
        for (int i = 0; i < procs; i++)
            if (i != root && oks[i] == 'n') {
                MPI_Send(bits, bytes, MPI_UNSIGNED_CHAR, i, i, MPI_COMM_WORLD);
                (*resend)++;
            }
        free(oks);
    } else if (crc_ok == 'n') {
        MPI_Recv(bits, bytes, MPI_UNSIGNED_CHAR, root, rank, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
    }
    double* dec;
    if (mode == BC_MASK) {
        char arr[65];
        doubletostr(&medium, arr);
        dec = myDecompress_bitwise_double_mask(bits, bytes, count, type, arr);
    } else {
        dec = myDecompress_bitwise_double(bits, bytes, count);
    }
    double gs = 0;
    for (int i = 0; i < count; i++) {
        if (rank == root) gs += fabs(dec[i] + mn - buffer[i]);
        else buffer[i] = dec[i] + mn;
    }
    *gosa += gs / count;
    free(dec);
    free(bits);
    if (c) { for (int i = 0; i < nblk; i++) free(c[i]); free(c); }
    free(r);
}

void MPI_Bcast_bitwise_crc(double* buffer, int count, int root, int rank, int procs, float* compress_ratio, double* gosa,
                           int* resend) {
    bcast64(BC_CRC, buffer, count, root, rank, procs, compress_ratio, gosa, resend);
}
void MPI_Bcast_bitwise_mask_crc(double* buffer, int count, int root, int rank, int procs, float* compress_ratio,
                                double* gosa, int* resend) {
    bcast64(BC_MASK, buffer, count, root, rank, procs, compress_ratio, gosa, resend);
}
void MPI_Bcast_bitwise_crc_hamming(double* buffer, int count, int root, int rank, int procs, float* compress_ratio,
                                   double* gosa, int* resend) {
    bcast64(BC_HAM, buffer, count, root, rank, procs, compress_ratio, gosa, resend);
}
