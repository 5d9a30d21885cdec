/*
 * dc_mpi.c -- float MPI send/recv wrappers over libdcamd (BASELINE north_star's
 * "MPI_COMPRESS send/recv wrapper").  Built with mpicc into lib/libdcamd_mpi.so (make mpi).
 *
 * The reference has this pair only for doubles (MPI_Send_bitwise_double / MPI_Recv_bitwise_double,
 * impl/dataCompression.c:226-353, used by impl/mycompress.c:44-50): toSmallDataset, compress, one
 * MPI_CHAR message framed [int bytes][min][stream]; the receiver decompresses and adds min back.  The
 * float apps inline the same sequence (impl/pingpong.c:128-209, impl/himenoBMTxps.c:644-706).  These
 * are the float versions with the same argument list and framing (float min), for CT5 (_bitwise),
 * CT6 (_np), CT11 (_op) and CT7 (_mask: [int bytes][float min][int type][char mask[17]][stream], type
 * and mask from med_dataset_float as pingpong does).  The codec work runs on the GPU behind the
 * reference C ABI; MPI moves host bytes exactly as in the reference.
 *
 * Differences from the double originals: the receiver stages the message in its own buffer instead
 * of receiving into `buf` (a stream larger than count floats cannot overflow it), and the sender frees
 * its temporaries.  Return value: the MPI_Send / MPI_Recv result, or MPI_ERR_OTHER when the codec
 * reports an error (dc_abi_status() after the ABI call; dc_last_error() explains).
 */
#include <mpi.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/dataCompression.h"
#include "../../include/dc_gpu.h"
#include "../../include/dc_mpi.h"

enum { HDR = (int)(sizeof(int) + sizeof(float)), MHDR = HDR + (int)sizeof(int) + 17 };

static int send_ct(int ct, const float* buf, int count, int dest, int tag, MPI_Comm comm) {
    float* small = NULL;
    const float mn = toSmallDataset_float((float*)buf, &small, count);
    if (!small) return MPI_ERR_OTHER;
    unsigned char* bits = NULL;
    int bytes = 0, pos = 8, type = 0;
    char mask[17];
    memset(mask, '0', sizeof mask);
    if (ct == 5) myCompress_bitwise(small, count, &bits, &bytes, &pos);
    else if (ct == 6) myCompress_bitwise_np(small, count, &bits, &bytes, &pos);
    else if (ct == 11) myCompress_bitwise_op(small, count, &bits, &bytes, &pos);
    else {                                                 /* ct 7, mask as impl/pingpong.c:198-206 */
        float mean = med_dataset_float(small, count, &type);
        char binary[33];
        floattostr(&mean, binary);
        memcpy(mask, binary, 17);
        myCompress_bitwise_mask(small, count, &bits, &bytes, &pos, type, mask);
    }
    free(small);
    if ((count > 0 && !bits) || dc_abi_status() != DC_OK) { free(bits); return MPI_ERR_OTHER; }
    const int hdr = ct == 7 ? MHDR : HDR;
    unsigned char* msg = (unsigned char*)malloc((size_t)hdr + (size_t)bytes);
    if (!msg) { free(bits); return MPI_ERR_OTHER; }
    memcpy(msg, &bytes, sizeof(int));
    memcpy(msg + sizeof(int), &mn, sizeof(float));
    if (ct == 7) {
        memcpy(msg + HDR, &type, sizeof(int));
        memcpy(msg + HDR + sizeof(int), mask, 17);
    }
    if (bytes) memcpy(msg + hdr, bits, (size_t)bytes);
    free(bits);
    const int ret = MPI_Send(msg, hdr + bytes, MPI_CHAR, dest, tag, comm);
    free(msg);
    return ret;
}

static int recv_ct(int ct, float* buf, int count, int source, int tag, MPI_Comm comm, MPI_Status* status) {
    MPI_Status st;
    MPI_Status* sp = status == MPI_STATUS_IGNORE ? &st : status;
    int ret = MPI_Probe(source, tag, comm, sp);
    if (ret != MPI_SUCCESS) return ret;
    int len = 0;
    MPI_Get_count(sp, MPI_CHAR, &len);
    unsigned char* msg = (unsigned char*)malloc(len > 0 ? (size_t)len : 1);
    if (!msg) return MPI_ERR_OTHER;
    ret = MPI_Recv(msg, len, MPI_CHAR, sp->MPI_SOURCE, sp->MPI_TAG, comm, sp);
    if (ret != MPI_SUCCESS) { free(msg); return ret; }
    const int hdr = ct == 7 ? MHDR : HDR;
    int bytes = 0, type = 0;
    float mn = 0.0f;
    char mask[17];
    if (len < hdr) { free(msg); return MPI_ERR_TRUNCATE; }
    memcpy(&bytes, msg, sizeof(int));
    memcpy(&mn, msg + sizeof(int), sizeof(float));
    if (ct == 7) {
        memcpy(&type, msg + HDR, sizeof(int));
        memcpy(mask, msg + HDR + sizeof(int), 17);
    }
    if (bytes < 0 || hdr + bytes > len) { free(msg); return MPI_ERR_TRUNCATE; }
    unsigned char* bits = msg + hdr;
    float* dec;
    if (ct == 5) dec = myDecompress_bitwise(bits, bytes, count);
    else if (ct == 6) dec = myDecompress_bitwise_np(bits, bytes, count);
    else if (ct == 11) dec = myDecompress_bitwise_op(bits, bytes, count);
    else dec = myDecompress_bitwise_mask(bits, bytes, count, type, mask);
    free(msg);
    if (!dec) return MPI_ERR_OTHER;
    if (dc_abi_status() != DC_OK) { free(dec); return MPI_ERR_OTHER; }
    for (int i = 0; i < count; i++) buf[i] = dec[i] + mn;   /* impl/dataCompression.c:245-248 (double) */
    free(dec);
    return ret;
}

#define DC_PAIR(SUF, CT)                                                                                 \
    int MPI_Send_bitwise_float##SUF(const void* buf, int count, MPI_Datatype datatype, int dest, int tag,   \
                                    MPI_Comm comm) {                                                    \
        (void)datatype;                                                                                 \
        return send_ct(CT, (const float*)buf, count, dest, tag, comm);                                  \
    }                                                                                                   \
    int MPI_Recv_bitwise_float##SUF(void* buf, int count, MPI_Datatype datatype, int source, int tag,       \
                                    MPI_Comm comm, MPI_Status* status) {                                \
        (void)datatype;                                                                                 \
        return recv_ct(CT, (float*)buf, count, source, tag, comm, status);                              \
    }

DC_PAIR(, 5)
DC_PAIR(_np, 6)
DC_PAIR(_op, 11)
DC_PAIR(_mask, 7)
