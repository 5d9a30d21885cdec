/*
 * dc_mpi.h -- float MPI send/recv wrappers of libdcamd_mpi.so (data-compression_amd/csrc/dc_mpi.c).
 *
 * Float counterparts of the reference's MPI_Send_bitwise_double / MPI_Recv_bitwise_double
 * (impl/dataCompression.h:57-62, impl/dataCompression.c:226-353): same argument list, one MPI_CHAR
 * message framed [int bytes][float min][stream] (CT7: [int bytes][float min][int type][char mask[17]]
 * [stream]); the receiver decodes into buf and adds min back.  The codec runs on the MI355X.
 * Include after <mpi.h>.
 */
#ifndef DC_MPI_H
#define DC_MPI_H
#include <mpi.h>

#ifdef __cplusplus
extern "C" {
#endif

/* CT5: zero / 3-predictor / raw tokens (myCompress_bitwise) */
int MPI_Send_bitwise_float(const void* buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm);
int MPI_Recv_bitwise_float(void* buf, int count, MPI_Datatype datatype, int source, int tag, MPI_Comm comm,
                           MPI_Status* status);
/* CT6: raw tokens only (myCompress_bitwise_np) */
int MPI_Send_bitwise_float_np(const void* buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm);
int MPI_Recv_bitwise_float_np(void* buf, int count, MPI_Datatype datatype, int source, int tag, MPI_Comm comm,
                              MPI_Status* status);
/* CT11: 3-bit codes or verbatim floats (myCompress_bitwise_op) */
int MPI_Send_bitwise_float_op(const void* buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm);
int MPI_Recv_bitwise_float_op(void* buf, int count, MPI_Datatype datatype, int source, int tag, MPI_Comm comm,
                              MPI_Status* status);
/* CT7: bitmask tokens, type / mask from med_dataset_float of the shifted data (impl/pingpong.c:198-206) */
int MPI_Send_bitwise_float_mask(const void* buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm);
int MPI_Recv_bitwise_float_mask(void* buf, int count, MPI_Datatype datatype, int source, int tag, MPI_Comm comm,
                                MPI_Status* status);

/* ---- the reference's double wrappers (impl/dataCompression.h:43-61, dataCompression.c:24-353, :800-1197),
 * same signatures; framing [int bytes][double min][stream]; _cn: the first len doubles compressed, the rest raw
 * (csrc/dc_mpi64.c) */
int MPI_Send_bitwise_double(const void* buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm);
int MPI_Recv_bitwise_double(void* buf, int count, MPI_Datatype datatype, int source, int tag, MPI_Comm comm,
                            MPI_Status* status);
int MPI_Send_bitwise_double_np(const void* buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm);
int MPI_Recv_bitwise_double_np(void* buf, int count, MPI_Datatype datatype, int source, int tag, MPI_Comm comm,
                               MPI_Status* status);
int MPI_Send_bitwise_double_op(const void* buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm);
int MPI_Recv_bitwise_double_op(void* buf, int count, MPI_Datatype datatype, int source, int tag, MPI_Comm comm,
                               MPI_Status* status);
int MPI_Send_bitwise_double_cn(const void* buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
                               int len);
int MPI_Recv_bitwise_double_cn(void* buf, int count, MPI_Datatype datatype, int source, int tag, MPI_Comm comm,
                               MPI_Status* status, int len);
int MPI_Send_bitwise_double_np_cn(const void* buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
                                  int len);
int MPI_Recv_bitwise_double_np_cn(void* buf, int count, MPI_Datatype datatype, int source, int tag, MPI_Comm comm,
                                  MPI_Status* status, int len);
int MPI_Send_bitwise_double_op_cn(const void* buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
                                  int len);
int MPI_Recv_bitwise_double_op_cn(void* buf, int count, MPI_Datatype datatype, int source, int tag, MPI_Comm comm,
                                  MPI_Status* status, int len);
/* CT8 (CRC-32), CT9 (bitmask + CRC-32), CT10 (CRC-32 + Hamming): broadcast from root, resend on failure */
/* h:50 c:165-224: root compresses (CT5), every rank receives [int bytes][double min][stream] padded to
 * count*8+12 bytes by one MPI_Bcast, non-roots decode and add min back into buf */
int MPI_Bcast_bitwise_double(void* buf, int count, MPI_Datatype datatype, int root, MPI_Comm comm);
void MPI_Bcast_bitwise_crc(double* buffer, int count, int root, int rank, int procs, float* compress_ratio,
                           double* gosa, int* resend);
void MPI_Bcast_bitwise_mask_crc(double* buffer, int count, int root, int rank, int procs, float* compress_ratio,
                                double* gosa, int* resend);
void MPI_Bcast_bitwise_crc_hamming(double* buffer, int count, int root, int rank, int procs, float* compress_ratio,
                                   double* gosa, int* resend);

#ifdef __cplusplus
}
#endif
#endif
