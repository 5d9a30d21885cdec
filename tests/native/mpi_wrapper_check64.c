/* mpirun -np 2 mpi_wrapper_check64 [n]: the double MPI wrappers of libdcamd_mpi (dc_mpi64.c).
 *  - MPI_Send/Recv_bitwise_double{,_np,_op} and their _cn variants (the first n/2 doubles compressed):
 *    rank 0 sends a U10 buffer, rank 1 compares what arrives bit for bit with the same round trip done
 *    locally through the reference C ABI (toSmallDataset_double, compress, decompress, + min);
 *  - MPI_Bcast_bitwise_crc / _mask_crc / _crc_hamming from root 0: rank 1's buffer must equal the local
 *    round trip (CT5, CT7 with the mean's mask, CT5), with whatever BER DC_BER sets (a damaged copy is
 *    resent or Hamming-corrected, so the result does not change).
 * Test program of tests/test_mpi_wrappers.py. */
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "dataCompression.h"
#include "dc_mpi.h"

static void gen_u10(double* x, int n) {                 /* the U10 generator, 53-bit variant */
    for (int i = 0; i < n; i++) {
        uint64_t z = 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1) + 42ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        x[i] = (double)(z >> 11) * 0x1p-53 * 10.0;
    }
}

static double* local_round_trip(int ct, const double* x, int n) {
    double* small = NULL;
    double mn = toSmallDataset_double((double*)x, &small, n);
    unsigned char* bits = NULL;
    int bytes = 0, pos = 8, type = 0;
    double* dec;
    if (ct == 7) {
        double mean = med_dataset_double(small, n, &type);
        char b[65];
        doubletostr(&mean, b);
        myCompress_bitwise_double_mask(small, n, &bits, &bytes, &pos, type, b);
        dec = myDecompress_bitwise_double_mask(bits, bytes, n, type, b);
    } else if (ct == 5) {
        myCompress_bitwise_double(small, n, &bits, &bytes, &pos);
        dec = myDecompress_bitwise_double(bits, bytes, n);
    } else if (ct == 6) {
        myCompress_bitwise_double_np(small, n, &bits, &bytes, &pos);
        dec = myDecompress_bitwise_double_np(bits, bytes, n);
    } else {
        myCompress_bitwise_double_op(small, n, &bits, &bytes, &pos);
        dec = myDecompress_bitwise_double_op(bits, bytes, n);
    }
    for (int i = 0; i < n; i++) dec[i] += mn;
    free(small);
    free(bits);
    return dec;
}

static int report(const char* what, int ct, int n, const double* want, const double* got, int m) {
    const int bad = memcmp(want, got, sizeof(double) * (size_t)m) != 0;
    printf("MPI_WRAPPER64 %s ct=%d n=%d %s\n", what, ct, n, bad ? "FAIL" : "OK");
    return bad;
}

int main(int argc, char** argv) {
    MPI_Init(&argc, &argv);
    int rank = 0, size = 0;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &size);
    const int n = argc > 1 ? atoi(argv[1]) : 1 << 20;
    const int half = n / 2;
    double* x = (double*)malloc(sizeof(double) * (size_t)n);
    double* y = (double*)malloc(sizeof(double) * (size_t)n);
    gen_u10(x, n);
    int fails = 0;
    const int cts[3] = {5, 6, 11};
    for (int k = 0; k < 3; k++) {
        const int ct = cts[k];
        for (int cn = 0; cn < 2; cn++) {
            const int tag = ct * 2 + cn;
            if (rank == 0) {
                int rc;
                if (!cn) rc = ct == 5 ? MPI_Send_bitwise_double(x, n, MPI_DOUBLE, 1, tag, MPI_COMM_WORLD)
                            : ct == 6 ? MPI_Send_bitwise_double_np(x, n, MPI_DOUBLE, 1, tag, MPI_COMM_WORLD)
                                      : MPI_Send_bitwise_double_op(x, n, MPI_DOUBLE, 1, tag, MPI_COMM_WORLD);
                else rc = ct == 5 ? MPI_Send_bitwise_double_cn(x, n, MPI_DOUBLE, 1, tag, MPI_COMM_WORLD, half)
                        : ct == 6 ? MPI_Send_bitwise_double_np_cn(x, n, MPI_DOUBLE, 1, tag, MPI_COMM_WORLD, half)
                                  : MPI_Send_bitwise_double_op_cn(x, n, MPI_DOUBLE, 1, tag, MPI_COMM_WORLD, half);
                if (rc != MPI_SUCCESS) { printf("send ct=%d cn=%d rc=%d\n", ct, cn, rc); fails++; }
            } else if (rank == 1) {
                MPI_Status st;
                int rc;
                if (!cn) rc = ct == 5 ? MPI_Recv_bitwise_double(y, n, MPI_DOUBLE, 0, tag, MPI_COMM_WORLD, &st)
                            : ct == 6 ? MPI_Recv_bitwise_double_np(y, n, MPI_DOUBLE, 0, tag, MPI_COMM_WORLD, &st)
                                      : MPI_Recv_bitwise_double_op(y, n, MPI_DOUBLE, 0, tag, MPI_COMM_WORLD, &st);
                else rc = ct == 5 ? MPI_Recv_bitwise_double_cn(y, n, MPI_DOUBLE, 0, tag, MPI_COMM_WORLD, &st, half)
                        : ct == 6 ? MPI_Recv_bitwise_double_np_cn(y, n, MPI_DOUBLE, 0, tag, MPI_COMM_WORLD, &st, half)
                                  : MPI_Recv_bitwise_double_op_cn(y, n, MPI_DOUBLE, 0, tag, MPI_COMM_WORLD, &st, half);
                const int m = cn ? half : n;
                double* want = local_round_trip(ct, x, m);
                int bad = rc != MPI_SUCCESS;
                if (cn) bad |= memcmp(x + half, y + half, sizeof(double) * (size_t)(n - half)) != 0;   /* raw tail */
                bad |= report(cn ? "sendrecv_cn" : "sendrecv", ct, n, want, y, m);
                fails += bad;
                free(want);
            }
        }
    }
    /* MPI_Bcast_bitwise_double (:165-224): CT5 from root 0 */
    memcpy(y, x, sizeof(double) * (size_t)n);
    if (rank != 0) memset(y, 0, sizeof(double) * (size_t)n);
    {
        const int rc = MPI_Bcast_bitwise_double(y, n, MPI_DOUBLE, 0, MPI_COMM_WORLD);
        if (rank == 1) {
            double* want = local_round_trip(5, x, n);
            fails += (rc != MPI_SUCCESS) | report("bcast_double", 5, n, want, y, n);
            free(want);
        } else if (rank == 0 && (rc != MPI_SUCCESS || memcmp(x, y, sizeof(double) * (size_t)n) != 0)) {
            printf("bcast_double root rc=%d (root buffer must stay unchanged)\n", rc);
            fails++;
        }
    }
    /* a root whose compress fails: every rank returns an error and no receiver touches its buffer */
    memset(y, 0, sizeof(double) * (size_t)n);
    if (rank == 0) { memcpy(y, x, sizeof(double) * (size_t)n); setenv("DC_TEST_FAIL_COMPRESS", "1", 1); }
    {
        const int rc = MPI_Bcast_bitwise_double(y, n, MPI_DOUBLE, 0, MPI_COMM_WORLD);
        if (rank == 0) unsetenv("DC_TEST_FAIL_COMPRESS");
        int touched = 0;
        if (rank != 0) for (int i = 0; i < n; i++) touched |= y[i] != 0.0;
        if (rc == MPI_SUCCESS || touched) {
            printf("bcast_double root failure: rank %d rc=%d touched=%d (want an error, buffer untouched)\n", rank, rc, touched);
            fails++;
        }
    }
    /* broadcasts: CT8 (crc), CT9 (mask_crc), CT10 (crc_hamming) */
    for (int mode = 8; mode <= 10; mode++) {
        memcpy(y, x, sizeof(double) * (size_t)n);
        float ratio = 0.0f;
        double gosa = 0.0;
        int resend = 0;
        if (rank != 0) memset(y, 0, sizeof(double) * (size_t)n);
        if (mode == 8) MPI_Bcast_bitwise_crc(y, n, 0, rank, size, &ratio, &gosa, &resend);
        else if (mode == 9) MPI_Bcast_bitwise_mask_crc(y, n, 0, rank, size, &ratio, &gosa, &resend);
        else MPI_Bcast_bitwise_crc_hamming(y, n, 0, rank, size, &ratio, &gosa, &resend);
        if (rank == 1) {
            double* want = local_round_trip(mode == 9 ? 7 : 5, x, n);
            fails += report(mode == 8 ? "bcast_crc" : mode == 9 ? "bcast_mask_crc" : "bcast_crc_hamming", mode, n, want, y, n);
            free(want);
        } else if (rank == 0) {
            printf("MPI_WRAPPER64 root mode=%d ratio=%f gosa=%g resend=%d\n", mode, 1.0 / ratio, gosa, resend);
        }
    }
    free(x);
    free(y);
    MPI_Finalize();
    return fails ? 1 : 0;
}
