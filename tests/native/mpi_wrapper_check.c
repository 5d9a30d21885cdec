/* mpirun -np 2 mpi_wrapper_check [n]: rank 0 sends one U10 buffer through each float wrapper of
 * libdcamd_mpi (CT5/6/11/7); rank 1 receives and compares bit for bit with the same round trip done
 * locally through the reference C ABI (toSmallDataset_float, compress, decompress, + min).  Test
 * program of tests/test_mpi_wrappers.py. */
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "dataCompression.h"
#include "dc_mpi.h"

static void gen_u10(float* x, int n) {                  /* SURVEY 8(d) U10, seed 42 */
    for (int i = 0; i < n; i++) {
        uint64_t z = 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1) + 42ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        x[i] = (float)(z >> 40) * (1.0f / 16777216.0f) * 10.0f;
    }
}

static float* local_round_trip(int ct, const float* x, int n) {
    float* small = NULL;
    float mn = toSmallDataset_float((float*)x, &small, n);
    unsigned char* bits = NULL;
    int bytes = 0, pos = 8, type = 0;
    char mask[17];
    float* dec;
    if (ct == 7) {
        float mean = med_dataset_float(small, n, &type);
        char b[33];
        floattostr(&mean, b);
        memcpy(mask, b, 17);
        myCompress_bitwise_mask(small, n, &bits, &bytes, &pos, type, mask);
        dec = myDecompress_bitwise_mask(bits, bytes, n, type, mask);
    } else if (ct == 5) {
        myCompress_bitwise(small, n, &bits, &bytes, &pos);
        dec = myDecompress_bitwise(bits, bytes, n);
    } else if (ct == 6) {
        myCompress_bitwise_np(small, n, &bits, &bytes, &pos);
        dec = myDecompress_bitwise_np(bits, bytes, n);
    } else {
        myCompress_bitwise_op(small, n, &bits, &bytes, &pos);
        dec = myDecompress_bitwise_op(bits, bytes, n);
    }
    for (int i = 0; i < n; i++) dec[i] += mn;
    free(small);
    free(bits);
    return dec;
}

int main(int argc, char** argv) {
    MPI_Init(&argc, &argv);
    int rank = 0, size = 0;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &size);
    const int n = argc > 1 ? atoi(argv[1]) : 1 << 20;
    float* x = (float*)malloc(sizeof(float) * (size_t)n);
    float* y = (float*)malloc(sizeof(float) * (size_t)n);
    gen_u10(x, n);
    const int cts[4] = {5, 6, 11, 7};
    int fails = 0;
    for (int k = 0; k < 4; k++) {
        const int ct = cts[k];
        if (rank == 0) {
            int rc = ct == 5 ? MPI_Send_bitwise_float(x, n, MPI_FLOAT, 1, ct, MPI_COMM_WORLD)
                   : ct == 6 ? MPI_Send_bitwise_float_np(x, n, MPI_FLOAT, 1, ct, MPI_COMM_WORLD)
                   : ct == 11 ? MPI_Send_bitwise_float_op(x, n, MPI_FLOAT, 1, ct, MPI_COMM_WORLD)
                              : MPI_Send_bitwise_float_mask(x, n, MPI_FLOAT, 1, ct, MPI_COMM_WORLD);
            if (rc != MPI_SUCCESS) { printf("send ct=%d rc=%d\n", ct, rc); fails++; }
        } else if (rank == 1) {
            MPI_Status st;
            int rc = ct == 5 ? MPI_Recv_bitwise_float(y, n, MPI_FLOAT, 0, ct, MPI_COMM_WORLD, &st)
                   : ct == 6 ? MPI_Recv_bitwise_float_np(y, n, MPI_FLOAT, 0, ct, MPI_COMM_WORLD, &st)
                   : ct == 11 ? MPI_Recv_bitwise_float_op(y, n, MPI_FLOAT, 0, ct, MPI_COMM_WORLD, &st)
                              : MPI_Recv_bitwise_float_mask(y, n, MPI_FLOAT, 0, ct, MPI_COMM_WORLD, &st);
            float* want = local_round_trip(ct, x, n);
            int bad = rc != MPI_SUCCESS || memcmp(want, y, sizeof(float) * (size_t)n) != 0;
            double maxerr = 0.0;
            for (int i = 0; i < n; i++) {
                double e = y[i] > x[i] ? y[i] - x[i] : x[i] - y[i];
                if (e > maxerr) maxerr = e;
            }
            printf("MPI_WRAPPER ct=%d n=%d %s maxerr=%g\n", ct, n, bad ? "MISMATCH" : "OK", maxerr);
            fails += bad;
            free(want);
        }
    }
    free(x);
    free(y);
    int all = 0;
    MPI_Allreduce(&fails, &all, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
    MPI_Finalize();
    return all ? 1 : 0;
}
