/* examples/rowwise_binding.c — the binding INTEGRATION.md §2 shows, as a compiled C99 program.
 *
 * It is the reference's multiplier_rowwise.c main loop (src/multiplier_rowwise.c:54-176) with
 * MPI replaced by libmatvec_gpu: same input files, same divisibility message, same 100-iteration
 * timed loop (distribution included), y printed with %.17g. Build: `make examples` (gcc, plain C:
 * proves include/matvec_gpu.h is a C header). Run from a directory holding ./data/.
 *   usage: rowwise_binding <n_rows> <n_cols> [n_gpus]
 */
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "../include/matvec_gpu.h"

static double wtime(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s <n_rows> <n_cols> [n_gpus]\n", argv[0]);
        return 1;
    }
    const long n_rows = strtol(argv[1], NULL, 10);
    const long n_cols = strtol(argv[2], NULL, 10);
    int ngpu = argc > 3 ? atoi(argv[3]) : 1;
    int devs[64];
    for (int i = 0; i < ngpu && i < 64; ++i) devs[i] = i;

    double* matrix = malloc(sizeof(double) * (size_t)n_rows * (size_t)n_cols);
    double* vector = malloc(sizeof(double) * (size_t)n_cols);
    double* result = malloc(sizeof(double) * (size_t)n_rows);
    if (mvg_load_matr("./data", n_rows, n_cols, matrix) != MVG_OK ||  /* load_matr, matr_utils.c:42 */
        mvg_load_vec("./data", n_cols, vector) != MVG_OK) {            /* load_vec,  matr_utils.c:65 */
        printf("Unable to load inputs: %s\n", mvg_last_error());
        return 0;
    }

    mvg_comm* comm;
    mvg_engine* eng;
    int rc = mvg_comm_init_all(&comm, ngpu, devs);                      /* MPI_Init / Comm_size */
    if (rc != MVG_OK) {
        fprintf(stderr, "%s: %s\n", mvg_strerror(rc), mvg_last_error());
        return 1;
    }
    rc = mvg_engine_create(&eng, MVG_ALG_ROWWISE, n_rows, n_cols, comm);
    if (rc == MVG_E_INDIVISIBLE) {
        printf("\nERROR!!!\n%s\n", mvg_last_error());                  /* rowwise.c:72-75 */
        return 0;
    }
    if (rc != MVG_OK) {
        fprintf(stderr, "%s: %s\n", mvg_strerror(rc), mvg_last_error());
        return 1;
    }
    double sum_time = 0.0;
    for (int i = 0; i < 100; i++) {                                     /* rowwise.c:135 */
        const double start = wtime();
        if ((rc = mvg_engine_distribute(eng, matrix, vector)) != MVG_OK) break;  /* distribute_data :139 */
        if ((rc = mvg_engine_multiply(eng)) != MVG_OK) break;                   /* multiply_std_rowwise :140 */
        if ((rc = mvg_engine_collect(eng, result)) != MVG_OK) break;            /* MPI_Gather :141 */
        sum_time += wtime() - start;
    }
    if (rc != MVG_OK) {
        fprintf(stderr, "%s: %s\n", mvg_strerror(rc), mvg_last_error());
        return 1;
    }
    mvg_engine_destroy(eng);
    mvg_comm_destroy(comm);                                             /* MPI_Finalize */
    for (long i = 0; i < n_rows; ++i) printf("%.17g\n", result[i]);
    fprintf(stderr, "%ld, %ld, %d, %lf\n", n_rows, n_cols, ngpu, sum_time / 100);  /* the CSV row */
    free(matrix);
    free(vector);
    free(result);
    return 0;
}
