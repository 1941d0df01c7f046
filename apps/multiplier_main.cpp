// multiplier_rowwise | multiplier_colwise | multiplier_blockwise  <n_rows> <n_cols>
//
// Drop-in for the reference's three MPI executables (src/multiplier_{rowwise,colwise,
// blockwise}.c): same argv, same ./data/matrix_<R>_<C>.txt + ./data/vector_<C>.txt inputs,
// same stdout banner and messages, same ./data/out/<alg>.csv row "%ld, %ld, %d, %lf", same
// timing semantics (A and x preloaded on the root; each iteration = distribute + multiply +
// root holds y; mean over iterations). One host process drives G GPUs instead of
// `mpiexec -n P` launching P ranks: G = $MVG_NGPUS or every visible device, and the CSV's
// n_processes column reports G.
//
// Extensions (all opt-in, environment):
//   MVG_NGPUS=G        GPUs to use (default: all visible)
//   MVG_ITERS=n        timed iterations (default 100, as the reference's loop, rowwise.c:135)
//   MVG_SYNTH=1        skip the text files and generate the synthetic inputs (spec in
//                      include/matvec_gpu.h) on the host — the large configs have no files
//   MVG_Y_OUT=path     write y, "%.17g" per line (the reference never writes y)
//   MVG_DATA_DIR=dir   input directory (default ./data, matr_utils.c:45,68)
//   MVG_ITER_LOG=path  write every timed iteration's end-to-end time (s), one per line
// Besides the CSV it prints the device-resident time (GEMV + collective only, A resident).
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include "../include/matvec_gpu.h"

#ifndef MVG_APP_ALG
#define MVG_APP_ALG MVG_ALG_ROWWISE
#endif

static const char* kAlgName[] = {"rowwise", "colwise", "blockwise"};

static long env_long(const char* name, long dflt) {
    const char* v = getenv(name);
    return (v && *v) ? strtol(v, nullptr, 10) : dflt;
}

static int die(int rc, const char* where) {
    fprintf(stderr, "%s failed: %s (%s)\n", where, mvg_strerror(rc), mvg_last_error());
    return 1;
}

static double now_s() {
    using namespace std::chrono;
    return duration<double>(steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const int alg = MVG_APP_ALG;
    if (argc < 3) {  // the reference dereferences argv[1..2] unchecked (rowwise.c:58-59)
        fprintf(stderr, "usage: %s <n_rows> <n_cols>\n", argv[0]);
        return 1;
    }
    const long n_rows = strtol(argv[1], nullptr, 10);
    const long n_cols = strtol(argv[2], nullptr, 10);
    if (n_rows < 0 || n_cols < 0) {
        fprintf(stderr, "n_rows and n_cols must be >= 0\n");
        return 1;
    }
    // G replaces mpiexec's P: $MVG_NGPUS, else every visible device (only then is the GPU
    // runtime touched before the divisibility check, as MPI_Init precedes it in the reference)
    int comm_sz = (int)env_long("MVG_NGPUS", 0);
    int ndev = 0;
    if (comm_sz <= 0) {
        int rc0 = mvg_device_count(&ndev);
        if (rc0 != MVG_OK || ndev == 0) {
            fprintf(stderr, "no GPU visible: %s\n", mvg_last_error());
            return 1;
        }
        comm_sz = ndev;
    }
    int rc = MVG_OK;
    const long iters = std::max(1L, env_long("MVG_ITERS", 100));
    const char* data_dir = getenv("MVG_DATA_DIR") ? getenv("MVG_DATA_DIR") : "./data";

    // Divisibility check, printed exactly like the reference's root (rowwise.c:72-75,
    // colwise.c:151-154, blockwise.c:277-281), exit status 0 as there.
    mvg_shard sh;
    rc = mvg_plan_shard(alg, n_rows, n_cols, comm_sz, 0, &sh);
    if (rc == MVG_E_INDIVISIBLE) {
        printf("\nERROR!!!\n%s\n", mvg_last_error());
        return 0;
    }
    if (rc != MVG_OK) return die(rc, "mvg_plan_shard");

    char csv[256];
    snprintf(csv, sizeof csv, "./data/out/%s.csv", kAlgName[alg]);
    {
        FILE* probe = fopen(csv, "r");
        if (!probe) {  // rowwise.c:80-88
            FILE* fp = fopen(csv, "w");
            if (!fp) {
                printf("Unable to create output file.\n");
                return 0;
            }
            fprintf(fp, "n_rows, n_cols, n_processes, time\n");
            fclose(fp);
        } else {
            fclose(probe);
        }
    }

    // banner (rowwise.c:100-104; blockwise.c:314-321)
    printf("n_rows = %ld\n", n_rows);
    printf("n_cols = %ld\n", n_cols);
    if (alg == MVG_ALG_BLOCKWISE) {
        printf("comm_sz = %d\n", comm_sz);
        printf("my_rank = %d\n", 0);
        printf("comm_sz_rows = %d\n", sh.grid_rows);
        printf("comm_sz_cols = %d\n", sh.grid_cols);
        printf("local_n_rows = %ld\n", (long)sh.n_rows);
        printf("local_n_cols = %ld\n", (long)sh.n_cols);
    } else {
        printf("local_n = %ld\n", (long)(alg == MVG_ALG_ROWWISE ? sh.n_rows : sh.n_cols));
        printf("comm_sz = %d\n", comm_sz);
        printf("my_rank = %d\n", 0);
    }
    fflush(stdout);

    const size_t nA = (size_t)n_rows * (size_t)n_cols;
    std::vector<double> A(std::max<size_t>(nA, 1)), x(std::max<long>(n_cols, 1)), y(std::max<long>(n_rows, 1));
    char name[128];
    if (env_long("MVG_SYNTH", 0)) {
        printf("Generating synthetic matrix %ld x %ld (seed %u) and vector (seed %u)...\n", n_rows, n_cols,
               MVG_SEED_A, MVG_SEED_X);
        if ((rc = mvg_synth_fill_host(A.data(), n_cols, n_rows, n_cols, 0, 0, n_cols, MVG_SEED_A)) != MVG_OK)
            return die(rc, "mvg_synth_fill_host");
        if ((rc = mvg_synth_fill_host(x.data(), n_cols, 1, n_cols, 0, 0, n_cols, MVG_SEED_X)) != MVG_OK)
            return die(rc, "mvg_synth_fill_host");
    } else {
        mvg_matrix_filename(n_rows, n_cols, name, sizeof name);
        printf("Reading matrix from file '%s/%s'...\n", data_dir, name);  // matr_utils.c:48
        fflush(stdout);
        if (mvg_load_matr(data_dir, n_rows, n_cols, A.data()) != MVG_OK) {
            printf("Unable to locate matrix file '%s'\n", name);  // rowwise.c:111-117
            return 0;
        }
        mvg_vector_filename(n_cols, name, sizeof name);
        printf("Reading vector from file '%s/%s'...\n", data_dir, name);
        fflush(stdout);
        if (mvg_load_vec(data_dir, n_cols, x.data()) != MVG_OK) {
            printf("Unable to locate vector file '%s'\n", name);
            return 0;
        }
    }
    if ((rc = mvg_device_count(&ndev)) != MVG_OK || comm_sz > ndev) {
        fprintf(stderr, "%d GPU(s) requested, %d visible: %s\n", comm_sz, ndev, mvg_last_error());
        return 1;
    }
    // pinned host memory: distribution runs at full PCIe rate on every GPU's own link
    const bool pinned = nA > 0 && mvg_host_register(A.data(), nA * sizeof(double)) == MVG_OK;
    // x and y too: a pageable 600-element y cost 22 us per collect against 13 us page-locked
    // (tools/e2e_small.py)
    const bool pinned_x = mvg_host_register(x.data(), x.size() * sizeof(double)) == MVG_OK;
    const bool pinned_y = mvg_host_register(y.data(), y.size() * sizeof(double)) == MVG_OK;

    std::vector<int> devs(comm_sz);
    for (int i = 0; i < comm_sz; ++i) devs[i] = i;
    mvg_comm* comm = nullptr;
    if ((rc = mvg_comm_init_all(&comm, comm_sz, devs.data())) != MVG_OK) return die(rc, "mvg_comm_init_all");
    mvg_engine* eng = nullptr;
    if ((rc = mvg_engine_create(&eng, alg, n_rows, n_cols, comm)) != MVG_OK) return die(rc, "mvg_engine_create");

    // the reference's timed loop (rowwise.c:135-151): distribution included, root holds y
    double sum_time = 0.0;
    std::vector<double> it_times;
    it_times.reserve((size_t)iters);
    for (long it = 0; it < iters; ++it) {
        if ((rc = mvg_engine_sync(eng)) != MVG_OK) return die(rc, "sync");
        const double t0 = now_s();
        if ((rc = mvg_engine_distribute(eng, A.data(), x.data())) != MVG_OK) return die(rc, "distribute");
        if ((rc = mvg_engine_multiply(eng)) != MVG_OK) return die(rc, "multiply");
        if ((rc = mvg_engine_collect(eng, y.data())) != MVG_OK) return die(rc, "collect");
        if ((rc = mvg_engine_sync(eng)) != MVG_OK) return die(rc, "sync");  // MPI_Barrier
        it_times.push_back(now_s() - t0);
        sum_time += it_times.back();
    }
    // device-resident: A already on the GPUs; GEMV + exchange only
    mvg_engine_kernel_timing(eng, 5);  // events on every 5th multiply (each pair costs ~6 us)
    const double t0 = now_s();
    for (long it = 0; it < iters; ++it)
        if ((rc = mvg_engine_multiply(eng)) != MVG_OK) return die(rc, "multiply");
    if ((rc = mvg_engine_sync(eng)) != MVG_OK) return die(rc, "sync");
    const double dev_s = (now_s() - t0) / (double)iters;
    double kms = 0.0;
    int64_t nk = 0;
    mvg_engine_kernel_ms(eng, &kms, &nk);
    const double bytes = 8.0 * ((double)nA + (double)n_cols * (alg == MVG_ALG_ROWWISE ? comm_sz : 1) + (double)n_rows);
    printf("end-to-end (distribute + multiply + y on root): mean %.6f s over %ld iterations\n", sum_time / iters, iters);
    printf("device-resident: %.4f ms per multiply, %.1f GB/s aggregate; GEMV kernel %.3f ms (max over GPUs)\n",
           dev_s * 1e3, bytes / dev_s / 1e9, kms);

    if (const char* tl = getenv("MVG_ITER_LOG")) {  // per-iteration end-to-end times, seconds
        if (FILE* f = fopen(tl, "w")) {
            for (double t : it_times) fprintf(f, "%.9f\n", t);
            fclose(f);
        }
    }
    if (const char* yo = getenv("MVG_Y_OUT")) {
        if ((rc = mvg_write_vec(yo, y.data(), n_rows)) != MVG_OK) return die(rc, "mvg_write_vec");
    }
    mvg_engine_destroy(eng);
    mvg_comm_destroy(comm);
    if (pinned) mvg_host_unregister(A.data());
    if (pinned_x) mvg_host_unregister(x.data());
    if (pinned_y) mvg_host_unregister(y.data());

    FILE* fp = fopen(csv, "a");  // rowwise.c:160-169
    if (!fp) {
        printf("Unable to open output file.\n");
        return 0;
    }
    fprintf(fp, "%ld, %ld, %d, %lf\n", n_rows, n_cols, comm_sz, sum_time / iters);
    fclose(fp);
    return 0;
}
