// multiplier_rowwise | multiplier_colwise | multiplier_blockwise  <n_rows> <n_cols>
//
// Drop-in for the reference's three MPI executables (src/multiplier_{rowwise,colwise,
// blockwise}.c): same argv, same ./data/matrix_<R>_<C>.txt + ./data/vector_<C>.txt inputs,
// same stdout banner and messages, same ./data/out/<alg>.csv row "%ld, %ld, %d, %lf", same
// timing semantics (A and x preloaded on the root; each iteration = Barrier, distribute +
// multiply + root holds y, Barrier; max over ranks; mean over iterations). Two launch modes:
//   mpiexec -n P bin/multiplier_<alg> R C   the reference's own launch line (test.sh:11): P
//       ranks, one GPU each (node-local rank -> device). Rank 0 loads A and x into an MPI-3
//       shared window every rank on the node maps, and each GPU pulls its own shard over its own
//       PCIe link (MVG_DIST=send: rank 0 alone reads A and ncclSends the shards over xGMI, the
//       reference's root-send pattern). MPI carries the bootstrap and timing only (apps/launch.h).
//   bin/multiplier_<alg> R C               one process drives G = $MVG_NGPUS GPUs (default all
//       visible); each GPU pulls its shard from the root's page-locked A concurrently.
// The CSV's n_processes column reports P (= G).
//
// Extensions (all opt-in, environment):
//   MVG_NGPUS=G        GPUs to use in the single-process mode (default: all visible)
//   MVG_DIST=send      rank mode: root-send distribution instead of the shared window
//   MVG_RANK_MODE=1    rank-mode code path even for P = 1 (tests; with MVG_MPI=1 no mpiexec)
//   MVG_SAME_DEVICE=1  rank mode with every rank on GPU 0 (tests on a one-GPU machine)
//   MVG_ITERS=n        timed iterations (default 100, as the reference's loop, rowwise.c:135)
//   MVG_SYNTH=1        skip the text files and generate the synthetic inputs (spec in
//                      include/matvec_gpu.h) on the host — the large configs have no files
//   MVG_SYNTH=device   generate each rank's shard of the same inputs on its GPU instead (no host
//                      A: config 4's 137 GB never exists on the host); nothing is distributed, so
//                      the timed loop is multiply + y on the root
//   MVG_Y_OUT=path     write y, "%.17g" per line (the reference never writes y)
//   MVG_EXACT=1        bit-exact mode (mvg_engine_set_exact): y, and so the MVG_Y_OUT file, is
//                      identical to the reference's (its sequential sums and combine orders)
//   MVG_OVERLAP=n      distribute A in n row chunks, each chunk's GEMV behind its copy
//   MVG_DATA_DIR=dir   input directory (default ./data, matr_utils.c:45,68)
//   MVG_ITER_LOG=path  write every timed iteration's end-to-end time (s), one per line
//   MVG_RUNTIME_ONLY=1 print the `runtime:` line (the RCCL and HIP runtime this executable binds,
//                      as after a device-resident run) and exit: no launcher, no device work
// Besides the CSV it prints the device-resident time (GEMV + collective only, A resident).
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <algorithm>
#include <memory>
#include <string>
#include <vector>

#include "../include/matvec_gpu.h"
#include "launch.h"

#ifndef MVG_APP_ALG
#define MVG_APP_ALG MVG_ALG_ROWWISE
#endif

static const char* kAlgName[] = {"rowwise", "colwise", "blockwise"};

static long env_long(const char* name, long dflt) {
    const char* v = getenv(name);
    return (v && *v) ? strtol(v, nullptr, 10) : dflt;
}


// every exit after launch_init goes through here (MPI_Finalize on all ranks)
static int finish(int code) {
    fflush(stdout);
    launch_finalize();
    return code;
}

static mvg_launch g_launch;

static int die(int rc, const char* where, int rank) {
    fprintf(stderr, "rank %d: %s failed: %s (%s)\n", rank, where, mvg_strerror(rc), mvg_last_error());
    fflush(stderr);
    return 1;
}

// a failure on one rank after the ranks started working together: the others may already wait
// in a collective, so the whole job is aborted (MPI_Abort); a single process just exits
static int fatal(int rc, const char* where) {
    die(rc, where, g_launch.rank);
    if (g_launch.size > 1) launch_abort(1);
    return finish(1);
}

int main(int argc, char** argv) {
    const int alg = MVG_APP_ALG;
    // one process per GPU: RCCL's intra-node IPC on this ROCm needs the dmabuf mode (the legacy
    // IPC handles fail with hipIpcGetMemHandle: invalid argument); before the HIP runtime starts
    setenv("HSA_ENABLE_IPC_MODE_LEGACY", "0", 0);
    if (const char* ro = getenv("MVG_RUNTIME_ONLY"); ro && ro[0] == '1') {
        // the RCCL and HIP runtime this executable binds, printed as the device-resident run's
        // `runtime:` line, and nothing else: no launcher, no device work
        int rccl_v = 0, hip_v = 0;
        const int rc = mvg_runtime_versions(&rccl_v, &hip_v);
        printf("runtime: RCCL %d (%s), HIP %d (%s)\n", rccl_v, mvg_runtime_path(1), hip_v, mvg_runtime_path(0));
        return rc == MVG_OK ? 0 : 1;
    }
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
    launch_init(&argc, &argv, &g_launch);
    const mvg_launch& L = g_launch;  // MPI_Init (rowwise.c:66), only under an MPI launcher
    const bool root = L.rank == 0;
    // rank mode: one GPU per MPI rank; P = the world size. Otherwise one process drives G GPUs:
    // $MVG_NGPUS, else every visible device (only then is the GPU runtime touched before the
    // divisibility check, as MPI_Init precedes it in the reference).
    const bool ranks = L.mpi && (L.size > 1 || env_long("MVG_RANK_MODE", 0) == 1);
    // MVG_SAME_DEVICE=1 (tests on a one-GPU machine): every rank uses GPU 0. RCCL refuses two
    // ranks on one device of one host, so each rank names its own host (NCCL_HOSTID) and the
    // ranks talk over loopback sockets — slow, but the multi-rank path runs end to end.
    const bool same_dev = ranks && env_long("MVG_SAME_DEVICE", 0) == 1;
    if (same_dev) {
        char hid[64];
        snprintf(hid, sizeof hid, "mvg-rank-%d", L.rank);
        setenv("NCCL_HOSTID", hid, 0);
        setenv("NCCL_SOCKET_IFNAME", "lo", 0);
        setenv("NCCL_IB_DISABLE", "1", 0);
    }
    const int my_device = same_dev ? 0 : L.local_rank;
    int comm_sz = L.mpi ? L.size : (int)env_long("MVG_NGPUS", 0);
    int ndev = 0;
    if (comm_sz <= 0) {
        int rc0 = mvg_device_count(&ndev);
        if (rc0 != MVG_OK || ndev == 0) {
            fprintf(stderr, "no GPU visible: %s\n", mvg_last_error());
            return finish(1);
        }
        comm_sz = ndev;
    }
    int rc = MVG_OK;
    const long iters = std::max(1L, env_long("MVG_ITERS", 100));
    const char* data_dir = getenv("MVG_DATA_DIR") ? getenv("MVG_DATA_DIR") : "./data";

    // Divisibility check, printed exactly like the reference's root (rowwise.c:72-75,
    // colwise.c:151-154, blockwise.c:277-281), exit status 0 as there. Every rank computes the
    // same verdict, so every rank leaves (the reference's other ranks would hang in MPI_Barrier).
    mvg_shard sh;
    rc = mvg_plan_shard(alg, n_rows, n_cols, comm_sz, L.rank, &sh);
    if (rc == MVG_E_INDIVISIBLE) {
        if (root) printf("\nERROR!!!\n%s\n", mvg_last_error());
        return finish(0);
    }
    if (rc != MVG_OK) return fatal(rc, "mvg_plan_shard");

    // root-only steps that can end the run (CSV, inputs) report a status every rank follows:
    // 1 = go on, 0 = stop with exit status 0 (the reference's `return 0` paths)
    int go = 1;
    char csv[256];
    snprintf(csv, sizeof csv, "./data/out/%s.csv", kAlgName[alg]);
    if (root) {
        FILE* probe = fopen(csv, "r");
        if (!probe) {  // rowwise.c:80-88
            FILE* fp = fopen(csv, "w");
            if (!fp) {
                printf("Unable to create output file.\n");
                go = 0;
            } else {
                fprintf(fp, "n_rows, n_cols, n_processes, time\n");
                fclose(fp);
            }
        } else {
            fclose(probe);
        }
    }
    launch_bcast(&go, sizeof go, 0);
    if (!go) return finish(0);

    mvg_shard sh0;  // the root's shard: the banner prints the root's view
    mvg_plan_shard(alg, n_rows, n_cols, comm_sz, 0, &sh0);
    if (root) {  // banner (rowwise.c:100-104; blockwise.c:314-321)
        printf("n_rows = %ld\n", n_rows);
        printf("n_cols = %ld\n", n_cols);
        if (alg == MVG_ALG_BLOCKWISE) {
            printf("comm_sz = %d\n", comm_sz);
            printf("my_rank = %d\n", 0);
            printf("comm_sz_rows = %d\n", sh0.grid_rows);
            printf("comm_sz_cols = %d\n", sh0.grid_cols);
            printf("local_n_rows = %ld\n", (long)sh0.n_rows);
            printf("local_n_cols = %ld\n", (long)sh0.n_cols);
        } else {
            printf("local_n = %ld\n", (long)(alg == MVG_ALG_ROWWISE ? sh0.n_rows : sh0.n_cols));
            printf("comm_sz = %d\n", comm_sz);
            printf("my_rank = %d\n", 0);
        }
        fflush(stdout);
    }

    // The root's A and x: in rank mode on one node, an MPI-3 shared window every rank maps (A,
    // then x); otherwise the root's own memory.
    const size_t nA = (size_t)n_rows * (size_t)n_cols;
    const char* synth_env = getenv("MVG_SYNTH");
    const bool synth_device = synth_env && strcmp(synth_env, "device") == 0;
    const char* dist_env = getenv("MVG_DIST");
    const bool want_shared = ranks && !synth_device && !(dist_env && strcmp(dist_env, "send") == 0);
    double* shared = want_shared ? (double*)launch_shared_alloc((nA + (size_t)n_cols + 1) * sizeof(double)) : nullptr;
    std::vector<double> x_own, y(root ? std::max(n_rows, 1L) : 1);
    std::unique_ptr<double, decltype(&free)> A_own(nullptr, &free);
    double* A = nullptr;
    double* x = nullptr;
    if (shared) {
        A = shared;
        x = shared + nA;
        // NUMA placement before the root fills the window: every rank first-touches its share of
        // A's rows from its GPU's socket, so each GPU later pulls its shard from local DRAM
        // instead of one socket's DRAM feeding every GPU across the inter-socket link
        const int64_t r0 = n_rows * L.rank / L.size, r1 = n_rows * (L.rank + 1) / L.size;
        (void)mvg_host_first_touch(A + r0 * n_cols, (size_t)(r1 - r0) * (size_t)n_cols * sizeof(double),
                                   my_device);
        launch_barrier();
    } else if (!synth_device && (root || !ranks)) {
        // left untouched by the allocation: the first write decides each page's NUMA node
        A_own.reset((double*)malloc(std::max<size_t>(nA, 1) * sizeof(double)));
        if (!A_own) {
            fprintf(stderr, "out of host memory for A (%zu doubles)\n", nA);
            return finish(1);
        }
        x_own.resize(std::max(n_cols, 1L));
        A = A_own.get();
        x = x_own.data();
        // one process driving G GPUs: GPU g's rows first-touched from GPU g's socket, as the
        // shared window is in rank mode (one socket's DRAM would otherwise feed every GPU)
        if (!ranks && comm_sz > 1)
            for (int g = 0; g < comm_sz; ++g) {
                const int64_t r0 = n_rows * g / comm_sz, r1 = n_rows * (g + 1) / comm_sz;
                (void)mvg_host_first_touch(A + r0 * n_cols, (size_t)(r1 - r0) * (size_t)n_cols * sizeof(double), g);
            }
    }
    if (root) {
        char name[128];
        if (synth_device) {
            printf("Generating synthetic matrix %ld x %ld (seed %u) and vector (seed %u) on the GPUs...\n", n_rows,
                   n_cols, MVG_SEED_A, MVG_SEED_X);
        } else if (env_long("MVG_SYNTH", 0)) {
            printf("Generating synthetic matrix %ld x %ld (seed %u) and vector (seed %u)...\n", n_rows, n_cols,
                   MVG_SEED_A, MVG_SEED_X);
            if ((rc = mvg_synth_fill_host(A, n_cols, n_rows, n_cols, 0, 0, n_cols, MVG_SEED_A)) != MVG_OK ||
                (rc = mvg_synth_fill_host(x, n_cols, 1, n_cols, 0, 0, n_cols, MVG_SEED_X)) != MVG_OK) {
                die(rc, "mvg_synth_fill_host", L.rank);
                go = -1;
            }
        } else {
            mvg_matrix_filename(n_rows, n_cols, name, sizeof name);
            printf("Reading matrix from file '%s/%s'...\n", data_dir, name);  // matr_utils.c:48
            fflush(stdout);
            if (mvg_load_matr(data_dir, n_rows, n_cols, A) != MVG_OK) {
                printf("Unable to locate matrix file '%s'\n", name);  // rowwise.c:111-117
                go = 0;
            } else {
                mvg_vector_filename(n_cols, name, sizeof name);
                printf("Reading vector from file '%s/%s'...\n", data_dir, name);
                fflush(stdout);
                if (mvg_load_vec(data_dir, n_cols, x) != MVG_OK) {
                    printf("Unable to locate vector file '%s'\n", name);
                    go = 0;
                }
            }
        }
        fflush(stdout);
    }
    launch_bcast(&go, sizeof go, 0);
    if (go <= 0) return finish(go < 0 ? 1 : 0);

    // devices: rank mode takes the node-local rank's GPU; the single process takes 0..G-1
    rc = mvg_device_count(&ndev);
    const int need = ranks ? my_device + 1 : comm_sz;
    if (launch_all_min(rc == MVG_OK && need <= ndev ? 1 : 0) == 0) {
        if (root || rc != MVG_OK || need > ndev)
            fprintf(stderr, "rank %d: %d GPU(s) needed on this node, %d visible: %s\n", L.rank,
                    ranks ? L.local_size : comm_sz, ndev, mvg_last_error());
        return finish(1);
    }
    // page-locked host memory: distribution runs at full PCIe rate on every GPU's own link; x and
    // y too (a pageable 600-element y cost 22 us per collect against 13 us page-locked,
    // tools/e2e_small.py). Rank mode: every rank locks the shared window (it pulls from it).
    std::vector<void*> pinned;
    auto pin = [&](void* p, size_t bytes) {
        if (p && bytes && mvg_host_register(p, bytes) == MVG_OK) pinned.push_back(p);
    };
    if (shared) {
        pin(shared, (nA + (size_t)n_cols + 1) * sizeof(double));
    } else if (A) {
        pin(A, nA * sizeof(double));
        pin(x, (size_t)n_cols * sizeof(double));
    }
    if (root) pin(y.data(), y.size() * sizeof(double));

    mvg_comm* comm = nullptr;
    if (ranks) {
        if ((rc = mvg_set_device(my_device)) != MVG_OK) return fatal(rc, "mvg_set_device");
        unsigned char uid[MVG_UNIQUE_ID_BYTES] = {0};
        int ok = 1;
        if (root && (rc = mvg_comm_unique_id(uid)) != MVG_OK) ok = die(rc, "mvg_comm_unique_id", L.rank) == 0;
        if (launch_all_min(ok) == 0) return finish(1);
        launch_bcast(uid, sizeof uid, 0);
        rc = mvg_comm_init_rank(&comm, uid, comm_sz, L.rank, my_device);
    } else {
        std::vector<int> devs(comm_sz);
        for (int i = 0; i < comm_sz; ++i) devs[i] = i;
        rc = mvg_comm_init_all(&comm, comm_sz, devs.data());
    }
    if (rc != MVG_OK) return fatal(rc, "mvg_comm_init");
    mvg_engine* eng = nullptr;
    if ((rc = mvg_engine_create(&eng, alg, n_rows, n_cols, comm)) != MVG_OK)
        return fatal(rc, "mvg_engine_create");

    if (synth_device && (rc = mvg_engine_fill_synth(eng, MVG_SEED_A, MVG_SEED_X)) != MVG_OK)
        return fatal(rc, "mvg_engine_fill_synth");
    auto distribute = [&]() {
        if (synth_device) return (int)MVG_OK;  // the shards were generated in place
        if (shared) return mvg_engine_distribute_shared(eng, A, x);
        return mvg_engine_distribute(eng, root ? A : nullptr, root ? x : nullptr);
    };
    // the reference's timed loop (rowwise.c:135-151): Barrier, t0, distribute + multiply +
    // collect, Barrier, t1, max over ranks on the root
    double sum_time = 0.0;
    std::vector<double> it_times;
    it_times.reserve((size_t)iters);
    for (long it = 0; it < iters; ++it) {
        if ((rc = mvg_engine_sync(eng)) != MVG_OK) return fatal(rc, "sync");
        launch_barrier();
        const double t0 = launch_wtime();
        if ((rc = distribute()) != MVG_OK) return fatal(rc, "distribute");
        if ((rc = mvg_engine_multiply(eng)) != MVG_OK) return fatal(rc, "multiply");
        if ((rc = mvg_engine_collect(eng, root ? y.data() : nullptr)) != MVG_OK)
            return fatal(rc, "collect");
        if ((rc = mvg_engine_sync(eng)) != MVG_OK) return fatal(rc, "sync");
        launch_barrier();
        const double elapsed = launch_max_to_root(launch_wtime() - t0);  // rowwise.c:146-147
        it_times.push_back(elapsed);
        sum_time += elapsed;
    }
    // device-resident: A already on the GPUs; GEMV + exchange only
    mvg_engine_kernel_timing(eng, 5);  // events on every 5th multiply (each pair costs ~6 us)
    launch_barrier();
    const double t0 = launch_wtime();
    for (long it = 0; it < iters; ++it)
        if ((rc = mvg_engine_multiply(eng)) != MVG_OK) return fatal(rc, "multiply");
    if ((rc = mvg_engine_sync(eng)) != MVG_OK) return fatal(rc, "sync");
    launch_barrier();
    const double dev_s = launch_max_to_root(launch_wtime() - t0) / (double)iters;
    double kms = 0.0;
    int64_t nk = 0;
    mvg_engine_kernel_ms(eng, &kms, &nk);
    kms = launch_max_to_root(kms);
    if (root) {
        const double bytes =
            8.0 * ((double)nA + (double)n_cols * (alg == MVG_ALG_ROWWISE ? comm_sz : 1) + (double)n_rows);
        printf("end-to-end (%s): mean %.6f s over %ld iterations\n",
               synth_device ? "multiply + y on root; inputs generated on the GPUs, nothing distributed"
                            : "distribute + multiply + y on root",
               sum_time / iters, iters);
        printf("device-resident: %.4f ms per multiply, %.1f GB/s aggregate; GEMV kernel %.3f ms (max over GPUs)\n",
               dev_s * 1e3, bytes / dev_s / 1e9, kms);
        int rccl_v = 0, hip_v = 0;
        if (mvg_runtime_versions(&rccl_v, &hip_v) == MVG_OK)  // which RCCL / HIP this process runs on
            printf("runtime: RCCL %d (%s), HIP %d (%s)\n", rccl_v, mvg_runtime_path(1), hip_v, mvg_runtime_path(0));
        if (ranks)
            printf("launch: %d ranks, one GPU each; distribution %s\n", comm_sz,
                   synth_device ? "none (inputs generated on every GPU)"
                   : shared     ? "from the root's A in a node-shared window, every GPU over its own link"
                                : "root H2D staging + ncclSend over xGMI");
        if (const char* tl = getenv("MVG_ITER_LOG")) {  // per-iteration end-to-end times, seconds
            if (FILE* f = fopen(tl, "w")) {
                for (double t : it_times) fprintf(f, "%.9f\n", t);
                fclose(f);
            }
        }
        if (const char* yo = getenv("MVG_Y_OUT")) {
            if ((rc = mvg_write_vec(yo, y.data(), n_rows)) != MVG_OK) {
                die(rc, "mvg_write_vec", L.rank);
                go = -1;
            }
        }
    }
    mvg_engine_destroy(eng);
    mvg_comm_destroy(comm);
    for (void* p : pinned) mvg_host_unregister(p);

    if (root && go > 0) {
        FILE* fp = fopen(csv, "a");  // rowwise.c:160-169
        if (!fp) {
            printf("Unable to open output file.\n");
        } else {
            fprintf(fp, "%ld, %ld, %d, %lf\n", n_rows, n_cols, comm_sz, sum_time / iters);
            fclose(fp);
        }
    }
    return finish(go < 0 ? 1 : 0);
}
