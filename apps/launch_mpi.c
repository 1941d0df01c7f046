/* Launcher over MPI (see launch.h). MPI is initialised only when the process was started by an
 * MPI launcher (MPICH/hydra exports PMI_RANK/PMI_SIZE/PMI_FD) or MVG_MPI=1 asks for it; a plain
 * start stays a single process and never touches MPI. */
#define _POSIX_C_SOURCE 200809L
#include <mpi.h>
#include <stdlib.h>
#include <string.h>
#include <sys/statvfs.h>
#include <time.h>

#include "launch.h"

static int g_mpi = 0;
static MPI_Comm g_node = MPI_COMM_NULL;
static MPI_Win g_win = MPI_WIN_NULL;

void launch_init(int* argc, char*** argv, mvg_launch* l) {
    memset(l, 0, sizeof *l);
    l->size = 1;
    l->local_size = 1;
    const char* force = getenv("MVG_MPI");
    const int launched = getenv("PMI_RANK") || getenv("PMI_SIZE") || getenv("PMI_FD");
    if (!(launched || (force && force[0] == '1'))) return;
    MPI_Init(argc, argv);
    g_mpi = 1;
    l->mpi = 1;
    MPI_Comm_rank(MPI_COMM_WORLD, &l->rank);
    MPI_Comm_size(MPI_COMM_WORLD, &l->size);
    MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, l->rank, MPI_INFO_NULL, &g_node);
    MPI_Comm_rank(g_node, &l->local_rank);
    MPI_Comm_size(g_node, &l->local_size);
}

void launch_finalize(void) {
    if (!g_mpi) return;
    launch_shared_free();
    if (g_node != MPI_COMM_NULL) MPI_Comm_free(&g_node);
    MPI_Finalize();
    g_mpi = 0;
}

void launch_abort(int code) {
    if (g_mpi) MPI_Abort(MPI_COMM_WORLD, code);
}

void launch_barrier(void) {
    if (g_mpi) MPI_Barrier(MPI_COMM_WORLD);
}

void launch_bcast(void* buf, size_t bytes, int root) {
    if (g_mpi) MPI_Bcast(buf, (int)bytes, MPI_BYTE, root, MPI_COMM_WORLD);
}

double launch_wtime(void) {
    if (g_mpi) return MPI_Wtime();
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

double launch_max_to_root(double v) {
    if (!g_mpi) return v;
    double out = 0.0;
    MPI_Reduce(&v, &out, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
    return out;
}

int launch_all_min(int v) {
    if (!g_mpi) return v;
    int out = v;
    MPI_Allreduce(&v, &out, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
    return out;
}

void* launch_shared_alloc(size_t bytes) {
    if (!g_mpi) return NULL;
    int world = 0, local = 0, rank = 0;
    MPI_Comm_size(MPI_COMM_WORLD, &world);
    MPI_Comm_size(g_node, &local);
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    if (local != world) return NULL; /* ranks on several nodes: every rank decides the same */
    /* rank 0 decides whether the window fits its /dev/shm (1 GiB spare) before any rank enters
     * the collective allocation */
    int ok = 0;
    if (rank == 0) {
        struct statvfs st;
        ok = statvfs("/dev/shm", &st) == 0 &&
             (double)st.f_bavail * (double)st.f_frsize > (double)bytes + (double)(1ull << 30);
    }
    MPI_Bcast(&ok, 1, MPI_INT, 0, MPI_COMM_WORLD);
    if (!ok) return NULL;
    void* mine = NULL;
    MPI_Comm_set_errhandler(g_node, MPI_ERRORS_RETURN);
    const int rc = MPI_Win_allocate_shared(rank == 0 ? (MPI_Aint)bytes : 0, 1, MPI_INFO_NULL, g_node,
                                           &mine, &g_win);
    if (launch_all_min(rc == MPI_SUCCESS ? 1 : 0) == 0) {
        if (rc == MPI_SUCCESS) MPI_Win_free(&g_win);
        g_win = MPI_WIN_NULL;
        return NULL;
    }
    MPI_Aint qbytes = 0;
    int disp = 0;
    void* base = NULL;
    MPI_Win_shared_query(g_win, 0, &qbytes, &disp, &base);
    return base;
}

void launch_shared_free(void) {
    if (g_mpi && g_win != MPI_WIN_NULL) MPI_Win_free(&g_win);
    g_win = MPI_WIN_NULL;
}
