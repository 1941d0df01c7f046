/* Process launcher seen by the executables: `mpiexec -n P bin/multiplier_<alg> R C` (the
 * reference's own launch line, test.sh:11) starts P ranks, one GPU each; a plain start is one
 * process driving MVG_NGPUS GPUs. MPI carries only process bootstrap and the timing brackets
 * (the RCCL unique id, barriers, the max-over-ranks reduce of each iteration's time) and maps
 * the root's A into every rank on the node; no matrix or vector data moves through MPI.
 *
 * Built as its own small C library, bin/libmvg_launch.so, from launch_mpi.c when an MPI is
 * found (MPI_Init only when the process was started by an MPI launcher) or from launch_none.c
 * (single process only). Keeping MPI in its own library keeps the MPI installation's directory
 * (and the C++ runtime it may carry) off the executables' own library search path. */
#ifndef MVG_LAUNCH_H
#define MVG_LAUNCH_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int rank;       /* world rank (MPI_COMM_WORLD) */
    int size;       /* world size = P */
    int local_rank; /* rank among the ranks on this node -> GPU index */
    int local_size;
    int mpi;        /* started by an MPI launcher (MPI initialised) */
} mvg_launch;

void launch_init(int* argc, char*** argv, mvg_launch* l);
void launch_finalize(void);
/* end every rank of the job (MPI_Abort); returns only without MPI */
void launch_abort(int code);
void launch_barrier(void);
void launch_bcast(void* buf, size_t bytes, int root);
double launch_wtime(void);
/* max of v over ranks, on rank 0 (MPI_Reduce MAX, as rowwise.c:147) */
double launch_max_to_root(double v);
/* min of v over every rank, returned everywhere (collective agreement on a status) */
int launch_all_min(int v);
/* `bytes` of host memory on the node, allocated by world rank 0 and mapped by every rank (the
 * MPI-3 shared window MPICH itself scatters through). Collective; NULL on every rank when the
 * ranks span nodes or the allocation does not fit. */
void* launch_shared_alloc(size_t bytes);
void launch_shared_free(void);

#ifdef __cplusplus
}
#endif
#endif
