/* Launcher without MPI (see launch.h): always one process; the GPU count comes from MVG_NGPUS. */
#define _POSIX_C_SOURCE 200809L
#include <string.h>
#include <time.h>

#include "launch.h"

void launch_init(int* argc, char*** argv, mvg_launch* l) {
    (void)argc;
    (void)argv;
    memset(l, 0, sizeof *l);
    l->size = 1;
    l->local_size = 1;
}
void launch_finalize(void) {}
void launch_abort(int code) { (void)code; }
void launch_barrier(void) {}
void launch_bcast(void* buf, size_t bytes, int root) {
    (void)buf;
    (void)bytes;
    (void)root;
}
double launch_wtime(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}
double launch_max_to_root(double v) { return v; }
int launch_all_min(int v) { return v; }
void* launch_shared_alloc(size_t bytes) {
    (void)bytes;
    return NULL;
}
void launch_shared_free(void) {}
