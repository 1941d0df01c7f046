/*
 * matvec_gpu.h — C-ABI of libmatvec_gpu.so, the MI355X (gfx950) replacement for the
 * compute + communication core of yaroslav-i-am/MatVec_MPI_Multiplier.
 *
 * Plain C types only (pointers, int64_t sizes, int return codes). No torch, no HIP
 * types in any signature: streams are passed as `void*` (a hipStream_t, NULL = the
 * library's own stream for that device).
 *
 * Every function returns MVG_OK (0) on success or a negative MVG_E* code; the text of
 * the last failure on the calling thread is available from mvg_last_error().
 *
 * Reference interfaces replaced (paths relative to the reference repository):
 *   mvg_gemv                 <- multiply_std_rowwise          src/matr_utils.c:86-96
 *                               (also the strip GEMV that multiply_colwise computes as
 *                                scale-then-row-sum,          src/multiplier_colwise.c:105-122)
 *   mvg_gemv_exact           <- the same, bit for bit (the reference's sequential sum)
 *   mvg_multiply_std_rowwise <- multiply_std_rowwise itself on host pointers (matr_utils.h:4-10)
 *   mvg_grid_shape           <- get_2_most_closest_multipliers src/utils.c:26-37
 *   mvg_plan_shard           <- local_n / local_n_rows / local_n_cols arithmetic
 *                               src/multiplier_rowwise.c:93, src/multiplier_colwise.c:349,
 *                               src/multiplier_blockwise.c:299-306 (+ divisibility checks
 *                               rowwise.c:72-75, colwise.c:151-154, blockwise.c:277-281)
 *   mvg_engine_distribute    <- distribute_data (Scatter/Bcast | Type_vector+Pack+Send |
 *                               block Pack+Send)  rowwise.c:12-51, colwise.c:11-102,
 *                               blockwise.c:17-141
 *   mvg_engine_multiply      <- local multiply + MPI_Gather / MPI_Reduce(SUM) /
 *                               gather_local_results
 *                               rowwise.c:140-141, colwise.c:105-129, blockwise.c:144-210,367-368
 *   mvg_engine_collect       <- root owning `result` after the timed region (the reference
 *                               never writes y; this is the opt-in y hand-back)
 *   mvg_load_matr / mvg_load_vec <- load_matr / load_vec       src/matr_utils.c:42-83
 *   mvg_comm_*               <- MPI_Init/Comm_size/Comm_rank/Finalize + the collectives
 *                               (RCCL over xGMI instead of MPI)
 */
#ifndef MATVEC_GPU_H
#define MATVEC_GPU_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ status codes */
#define MVG_OK              0
#define MVG_E_INVALID      -1   /* bad argument (null pointer, negative size, ...)   */
#define MVG_E_INDIVISIBLE  -2   /* shape does not split over the rank count          */
#define MVG_E_HIP          -3   /* HIP runtime failure                                */
#define MVG_E_RCCL         -4   /* RCCL failure                                       */
#define MVG_E_IO           -5   /* file missing / unreadable                          */
#define MVG_E_NOMEM        -6   /* host or device allocation failed                   */
#define MVG_E_STATE        -7   /* call out of order (e.g. multiply before distribute)*/

/* ------------------------------------------------------------------ algorithms   */
#define MVG_ALG_ROWWISE    0    /* src/multiplier_rowwise.c   */
#define MVG_ALG_COLWISE    1    /* src/multiplier_colwise.c   */
#define MVG_ALG_BLOCKWISE  2    /* src/multiplier_blockwise.c */

const char* mvg_version(void);
const char* mvg_strerror(int code);
const char* mvg_last_error(void);

/* The runtimes this library is bound to in the calling process (no counterpart in the
 * reference, whose MPI is fixed at build time). The library needs libamdhip64.so.7 and
 * librccl.so.1 by soname, so a process that loaded another copy first (PyTorch's ROCm wheel
 * bundles its own HIP and RCCL) runs the library on that copy. mvg_runtime_versions: RCCL's
 * ncclGetVersion code (e.g. 22705 = 2.27.5) and HIP's hipRuntimeGetVersion; either pointer may
 * be NULL. mvg_runtime_path: the file the bound copy was loaded from (which: 0 = the HIP
 * runtime, 1 = RCCL), "" when unknown. Neither call runs anything on a device (asking for the
 * HIP version may start the HIP runtime; mvg_runtime_path and the RCCL version do not). */
int mvg_runtime_versions(int* rccl_version, int* hip_runtime_version);
const char* mvg_runtime_path(int which);

/* ------------------------------------------------------------------ planner (host only, no GPU)
 * get_2_most_closest_multipliers (src/utils.c:26-37): rows = largest d <= floor(sqrt(p))
 * with p % d == 0, cols = p / d.  p <= 0 -> MVG_E_INVALID. */
int mvg_grid_shape(int64_t p, int* grid_rows, int* grid_cols);

/* The slice of the global R x C problem that rank `rank` of `nranks` owns.
 * row_off/col_off/n_rows/n_cols: the block of A (and col_off/n_cols: the x segment);
 * y_off/y_len: the slice of y its partial result contributes to.
 * grid_r/grid_c: rank's coordinate in the grid (row-split: (rank,0), col-split: (0,rank)).
 * Returns MVG_E_INDIVISIBLE exactly where the reference prints "ERROR!!!", and also
 * (deliberate deviation) where the reference would silently compute a
 * wrong y: block-split with R % r != 0 or C % c != 0. */
typedef struct mvg_shard {
    int     alg, nranks, rank;
    int     grid_rows, grid_cols, grid_r, grid_c;
    int64_t R, C;
    int64_t row_off, col_off, n_rows, n_cols;
    int64_t y_off, y_len;
} mvg_shard;
int mvg_plan_shard(int alg, int64_t R, int64_t C, int nranks, int rank, mvg_shard* out);

/* The exchange step after the local product, as the collective schedule rank `rank` runs
 * (the engine drives RCCL from exactly this plan; tests replay it over gloo).
 *   row  : GATHER(world, count = R/P, PART -> Y)                    rowwise.c:141
 *   col  : REDUCE(world, count = R, PART -> Y)                       colwise.c:124
 *   block: REDUCE(row comm: color grid_r, key grid_c; count = R/r, PART -> ROW on the leader),
 *          GATHER(col comm: the grid-column-0 leaders, key grid_r; ROW -> Y)  blockwise.c:144-210
 *          (one grid row: a single REDUCE straight into Y).
 * P == 1 has no steps (the product is written straight into Y) unless force_collect != 0.
 * A communicator is identified by (comm kind, color); ranks order by key; root is the rank
 * within that communicator (always 0, i.e. world rank 0 / the grid-row leader). */
#define MVG_X_GATHER    0
#define MVG_X_REDUCE    1
#define MVG_X_WORLD     0
#define MVG_X_ROW       1
#define MVG_X_COL       2
#define MVG_X_BUF_PART  0   /* the local product (y_len doubles; R for column split) */
#define MVG_X_BUF_ROW   1   /* the grid-row sum on the row leader (y_len doubles)       */
#define MVG_X_BUF_Y     2   /* the full y on world rank 0 (R doubles)                   */
typedef struct mvg_xstep {
    int     op, comm, color, key, member, root, src, dst;
    int64_t count;
} mvg_xstep;
#define MVG_MAX_XSTEPS 4
int mvg_plan_exchange(int alg, int64_t R, int64_t C, int nranks, int rank, int force_collect,
                      mvg_xstep* steps, int max_steps, int* nsteps);

/* Test hook: the calls one process driving `ndev` devices issues (the executables'
 * MVG_NGPUS=G form: ncclCommSplit of the schedule's sub-communicators, then one multiply's
 * exchange), produced by the engine's own exchange code with a recorder in place of RCCL, so no
 * device is needed. `exact` != 0: exact mode's exchange (rank-order gather to rank 0 + the
 * combine kernel there). Calls are listed in issue order; `group` numbers the
 * ncclGroupStart/End bracket each was issued in (-1: outside any, the combine kernel); `comm`
 * is -1 for the world communicator, else the group whose split created it;
 * color -1 = NCCL_SPLIT_NOCOLOR; src/dst are MVG_X_BUF_*
 * (MVG_X_BUF_GATHERED: rank 0's gather buffer in exact mode), -1 where the call has none.
 * Reference interface it stands for: multiplier_blockwise.c:144-210 (gather_local_results),
 * multiplier_colwise.c:124, multiplier_rowwise.c:141. */
#define MVG_XCALL_SPLIT   0
#define MVG_XCALL_GATHER  1
#define MVG_XCALL_REDUCE  2
#define MVG_XCALL_COMBINE 3
#define MVG_X_BUF_GATHERED 3
typedef struct mvg_xcall {
    int     group, kind, rank, comm, color, key, root, src, dst;
    int64_t count;
} mvg_xcall;
int mvg_debug_trace_exchange(int alg, int64_t R, int64_t C, int ndev, int exact, mvg_xcall* calls, int max_calls,
                             int* ncalls);

/* ------------------------------------------------------------------ synthetic inputs
 * value(seed, idx) = (double)k / 10000.0, k = floor(splitmix64(s0 + idx*gamma) * 10000 / 2^64),
 * s0 = splitmix64(seed), gamma = 0x9E3779B97F4A7C15. Every value is exactly what "%.4f" text
 * of it parses back to (the reference's data format, README.md:32), so synthetic and text
 * inputs are interchangeable bit for bit. A uses idx = i*C + j of the GLOBAL matrix; x uses
 * its own seed.  The device fill writes a shard [row_off, +m) x [col_off, +k) of a global
 * R x C matrix (n_cols_global = C) into dst with leading dimension ld. */
#define MVG_SEED_A 42u
#define MVG_SEED_X 4242u
double mvg_synth_value(uint64_t seed, uint64_t idx);
int    mvg_synth_fill_host(double* dst, int64_t ld, int64_t m, int64_t k,
                           int64_t row_off, int64_t col_off, int64_t n_cols_global, uint64_t seed);
int    mvg_synth_fill_device(double* d_dst, int64_t ld, int64_t m, int64_t k,
                             int64_t row_off, int64_t col_off, int64_t n_cols_global,
                             uint64_t seed, void* stream);

/* ------------------------------------------------------------------ device helpers */
int mvg_device_count(int* n);
int mvg_set_device(int dev);
int mvg_malloc(void** dptr, size_t bytes);
int mvg_free(void* dptr);
int mvg_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream);
int mvg_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream);
int mvg_stream_sync(void* stream);
int mvg_host_register(void* ptr, size_t bytes);     /* pin caller-owned host memory */
int mvg_host_unregister(void* ptr);
/* NUMA node of GPU `device` (from its PCI address; -1 when unknown). */
int mvg_device_numa_node(int device, int* node);
/* Zero [ptr, ptr + bytes) from threads bound to the CPUs of GPU `device`'s NUMA node, so the
 * pages land in that socket's DRAM (first-touch placement of host memory the GPU will pull
 * from; the executables' shared window). Falls back to the caller's CPUs. */
int mvg_host_first_touch(void* ptr, size_t bytes, int device);

/* ------------------------------------------------------------------ the hot kernel
 * y[i] = sum_j A[i*lda + j] * x[j], i < m, j < k (fp64, row-major, lda >= k).
 * Device pointers; asynchronous on `stream`. Results match the reference's sequential
 * left-to-right sum (src/matr_utils.c:87-93) to <= 1e-12 relative per element for
 * non-negative data (different, fixed, run-to-run deterministic summation order).
 * m == 0 or k == 0 is valid (k == 0 writes zeros, as the reference's `sum = 0`). */
int mvg_gemv(const double* d_A, int64_t lda, const double* d_x, double* d_y,
             int64_t m, int64_t k, void* stream);

/* Same, with an explicit kernel variant (benchmarks / tests):
 *   0 = auto (shape-adaptive), 1.. = the table in csrc/gemv.hip (names via
 *   mvg_gemv_variant_name: vec_* wave-owns-rows, rowblk_* row-per-workgroup, scl_* 8-B loads). */
int mvg_gemv_variant(const double* d_A, int64_t lda, const double* d_x, double* d_y,
                     int64_t m, int64_t k, int variant, void* stream);
int mvg_gemv_variant_count(void);
/* the variant mvg_gemv picks for a 16-B-aligned A, x with this lda, m and k */
int mvg_gemv_auto_variant(int64_t lda, int64_t m, int64_t k);
const char* mvg_gemv_variant_name(int variant);

/* Several x per pass over A (beyond the reference's surface):
 * Y[:, v] = A X[:, v] for v < nv, X k x nv and Y m x nv column-major (vector v at X + v*ldx,
 * Y + v*ldy; ldx >= k, ldy >= m). A is streamed once per group of 8 vectors (16 from 8192 rows
 * of >= 1024 columns, on the matrix cores), so the HBM cost
 * of nv products approaches that of one. Same numerics contract as mvg_gemv. */
int mvg_gemv_multi(const double* d_A, int64_t lda, const double* d_X, int64_t ldx, double* d_Y,
                   int64_t ldy, int64_t m, int64_t k, int nv, void* stream);
/* mvg_gemv_multi with an explicit kernel variant (0 = automatic; tests and sweeps) */
int mvg_gemv_multi_variant(const double* d_A, int64_t lda, const double* d_X, int64_t ldx, double* d_Y,
                           int64_t ldy, int64_t m, int64_t k, int nv, int variant, void* stream);
int mvg_gemv_multi_variant_count(void);
/* the variant mvg_gemv_multi picks for the first group of nv >= 2 vectors (16-B aligned A and X,
 * even lda and ldx): up to 16 vectors per pass on long enough shapes, else up to 8; 0 for nv < 2
 * (the single-vector dispatch) */
int mvg_gemv_multi_auto_variant(int64_t lda, int64_t ldx, int64_t m, int64_t k, int nv);
const char* mvg_gemv_multi_variant_name(int variant);

/* Bit-exact form of mvg_gemv: every row is the reference's own chain
 *   sum = 0; for j < k: sum = round(sum + round(A[i*lda + j] * x[j]))
 * (src/matr_utils.c:87-93: a rounded multiply then a rounded add, left to right, no FMA), so
 * y is bit-identical to multiply_std_rowwise on the same inputs (and to the strip sums of
 * multiply_colwise, src/multiplier_colwise.c:107-122). Tall shapes whose rows start on 128-B
 * lines: one lane per row, rows streamed through LDS; everything else: several lanes per row,
 * the running sum handed lane to lane in column order (csrc/gemv_exact.hip). Any lda >= k and
 * any alignment. */
int mvg_gemv_exact(const double* d_A, int64_t lda, const double* d_x, double* d_y,
                   int64_t m, int64_t k, void* stream);
/* The reference's in-process call on host pointers, src/matr_utils.h:4-10:
 *   void multiply_std_rowwise(double* matrix, double* vector, long n_rows, long n_cols, double* result);
 * row-major matrix (n_rows x n_cols), vector (n_cols), result (n_rows), all caller-owned host
 * memory, on the calling thread's current device: copies A and x over, runs mvg_gemv_exact
 * (exact != 0: result bit-identical to the reference's) or mvg_gemv (exact == 0: within 1e-12),
 * copies y back and waits. Device buffers are kept per thread and grown as needed; all-zero /
 * null arguments release them. */
int mvg_multiply_std_rowwise(const double* matrix, const double* vector, int64_t n_rows, int64_t n_cols,
                             double* result, int exact);
/* explicit exact variant (0 = auto; names via mvg_gemv_exact_variant_name: seq_r<RW>_t<T>_b<NB>
 * and seqx_* RW-row LDS-DMA tiles of 2T columns with NB buffers, hop_l<L>_w<W>_u<U> L lanes per
 * row holding W columns each with U segments in flight, hop8_* the same with 8-B loads (any
 * alignment, any lda), seq_scalar a lane per row with 8-B loads) */
int mvg_gemv_exact_variant(const double* d_A, int64_t lda, const double* d_x, double* d_y,
                           int64_t m, int64_t k, int variant, void* stream);
int mvg_gemv_exact_variant_count(void);
int mvg_gemv_exact_auto_variant(int64_t lda, int64_t m, int64_t k);
const char* mvg_gemv_exact_variant_name(int variant);
/* Test hooks of the exact dispatch (no counterpart in the reference). mvg_debug_set_cu_count:
 * the CU count the dispatch plans whole rounds of workgroups for (0 = the current device's).
 * mvg_debug_set_exact_even_lds: the LDS reservation of the evenly placed form in bytes (0 = its
 * own 96 KiB); above the CU's 160 KiB the runtime refuses the launch, which drives the fallback
 * to the one-wave form (same sums); it also forgets earlier refusals. */
int mvg_debug_set_cu_count(int n);
int mvg_debug_set_exact_even_lds(int64_t bytes);
/* 1 when the runtime has refused the evenly placed exact form's LDS on `device` in this process
 * (a request above the device's per-workgroup LDS, confirmed against
 * hipDeviceAttributeMaxSharedMemoryPerBlock, logged once on stderr): the auto dispatch there
 * then runs the one-wave forms. 0 otherwise; MVG_E_INVALID for a device index outside 0..63. */
int mvg_gemv_exact_even_refused(int device);

/* The same bit-exact product over A in column panels (the engine's device layout in exact mode,
 * DESIGN §4b): panel p holds columns [p*P, p*P + P) of all m rows, row i of it at
 * d_Ap + p*pstride + i*P (pstride >= m*P doubles; the last panel may be narrower than P and is
 * padded to P). Same sums in the same order as mvg_gemv_exact (multiply_std_rowwise,
 * src/matr_utils.c:86-96), so y is the same bit for bit; streaming the rows panel by panel reads
 * one contiguous region at a time instead of m scattered ones. P a power of two, a multiple of
 * 16 (32 for panel_l16_*); d_Ap and d_x 16-B aligned. variant 0 = auto (names:
 * mvg_gemv_exact_panel_variant_name, panel_l<L>_w<W>_u<U> as the hop forms). */
int mvg_gemv_exact_panels(const double* d_Ap, int64_t pstride, int64_t P, const double* d_x, double* d_y,
                          int64_t m, int64_t k, int variant, void* stream);
/* Rows [0, m) of a row-major A (lda) into rows [0, m) of the panel layout above (device to
 * device, HBM-bound; any lda and alignment). Row ranges map onto row ranges: offset d_A by
 * r0*lda and d_Ap by r0*P, keep pstride. */
int mvg_panel_relayout(const double* d_A, int64_t lda, int64_t m, int64_t k, double* d_Ap, int64_t pstride,
                       int64_t P, void* stream);
/* P the engine uses for an m x k shard in exact mode (0: it keeps the row-major kernels). */
int64_t mvg_exact_panel_width(int64_t m, int64_t k);
int mvg_gemv_exact_panel_variant_count(void);
int mvg_gemv_exact_panel_auto_variant(int64_t m, int64_t k);
const char* mvg_gemv_exact_panel_variant_name(int variant);

/* Read-only streaming microkernel over `bytes` of device memory (HBM ceiling calibration). */
int mvg_stream_read(const double* d_src, int64_t n, double* d_sink, void* stream);

/* ------------------------------------------------------------------ communicators (RCCL)
 * One communicator object per process covers all devices this process drives:
 *   mvg_comm_init_all : single process, G devices (the executables' model; ncclCommInitAll)
 *   mvg_comm_init_rank: one process per device (torch.distributed.run model); the caller
 *                       moves the 128-byte unique id from rank 0 to every rank. */
typedef struct mvg_comm mvg_comm;
#define MVG_UNIQUE_ID_BYTES 128
int mvg_comm_unique_id(unsigned char out[MVG_UNIQUE_ID_BYTES]);
int mvg_comm_init_all(mvg_comm** out, int ndev, const int* devlist);
int mvg_comm_init_rank(mvg_comm** out, const unsigned char id[MVG_UNIQUE_ID_BYTES],
                       int nranks, int rank, int device);
int mvg_comm_size(const mvg_comm* c, int* nranks);
int mvg_comm_local_count(const mvg_comm* c, int* nlocal);
int mvg_comm_local_rank(const mvg_comm* c, int local_index, int* rank, int* device);
int mvg_comm_destroy(mvg_comm* c);

/* ------------------------------------------------------------------ engine
 * The distributed multiplier: one object per (alg, R, C, comm). Holds, per local device,
 * the shard of A, the x segment, the partial y and (on rank 0) the full y.
 *   distribute : host A/x on the root (rank 0's process) -> device shards (H2D, the
 *                Scatter/Bcast/Pack+Send of the reference). A_host == NULL on non-root.
 *   fill_synth : device-resident inputs, generated on each device (no host copy).
 *   multiply   : local GEMV on every device + the exchange step
 *                (row: ncclGather of y; col: ncclReduce(SUM); block: ncclReduce(SUM) on each
 *                 grid-row communicator, then ncclGather of the row leaders' slices).
 *                Asynchronous on the engine's streams; mvg_engine_sync waits. The exchange
 *                runs on a second stream per device and overlaps the next multiply's GEMV
 *                (partial y double-buffered); collect and sync wait for it.
 *   collect    : y (R doubles) -> host on the root.  */
typedef struct mvg_engine mvg_engine;
int mvg_engine_create(mvg_engine** out, int alg, int64_t R, int64_t C, mvg_comm* comm);
int mvg_engine_shard(const mvg_engine* e, int local_index, mvg_shard* out);
int mvg_engine_distribute(mvg_engine* e, const double* A_host, const double* x_host);
/* One process per GPU on one node: the root's A, x live in host memory every rank maps
 * (shared memory); each GPU pulls its own shard over its own PCIe link, all in parallel (the
 * analog of MPICH's shared-memory MPI_Scatter on one host). Every rank passes the full A, x.
 * In single-process mode identical to mvg_engine_distribute. */
int mvg_engine_distribute_shared(mvg_engine* e, const double* A_shared, const double* x_shared);
int mvg_engine_fill_synth(mvg_engine* e, uint64_t seed_a, uint64_t seed_x);
int mvg_engine_multiply(mvg_engine* e);
int mvg_engine_sync(mvg_engine* e);
int mvg_engine_collect(mvg_engine* e, double* y_host);
/* per-local-device GEMV stream (hipStream_t as void*), e.g. for hipEvent timing of the GEMV by
 * the caller; y on the root is complete only after mvg_engine_sync / mvg_engine_collect */
int mvg_engine_stream(const mvg_engine* e, int local_index, void** stream);
/* Average GEMV kernel time (ms) over the multiply calls since the last reset, measured with
 * hipEvents bracketing the kernel on each local device's stream (max over local devices).
 * every = N > 0 brackets every Nth multiply call (1 = all); 0 turns timing off; -1 times spans:
 * one event before the first GEMV after a reset or a sync and one at the next mvg_engine_sync,
 * nothing between the GEMVs of the span (a bracketing marker stalls the stream around its
 * kernel), so the average is the span over its multiplies (the GEMVs back to back, with their
 * dispatch gaps; at more than one rank it also holds the GEMV stream's waits on the exchange).
 * A span that also holds other writes to the shard — a distribution, a synthetic fill, exact
 * mode's panel relayout after the span's first GEMV, a chunked distribution's copies — is
 * dropped: it adds no launches and no time to the average. */
int mvg_engine_kernel_timing(mvg_engine* e, int every);
int mvg_engine_kernel_ms(mvg_engine* e, double* avg_ms, int64_t* launches);
int mvg_engine_destroy(mvg_engine* e);
/* Bit-exact mode (off by default; MVG_EXACT=1 in the environment turns it on at creation):
 * local products by mvg_gemv_exact, and the exchange adds the partials in the reference's own
 * order — the column split's MPI_Reduce as MPICH 3.3.2 sums it (binomial tree, or reduce-scatter
 * + gather for buffers over 2 KiB, oracle/cpu_ref.c ref_mpich_reduce)
 * (colwise.c:124), the block split's partials into a zeroed y in rank order
 * (blockwise.c:150-207) — after an ncclGather of every partial to rank 0. y is then
 * bit-identical to the reference's (block split with > 2 grid columns: to the reference's
 * result for rank-order message arrival; its own order varies run to run). */
int mvg_engine_set_exact(mvg_engine* e, int on);
int mvg_engine_exact(const mvg_engine* e, int* on);
/* Exact mode keeps a column-panel copy of a tall long-row shard (mvg_exact_panel_width) and
 * multiplies it with mvg_gemv_exact_panels: the copy is allocated (if it fits in free HBM with
 * 8 GiB to spare) and rebuilt from the row-major shard by the second multiply after each
 * distribute / fill — a distribution multiplied once never pays for it — and released when exact
 * mode is switched off; MVG_NO_PANELS=1 turns it off. *P = the panel width of local shard i's
 * copy, 0 while it runs the row-major kernels. */
int mvg_engine_exact_panels(const mvg_engine* e, int local_index, int64_t* P);
/* Chunked distribution (off by default; MVG_OVERLAP=n in the environment sets it at creation):
 * chunks > 1 makes distribute / distribute_shared move each shard's rows in that many chunks on
 * a copy stream, and the next multiply runs each chunk's GEMV as soon as its rows have landed,
 * so only the last chunk's GEMV follows the transfer (the root-send distribution of one process
 * per GPU is unchanged). 0 or 1 = one copy, then the GEMV. y is the same either way (row chunks
 * are independent products; bit for bit in exact mode). */
int mvg_engine_set_overlap(mvg_engine* e, int chunks);

/* ------------------------------------------------------------------ text I/O (src/matr_utils.c)
 * Same file names under the same directory convention: <dir>/matrix_<R>_<C>.txt,
 * <dir>/vector_<n>.txt (dir "./data" in the executables, matr_utils.c:45,68). Whitespace
 * separated "%lf" tokens, row-major. Parsing is strtod (== fscanf "%lf") on an mmap'd file,
 * split over threads; 64-bit indexing. Returns MVG_E_IO if the file is missing or short. */
int mvg_matrix_filename(int64_t R, int64_t C, char* buf, size_t buflen);
int mvg_vector_filename(int64_t n, char* buf, size_t buflen);
int mvg_load_matr(const char* dir, int64_t R, int64_t C, double* A);
/* Binary cache beside the text (<dir>/matrix_<R>_<C>.bin: "MVGBIN1\0", int64 R, int64 C, R*C
 * native fp64). mvg_load_matr reads it instead of the text when it exists, matches (R, C) and is
 * not older than the text; with MVG_BIN_CACHE=1 it also writes it after parsing the text;
 * MVG_BIN_CACHE=0 ignores it. Parsing a 30-120 GB text file once is then enough. */
int mvg_write_matr_bin(const char* path, const double* A, int64_t R, int64_t C);
int mvg_load_vec(const char* dir, int64_t n, double* x);
int mvg_write_vec(const char* path, const double* v, int64_t n);   /* "%.17g\n" per value */
int mvg_write_matr_synth(const char* path, int64_t R, int64_t C, uint64_t seed); /* "%.4f " */

#ifdef __cplusplus
}
#endif
#endif /* MATVEC_GPU_H */
