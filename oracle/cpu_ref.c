/*
 * oracle/cpu_ref.c — CPU restatement of the reference's three distributed multipliers.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this (as the checker / the CPU baseline), never the product
 * path. It is pinned against golden y vectors produced by the real reference (compiled
 * from /root/reference/src with MPICH by oracle/build_ref.sh; tests/golden/make_golden.py and
 * tests/golden/make_config_slices.py run it).
 *
 * Every function cites the reference file:line it restates. Arithmetic is plain C with
 * -ffp-contract=off (no FMA), exactly the operation order of the reference:
 *   - the local product is a left-to-right sum from 0 (src/matr_utils.c:86-96),
 *   - column split scales in place then row-sums (src/multiplier_colwise.c:107-122) and
 *     combines the strips with MPI_Reduce(SUM) (colwise.c:124), restated as the image's MPICH
 *     3.3.2 runs it: binomial tree or reduce-scatter + gather by message size (ref_mpich_reduce),
 *   - block split accumulates y[(src/c)*lr + j] += partial into a zeroed y, the root's own
 *     block first, then the others (src/multiplier_blockwise.c:150-207). The reference takes
 *     them in MPI_ANY_SOURCE arrival order (nondeterministic); this oracle uses rank order.
 * Sizes are 64-bit throughout (the reference's int counts overflow at the large configs).
 */
#define _GNU_SOURCE
#include "cpu_ref.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* src/matr_utils.c:86-96 */
void ref_multiply_std_rowwise(const double* matrix, const double* vector, int64_t n_rows,
                              int64_t n_cols, double* result) {
    for (int64_t i = 0; i < n_rows; ++i) {
        double sum = 0;
        for (int64_t j = 0; j < n_cols; ++j) sum += matrix[i * n_cols + j] * vector[j];
        result[i] = sum;
    }
}

/* src/utils.c:26-37 */
void ref_grid_shape(int64_t number, int* dividers) {
    int sroot = (int)sqrt_floor(number); /* = (int)sqrt((double)number) */
    for (int cur_div = sroot; cur_div > 0; --cur_div) {
        if (number % cur_div == 0) {
            dividers[0] = cur_div;
            dividers[1] = (int)(number / cur_div);
            return;
        }
    }
}

int64_t sqrt_floor(int64_t n) {
    int64_t s = 0;
    while ((s + 1) * (s + 1) <= n) ++s;
    return s;
}

/* MPI_Reduce(SUM, root 0) over P rank buffers of n doubles, as the image's MPICH 3.3.2 runs it
 * for the reference's colwise.c:124 (MPIR_Reduce_intra_auto; on one node the SMP path hands the
 * same communicator to the same choice):
 *   - n * 8 > 2048 bytes and n >= pof2 (pof2 = largest power of two <= P): reduce-scatter +
 *     gather. With rem = P - pof2, ranks 2i and 2i+1 (i < rem) first fold into one new rank i,
 *     the others become new rank r - rem; the recursive halving then sums the pof2 new ranks as a
 *     binomial tree ((n0 + n1) + (n2 + n3)) + ...;
 *   - otherwise the binomial tree over the P ranks: at mask = 1, 2, 4, ... rank r (r % 2mask == 0)
 *     adds rank r + mask's buffer.
 * The two agree whenever P is a power of two (and at P = 3, 6, 7, 12); they differ at P = 5, 9,
 * 10, 11, 13, ... (golden sq_720/colwise/P5, P9, P10 pin both branches). fp64 addition is
 * commutative bit for bit, so only the association matters. Result in bufs[0]. */
static void binomial_over(double** bufs, const int* idx, int n_idx, int64_t n) {
    for (int mask = 1; mask < n_idx; mask <<= 1)
        for (int r = 0; r + mask < n_idx; r += 2 * mask) {
            double* a = bufs[idx[r]];
            const double* b = bufs[idx[r + mask]];
            for (int64_t i = 0; i < n; ++i) a[i] = a[i] + b[i];
        }
}

void ref_mpich_reduce(double** bufs, int P, int64_t n) {
    int pof2 = 1;
    while (pof2 * 2 <= P) pof2 *= 2;
    int* idx = (int*)malloc(sizeof(int) * (size_t)P);
    int m = P;
    if (n * 8 > 2048 && n >= pof2 && pof2 != P) {
        const int rem = P - pof2;
        for (int i = 0; i < rem; ++i)
            for (int64_t k = 0; k < n; ++k) bufs[2 * i][k] = bufs[2 * i][k] + bufs[2 * i + 1][k];
        for (int i = 0; i < pof2; ++i) idx[i] = i < rem ? 2 * i : i + rem;
        m = pof2;
    } else {
        for (int i = 0; i < P; ++i) idx[i] = i;
    }
    binomial_over(bufs, idx, m, n);
    free(idx);
}

/* src/multiplier_rowwise.c:93,139-141: scatter rows, local product, gather in rank order.
 * Each row's sum is independent of P, so this equals the serial product bit for bit. */
int ref_rowwise(const double* A, const double* x, int64_t R, int64_t C, int P, double* y) {
    if (P <= 0 || R % P != 0) return -2;
    const int64_t ln = R / P;
    for (int r = 0; r < P; ++r) ref_multiply_std_rowwise(A + r * ln * C, x, ln, C, y + r * ln);
    return 0;
}

/* src/multiplier_colwise.c:11-129. Strip i = columns [i*ln, +ln) packed row-major
 * (MPI_Type_vector(R, ln, C) + MPI_Pack, :15-45), x segment i (MPI_Scatter :86-95). */
int ref_colwise(const double* A, const double* x, int64_t R, int64_t C, int P, double* y) {
    if (P <= 0 || C % P != 0) return -2;
    const int64_t ln = C / P;
    double** part = (double**)malloc(sizeof(double*) * (size_t)P);
    double* strip = (double*)malloc(sizeof(double) * (size_t)(R * ln > 0 ? R * ln : 1));
    for (int p = 0; p < P; ++p) {
        part[p] = (double*)malloc(sizeof(double) * (size_t)(R > 0 ? R : 1));
        for (int64_t i = 0; i < R; ++i) memcpy(strip + i * ln, A + i * C + p * ln, sizeof(double) * (size_t)ln);
        const double* xs = x + p * ln;
        /* :107-111 scale in place, j outer / i inner */
        for (int64_t j = 0; j < ln; ++j)
            for (int64_t i = 0; i < R; ++i) strip[i * ln + j] *= xs[j];
        /* :116-122 row sums from 0.0 */
        for (int64_t i = 0; i < R; ++i) {
            double sum = 0.0;
            for (int64_t j = 0; j < ln; ++j) sum += strip[i * ln + j];
            part[p][i] = sum;
        }
    }
    ref_mpich_reduce(part, P, R); /* :124 */
    memcpy(y, part[0], sizeof(double) * (size_t)R);
    for (int p = 0; p < P; ++p) free(part[p]);
    free(part);
    free(strip);
    return 0;
}

/* src/multiplier_blockwise.c:17-210,299-306,367-368 (with 64-bit sizes and the deliberate
 * refusal of R % r != 0 or C % c != 0 that the build's planner also applies). */
int ref_blockwise(const double* A, const double* x, int64_t R, int64_t C, int P, double* y) {
    if (P <= 0 || ((uint64_t)R * (uint64_t)C) % (uint64_t)P != 0) return -2;
    int g[2] = {1, 1};
    ref_grid_shape(P, g);
    const int gr = g[0], gc = g[1];
    if (R % gr != 0 || C % gc != 0) return -2;
    const int64_t lr = R / gr, lc = C / gc;
    double* blk = (double*)malloc(sizeof(double) * (size_t)(lr * lc > 0 ? lr * lc : 1));
    double* part = (double*)malloc(sizeof(double) * (size_t)(lr > 0 ? lr : 1));
    for (int64_t i = 0; i < R; ++i) y[i] = 0.0; /* :150-154 */
    for (int src = 0; src < P; ++src) {         /* :179-207, rank order */
        const int bi = src / gc, bj = src % gc;
        for (int64_t i = 0; i < lr; ++i)
            memcpy(blk + i * lc, A + (bi * lr + i) * C + bj * lc, sizeof(double) * (size_t)lc);
        ref_multiply_std_rowwise(blk, x + bj * lc, lr, lc, part); /* :367 */
        for (int64_t j = 0; j < lr; ++j) y[bi * lr + j] += part[j]; /* :206 */
    }
    free(blk);
    free(part);
    return 0;
}

int ref_multiply(int alg, const double* A, const double* x, int64_t R, int64_t C, int P, double* y) {
    switch (alg) {
        case 0: return ref_rowwise(A, x, R, C, P, y);
        case 1: return ref_colwise(A, x, R, C, P, y);
        case 2: return ref_blockwise(A, x, R, C, P, y);
        default: return -1;
    }
}

/* ---------------------------------------------------------------- synthetic generator
 * Same spec as include/matvec_gpu.h (an input-format spec, restated independently here). */
static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

double ref_synth_value(uint64_t seed, uint64_t idx) {
    const uint64_t g = 0x9E3779B97F4A7C15ULL;
    const uint64_t s0 = mix64(seed + g);
    const uint64_t z = mix64(s0 + idx * g + g);
    const uint64_t k = (uint64_t)(((unsigned __int128)z * 10000u) >> 64);
    return (double)k / 10000.0;
}

void ref_synth_fill(double* dst, int64_t R, int64_t C, uint64_t seed) {
    for (int64_t i = 0; i < R; ++i)
        for (int64_t j = 0; j < C; ++j) dst[i * C + j] = ref_synth_value(seed, (uint64_t)(i * C + j));
}

/* rows [r0, r0+nr) x cols [c0, c0+nc) of a global matrix with C columns, packed (ld = nc) */
void ref_synth_block(double* dst, int64_t r0, int64_t nr, int64_t c0, int64_t nc, int64_t C, uint64_t seed) {
    for (int64_t i = 0; i < nr; ++i)
        for (int64_t j = 0; j < nc; ++j)
            dst[i * nc + j] = ref_synth_value(seed, (uint64_t)((r0 + i) * C + c0 + j));
}

/* ---------------------------------------------------------------- CPU baseline timing
 * The reference's timed loop (rowwise.c:135-151, colwise.c:218-233, blockwise.c:361-378)
 * with P threads standing in for P MPI ranks on one host: every iteration is
 * barrier -> t0 -> distribute (each rank copies its shard out of the root's A; root's x
 * segments likewise) -> local product -> collect on the root -> barrier -> t1, the
 * iteration time is the max over ranks, and the result is the mean over iterations.
 * Distribution is done by each rank in parallel, which is optimistic for the reference's
 * sequential root sends (so the baseline errs on the fast side). */
typedef struct {
    int alg, P, rank, iters;
    int64_t R, C;
    const double* A;
    const double* x;
    double* y;
    double** parts;   /* col: per-rank partial y; block: per-rank partial slice */
    pthread_barrier_t* bar;
    double* elapsed;  /* [iters * P] */
} tjob;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void* rank_main(void* arg) {
    tjob* j = (tjob*)arg;
    const int64_t R = j->R, C = j->C;
    const int P = j->P, rk = j->rank;
    int64_t lr = R, lc = C, r0 = 0, c0 = 0, gc = 1;
    if (j->alg == 0) { lr = R / P; r0 = rk * lr; }
    else if (j->alg == 1) { lc = C / P; c0 = rk * lc; }
    else {
        int g[2];
        ref_grid_shape(P, g);
        gc = g[1];
        lr = R / g[0]; lc = C / g[1];
        r0 = (rk / gc) * lr; c0 = (rk % gc) * lc;
    }
    double* loc = (double*)malloc(sizeof(double) * (size_t)(lr * lc > 0 ? lr * lc : 1));
    double* xs = (double*)malloc(sizeof(double) * (size_t)(lc > 0 ? lc : 1));
    double* part = j->parts[rk];
    for (int it = 0; it < j->iters; ++it) {
        pthread_barrier_wait(j->bar);
        const double t0 = now_s();
        for (int64_t i = 0; i < lr; ++i) memcpy(loc + i * lc, j->A + (r0 + i) * C + c0, sizeof(double) * (size_t)lc);
        memcpy(xs, j->x + c0, sizeof(double) * (size_t)lc);
        if (j->alg == 1) {
            for (int64_t c = 0; c < lc; ++c)
                for (int64_t i = 0; i < lr; ++i) loc[i * lc + c] *= xs[c];
            for (int64_t i = 0; i < lr; ++i) {
                double s = 0.0;
                for (int64_t c = 0; c < lc; ++c) s += loc[i * lc + c];
                part[i] = s;
            }
        } else {
            ref_multiply_std_rowwise(loc, xs, lr, lc, part);
        }
        pthread_barrier_wait(j->bar); /* partials ready: the collective */
        if (rk == 0) {
            if (j->alg == 0) {
                for (int p = 0; p < P; ++p) memcpy(j->y + p * lr, j->parts[p], sizeof(double) * (size_t)lr);
            } else if (j->alg == 1) {
                ref_mpich_reduce(j->parts, P, R);
                memcpy(j->y, j->parts[0], sizeof(double) * (size_t)R);
            } else {
                for (int64_t i = 0; i < R; ++i) j->y[i] = 0.0;
                for (int p = 0; p < P; ++p)
                    for (int64_t i = 0; i < lr; ++i) j->y[(p / gc) * lr + i] += j->parts[p][i];
            }
        }
        pthread_barrier_wait(j->bar);
        j->elapsed[it * P + rk] = now_s() - t0;
    }
    free(loc);
    free(xs);
    return NULL;
}

double ref_time_multiply(int alg, const double* A, const double* x, int64_t R, int64_t C, int P,
                         int iters, double* y) {
    if (P <= 0 || iters <= 0) return -1.0;
    if (alg == 0 && R % P) return -1.0;
    if (alg == 1 && C % P) return -1.0;
    if (alg == 2) {
        int g[2];
        ref_grid_shape(P, g);
        if (R % g[0] || C % g[1]) return -1.0;
    }
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)P);
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)P);
    tjob* jobs = (tjob*)malloc(sizeof(tjob) * (size_t)P);
    double** parts = (double**)malloc(sizeof(double*) * (size_t)P);
    double* el = (double*)calloc((size_t)iters * (size_t)P, sizeof(double));
    for (int p = 0; p < P; ++p) parts[p] = (double*)malloc(sizeof(double) * (size_t)(R > 0 ? R : 1));
    for (int p = 0; p < P; ++p) {
        jobs[p] = (tjob){alg, P, p, iters, R, C, A, x, y, parts, &bar, el};
        pthread_create(&th[p], NULL, rank_main, &jobs[p]);
    }
    for (int p = 0; p < P; ++p) pthread_join(th[p], NULL);
    double sum = 0.0;
    for (int it = 0; it < iters; ++it) {
        double mx = 0.0;
        for (int p = 0; p < P; ++p)
            if (el[it * P + p] > mx) mx = el[it * P + p];
        sum += mx; /* MPI_Reduce(MAX) per iteration, summed (rowwise.c:147-150) */
    }
    for (int p = 0; p < P; ++p) free(parts[p]);
    free(parts);
    free(el);
    free(jobs);
    free(th);
    pthread_barrier_destroy(&bar);
    return sum / iters;
}
