/* oracle/cpu_ref.h — TEST INFRASTRUCTURE ONLY (see cpu_ref.c header). */
#ifndef MVG_ORACLE_CPU_REF_H
#define MVG_ORACLE_CPU_REF_H
#include <stdint.h>

void ref_multiply_std_rowwise(const double* matrix, const double* vector, int64_t n_rows,
                              int64_t n_cols, double* result);
void ref_grid_shape(int64_t number, int* dividers);
int64_t sqrt_floor(int64_t n);
void ref_mpich_reduce(double** bufs, int P, int64_t n);
int ref_rowwise(const double* A, const double* x, int64_t R, int64_t C, int P, double* y);
int ref_colwise(const double* A, const double* x, int64_t R, int64_t C, int P, double* y);
int ref_blockwise(const double* A, const double* x, int64_t R, int64_t C, int P, double* y);
int ref_multiply(int alg, const double* A, const double* x, int64_t R, int64_t C, int P, double* y);
double ref_synth_value(uint64_t seed, uint64_t idx);
void ref_synth_fill(double* dst, int64_t R, int64_t C, uint64_t seed);
void ref_synth_block(double* dst, int64_t r0, int64_t nr, int64_t c0, int64_t nc, int64_t C, uint64_t seed);
double ref_time_multiply(int alg, const double* A, const double* x, int64_t R, int64_t C, int P,
                         int iters, double* y);

#endif
