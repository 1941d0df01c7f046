// Calibration microkernels (development tool, not part of the product): how fast can one MI355X
// read a large buffer once, by access order?
//   seq_read<UNR>    : grid-stride over 1-KiB wave chunks in address order — all workgroups
//                      together sweep memory front to back (the ideal sliding window);
//   range_read<UNR>  : every wave reads its own contiguous range (n / waves), the pattern of
//                      the product's mvg_stream_read and of the exact forms' all-rows-at-once
//                      stream.
// Both: 16-B non-temporal loads, UNR loads in flight per lane, sums kept live.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef double dbl2 __attribute__((ext_vector_type(2)));

template <int UNR>
__global__ __launch_bounds__(256) void seq_read(const dbl2* __restrict__ s, int64_t n2, double* sink) {
    const int64_t nthreads = (int64_t)gridDim.x * 256;
    dbl2 acc = {0.0, 0.0};
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + nthreads * (UNR - 1) < n2; i += nthreads * UNR) {
        dbl2 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) v[u] = __builtin_nontemporal_load(s + i + nthreads * u);
#pragma unroll
        for (int u = 0; u < UNR; ++u) acc += v[u];
    }
    for (; i < n2; i += nthreads) acc += s[i];
    if (acc.x == -1.0 && acc.y == -2.0) sink[threadIdx.x] = acc.x;
}

template <int UNR>
__global__ __launch_bounds__(256) void range_read(const dbl2* __restrict__ s, int64_t n2, double* sink) {
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    const int lane = threadIdx.x & 63;
    const int64_t per = (n2 + nwaves - 1) / nwaves;
    const int64_t b = wave * per;
    const int64_t e = b + per < n2 ? b + per : n2;
    dbl2 acc = {0.0, 0.0};
    int64_t i = b + lane;
    for (; i + 64 * (UNR - 1) < e; i += 64 * UNR) {
        dbl2 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) v[u] = __builtin_nontemporal_load(s + i + 64 * u);
#pragma unroll
        for (int u = 0; u < UNR; ++u) acc += v[u];
    }
    for (; i < e; i += 64) acc += s[i];
    if (acc.x == -1.0 && acc.y == -2.0) sink[threadIdx.x] = acc.x;
}

extern "C" int read_kernel(int kind, int unr, int blocks, const double* src, int64_t n, double* sink, void* stream) {
    if (n & 1 || ((uintptr_t)src & 15) || blocks <= 0) return -1;
    const dbl2* s = reinterpret_cast<const dbl2*>(src);
    hipStream_t st = (hipStream_t)stream;
#define L(K, U) hipLaunchKernelGGL((K<U>), dim3(blocks), dim3(256), 0, st, s, n / 2, sink)
    if (kind == 0 && unr == 4) L(seq_read, 4);
    else if (kind == 0 && unr == 8) L(seq_read, 8);
    else if (kind == 0 && unr == 16) L(seq_read, 16);
    else if (kind == 1 && unr == 4) L(range_read, 4);
    else if (kind == 1 && unr == 8) L(range_read, 8);
    else return -1;
#undef L
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
