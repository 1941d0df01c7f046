// Read-only calibration of the bit-exact kernels' memory pattern (development tool, not part of
// the product): how fast can one MI355X read a row-major M x K fp64 matrix when every wave walks
// R whole rows from column 0 to K in 128-B (or 256-B) segments per row, as gemv_seq_hop does —
// and does capping the resident waves (a sliding window over the rows, the tree kernel's access
// order) with deeper prefetch per row read faster than all rows at once?
//   hipcc --offload-arch=gfx950 -O3 tools/micro/window_read.hip -o /tmp/window_read
//   /tmp/window_read [M] [K]
// One JSON line per (lanes per row, segments in flight, waves per CU cap).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef double dbl2 __attribute__((ext_vector_type(2)));

// L lanes per row (64 / L rows per wave), lane c reads 16 B at column 2c of each L*2-column
// segment; U segments in flight per row; every row read from column 0 to K in order.
template <int L, int U>
__global__ __launch_bounds__(64) void rows_read(const double* __restrict__ A, int64_t lda, int64_t M, int64_t K,
                                                double* sink) {
    extern __shared__ double cap[];  // sized at launch only to cap residency
    constexpr int S = 2 * L;         // columns per segment
    const int lane = threadIdx.x;
    const int64_t row = (int64_t)blockIdx.x * (64 / L) + lane / L;
    const int64_t rr = row < M ? row : M - 1;
    const dbl2* p = reinterpret_cast<const dbl2*>(A + rr * lda + 2 * (lane % L));
    const int64_t nseg = K / S;
    dbl2 v[U];
    dbl2 acc = {0.0, 0.0};
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + (int64_t)(u < nseg ? u : 0) * L);
    int64_t s = U;
    for (; s + U <= nseg; s += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            acc += v[u];
            v[u] = __builtin_nontemporal_load(p + (s + u) * L);
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
    for (; s < nseg; ++s) acc += __builtin_nontemporal_load(p + s * L);
    if (acc.x == -1.0 && acc.y == -2.0) {
        cap[lane] = acc.x;
        sink[lane] = cap[lane ^ 1];
    }
}

// the ideal sliding window: all workgroups sweep memory front to back in 1-KiB wave chunks
__global__ __launch_bounds__(256) void seq_read(const dbl2* __restrict__ s, int64_t n2, double* sink) {
    const int64_t nthreads = (int64_t)gridDim.x * 256;
    dbl2 acc = {0.0, 0.0};
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + nthreads * 7 < n2; i += nthreads * 8) {
        dbl2 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(s + i + nthreads * u);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; i < n2; i += nthreads) acc += s[i];
    if (acc.x == -1.0 && acc.y == -2.0) sink[threadIdx.x] = acc.x;
}

template <int L, int U>
static void run(const double* A, int64_t M, int64_t K, double* sink, int cap_waves, hipEvent_t e0, hipEvent_t e1) {
    const size_t lds = cap_waves >= 32 ? 0 : (size_t)(160 * 1024 / cap_waves) & ~(size_t)1023;
    const int64_t grid = (M + 64 / L - 1) / (64 / L);
    auto launch = [&] { hipLaunchKernelGGL((rows_read<L, U>), dim3(grid), dim3(64), lds, 0, A, K, M, K, sink); };
    launch();
    float best = 1e30f, tot = 0.f;
    const int reps = 5, per = 10;
    for (int r = 0; r < reps; ++r) {
        hipEventRecord(e0);
        for (int i = 0; i < per; ++i) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms / per < best ? ms / per : best;
        tot += ms / per;
    }
    const double bytes = 8.0 * (double)M * (double)K;
    printf("{\"kernel\": \"rows_read\", \"lanes_per_row\": %d, \"rows_per_wave\": %d, \"segments_in_flight\": %d, "
           "\"bytes_in_flight_per_row\": %d, \"waves_per_cu_cap\": %d, \"M\": %ld, \"K\": %ld, \"best_us\": %.2f, "
           "\"mean_us\": %.2f, \"TBps_best\": %.3f, \"err\": \"%s\"}\n",
           L, 64 / L, U, U * L * 16, cap_waves, (long)M, (long)K, best * 1e3, tot / reps * 1e3, bytes / (best * 1e-3) / 1e12,
           hipGetErrorString(hipGetLastError()));
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int64_t M = argc > 1 ? atol(argv[1]) : 16384;
    const int64_t K = argc > 2 ? atol(argv[2]) : 16384;
    double *A, *sink;
    hipMalloc(&A, (size_t)(M * K) * sizeof(double));
    hipMalloc(&sink, 4096);
    hipMemset(A, 0, (size_t)(M * K) * sizeof(double));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    {  // contiguous sweep, the sliding-window ideal
        const int64_t n2 = M * K / 2;
        auto launch = [&] { hipLaunchKernelGGL(seq_read, dim3(8192), dim3(256), 0, 0, (const dbl2*)A, n2, sink); };
        launch();
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            hipEventRecord(e0);
            for (int i = 0; i < 10; ++i) launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms / 10 < best ? ms / 10 : best;
        }
        printf("{\"kernel\": \"seq_read\", \"M\": %ld, \"K\": %ld, \"best_us\": %.2f, \"TBps_best\": %.3f}\n", (long)M,
               (long)K, best * 1e3, 8.0 * M * K / (best * 1e-3) / 1e12);
    }
    // the exact kernel's pattern (8 lanes x 16 B per row, 16 segments in flight, all rows at once)
    // and sliding windows: fewer resident waves, deeper prefetch per row
    for (int cap : {32, 8, 4, 2}) {
        run<8, 16>(A, M, K, sink, cap, e0, e1);
        run<8, 32>(A, M, K, sink, cap, e0, e1);
        run<8, 64>(A, M, K, sink, cap, e0, e1);
        run<16, 16>(A, M, K, sink, cap, e0, e1);
        run<16, 32>(A, M, K, sink, cap, e0, e1);
    }
    hipFree(A);
    hipFree(sink);
    return 0;
}
