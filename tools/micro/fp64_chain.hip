// Dependent fp64 add chain latency on one wave (development microbenchmark): how long the
// bit-exact kernel's per-row chain of rounded adds must take at minimum.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/micro/fp64_chain.hip -o fp64_chain
#include <hip/hip_runtime.h>
#include <stdio.h>
#pragma clang fp contract(off)

// chain: s = s + p[j % 16] with the products already in registers (pure add latency)
__global__ void add_chain(double* out, int n, double seed) {
    double p[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) p[i] = seed * (i + threadIdx.x + 1);
    double s = 0.0;
    for (int j = 0; j < n; j += 16) {
#pragma unroll
        for (int i = 0; i < 16; ++i) s = s + p[i];
    }
    out[threadIdx.x] = s;
}

// chain with the multiply inside: s = s + a[i] * x[i] (products independent of s)
__global__ void muladd_chain(double* out, int n, double seed) {
    double a[16], x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        a[i] = seed * (i + threadIdx.x + 1);
        x[i] = seed / (i + 3);
    }
    double s = 0.0;
    for (int j = 0; j < n; j += 16) {
#pragma unroll
        for (int i = 0; i < 16; ++i) s = s + a[i] * x[i];
    }
    out[threadIdx.x] = s;
}

int main() {
    double* d;
    hipMalloc(&d, 64 * sizeof(double));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int n = 1 << 22;
    for (int k = 0; k < 2; ++k) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            if (k == 0)
                hipLaunchKernelGGL(add_chain, dim3(1), dim3(64), 0, 0, d, n, 1e-3);
            else
                hipLaunchKernelGGL(muladd_chain, dim3(1), dim3(64), 0, 0, d, n, 1e-3);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep) printf("{\"chain\": \"%s\", \"steps\": %d, \"ns_per_step\": %.3f}\n", k ? "mul+add" : "add", n,
                            ms * 1e6 / n);
        }
    }
    return 0;
}
