// What the HIP runtime returns when a launch asks for more dynamic LDS than a gfx950 CU has
// (160 KiB), and whether a stale error from an earlier call is visible to hipPeekAtLastError
// before the launch. Decides which error codes the exact dispatch's fallback may treat as a
// refused reservation (gemv_exact.hip). Nothing is launched that could run: the kernel body is
// empty and the oversized launches are expected to be refused before dispatch.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void empty_kernel(int* p) {
    extern __shared__ int lds[];
    if (p && threadIdx.x == 0) p[blockIdx.x] = lds[0] * 0;
}

static void try_launch(size_t lds_bytes, int threads) {
    int* d = nullptr;
    (void)hipMalloc(&d, 4096 * sizeof(int));
    hipLaunchKernelGGL(empty_kernel, dim3(64), dim3(threads), lds_bytes, 0, d);
    hipError_t launch = hipGetLastError();
    hipError_t sync = hipDeviceSynchronize();
    printf("lds %zu B threads %d: launch %d (%s), sync %d (%s)\n", lds_bytes, threads, (int)launch,
           hipGetErrorName(launch), (int)sync, hipGetErrorName(sync));
    (void)hipFree(d);
}

int main() {
    int dev = 0, max_lds = 0, max_optin = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev);
    (void)hipDeviceGetAttribute(&max_optin, hipDeviceAttributeSharedMemPerBlockOptin, dev);
    printf("max shared per block %d, optin %d\n", max_lds, max_optin);
    try_launch(96 * 1024, 512);
    try_launch(160 * 1024, 512);
    try_launch(160 * 1024 + 8, 512);
    try_launch(256 * 1024, 512);
    // a stale error from an earlier call: visible to peek, cleared by get
    hipError_t bad = hipSetDevice(1 << 20);
    hipError_t peek = hipPeekAtLastError();
    hipError_t got = hipGetLastError();
    hipError_t after = hipGetLastError();
    printf("stale: set %d (%s) peek %d get %d after %d\n", (int)bad, hipGetErrorName(bad), (int)peek, (int)got,
           (int)after);
    try_launch(96 * 1024, 512);
    return 0;
}
