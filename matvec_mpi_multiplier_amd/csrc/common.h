// Internal helpers shared by the libmatvec_gpu translation units (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string>
#include <thread>
#include <vector>

#include "../../include/matvec_gpu.h"

namespace mvg {

// Last error text for mvg_last_error(); thread-local like errno.
void set_error(const std::string& msg);
const std::string& get_error();

int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

// An error that an earlier HIP call on this thread left pending belongs to that call. Every
// public launch entry point (tree, multi-vector, exact, panels, relayout, fill, stream read)
// takes it after its argument checks (pure host logic) and before its first HIP call, and
// reports it as such — the call fails, nothing is launched — so the hipGetLastError after its
// own launch only ever sees that launch's error.
int take_pending_error(const char* where);

#define MVG_HIP(call)                                                     \
    do {                                                                  \
        hipError_t _e = (call);                                           \
        if (_e != hipSuccess) return ::mvg::hip_fail(_e, #call);          \
    } while (0)

// ----- exact exchange (gemv_exact.hip): the reference's own combine orders on the root
// MPI_Reduce(SUM) as the reference's MPICH runs it (colwise.c:124): binomial tree or, for long
// buffers, reduce-scatter + gather, by MPICH 3.3.2's own rule (gemv_exact.hip); overwrites parts
int launch_combine_mpich_reduce(double* parts, int P, int64_t n, double* y, hipStream_t s);
// gather_local_results (blockwise.c:150-207): y = ((0 + p[gi*gc]) + p[gi*gc+1]) + ... per grid row
int launch_combine_grid_rows(const double* parts, int gr, int gc, int64_t lr, double* y, hipStream_t s);

// ----- synthetic generator (spec in include/matvec_gpu.h) ---------------------------
constexpr uint64_t kGamma = 0x9E3779B97F4A7C15ULL;

__host__ __device__ inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
__host__ __device__ inline uint64_t splitmix64(uint64_t x) { return mix64(x + kGamma); }

__host__ __device__ inline uint64_t mulhi_10000(uint64_t z) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(z, 10000ULL);
#else
    return (uint64_t)(((unsigned __int128)z * 10000u) >> 64);
#endif
}

// s0 = splitmix64(seed); value = floor(splitmix64(s0 + idx*gamma) * 1e4 / 2^64) / 1e4
__host__ __device__ inline double synth_value(uint64_t s0, uint64_t idx) {
    const uint64_t z = splitmix64(s0 + idx * kGamma);
    return (double)mulhi_10000(z) / 10000.0;
}

// Host threads the library's CPU work (loader, host generator, first touch) uses: $MVG_THREADS
// if set, else the CPUs this process may actually run on — its affinity mask, capped by its
// cgroup's CPU quota (a job given 16 CPUs of a 256-CPU host sees 256 in hardware_concurrency) —
// at most 64 (host.cpp).
int host_thread_count();

// Static split of [0, n) over host_thread_count() threads. `serial` forces one thread.
template <class F>
void parallel_for(int64_t n, F&& body, bool serial = false) {
    int nt = host_thread_count();
    if (nt > n) nt = (int)(n > 0 ? n : 1);
    if (serial || nt == 1) {
        body((int64_t)0, n);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) {
        const int64_t b = n * t / nt, e = n * (t + 1) / nt;
        th.emplace_back([&body, b, e] { body(b, e); });
    }
    for (auto& t : th) t.join();
}

}  // namespace mvg
