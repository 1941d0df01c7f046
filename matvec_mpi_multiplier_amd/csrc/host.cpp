// Host-side parts of the C-ABI: status/error text, device helpers, the synthetic generator
// on the host, and the shard planner (pure integer work, no GPU needed).
#include <ctype.h>
#include <math.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>

#include <string>

#include "common.h"

namespace mvg {

static thread_local std::string t_err;

void set_error(const std::string& msg) { t_err = msg; }
const std::string& get_error() { return t_err; }

int fail(int code, const std::string& msg) {
    t_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    t_err = std::string(what) + ": " + hipGetErrorString(e);
    return MVG_E_HIP;
}

int take_pending_error(const char* where) {
    const hipError_t e = hipGetLastError();
    if (e == hipSuccess) return MVG_OK;
    t_err = std::string(where) + ": HIP error pending from an earlier call: " + hipGetErrorString(e);
    return MVG_E_HIP;
}

// ------------------------------------------------------------------ host threads
int host_thread_count() {
    if (const char* e = getenv("MVG_THREADS")) {
        const int v = atoi(e);
        return v < 1 ? 1 : v > 64 ? 64 : v;
    }
    static const int n = [] {
        int nt = (int)std::thread::hardware_concurrency();
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof set, &set) == 0 && CPU_COUNT(&set) > 0) nt = CPU_COUNT(&set);
        // cgroup v2 quota: "<max> <period>" in cpu.max ("max" = unlimited)
        if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
            char q[32] = {0};
            long long period = 0;
            if (fscanf(f, "%31s %lld", q, &period) == 2 && period > 0 && strcmp(q, "max") != 0) {
                const long long cpus = (atoll(q) + period - 1) / period;
                if (cpus >= 1 && cpus < nt) nt = (int)cpus;
            }
            fclose(f);
        }
        return nt < 1 ? 1 : nt > 64 ? 64 : nt;
    }();
    return n;
}

}  // namespace mvg

using namespace mvg;

extern "C" {

const char* mvg_version(void) { return "matvec_gpu 0.1.0 (gfx950)"; }

const char* mvg_strerror(int code) {
    switch (code) {
        case MVG_OK: return "ok";
        case MVG_E_INVALID: return "invalid argument";
        case MVG_E_INDIVISIBLE: return "shape does not divide over the rank count";
        case MVG_E_HIP: return "HIP runtime error";
        case MVG_E_RCCL: return "RCCL error";
        case MVG_E_IO: return "I/O error";
        case MVG_E_NOMEM: return "out of memory";
        case MVG_E_STATE: return "call out of order";
        default: return "unknown error";
    }
}

const char* mvg_last_error(void) { return t_err.c_str(); }

// ------------------------------------------------------------------ planner
// get_2_most_closest_multipliers (reference src/utils.c:26-37). The reference computes
// (int)sqrt((double)p) and walks down to the first divisor; same here, with the float
// sqrt result corrected so a rounding error can never skip the true floor(sqrt(p)).
int mvg_grid_shape(int64_t p, int* gr, int* gc) {
    if (p <= 0 || !gr || !gc) return fail(MVG_E_INVALID, "mvg_grid_shape: p must be > 0");
    int64_t s = (int64_t)sqrt((double)p);
    while (s * s > p) --s;
    while ((s + 1) * (s + 1) <= p) ++s;
    for (int64_t d = s; d > 0; --d) {
        if (p % d == 0) {
            *gr = (int)d;
            *gc = (int)(p / d);
            return MVG_OK;
        }
    }
    return fail(MVG_E_INVALID, "mvg_grid_shape: unreachable");
}

// Shard arithmetic of the three drivers:
//   row-split  : local_n = R / P rows each (rowwise.c:93), rank i owns rows [i*local_n, +local_n)
//                (MPI_Scatter rank order, rowwise.c:16-37), y slice = its rows (MPI_Gather :141).
//   col-split  : local_n = C / P columns each (colwise.c:349), rank i owns strip
//                [i*local_n, +local_n) (Pack offset &matrix[i*local_n], colwise.c:37-38), x segment
//                i (MPI_Scatter :86-95), partial y over all R rows (MPI_Reduce :124).
//   block-split: (r, c) = get_2_most_closest_multipliers(P) (blockwise.c:299-302); rank
//                i*c + j owns block (i, j) of lr x lc (blockwise.c:56,71), x segment j (:79),
//                partial y slice rows [i*lr, +lr) (blockwise.c:206).
int mvg_plan_shard(int alg, int64_t R, int64_t C, int P, int rank, mvg_shard* o) {
    if (!o || R < 0 || C < 0 || P <= 0 || rank < 0 || rank >= P)
        return fail(MVG_E_INVALID, "mvg_plan_shard: bad arguments");
    memset(o, 0, sizeof(*o));
    o->alg = alg;
    o->nranks = P;
    o->rank = rank;
    o->R = R;
    o->C = C;
    char msg[256];
    switch (alg) {
        case MVG_ALG_ROWWISE: {
            // rowwise.c:72-75
            if (R % P != 0) {
                snprintf(msg, sizeof msg, "%lld mod %d = %lld. Unable to parallellize task.",
                         (long long)R, P, (long long)(R % P));
                return fail(MVG_E_INDIVISIBLE, msg);
            }
            const int64_t ln = R / P;
            o->grid_rows = P;
            o->grid_cols = 1;
            o->grid_r = rank;
            o->grid_c = 0;
            o->row_off = rank * ln;
            o->n_rows = ln;
            o->col_off = 0;
            o->n_cols = C;
            o->y_off = o->row_off;
            o->y_len = ln;
            return MVG_OK;
        }
        case MVG_ALG_COLWISE: {
            // colwise.c:151-154 checks C % P (its message prints R % P by mistake; we print
            // the quantity that was actually checked).
            if (C % P != 0) {
                snprintf(msg, sizeof msg, "%lld mod %d = %lld. Unable to parallellize task.",
                         (long long)C, P, (long long)(C % P));
                return fail(MVG_E_INDIVISIBLE, msg);
            }
            const int64_t ln = C / P;
            o->grid_rows = 1;
            o->grid_cols = P;
            o->grid_r = 0;
            o->grid_c = rank;
            o->row_off = 0;
            o->n_rows = R;
            o->col_off = rank * ln;
            o->n_cols = ln;
            o->y_off = 0;
            o->y_len = R;
            return MVG_OK;
        }
        case MVG_ALG_BLOCKWISE: {
            // blockwise.c:277-281 checks only (R*C) % P ...
            if (((uint64_t)R * (uint64_t)C) % (uint64_t)P != 0) {
                snprintf(msg, sizeof msg, "%llu mod %d = %llu. Unable to parallellize task.",
                         (unsigned long long)((uint64_t)R * (uint64_t)C), P,
                         (unsigned long long)(((uint64_t)R * (uint64_t)C) % (uint64_t)P));
                return fail(MVG_E_INDIVISIBLE, msg);
            }
            int gr = 1, gc = 1;
            mvg_grid_shape(P, &gr, &gc);
            // ... deliberate deviation: the reference then truncates R/r and C/c and silently
            // drops trailing rows/columns (SURVEY §4 bug 1); we refuse instead.
            if (R % gr != 0 || C % gc != 0) {
                snprintf(msg, sizeof msg,
                         "%lld x %lld does not split over a %d x %d grid. Unable to parallellize task.",
                         (long long)R, (long long)C, gr, gc);
                return fail(MVG_E_INDIVISIBLE, msg);
            }
            const int64_t lr = R / gr, lc = C / gc;
            o->grid_rows = gr;
            o->grid_cols = gc;
            o->grid_r = rank / gc;
            o->grid_c = rank % gc;
            o->row_off = o->grid_r * lr;
            o->n_rows = lr;
            o->col_off = o->grid_c * lc;
            o->n_cols = lc;
            o->y_off = o->row_off;
            o->y_len = lr;
            return MVG_OK;
        }
        default:
            return fail(MVG_E_INVALID, "mvg_plan_shard: unknown algorithm");
    }
}

int mvg_plan_exchange(int alg, int64_t R, int64_t C, int P, int rank, int force,
                      mvg_xstep* steps, int max_steps, int* nsteps) {
    if (!steps || !nsteps || max_steps < 0) return fail(MVG_E_INVALID, "mvg_plan_exchange: null");
    *nsteps = 0;
    mvg_shard s;
    int rc = mvg_plan_shard(alg, R, C, P, rank, &s);
    if (rc != MVG_OK) return rc;
    if (P == 1 && !force) return MVG_OK;
    mvg_xstep v[2];
    int n = 0;
    memset(v, 0, sizeof v);
    if (alg == MVG_ALG_ROWWISE || alg == MVG_ALG_COLWISE) {
        v[0].op = alg == MVG_ALG_ROWWISE ? MVG_X_GATHER : MVG_X_REDUCE;
        v[0].comm = MVG_X_WORLD;
        v[0].color = 0;
        v[0].key = rank;
        v[0].member = 1;
        v[0].root = 0;
        v[0].src = MVG_X_BUF_PART;
        v[0].dst = MVG_X_BUF_Y;
        v[0].count = s.y_len;
        n = 1;
    } else {
        const bool one_row = s.grid_rows == 1;
        v[0].op = MVG_X_REDUCE;
        v[0].comm = MVG_X_ROW;
        v[0].color = s.grid_r;
        v[0].key = s.grid_c;
        v[0].member = 1;
        v[0].root = 0;
        v[0].src = MVG_X_BUF_PART;
        v[0].dst = one_row ? MVG_X_BUF_Y : MVG_X_BUF_ROW;
        v[0].count = s.y_len;
        n = 1;
        if (!one_row) {
            v[1].op = MVG_X_GATHER;
            v[1].comm = MVG_X_COL;
            v[1].color = 0;
            v[1].key = s.grid_r;
            v[1].member = s.grid_c == 0;
            v[1].root = 0;
            v[1].src = MVG_X_BUF_ROW;
            v[1].dst = MVG_X_BUF_Y;
            v[1].count = s.y_len;
            n = 2;
        }
    }
    if (n > max_steps) return fail(MVG_E_INVALID, "mvg_plan_exchange: steps buffer too small");
    for (int i = 0; i < n; ++i) steps[i] = v[i];
    *nsteps = n;
    return MVG_OK;
}

// ------------------------------------------------------------------ synthetic (host)
double mvg_synth_value(uint64_t seed, uint64_t idx) { return synth_value(splitmix64(seed), idx); }

int mvg_synth_fill_host(double* dst, int64_t ld, int64_t m, int64_t k, int64_t row_off,
                        int64_t col_off, int64_t ncols, uint64_t seed) {
    if (m < 0 || k < 0 || ld < k || row_off < 0 || col_off < 0 || col_off + k > ncols)
        return fail(MVG_E_INVALID, "mvg_synth_fill_host: bad shape");
    if (m == 0 || k == 0) return MVG_OK;
    if (!dst) return fail(MVG_E_INVALID, "mvg_synth_fill_host: null dst");
    const uint64_t s0 = splitmix64(seed);
    parallel_for(m, [&](int64_t r0, int64_t r1) {
        for (int64_t r = r0; r < r1; ++r) {
            const uint64_t gbase = (uint64_t)(row_off + r) * (uint64_t)ncols + (uint64_t)col_off;
            double* d = dst + r * ld;
            for (int64_t c = 0; c < k; ++c) d[c] = synth_value(s0, gbase + c);
        }
    }, m * k < (1 << 20));
    return MVG_OK;
}

// ------------------------------------------------------------------ device helpers
int mvg_device_count(int* n) {
    if (!n) return fail(MVG_E_INVALID, "null");
    MVG_HIP(hipGetDeviceCount(n));
    return MVG_OK;
}
int mvg_set_device(int dev) {
    MVG_HIP(hipSetDevice(dev));
    return MVG_OK;
}
int mvg_malloc(void** p, size_t bytes) {
    if (!p) return fail(MVG_E_INVALID, "null");
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) {
        hip_fail(e, "hipMalloc");
        return MVG_E_NOMEM;
    }
    return MVG_OK;
}
int mvg_free(void* p) {
    MVG_HIP(hipFree(p));
    return MVG_OK;
}
int mvg_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream) {
    MVG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
    return MVG_OK;
}
int mvg_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream) {
    MVG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
    return MVG_OK;
}
int mvg_stream_sync(void* stream) {
    MVG_HIP(hipStreamSynchronize((hipStream_t)stream));
    return MVG_OK;
}
// ------------------------------------------------------------------ the reference's in-process call
// multiply_std_rowwise(matrix, vector, n_rows, n_cols, result) (src/matr_utils.h:4-10,
// src/matr_utils.c:86-96) on host pointers, on the calling thread's current device: A and x go
// over, the GEMV runs (exact != 0: the reference's own sequential sums, bit for bit; 0: the
// tree-summed kernel, within 1e-12), y comes back. The device buffers stay with the thread and
// grow as needed, so a loop of calls allocates once; they are released by a call with
// n_rows = n_cols = 0 and null pointers, or at process exit.
int mvg_multiply_std_rowwise(const double* matrix, const double* vector, int64_t n_rows, int64_t n_cols,
                             double* result, int exact) {
    struct Workspace {
        int dev = -1;
        double* buf = nullptr;
        size_t cap = 0;  // doubles
    };
    thread_local Workspace ws;
    if (n_rows < 0 || n_cols < 0) return fail(MVG_E_INVALID, "mvg_multiply_std_rowwise: negative size");
    if (n_rows == 0 && n_cols == 0 && !matrix && !vector && !result) {
        if (ws.buf) {
            int cur = 0;
            MVG_HIP(hipGetDevice(&cur));
            MVG_HIP(hipSetDevice(ws.dev));
            const hipError_t e = hipFree(ws.buf);
            MVG_HIP(hipSetDevice(cur));
            ws = Workspace{};
            MVG_HIP(e);
        }
        return MVG_OK;
    }
    if (n_rows == 0) return MVG_OK;
    if (!result || (n_cols > 0 && (!matrix || !vector)))
        return fail(MVG_E_INVALID, "mvg_multiply_std_rowwise: null pointer");
    int dev = 0;
    MVG_HIP(hipGetDevice(&dev));
    auto even = [](int64_t n) { return (size_t)((n + 1) & ~(int64_t)1); };  // 16-B aligned parts
    const size_t na = even(n_rows * n_cols), nx = even(n_cols), need = na + nx + even(n_rows);
    if (ws.dev != dev || ws.cap < need) {
        if (ws.buf) {
            MVG_HIP(hipSetDevice(ws.dev));
            (void)hipFree(ws.buf);
            MVG_HIP(hipSetDevice(dev));
            ws = Workspace{};
        }
        void* p = nullptr;
        if (const int rc = mvg_malloc(&p, need * sizeof(double)); rc != MVG_OK) return rc;
        ws.dev = dev, ws.buf = (double*)p, ws.cap = need;
    }
    double *dA = ws.buf, *dx = dA + na, *dy = dx + nx;
    MVG_HIP(hipMemcpyAsync(dA, matrix, (size_t)(n_rows * n_cols) * sizeof(double), hipMemcpyHostToDevice, nullptr));
    MVG_HIP(hipMemcpyAsync(dx, vector, (size_t)n_cols * sizeof(double), hipMemcpyHostToDevice, nullptr));
    const int rc = exact ? mvg_gemv_exact(dA, n_cols, dx, dy, n_rows, n_cols, nullptr)
                         : mvg_gemv(dA, n_cols, dx, dy, n_rows, n_cols, nullptr);
    if (rc != MVG_OK) return rc;
    MVG_HIP(hipMemcpyAsync(result, dy, (size_t)n_rows * sizeof(double), hipMemcpyDeviceToHost, nullptr));
    MVG_HIP(hipStreamSynchronize(nullptr));
    return MVG_OK;
}

int mvg_host_register(void* ptr, size_t bytes) {
    MVG_HIP(hipHostRegister(ptr, bytes, hipHostRegisterDefault));
    return MVG_OK;
}
// NUMA placement of host memory a GPU will pull from (the shared window of the executables):
// the pages of [p, p + bytes) are first-touched (zeroed) by threads bound to the CPUs of the
// NUMA node `device` hangs off (PCI bus id -> sysfs numa_node), so the kernel places them in
// that socket's DRAM. Placement only: when the node is unknown the caller's CPUs touch them.
int mvg_device_numa_node(int device, int* node) {
    if (!node) return fail(MVG_E_INVALID, "null");
    *node = -1;
    char bus[64] = {0};
    MVG_HIP(hipDeviceGetPCIBusId(bus, (int)sizeof bus, device));
    for (char* c = bus; *c; ++c) *c = (char)tolower(*c);
    char path[160];
    snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
    if (FILE* f = fopen(path, "r")) {
        if (fscanf(f, "%d", node) != 1) *node = -1;
        fclose(f);
    }
    return MVG_OK;
}

int mvg_host_first_touch(void* p, size_t bytes, int device) {
    if (!p || bytes == 0) return MVG_OK;
    int node = -1;
    (void)mvg_device_numa_node(device, &node);
    cpu_set_t keep, want;
    CPU_ZERO(&want);
    bool bound = false;
    if (node >= 0 && pthread_getaffinity_np(pthread_self(), sizeof keep, &keep) == 0) {
        char path[96];
        snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
        if (FILE* f = fopen(path, "r")) {
            int a = 0, b = 0;
            char sep = 0;
            while (fscanf(f, "%d", &a) == 1) {
                b = a;
                if (fscanf(f, "%c", &sep) == 1 && sep == '-') {
                    if (fscanf(f, "%d", &b) != 1) b = a;
                    if (fscanf(f, "%c", &sep) != 1) sep = 0;
                }
                for (int c = a; c <= b && c < CPU_SETSIZE; ++c)
                    if (CPU_ISSET(c, &keep)) CPU_SET(c, &want);
                if (sep != ',') break;
            }
            fclose(f);
        }
        // threads created below inherit the calling thread's mask
        bound = CPU_COUNT(&want) > 0 && pthread_setaffinity_np(pthread_self(), sizeof want, &want) == 0;
    }
    const size_t page = 1 << 21;
    const int64_t chunks = (int64_t)((bytes + page - 1) / page);
    char* base = (char*)p;
    parallel_for(chunks, [&](int64_t c0, int64_t c1) {
        const size_t b0 = (size_t)c0 * page;
        const size_t b1 = std::min(bytes, (size_t)c1 * page);
        memset(base + b0, 0, b1 - b0);
    }, bytes < (64u << 20));
    if (bound) (void)pthread_setaffinity_np(pthread_self(), sizeof keep, &keep);
    return MVG_OK;
}

int mvg_host_unregister(void* ptr) {
    MVG_HIP(hipHostUnregister(ptr));
    return MVG_OK;
}

}  // extern "C"
