// Communicators (RCCL over xGMI) and the distributed multiplier engine.
//
// The engine is the MI355X replacement for what the three reference drivers do around the
// local product, one algorithm per object:
//
//   ROWWISE   distribute: MPI_Scatter(rows) + MPI_Bcast(x)          rowwise.c:12-51
//             exchange  : MPI_Gather(y pieces, rank order)          rowwise.c:141
//             here      : H2D row shard (or root->peer ncclSend), ncclGather of y to rank 0
//   COLWISE   distribute: MPI_Type_vector + MPI_Pack + MPI_Send strips, MPI_Scatter(x)
//                                                                   colwise.c:11-102
//             exchange  : MPI_Reduce(SUM) of partial y              colwise.c:124
//             here      : 2-D H2D into a packed strip, ncclReduce(fp64, sum) to rank 0
//   BLOCKWISE distribute: block Pack + Send, x segment Send         blockwise.c:17-141
//             exchange  : root Recv(ANY_SOURCE) + y[(src/c)*lr+j] += partial
//                                                                   blockwise.c:144-210
//             here      : ncclReduce(sum) over each grid-row communicator to the row leader
//                         (grid column 0), then ncclGather of the r leader slices to rank 0.
//                         Fixed order: deterministic, unlike the reference's arrival order.
//
// One process may drive several devices (mvg_comm_init_all: the executables) or exactly one
// (mvg_comm_init_rank: one process per GPU under torch.distributed.run). Every collective
// is issued for all local devices inside ncclGroupStart/End, so both models share one path.
#include <dlfcn.h>
#include <rccl/rccl.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "common.h"

using namespace mvg;

namespace {

int nccl_fail(ncclResult_t r, const char* what) {
    set_error(std::string(what) + ": " + ncclGetErrorString(r));
    return MVG_E_RCCL;
}

#define MVG_NCCL(call)                                                  \
    do {                                                                \
        ncclResult_t _r = (call);                                       \
        if (_r != ncclSuccess) return nccl_fail(_r, #call);             \
    } while (0)

struct LocalRank {
    int rank = 0;
    int device = 0;
    ncclComm_t comm = nullptr;
};

}  // namespace

struct mvg_comm {
    int nranks = 0;
    std::vector<LocalRank> locals;
};

namespace {

constexpr int kRing = 8;

struct Shard {
    mvg_shard plan{};
    int device = 0;
    int rank = 0;
    ncclComm_t world = nullptr;
    // exchange schedule (mvg_plan_exchange) and the communicator each step runs on:
    // the world, or a split of it (block-split: grid-row comm, grid-column-0 leaders' comm)
    mvg_xstep steps[MVG_MAX_XSTEPS];
    int nsteps = 0;
    ncclComm_t xcomm[MVG_MAX_XSTEPS] = {};
    bool owns_xcomm[MVG_MAX_XSTEPS] = {};
    hipStream_t stream = nullptr;       // GEMV (and the root's distribution sends)
    hipStream_t copy_stream = nullptr;  // H2D staging
    hipStream_t xstream = nullptr;      // the exchange step (collectives), overlapping the next GEMV
    double* dA = nullptr;
    double* dx = nullptr;
    // exact mode, tall long-row shards: the same A in column panels (mvg_gemv_exact_panels),
    // allocated and rebuilt from dA by the second multiply after a write to dA
    double* dAp = nullptr;
    int64_t panelP = 0, pstride = 0;
    bool panels_fresh = false;
    int64_t uses = 0;  // multiplies since dA was last written
    // local product: y_len (row/block) or R (col) doubles; a ring of kRing buffers when an
    // exchange follows: multiply n writes dy_parts[n % ring] while earlier exchanges still read
    // the others
    double* dy_parts[kRing] = {};
    hipEvent_t gemv_done[kRing] = {};  // GEMV into dy_parts[b] finished
    hipEvent_t x_done[kRing] = {};     // exchange reading dy_parts[b] finished
    // chunked distribution (mvg_engine_set_overlap): row chunk c of A landed (copy_stream); the
    // next multiply runs the GEMV of chunk c behind it, while later chunks are still copying
    std::vector<hipEvent_t> chunk_ev;
    std::vector<int64_t> chunk_row;   // chunk c = rows [chunk_row[c], chunk_row[c + 1])
    hipEvent_t copy_ready = nullptr;  // s.stream's work before the copies (the last GEMV reads dA)
    bool chunks_pending = false;
    double* dy_row = nullptr;   // block-split row leader: reduced slice (lr doubles)
    double* dy = nullptr;       // rank 0: the full y (R doubles)
    double* stage[2] = {nullptr, nullptr};  // root: staging for root->peer sends (rank mode)
    double* gbuf = nullptr;     // rank 0, exact mode: every rank's partial, gathered in rank order
    size_t stage_elems = 0;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pool;
    size_t ev_used = 0;
    hipEvent_t span_t0 = nullptr, span_t1 = nullptr;  // span timing (mvg_engine_kernel_timing(-1))
};

}  // namespace

struct mvg_engine {
    int alg = 0;
    int64_t R = 0, C = 0;
    int nranks = 0;
    bool single_process = false;  // all ranks in this process
    bool always_collect = false;  // run the collectives even at nranks == 1 (tests)
    bool distributed = false;
    bool exact = false;         // bit-exact mode: mvg_gemv_exact + the reference's combine orders
    int overlap_chunks = 0;     // > 1: distribute in row chunks, each chunk's GEMV behind its copy
    int timing_every = 0;       // record kernel events on every Nth multiply (0 = off, -1 = span)
    int64_t span_multiplies = 0;  // span timing: multiplies since the span's first event (0 = none open)
    bool span_valid = true;       // no chunked distribution's copies inside the open span
    int64_t nx = 0;             // multiplies with an exchange issued so far
    bool x_pending = false;     // an exchange may still run (slot (nx - 1) % ring)
    int ring = kRing;           // ring length in use (MVG_XRING, 1 = exchange on the GEMV stream)
    int64_t multiply_calls = 0;
    double kernel_ms_sum = 0.0;
    int64_t kernel_launches = 0;
    std::vector<Shard> shards;
};

namespace {

// The exchange's device-side calls — RCCL's communicator splits and collectives, and exact
// mode's combine kernel on rank 0 — go through one interface: RCCL and the kernels on the
// devices (DeviceXOps), or a recorder that lists them in issue order (TraceXOps,
// mvg_debug_trace_exchange: the single-process G-device schedule, run on a host without GPUs).
struct XOps {
    virtual ~XOps() = default;
    virtual ncclResult_t group_start() = 0;
    virtual ncclResult_t group_end() = 0;
    virtual void set_device(int dev) = 0;
    virtual ncclResult_t split(ncclComm_t world, int color, int key, ncclComm_t* out) = 0;
    virtual ncclResult_t gather(const double* src, double* dst, size_t count, int root, ncclComm_t comm,
                                hipStream_t st) = 0;
    virtual ncclResult_t reduce(const double* src, double* dst, size_t count, int root, ncclComm_t comm,
                                hipStream_t st) = 0;
    virtual int combine(const mvg_engine* e, const Shard& s, hipStream_t st) = 0;
};

struct DeviceXOps final : XOps {
    ncclResult_t group_start() override { return ncclGroupStart(); }
    ncclResult_t group_end() override { return ncclGroupEnd(); }
    void set_device(int dev) override { (void)hipSetDevice(dev); }
    ncclResult_t split(ncclComm_t world, int color, int key, ncclComm_t* out) override {
        return ncclCommSplit(world, color, key, out, nullptr);
    }
    ncclResult_t gather(const double* src, double* dst, size_t count, int root, ncclComm_t comm,
                        hipStream_t st) override {
        return ncclGather(src, dst, count, ncclFloat64, root, comm, st);
    }
    ncclResult_t reduce(const double* src, double* dst, size_t count, int root, ncclComm_t comm,
                        hipStream_t st) override {
        return ncclReduce(src, dst, count, ncclFloat64, ncclSum, root, comm, st);
    }
    int combine(const mvg_engine* e, const Shard& s, hipStream_t st) override {
        return e->alg == MVG_ALG_COLWISE ? launch_combine_mpich_reduce(s.gbuf, e->nranks, e->R, s.dy, st)
                                         : launch_combine_grid_rows(s.gbuf, s.plan.grid_rows, s.plan.grid_cols,
                                                                    s.plan.y_len, s.dy, st);
    }
};

DeviceXOps g_device_ops;

// A shard keeps a grid-row buffer when a step of its schedule reads or writes one.
bool needs_row_buffer(const Shard& s) {
    bool need = false;
    for (int k = 0; k < s.nsteps; ++k)
        need |= s.steps[k].member && (s.steps[k].dst == MVG_X_BUF_ROW || s.steps[k].src == MVG_X_BUF_ROW);
    return need;
}

// Sub-communicators of the exchange schedule. ncclCommSplit is collective over the world, so
// every local rank calls it for every split step, inside one group per step.
int split_steps(std::vector<Shard>& shards, XOps& ops) {
    const int nsteps = shards.empty() ? 0 : shards[0].nsteps;
    for (int k = 0; k < nsteps; ++k) {
        if (shards[0].steps[k].comm == MVG_X_WORLD) {
            for (auto& s : shards) s.xcomm[k] = s.world;
            continue;
        }
        ncclResult_t r = ops.group_start();
        if (r != ncclSuccess) return nccl_fail(r, "ncclGroupStart");
        for (auto& s : shards) {
            ops.set_device(s.device);
            const mvg_xstep& st = s.steps[k];
            r = ops.split(s.world, st.member ? st.color : NCCL_SPLIT_NOCOLOR, st.key, &s.xcomm[k]);
            s.owns_xcomm[k] = true;
            if (r != ncclSuccess) break;
        }
        const ncclResult_t r2 = ops.group_end();
        if (r != ncclSuccess) return nccl_fail(r, "ncclCommSplit");
        if (r2 != ncclSuccess) return nccl_fail(r2, "ncclCommSplit group");
    }
    return MVG_OK;
}

// Exact mode's column-panel copy of a shard (s.panelP > 0), allocated when first needed if it
// fits in free HBM with 8 GiB to spare; otherwise the shard keeps the row-major exact kernels
// (panelP = 0 until exact mode is switched on again).
void alloc_panels(Shard& s) {
    const int64_t elems = s.pstride * ((s.plan.n_cols + s.panelP - 1) / s.panelP);
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess ||
        (double)elems * sizeof(double) + (double)(8ll << 30) > (double)free_b ||
        hipMalloc((void**)&s.dAp, (size_t)elems * sizeof(double)) != hipSuccess) {
        (void)hipGetLastError();
        s.dAp = nullptr;
        s.panelP = s.pstride = 0;
    }
}

bool getenv_flag(const char* name) {
    const char* v = getenv(name);
    return v && v[0] == '1';
}

struct DeviceGuard {
    int prev = 0;
    DeviceGuard() { (void)hipGetDevice(&prev); }
    ~DeviceGuard() { (void)hipSetDevice(prev); }
};

int alloc_doubles(double** p, int64_t n) {
    if (n <= 0) {
        *p = nullptr;
        return MVG_OK;
    }
    hipError_t e = hipMalloc((void**)p, (size_t)n * sizeof(double));
    if (e != hipSuccess) {
        hip_fail(e, "hipMalloc");
        return MVG_E_NOMEM;
    }
    return MVG_OK;
}

void free_shard(Shard& s) {
    (void)hipSetDevice(s.device);
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    if (s.copy_stream) (void)hipStreamSynchronize(s.copy_stream);
    if (s.xstream) (void)hipStreamSynchronize(s.xstream);
    for (double* p : {s.dA, s.dAp, s.dx, s.dy_row, s.dy, s.stage[0], s.stage[1], s.gbuf})
        if (p) (void)hipFree(p);
    for (int b = 0; b < kRing; ++b) {
        if (s.dy_parts[b]) (void)hipFree(s.dy_parts[b]);
        if (s.gemv_done[b]) (void)hipEventDestroy(s.gemv_done[b]);
        if (s.x_done[b]) (void)hipEventDestroy(s.x_done[b]);
    }
    for (auto& ev : s.ev_pool) {
        (void)hipEventDestroy(ev.first);
        (void)hipEventDestroy(ev.second);
    }
    for (hipEvent_t ev : s.chunk_ev) (void)hipEventDestroy(ev);
    if (s.span_t0) (void)hipEventDestroy(s.span_t0);
    if (s.span_t1) (void)hipEventDestroy(s.span_t1);
    if (s.copy_ready) (void)hipEventDestroy(s.copy_ready);
    s.ev_pool.clear();
    for (int k = 0; k < MVG_MAX_XSTEPS; ++k)
        if (s.owns_xcomm[k] && s.xcomm[k]) (void)ncclCommDestroy(s.xcomm[k]);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    if (s.copy_stream) (void)hipStreamDestroy(s.copy_stream);
    if (s.xstream) (void)hipStreamDestroy(s.xstream);
    s = Shard{};
}

// 2-D host -> device copy of a shard region into a packed device buffer (pitch = cols).
int h2d_region(double* dst, const double* host, int64_t ld_host, int64_t rows, int64_t cols,
               hipStream_t s) {
    if (rows == 0 || cols == 0) return MVG_OK;
    if (cols == ld_host) {
        MVG_HIP(hipMemcpyAsync(dst, host, (size_t)(rows * cols) * sizeof(double),
                               hipMemcpyHostToDevice, s));
    } else {
        MVG_HIP(hipMemcpy2DAsync(dst, (size_t)cols * sizeof(double), host,
                                 (size_t)ld_host * sizeof(double), (size_t)cols * sizeof(double),
                                 (size_t)rows, hipMemcpyHostToDevice, s));
    }
    return MVG_OK;
}

// A chunked distribution's copies into dA / dx may still be running on the copy stream. Any
// other writer of those buffers on s.stream (the synthetic fill, the root-send receives) first
// waits for the last of them (the copy stream runs in order), and the pending chunks are dropped:
// the next multiply then reads the whole new shard.
int drain_chunks(Shard& s) {
    if (s.chunks_pending && !s.chunk_ev.empty()) {
        const size_t last = s.chunk_row.size() >= 2 ? s.chunk_row.size() - 2 : 0;
        MVG_HIP(hipStreamWaitEvent(s.stream, s.chunk_ev[last], 0));
    }
    s.chunks_pending = false;
    return MVG_OK;
}

// x segment that a shard needs: full x (row), strip segment (col), block column segment.
inline int64_t x_off(const mvg_shard& p) { return p.col_off; }
inline int64_t x_len(const mvg_shard& p) { return p.n_cols; }

// Every local device pulls its own shard (and x segment) from host memory that holds the
// whole A and x, over its own PCIe link, concurrently (one stream per device). With
// overlap_chunks > 1 the shard's rows go over in that many chunks on the copy stream, each
// followed by an event, and the next multiply runs each chunk's GEMV as soon as the chunk has
// landed: only the last chunk's GEMV is left after the transfer.
int distribute_direct(mvg_engine* e, const double* A, const double* x) {
    const int64_t C = e->C;
    for (auto& s : e->shards) {
        MVG_HIP(hipSetDevice(s.device));
        const mvg_shard& p = s.plan;
        const int nch = e->overlap_chunks > 1 && p.n_rows >= 2 * (int64_t)e->overlap_chunks ? e->overlap_chunks : 0;
        if (int rc0 = drain_chunks(s); rc0 != MVG_OK) return rc0;
        if (nch == 0) {
            int rc = h2d_region(s.dA, A + p.row_off * C + p.col_off, C, p.n_rows, p.n_cols, s.stream);
            if (rc != MVG_OK) return rc;
            rc = h2d_region(s.dx, x + x_off(p), x_len(p), 1, x_len(p), s.stream);
            if (rc != MVG_OK) return rc;
            continue;
        }
        if (!s.copy_ready) MVG_HIP(hipEventCreateWithFlags(&s.copy_ready, hipEventDisableTiming));
        while ((int)s.chunk_ev.size() < nch) {
            hipEvent_t ev;
            MVG_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            s.chunk_ev.push_back(ev);
        }
        // the copies overwrite dA and dx, which the GEMV last queued on s.stream still reads
        MVG_HIP(hipEventRecord(s.copy_ready, s.stream));
        MVG_HIP(hipStreamWaitEvent(s.copy_stream, s.copy_ready, 0));
        int rc = h2d_region(s.dx, x + x_off(p), x_len(p), 1, x_len(p), s.copy_stream);
        if (rc != MVG_OK) return rc;
        s.chunk_row.assign(nch + 1, 0);
        for (int c = 0; c <= nch; ++c) s.chunk_row[c] = p.n_rows * c / nch;
        for (int c = 0; c < nch; ++c) {
            const int64_t r0 = s.chunk_row[c], r1 = s.chunk_row[c + 1];
            rc = h2d_region(s.dA + r0 * p.n_cols, A + (p.row_off + r0) * C + p.col_off, C, r1 - r0, p.n_cols,
                            s.copy_stream);
            if (rc != MVG_OK) return rc;
            MVG_HIP(hipEventRecord(s.chunk_ev[c], s.copy_stream));
        }
        s.chunks_pending = true;
    }
    return MVG_OK;
}

// The exchange step from the shared schedule (mvg_plan_exchange): one group per step, every
// local member issuing its call in it. A failing call inside the group still closes the group
// before the error is reported.
int exchange_plan(mvg_engine* e, int b, bool serial, XOps& ops) {
    const int nsteps = e->shards[0].nsteps;
    for (int k = 0; k < nsteps; ++k) {
        MVG_NCCL(ops.group_start());
        ncclResult_t r = ncclSuccess;
        const char* what = "";
        for (auto& s : e->shards) {
            const mvg_xstep& st = s.steps[k];
            if (!st.member) continue;
            ops.set_device(s.device);
            double* bufs[3] = {s.dy_parts[b], s.dy_row, s.dy};
            const double* src = bufs[st.src];
            double* dst = bufs[st.dst];
            if (!dst) dst = s.dy_parts[b];  // recvbuff is only written on the root
            hipStream_t stream = serial ? s.stream : s.xstream;
            if (st.op == MVG_X_GATHER) {
                r = ops.gather(src, dst, (size_t)st.count, st.root, s.xcomm[k], stream);
                what = "ncclGather";
            } else {
                r = ops.reduce(src, dst, (size_t)st.count, st.root, s.xcomm[k], stream);
                what = "ncclReduce";
            }
            if (r != ncclSuccess) break;
        }
        const ncclResult_t r2 = ops.group_end();
        if (r != ncclSuccess) return nccl_fail(r, what);
        if (r2 != ncclSuccess) return nccl_fail(r2, "ncclGroupEnd");
    }
    return MVG_OK;
}

// Exact mode (mvg_engine_set_exact): every partial gathered to rank 0 in rank order, then added
// there in the reference's order.
int exchange_exact(mvg_engine* e, int b, bool serial, XOps& ops) {
    const int64_t count = e->alg == MVG_ALG_COLWISE ? e->R : e->shards[0].plan.y_len;
    MVG_NCCL(ops.group_start());
    ncclResult_t r = ncclSuccess;
    for (auto& s : e->shards) {
        ops.set_device(s.device);
        // recvbuff is only written on the root
        r = ops.gather(s.dy_parts[b], s.rank == 0 ? s.gbuf : s.dy_parts[b], (size_t)count, 0, s.world,
                       serial ? s.stream : s.xstream);
        if (r != ncclSuccess) break;
    }
    const ncclResult_t r2 = ops.group_end();
    if (r != ncclSuccess) return nccl_fail(r, "ncclGather (exact)");
    if (r2 != ncclSuccess) return nccl_fail(r2, "ncclGroupEnd");
    for (auto& s : e->shards) {
        if (s.rank != 0) continue;
        ops.set_device(s.device);
        const int rc = ops.combine(e, s, serial ? s.stream : s.xstream);
        if (rc != MVG_OK) return rc;
    }
    return MVG_OK;
}

// The recorder behind mvg_debug_trace_exchange. Communicators and buffers are stand-in handles
// the trace hands out; every call is listed with the group it was issued in.
struct TraceXOps final : XOps {
    std::vector<mvg_xcall> calls;
    int group = -1, depth = 0, device = 0;
    std::vector<std::pair<uintptr_t, int>> comm_step;  // handle -> group that created it (-1 world)
    std::vector<std::pair<uintptr_t, std::pair<int, int>>> buffers;  // address -> (rank, MVG_X_BUF_*)
    uintptr_t next_comm = 0x7e0000;

    int comm_of(ncclComm_t c) const {
        for (auto& kv : comm_step)
            if (kv.first == (uintptr_t)c) return kv.second;
        return -2;
    }
    int buf_of(const double* p) const {
        for (auto& kv : buffers)
            if (kv.first == (uintptr_t)p) return kv.second.second;
        return -1;
    }
    mvg_xcall base(int kind) const {
        mvg_xcall c{};
        c.group = depth > 0 ? group : -1;  // -1: outside any group (the combine kernel)
        c.kind = kind;
        c.rank = device;  // the trace's devices are its ranks
        c.comm = -1;
        c.color = c.key = c.root = -1;
        c.src = c.dst = -1;
        return c;
    }
    ncclResult_t group_start() override {
        if (depth++ == 0) ++group;
        return ncclSuccess;
    }
    ncclResult_t group_end() override {
        if (depth > 0) --depth;
        return ncclSuccess;
    }
    void set_device(int dev) override { device = dev; }
    ncclResult_t split(ncclComm_t world, int color, int key, ncclComm_t* out) override {
        mvg_xcall c = base(MVG_XCALL_SPLIT);
        c.comm = comm_of(world);
        c.color = color == NCCL_SPLIT_NOCOLOR ? -1 : color;
        c.key = key;
        calls.push_back(c);
        *out = (ncclComm_t)(next_comm++);
        comm_step.push_back({(uintptr_t)*out, group});
        return ncclSuccess;
    }
    ncclResult_t coll(int kind, const double* src, double* dst, size_t count, int root, ncclComm_t comm) {
        mvg_xcall c = base(kind);
        c.comm = comm_of(comm);
        c.root = root;
        c.count = (int64_t)count;
        c.src = buf_of(src);
        c.dst = buf_of(dst);
        calls.push_back(c);
        return ncclSuccess;
    }
    ncclResult_t gather(const double* src, double* dst, size_t count, int root, ncclComm_t comm,
                        hipStream_t) override {
        return coll(MVG_XCALL_GATHER, src, dst, count, root, comm);
    }
    ncclResult_t reduce(const double* src, double* dst, size_t count, int root, ncclComm_t comm,
                        hipStream_t) override {
        return coll(MVG_XCALL_REDUCE, src, dst, count, root, comm);
    }
    int combine(const mvg_engine* e, const Shard& s, hipStream_t) override {
        mvg_xcall c = base(MVG_XCALL_COMBINE);
        c.count = (e->alg == MVG_ALG_COLWISE ? e->R : s.plan.y_len) * e->nranks;
        c.src = buf_of(s.gbuf);
        c.dst = buf_of(s.dy);
        calls.push_back(c);
        return MVG_OK;
    }
};

}  // namespace

extern "C" {

// ------------------------------------------------------------------ bound runtimes
int mvg_runtime_versions(int* rccl_version, int* hip_runtime_version) {
    if (rccl_version) MVG_NCCL(ncclGetVersion(rccl_version));
    if (hip_runtime_version) MVG_HIP(hipRuntimeGetVersion(hip_runtime_version));
    return MVG_OK;
}

// The object that defines one symbol of each runtime as this library resolved it: the copy the
// process actually calls, whichever loaded first with the same soname.
const char* mvg_runtime_path(int which) {
    const void* sym = which == 0 ? (const void*)&hipGetDeviceCount
                    : which == 1 ? (const void*)&ncclGetVersion : nullptr;
    Dl_info info;
    if (!sym || dladdr(sym, &info) == 0 || !info.dli_fname) return "";
    return info.dli_fname;
}

// ------------------------------------------------------------------ communicators
int mvg_comm_unique_id(unsigned char out[MVG_UNIQUE_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == MVG_UNIQUE_ID_BYTES, "ncclUniqueId size");
    if (!out) return fail(MVG_E_INVALID, "null");
    ncclUniqueId id;
    MVG_NCCL(ncclGetUniqueId(&id));
    memcpy(out, &id, sizeof id);
    return MVG_OK;
}

int mvg_comm_init_all(mvg_comm** out, int ndev, const int* devlist) {
    if (!out || ndev <= 0) return fail(MVG_E_INVALID, "mvg_comm_init_all: bad arguments");
    *out = nullptr;
    std::vector<int> devs(ndev);
    for (int i = 0; i < ndev; ++i) devs[i] = devlist ? devlist[i] : i;
    std::vector<ncclComm_t> comms(ndev, nullptr);
    DeviceGuard g;
    // One device needs no collective (the exchange plan is empty), so RCCL is not initialised
    // at all — no bootstrap cost, no RCCL banner on the executables' stdout — unless
    // MVG_ALWAYS_COLLECT=1 asks for the collectives to run anyway.
    const char* ac = getenv("MVG_ALWAYS_COLLECT");
    if (ndev > 1 || (ac && ac[0] == '1')) {
        MVG_NCCL(ncclCommInitAll(comms.data(), ndev, devs.data()));
    } else {
        MVG_HIP(hipSetDevice(devs[0]));
    }
    mvg_comm* c = new mvg_comm;
    c->nranks = ndev;
    for (int i = 0; i < ndev; ++i) c->locals.push_back(LocalRank{i, devs[i], comms[i]});
    *out = c;
    return MVG_OK;
}

int mvg_comm_init_rank(mvg_comm** out, const unsigned char id[MVG_UNIQUE_ID_BYTES], int nranks,
                       int rank, int device) {
    if (!out || !id || nranks <= 0 || rank < 0 || rank >= nranks)
        return fail(MVG_E_INVALID, "mvg_comm_init_rank: bad arguments");
    *out = nullptr;
    MVG_HIP(hipSetDevice(device));
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof uid);
    ncclComm_t comm;
    MVG_NCCL(ncclCommInitRank(&comm, nranks, uid, rank));
    mvg_comm* c = new mvg_comm;
    c->nranks = nranks;
    c->locals.push_back(LocalRank{rank, device, comm});
    *out = c;
    return MVG_OK;
}

int mvg_comm_size(const mvg_comm* c, int* n) {
    if (!c || !n) return fail(MVG_E_INVALID, "null");
    *n = c->nranks;
    return MVG_OK;
}
int mvg_comm_local_count(const mvg_comm* c, int* n) {
    if (!c || !n) return fail(MVG_E_INVALID, "null");
    *n = (int)c->locals.size();
    return MVG_OK;
}
int mvg_comm_local_rank(const mvg_comm* c, int i, int* rank, int* device) {
    if (!c || i < 0 || i >= (int)c->locals.size()) return fail(MVG_E_INVALID, "bad local index");
    if (rank) *rank = c->locals[i].rank;
    if (device) *device = c->locals[i].device;
    return MVG_OK;
}
int mvg_comm_destroy(mvg_comm* c) {
    if (!c) return MVG_OK;
    DeviceGuard g;
    for (auto& l : c->locals) {
        (void)hipSetDevice(l.device);
        if (l.comm) (void)ncclCommDestroy(l.comm);
    }
    delete c;
    return MVG_OK;
}

// ------------------------------------------------------------------ engine
int mvg_engine_destroy(mvg_engine* e) {
    if (!e) return MVG_OK;
    DeviceGuard g;
    for (auto& s : e->shards) free_shard(s);
    delete e;
    return MVG_OK;
}

int mvg_engine_create(mvg_engine** out, int alg, int64_t R, int64_t C, mvg_comm* comm) {
    if (!out || !comm || R < 0 || C < 0) return fail(MVG_E_INVALID, "mvg_engine_create: bad arguments");
    *out = nullptr;
    // Validate the whole grid first (the reference's root-only divisibility check).
    mvg_shard probe;
    int rc = mvg_plan_shard(alg, R, C, comm->nranks, 0, &probe);
    if (rc != MVG_OK) return rc;

    DeviceGuard g;
    mvg_engine* e = new mvg_engine;
    e->alg = alg;
    e->R = R;
    e->C = C;
    e->nranks = comm->nranks;
    e->single_process = (int)comm->locals.size() == comm->nranks;
    const char* ac = getenv("MVG_ALWAYS_COLLECT");
    // forced collectives need an RCCL communicator (a one-device comm made without the
    // variable has none)
    e->always_collect = ac && ac[0] == '1' && comm->locals[0].comm != nullptr;
    if (const char* v = getenv("MVG_XRING")) e->ring = std::max(1, std::min(kRing, atoi(v)));
    const char* ex = getenv("MVG_EXACT");
    const bool want_exact = ex && ex[0] == '1';
    if (const char* ov = getenv("MVG_OVERLAP")) e->overlap_chunks = std::max(0, atoi(ov));

    e->shards.resize(comm->locals.size());
    auto bail = [&](int code) {
        mvg_engine_destroy(e);
        return code;
    };
    for (size_t i = 0; i < comm->locals.size(); ++i) {
        Shard& s = e->shards[i];
        const LocalRank& l = comm->locals[i];
        s.device = l.device;
        s.rank = l.rank;
        s.world = l.comm;
        if ((rc = mvg_plan_shard(alg, R, C, comm->nranks, l.rank, &s.plan)) != MVG_OK) return bail(rc);
        if (hipSetDevice(s.device) != hipSuccess) return bail(fail(MVG_E_HIP, "hipSetDevice"));
        if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&s.copy_stream, hipStreamNonBlocking) != hipSuccess)
            return bail(fail(MVG_E_HIP, "hipStreamCreate"));
        const mvg_shard& p = s.plan;
        if ((rc = alloc_doubles(&s.dA, p.n_rows * p.n_cols)) != MVG_OK) return bail(rc);
        if ((rc = alloc_doubles(&s.dx, x_len(p))) != MVG_OK) return bail(rc);
        const int64_t part = alg == MVG_ALG_COLWISE ? R : p.y_len;
        if ((rc = mvg_plan_exchange(alg, R, C, comm->nranks, l.rank, e->always_collect, s.steps,
                                    MVG_MAX_XSTEPS, &s.nsteps)) != MVG_OK)
            return bail(rc);
        if ((rc = alloc_doubles(&s.dy_parts[0], part)) != MVG_OK) return bail(rc);
        if (s.nsteps > 0) {
            for (int b = 1; b < e->ring; ++b)
                if ((rc = alloc_doubles(&s.dy_parts[b], part)) != MVG_OK) return bail(rc);
            if (hipStreamCreateWithFlags(&s.xstream, hipStreamNonBlocking) != hipSuccess)
                return bail(fail(MVG_E_HIP, "hipStreamCreate"));
            for (int b = 0; b < e->ring; ++b)
                // GEMV -> exchange kernel on the same device: no system-scope fence needed (the
                // marker with one cost ~2 us of idle GPU per multiply); exchange -> collect's
                // D2H copy keeps the default (host-visible) fence
                if (hipEventCreateWithFlags(&s.gemv_done[b], hipEventDisableTiming | hipEventDisableSystemFence) !=
                        hipSuccess ||
                    hipEventCreateWithFlags(&s.x_done[b], hipEventDisableTiming) != hipSuccess)
                    return bail(fail(MVG_E_HIP, "hipEventCreate"));
        }
        if (needs_row_buffer(s))
            if ((rc = alloc_doubles(&s.dy_row, p.y_len)) != MVG_OK) return bail(rc);
        if (l.rank == 0)
            if ((rc = alloc_doubles(&s.dy, R)) != MVG_OK) return bail(rc);
        // Warm the device before any timed loop: first-touch every buffer (the first H2D into
        // never-touched HBM ran at 11 GB/s instead of 56, profiles/r01/e2e_small/numa_h2d.jsonl) and launch the
        // shard's GEMV once (loads its code object and any split-K workspace). These one-time
        // costs are the GPU runtime's analogue of MPI_Init; without this they landed in the
        // executables' first timed iteration (+0.1 ms on the mean at 600 x 600).
        auto zero = [&](double* p, int64_t n) {
            return p && n > 0 ? hipMemsetAsync(p, 0, (size_t)n * sizeof(double), s.stream) : hipSuccess;
        };
        hipError_t ze = zero(s.dA, p.n_rows * p.n_cols);
        if (ze == hipSuccess) ze = zero(s.dx, x_len(p));
        for (int b = 0; b < kRing && ze == hipSuccess; ++b) ze = zero(s.dy_parts[b], part);
        if (ze == hipSuccess) ze = zero(s.dy_row, p.y_len);
        if (ze == hipSuccess) ze = zero(s.dy, R);
        if (ze != hipSuccess) return bail(hip_fail(ze, "hipMemsetAsync"));
        if ((rc = mvg_gemv(s.dA, p.n_cols, s.dx, s.dy_parts[0], p.n_rows, p.n_cols, s.stream)) != MVG_OK)
            return bail(rc);
        // ... and one page-locked H2D into A's buffer and D2H out of y's, as large as those
        // transfers will be up to 4 MiB, on each stream that distributes or collects. The
        // runtime brings its large-copy path up on the first such transfer of the process:
        // 8.2 ms once (tools/probes/first_copy.py: 2.88 MB from any page-locked buffer, 8.2 ms first,
        // 66 us after; 512-B copies do not trigger it), which otherwise landed in the
        // executables' first timed iteration (bin/multiplier_rowwise 600 600, MVG_ITER_LOG).
        const int64_t a_elems = std::min<int64_t>(p.n_rows * p.n_cols, 1 << 19);
        const int64_t y_elems = std::min<int64_t>(part, 1 << 19);
        const size_t wbytes = (size_t)std::max<int64_t>({a_elems, y_elems, 1}) * sizeof(double);
        double* pinned = nullptr;
        if (hipHostMalloc((void**)&pinned, wbytes, hipHostMallocDefault) != hipSuccess)
            return bail(fail(MVG_E_NOMEM, "hipHostMalloc (engine warm-up)"));
        memset(pinned, 0, wbytes);
        hipError_t we = hipSuccess;
        for (hipStream_t st : {s.stream, s.copy_stream}) {
            if (we == hipSuccess && a_elems > 0)
                we = hipMemcpyAsync(s.dA, pinned, (size_t)a_elems * sizeof(double), hipMemcpyHostToDevice, st);
            if (we == hipSuccess && y_elems > 0)
                we = hipMemcpyAsync(pinned, s.dy_parts[0], (size_t)y_elems * sizeof(double), hipMemcpyDeviceToHost, st);
            if (we == hipSuccess) we = hipStreamSynchronize(st);
        }
        (void)hipHostFree(pinned);
        if (we != hipSuccess) return bail(hip_fail(we, "engine warm-up"));
    }
    if ((rc = split_steps(e->shards, g_device_ops)) != MVG_OK) return bail(rc);
    if (want_exact && (rc = mvg_engine_set_exact(e, 1)) != MVG_OK) return bail(rc);
    *out = e;
    return MVG_OK;
}

// Exact mode: the local products come from mvg_gemv_exact (the reference's sequential sums) and
// the exchange reproduces the reference's combine order instead of RCCL's: every rank's partial
// is gathered to rank 0 in rank order (one ncclGather) and a small kernel there adds them as
// the reference does — MPI_Reduce's tree as MPICH picks it for the column split (colwise.c:124), the
// grid row's blocks into a zeroed y in rank order for the block split (blockwise.c:150-207).
// The row split's gather is a copy and stays as it is. y is then bit-identical to the
// reference's (block split: to its result for rank-order arrival, which is every arrival order
// when the grid has at most two columns).
int mvg_engine_set_exact(mvg_engine* e, int on) {
    if (!e) return fail(MVG_E_INVALID, "null engine");
    int rc = mvg_engine_sync(e);
    if (rc != MVG_OK) return rc;
    e->exact = on != 0;
    DeviceGuard g;
    for (auto& s : e->shards) {
        MVG_HIP(hipSetDevice(s.device));
        if (!e->exact) {
            if (s.dAp) (void)hipFree(s.dAp);
            s.dAp = nullptr;
            s.panelP = s.pstride = 0;
            continue;
        }
        if (s.dAp || getenv_flag("MVG_NO_PANELS")) continue;
        // the panel copy where it pays (mvg_exact_panel_width); allocated by the multiply that
        // first needs it (alloc_panels), so a distribute-per-multiply loop never holds one
        s.panelP = mvg_exact_panel_width(s.plan.n_rows, s.plan.n_cols);
        s.pstride = s.plan.n_rows * s.panelP;
        s.panels_fresh = false;
    }
    if (!e->exact || e->alg == MVG_ALG_ROWWISE) return MVG_OK;
    for (auto& s : e->shards) {
        if (s.rank != 0 || s.nsteps == 0 || s.gbuf) continue;
        MVG_HIP(hipSetDevice(s.device));
        const int64_t part = e->alg == MVG_ALG_COLWISE ? e->R : s.plan.y_len;
        if ((rc = alloc_doubles(&s.gbuf, part * e->nranks)) != MVG_OK) return rc;
    }
    return MVG_OK;
}

int mvg_engine_exact_panels(const mvg_engine* e, int i, int64_t* P) {
    if (!e || !P || i < 0 || i >= (int)e->shards.size()) return fail(MVG_E_INVALID, "bad index");
    *P = e->exact && e->shards[i].dAp ? e->shards[i].panelP : 0;
    return MVG_OK;
}

int mvg_engine_exact(const mvg_engine* e, int* on) {
    if (!e || !on) return fail(MVG_E_INVALID, "null");
    *on = e->exact ? 1 : 0;
    return MVG_OK;
}

int mvg_engine_set_overlap(mvg_engine* e, int chunks) {
    if (!e || chunks < 0) return fail(MVG_E_INVALID, "mvg_engine_set_overlap: bad arguments");
    int rc = mvg_engine_sync(e);
    if (rc != MVG_OK) return rc;
    e->overlap_chunks = chunks;
    return MVG_OK;
}

int mvg_engine_shard(const mvg_engine* e, int i, mvg_shard* out) {
    if (!e || !out || i < 0 || i >= (int)e->shards.size()) return fail(MVG_E_INVALID, "bad index");
    *out = e->shards[i].plan;
    return MVG_OK;
}

int mvg_engine_stream(const mvg_engine* e, int i, void** stream) {
    if (!e || !stream || i < 0 || i >= (int)e->shards.size()) return fail(MVG_E_INVALID, "bad index");
    *stream = (void*)e->shards[i].stream;
    return MVG_OK;
}

// A write of the shard (distribution, synthetic fill) while a kernel-timing span is open would
// land on the GEMV stream between the span's events: the span no longer times GEMVs alone.
static void void_open_span(mvg_engine* e) {
    if (e->timing_every == -1 && e->span_multiplies > 0) e->span_valid = false;
}

int mvg_engine_fill_synth(mvg_engine* e, uint64_t seed_a, uint64_t seed_x) {
    if (!e) return fail(MVG_E_INVALID, "null engine");
    void_open_span(e);
    DeviceGuard g;
    int rc;
    for (auto& s : e->shards) {
        s.panels_fresh = false;
        s.uses = 0;
        MVG_HIP(hipSetDevice(s.device));
        if ((rc = drain_chunks(s)) != MVG_OK) return rc;
        const mvg_shard& p = s.plan;
        if ((rc = mvg_synth_fill_device(s.dA, p.n_cols, p.n_rows, p.n_cols, p.row_off, p.col_off,
                                        e->C, seed_a, s.stream)) != MVG_OK)
            return rc;
        if ((rc = mvg_synth_fill_device(s.dx, x_len(p), 1, x_len(p), 0, x_off(p), e->C, seed_x,
                                        s.stream)) != MVG_OK)
            return rc;
    }
    for (auto& s : e->shards) {
        MVG_HIP(hipSetDevice(s.device));
        MVG_HIP(hipStreamSynchronize(s.stream));
    }
    e->distributed = true;
    return MVG_OK;
}

// Root (rank 0's process) holds A and x in host memory, as in every reference driver.
// Single-process: each device pulls its own shard over its own PCIe link, concurrently.
// One process per GPU: rank 0 stages each peer's shard through two device buffers and
// ncclSend's it over xGMI (the reference's sequential root Send loop, colwise.c:33-57),
// overlapping the next chunk's H2D with the current chunk's send.
int mvg_engine_distribute(mvg_engine* e, const double* A, const double* x) {
    if (!e) return fail(MVG_E_INVALID, "null engine");
    void_open_span(e);
    DeviceGuard g;
    const int64_t C = e->C;
    Shard* root = nullptr;
    for (auto& s : e->shards)
        if (s.rank == 0) root = &s;
    if (root && (!x || (!A && e->R * C > 0))) return fail(MVG_E_INVALID, "root needs A and x");
    for (auto& s : e->shards) s.panels_fresh = false, s.uses = 0;

    if (e->single_process) {
        int rc = distribute_direct(e, A, x);
        if (rc != MVG_OK) return rc;
    } else {
        // exactly one local shard
        Shard& s = e->shards[0];
        MVG_HIP(hipSetDevice(s.device));
        // the root-send form always lands whole shards on s.stream, after any chunked copies
        if (int rc0 = drain_chunks(s); rc0 != MVG_OK) return rc0;
        // the sends/recvs below use the world communicator on s.stream: order them after any
        // exchange still running on s.xstream (one communicator, one order of operations)
        if (e->x_pending) MVG_HIP(hipStreamWaitEvent(s.stream, s.x_done[(e->nx - 1) % e->ring], 0));
        if (s.rank == 0) {
            const int64_t chunk_bytes = 256ll << 20;
            if (!s.stage[0]) {
                s.stage_elems = (size_t)(chunk_bytes / (int64_t)sizeof(double));
                int rc;
                if ((rc = alloc_doubles(&s.stage[0], (int64_t)s.stage_elems)) != MVG_OK) return rc;
                if ((rc = alloc_doubles(&s.stage[1], (int64_t)s.stage_elems)) != MVG_OK) return rc;
            }
            // sent[b] starts recorded on s.stream, behind the previous GEMV (which reads dA, dx)
            // and the exchange wait above: every copy_stream write below is ordered after those
            hipEvent_t copied[2], sent[2];
            for (int b = 0; b < 2; ++b) {
                MVG_HIP(hipEventCreateWithFlags(&copied[b], hipEventDisableTiming));
                MVG_HIP(hipEventCreateWithFlags(&sent[b], hipEventDisableTiming));
                MVG_HIP(hipEventRecord(sent[b], s.stream));
            }
            // the own shard's copy into dA/dx needs that order even when no peer piece is sent
            // (every peer shard empty); waiting on the initial record keeps it overlapping the
            // last peer sends
            hipEvent_t ready;
            MVG_HIP(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
            MVG_HIP(hipEventRecord(ready, s.stream));
            int buf = 0;
            for (int peer = 1; peer < e->nranks; ++peer) {
                mvg_shard p;
                int rc = mvg_plan_shard(e->alg, e->R, C, e->nranks, peer, &p);
                if (rc != MVG_OK) return rc;
                // x segment first, then A rows in chunks
                struct Piece { const double* src; int64_t ld, rows, cols; };
                std::vector<Piece> pieces;
                pieces.push_back({x + x_off(p), x_len(p), 1, x_len(p)});
                const int64_t rows_per = p.n_cols > 0
                    ? std::max<int64_t>(1, (int64_t)s.stage_elems / p.n_cols) : p.n_rows;
                for (int64_t r0 = 0; r0 < p.n_rows; r0 += rows_per)
                    pieces.push_back({A + (p.row_off + r0) * C + p.col_off, C,
                                      std::min(rows_per, p.n_rows - r0), p.n_cols});
                for (const Piece& pc : pieces) {
                    const int64_t n = pc.rows * pc.cols;
                    if (n == 0) continue;
                    if (n > (int64_t)s.stage_elems) return fail(MVG_E_INVALID, "row larger than staging");
                    MVG_HIP(hipStreamWaitEvent(s.copy_stream, sent[buf], 0));
                    if ((rc = h2d_region(s.stage[buf], pc.src, pc.ld, pc.rows, pc.cols, s.copy_stream)) != MVG_OK)
                        return rc;
                    MVG_HIP(hipEventRecord(copied[buf], s.copy_stream));
                    MVG_HIP(hipStreamWaitEvent(s.stream, copied[buf], 0));
                    MVG_NCCL(ncclSend(s.stage[buf], (size_t)n, ncclFloat64, peer, s.world, s.stream));
                    MVG_HIP(hipEventRecord(sent[buf], s.stream));
                    buf ^= 1;
                }
            }
            // own shard last (MPI_Pack of the root's own strip comes last too, colwise.c:61-69)
            const mvg_shard& p = s.plan;
            MVG_HIP(hipStreamWaitEvent(s.copy_stream, ready, 0));
            (void)hipEventDestroy(ready);
            int rc = h2d_region(s.dA, A + p.row_off * C + p.col_off, C, p.n_rows, p.n_cols, s.copy_stream);
            if (rc != MVG_OK) return rc;
            if ((rc = h2d_region(s.dx, x + x_off(p), x_len(p), 1, x_len(p), s.copy_stream)) != MVG_OK) return rc;
            MVG_HIP(hipEventRecord(copied[0], s.copy_stream));
            MVG_HIP(hipStreamWaitEvent(s.stream, copied[0], 0));
            for (int b = 0; b < 2; ++b) {
                (void)hipEventDestroy(copied[b]);
                (void)hipEventDestroy(sent[b]);
            }
        } else {
            const mvg_shard& p = s.plan;
            if (x_len(p) > 0)
                MVG_NCCL(ncclRecv(s.dx, (size_t)x_len(p), ncclFloat64, 0, s.world, s.stream));
            const int64_t rows_per = p.n_cols > 0
                ? std::max<int64_t>(1, (int64_t)((256ll << 20) / (int64_t)sizeof(double)) / p.n_cols)
                : p.n_rows;
            for (int64_t r0 = 0; r0 < p.n_rows; r0 += rows_per) {
                const int64_t n = std::min(rows_per, p.n_rows - r0) * p.n_cols;
                if (n == 0) continue;
                MVG_NCCL(ncclRecv(s.dA + r0 * p.n_cols, (size_t)n, ncclFloat64, 0, s.world, s.stream));
            }
        }
    }
    e->distributed = true;
    return MVG_OK;
}

int mvg_engine_distribute_shared(mvg_engine* e, const double* A, const double* x) {
    if (!e) return fail(MVG_E_INVALID, "null engine");
    if (!x || (!A && e->R * e->C > 0)) return fail(MVG_E_INVALID, "every rank needs the shared A and x");
    void_open_span(e);
    for (auto& s : e->shards) s.panels_fresh = false, s.uses = 0;
    DeviceGuard g;
    int rc = distribute_direct(e, A, x);
    if (rc != MVG_OK) return rc;
    e->distributed = true;
    return MVG_OK;
}

int mvg_engine_kernel_timing(mvg_engine* e, int enable) {
    if (!e) return fail(MVG_E_INVALID, "null engine");
    int rc = mvg_engine_sync(e);
    if (rc != MVG_OK) return rc;
    e->timing_every = enable > 0 ? enable : enable == -1 ? -1 : 0;
    e->span_multiplies = 0;
    e->span_valid = true;
    e->multiply_calls = 0;
    e->kernel_ms_sum = 0.0;
    e->kernel_launches = 0;
    return MVG_OK;
}

int mvg_engine_multiply(mvg_engine* e) {
    if (!e) return fail(MVG_E_INVALID, "null engine");
    if (!e->distributed) return fail(MVG_E_STATE, "mvg_engine_multiply before distribute/fill");
    DeviceGuard g;
    const int nsteps = e->shards[0].nsteps;
    const bool solo = nsteps == 0;  // P == 1: the product goes straight into y
    bool chunked = false;  // a chunked distribution is pending: the GEMVs wait on copies, not timed
    for (auto& s : e->shards) chunked |= s.chunks_pending;
    const bool timed = e->timing_every > 0 && (e->multiply_calls++ % e->timing_every) == 0 && !chunked;
    // span timing: one event before the first GEMV of the span, one at the next sync, no marker
    // between the GEMVs in between (a timing marker costs the stream ~6 us around the kernel it
    // brackets, profiles/r05/t5c); a chunked distribution's copies inside the span void it
    const bool span_open = e->timing_every == -1 && e->span_multiplies == 0 && !chunked;
    if (e->timing_every == -1) {
        if (chunked) e->span_valid = false;
        ++e->span_multiplies;
    }
    const bool serial = e->ring == 1;
    const int b = solo ? 0 : (int)(e->nx % e->ring);
    // The GEMV writes dy_parts[b]; the exchange that last read it was multiply nx - ring's. The
    // GEMV stream waits once per ring, on the latest exchange (nx - 1): every slot is then free
    // for the next `ring` GEMVs (the exchange stream runs in order), so one cross-stream wait is
    // paid per ring instead of per multiply (measured: a wait per multiply cost more than the
    // overlap saved at world size 1).
    int wait_slot = -1;
    if (!solo && !serial && e->x_pending && b == 0) wait_slot = (int)((e->nx - 1) % e->ring);
    // 1) local product on every device
    for (auto& s : e->shards) {
        MVG_HIP(hipSetDevice(s.device));
        const mvg_shard& p = s.plan;
        if (wait_slot >= 0) MVG_HIP(hipStreamWaitEvent(s.stream, s.x_done[wait_slot], 0));
        double* out = solo ? s.dy : s.dy_parts[b];
        // exact mode's panel copy of A, rebuilt from dA by the second multiply after a write:
        // the rebuild moves the shard twice through HBM (about ten multiplies' worth of the
        // panels' gain), so a distribution that is multiplied once (the reference's timed loop:
        // distribute + multiply per iteration) never pays for it, and repeated multiplies of
        // the same A (device-resident) run on panels from the second one on
        if (e->exact && s.panelP && !s.panels_fresh && s.uses >= 1 && !s.chunks_pending) {
            if (!s.dAp) alloc_panels(s);
            if (s.dAp) {
                int rc = mvg_panel_relayout(s.dA, p.n_cols, p.n_rows, p.n_cols, s.dAp, s.pstride, s.panelP, s.stream);
                if (rc != MVG_OK) return rc;
                s.panels_fresh = true;
                // a relayout after the span's first event would be counted as GEMV time
                if (e->timing_every == -1 && !span_open) e->span_valid = false;
            }
        }
        const bool panels = e->exact && s.dAp && s.panels_fresh;
        ++s.uses;
        if (span_open) {
            if (!s.span_t0) MVG_HIP(hipEventCreate(&s.span_t0));
            if (!s.span_t1) MVG_HIP(hipEventCreate(&s.span_t1));
            MVG_HIP(hipEventRecord(s.span_t0, s.stream));
        }
        hipEvent_t t0 = nullptr, t1 = nullptr;
        if (timed) {
            if (s.ev_used == s.ev_pool.size()) {
                hipEvent_t a, b;
                MVG_HIP(hipEventCreate(&a));
                MVG_HIP(hipEventCreate(&b));
                s.ev_pool.emplace_back(a, b);
            }
            t0 = s.ev_pool[s.ev_used].first;
            t1 = s.ev_pool[s.ev_used].second;
            ++s.ev_used;
            MVG_HIP(hipEventRecord(t0, s.stream));
        }
        auto gemv = [&](int64_t r0, int64_t rows) {
            if (panels)
                return mvg_gemv_exact_panels(s.dAp + r0 * s.panelP, s.pstride, s.panelP, s.dx, out + r0, rows,
                                             p.n_cols, 0, s.stream);
            return e->exact ? mvg_gemv_exact(s.dA + r0 * p.n_cols, p.n_cols, s.dx, out + r0, rows, p.n_cols, s.stream)
                            : mvg_gemv(s.dA + r0 * p.n_cols, p.n_cols, s.dx, out + r0, rows, p.n_cols, s.stream);
        };
        int rc = MVG_OK;
        if (s.chunks_pending) {
            // row chunks are independent products: each runs once its rows have landed
            for (size_t c = 0; c + 1 < s.chunk_row.size() && rc == MVG_OK; ++c) {
                MVG_HIP(hipStreamWaitEvent(s.stream, s.chunk_ev[c], 0));
                rc = gemv(s.chunk_row[c], s.chunk_row[c + 1] - s.chunk_row[c]);
            }
            s.chunks_pending = false;
        } else {
            rc = gemv(0, p.n_rows);
        }
        if (rc != MVG_OK) return rc;
        if (timed) MVG_HIP(hipEventRecord(t1, s.stream));
        if (!solo && !serial) {
            MVG_HIP(hipEventRecord(s.gemv_done[b], s.stream));
            MVG_HIP(hipStreamWaitEvent(s.xstream, s.gemv_done[b], 0));
        }
    }
    if (solo) return MVG_OK;
    // 2) the exchange step on the exchange stream, overlapping the next multiply's GEMV
    const int rc_x = e->exact && e->alg != MVG_ALG_ROWWISE ? exchange_exact(e, b, serial, g_device_ops)
                                                            : exchange_plan(e, b, serial, g_device_ops);
    if (rc_x != MVG_OK) return rc_x;
    for (auto& s : e->shards) {
        MVG_HIP(hipSetDevice(s.device));
        if (!serial) MVG_HIP(hipEventRecord(s.x_done[b], s.xstream));
    }
    e->x_pending = !serial;
    ++e->nx;
    return MVG_OK;
}

int mvg_engine_sync(mvg_engine* e) {
    if (!e) return fail(MVG_E_INVALID, "null engine");
    DeviceGuard g;
    const bool span = e->timing_every == -1 && e->span_multiplies > 0;
    for (auto& s : e->shards) {
        MVG_HIP(hipSetDevice(s.device));
        if (span && s.span_t1) MVG_HIP(hipEventRecord(s.span_t1, s.stream));
        MVG_HIP(hipStreamSynchronize(s.copy_stream));
        MVG_HIP(hipStreamSynchronize(s.stream));
        if (s.xstream) MVG_HIP(hipStreamSynchronize(s.xstream));
    }
    e->x_pending = false;
    if (span) {
        // the span's GEMV time per multiply: first GEMV's start to the stream's end, max over
        // the local devices (the GEMV stream holds nothing else at one rank per process; with an
        // exchange it also holds the once-per-ring waits on the exchange stream)
        float worst = 0.f;
        for (auto& s : e->shards) {
            if (!s.span_t0 || !s.span_t1) continue;
            float ms = 0.f;
            MVG_HIP(hipEventElapsedTime(&ms, s.span_t0, s.span_t1));
            worst = std::max(worst, ms);
        }
        if (e->span_valid) {
            e->kernel_ms_sum += worst;
            e->kernel_launches += e->span_multiplies;
        }
        e->span_multiplies = 0;
        e->span_valid = true;
    }
    if (e->timing_every > 0) {
        // per timed multiply call: max over local devices, then summed
        size_t n = e->shards.empty() ? 0 : e->shards[0].ev_used;
        for (size_t k = 0; k < n; ++k) {
            float worst = 0.f;
            for (auto& s : e->shards) {
                if (k >= s.ev_used) continue;
                float ms = 0.f;
                MVG_HIP(hipEventElapsedTime(&ms, s.ev_pool[k].first, s.ev_pool[k].second));
                worst = std::max(worst, ms);
            }
            e->kernel_ms_sum += worst;
            ++e->kernel_launches;
        }
    }
    for (auto& s : e->shards) s.ev_used = 0;
    return MVG_OK;
}

int mvg_engine_kernel_ms(mvg_engine* e, double* avg_ms, int64_t* launches) {
    if (!e || !avg_ms) return fail(MVG_E_INVALID, "null");
    int rc = mvg_engine_sync(e);
    if (rc != MVG_OK) return rc;
    *avg_ms = e->kernel_launches ? e->kernel_ms_sum / (double)e->kernel_launches : 0.0;
    if (launches) *launches = e->kernel_launches;
    return MVG_OK;
}

int mvg_engine_collect(mvg_engine* e, double* y) {
    if (!e) return fail(MVG_E_INVALID, "null engine");
    DeviceGuard g;
    for (auto& s : e->shards) {
        if (s.rank != 0) continue;
        if (!y) return fail(MVG_E_INVALID, "root needs a y buffer");
        MVG_HIP(hipSetDevice(s.device));
        if (e->x_pending)  // y is complete once the last exchange is
            MVG_HIP(hipStreamWaitEvent(s.stream, s.x_done[(e->nx - 1) % e->ring], 0));
        if (e->R > 0)
            MVG_HIP(hipMemcpyAsync(y, s.dy, (size_t)e->R * sizeof(double), hipMemcpyDeviceToHost, s.stream));
        MVG_HIP(hipStreamSynchronize(s.stream));
    }
    return MVG_OK;
}

// The single-process G-device exchange (the executables' MVG_NGPUS=G form) without devices:
// the shards the engine would create over G local devices (the same planner, the same buffer
// choices), their communicator splits and one multiply's exchange, issued through the recorder
// instead of RCCL (split_steps, exchange_plan / exchange_exact: the engine's own code).
int mvg_debug_trace_exchange(int alg, int64_t R, int64_t C, int ndev, int exact, mvg_xcall* calls, int max_calls,
                             int* ncalls) {
    if (!calls || !ncalls || ndev <= 0 || max_calls < 0) return fail(MVG_E_INVALID, "mvg_debug_trace_exchange: bad arguments");
    *ncalls = 0;
    mvg_shard probe;
    int rc = mvg_plan_shard(alg, R, C, ndev, 0, &probe);
    if (rc != MVG_OK) return rc;
    mvg_engine e;
    e.alg = alg;
    e.R = R;
    e.C = C;
    e.nranks = ndev;
    e.single_process = true;
    e.exact = exact != 0;
    e.shards.resize(ndev);
    TraceXOps ops;
    auto fake = [&](int r, int id) {
        const uintptr_t a = ((uintptr_t)(r + 1) << 24) + ((uintptr_t)(id + 1) << 16);
        ops.buffers.push_back({a, {r, id}});
        return (double*)a;
    };
    for (int r = 0; r < ndev; ++r) {
        Shard& s = e.shards[r];
        s.device = r;
        s.rank = r;
        s.world = (ncclComm_t)((uintptr_t)0x7d0000 + r);
        ops.comm_step.push_back({(uintptr_t)s.world, -1});
        if ((rc = mvg_plan_shard(alg, R, C, ndev, r, &s.plan)) != MVG_OK) return rc;
        if ((rc = mvg_plan_exchange(alg, R, C, ndev, r, 0, s.steps, MVG_MAX_XSTEPS, &s.nsteps)) != MVG_OK) return rc;
        s.dy_parts[0] = fake(r, MVG_X_BUF_PART);
        if (needs_row_buffer(s)) s.dy_row = fake(r, MVG_X_BUF_ROW);
        if (r == 0) s.dy = fake(r, MVG_X_BUF_Y);
        if (e.exact && alg != MVG_ALG_ROWWISE && r == 0 && s.nsteps > 0) s.gbuf = fake(r, MVG_X_BUF_GATHERED);
    }
    if ((rc = split_steps(e.shards, ops)) != MVG_OK) return rc;
    if (e.shards[0].nsteps > 0) {
        rc = e.exact && alg != MVG_ALG_ROWWISE ? exchange_exact(&e, 0, false, ops) : exchange_plan(&e, 0, false, ops);
        if (rc != MVG_OK) return rc;
    }
    if ((int)ops.calls.size() > max_calls) return fail(MVG_E_INVALID, "mvg_debug_trace_exchange: calls buffer too small");
    for (size_t i = 0; i < ops.calls.size(); ++i) calls[i] = ops.calls[i];
    *ncalls = (int)ops.calls.size();
    return MVG_OK;
}

}  // extern "C"
