// Experiment (development tool, not part of the product): the chain-hopping exact GEMV over a
// column-panel device layout of A.
//
// Hypothesis. Every exact form streams all M rows at once (each row's sequential chain is too
// slow for a sliding window of rows), so at any moment it reads M scattered 128-B pieces, one per
// row, 2 GiB apart end to end at config 2 — the access pattern of a plain streaming read of
// thousands of separate ranges, which runs at the same rate (309 us at 16384^2 against the tree
// kernel's 294; profiles/r02/sweep_exact15_stream_cal.jsonl). With A stored as column panels —
// panel p holds columns [p*P, p*P + P) of every row, rows P doubles apart, panels M*P doubles
// apart — the same all-rows-at-once chain order reads one compact, contiguous M*P*8-byte region
// at a time: a sliding window again, now over panels. The layout is the engine's to choose (its
// H2D of each shard can write panels with one 2-D copy per panel); the arithmetic and its order
// are unchanged, so y stays bit-identical to the row-major exact kernel.
//
// hop_panel<L, W, U>: L lanes per row, W columns per lane per segment, U segments in flight,
// exactly as gemv_seq_hop (csrc/gemv_exact.hip) without the head/tail machinery: K % P == 0,
// P % (L*W) == 0, P a power of two, 16-B aligned A and x.
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

typedef double dbl2x __attribute__((ext_vector_type(2)));

template <int L, bool FWD>
__device__ __forceinline__ double hop(double v) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    constexpr int kCtrl = L <= 16 ? (FWD ? 0x111 : 0x101) : (FWD ? 0x138 : 0x130);
    const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)b, kCtrl, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), kCtrl, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

template <int L, int W, bool FWD>
__device__ __forceinline__ double hop_segment(double sum, const dbl2x (&a)[W / 2], const dbl2x (&xv)[W / 2]) {
    double p[W];
#pragma unroll
    for (int v = 0; v < W / 2; ++v) p[2 * v] = a[v].x * xv[v].x, p[2 * v + 1] = a[v].y * xv[v].y;
#pragma unroll
    for (int t = 0; t < L; ++t) {
#pragma unroll
        for (int j = 0; j < W; ++j) sum = sum + p[j];
        if (t + 1 < L) sum = hop<L, FWD>(sum);
    }
    return sum;
}

template <int V, bool NT>
__device__ __forceinline__ void load_run(const double* p, dbl2x (&d)[V]) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
        if constexpr (NT)
            d[v] = __builtin_nontemporal_load(reinterpret_cast<const dbl2x*>(p) + v);
        else
            d[v] = reinterpret_cast<const dbl2x*>(p)[v];
    }
}

// lp = log2(P); segment g of row r lives at A + (gS >> lp) * M * P + r * P + (gS & (P - 1))
template <int L, int W, int U>
__global__ __launch_bounds__(64) void hop_panel(const double* __restrict__ A, int64_t M, int64_t K, int lp,
                                                const double* __restrict__ x, double* __restrict__ y) {
    constexpr int R = 64 / L, S = L * W, V = W / 2;
    const int lane = threadIdx.x;
    const int c = lane % L;
    const int64_t row = (int64_t)blockIdx.x * R + lane / L;
    const int64_t rr = row < M ? row : M - 1;
    const int64_t P = 1ll << lp;
    const double* arow = A + rr * P;
    const int64_t pstride = M * P;
    const int off[2] = {c * W, (L - 1 - c) * W};
    auto seg = [&](int64_t g) { return arow + ((g * S) >> lp) * pstride + ((g * S) & (P - 1)); };
    const int64_t nseg = K / S;
    double sum = 0.0;
    dbl2x a[U][V], xv[U][V];
#pragma unroll
    for (int i = 0; i < U; ++i) {
        const int64_t g = i < nseg ? i : nseg - 1;
        load_run<V, true>(seg(g) + off[i & 1], a[i]);
        load_run<V, false>(x + g * S + off[i & 1], xv[i]);
        __builtin_amdgcn_sched_barrier(0);
    }
    int64_t base = 0;
    for (; base + U <= nseg; base += U) {
#pragma unroll
        for (int i = 0; i < U; ++i) {
            sum = (i & 1) ? hop_segment<L, W, false>(sum, a[i], xv[i]) : hop_segment<L, W, true>(sum, a[i], xv[i]);
            __builtin_amdgcn_sched_barrier(0);
            const int64_t g = base + i + U < nseg ? base + i + U : nseg - 1;
            load_run<V, true>(seg(g) + off[i & 1], a[i]);
            load_run<V, false>(x + g * S + off[i & 1], xv[i]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#pragma unroll
    for (int i = 0; i < U; ++i)
        if (base + i < nseg)
            sum = (i & 1) ? hop_segment<L, W, false>(sum, a[i], xv[i]) : hop_segment<L, W, true>(sum, a[i], xv[i]);
    const int holder = (nseg & 1) ? L - 1 : 0;
    if (c == holder && row < M) y[row] = sum;
}

typedef void (*panel_fn)(const double*, int64_t, int64_t, int, const double*, double*);
struct PanelVariant { const char* name; panel_fn fn; int lanes, cols; };
static const PanelVariant kPanel[] = {
    {"panel_l8_w2_u16", hop_panel<8, 2, 16>, 8, 2},
    {"panel_l8_w2_u24", hop_panel<8, 2, 24>, 8, 2},
    {"panel_l8_w2_u8", hop_panel<8, 2, 8>, 8, 2},
    {"panel_l16_w2_u16", hop_panel<16, 2, 16>, 16, 2},
};
static const int kNumPanel = (int)(sizeof(kPanel) / sizeof(kPanel[0]));

extern "C" {
int panel_variant_count(void) { return kNumPanel; }
const char* panel_variant_name(int v) { return v >= 0 && v < kNumPanel ? kPanel[v].name : "invalid"; }

// 0 = launched; -1 = shape/operands outside the experiment's assumptions
int panel_hop(const double* A, int64_t M, int64_t K, int64_t P, const double* x, double* y, int v, void* stream) {
    if (v < 0 || v >= kNumPanel || M <= 0 || K <= 0 || P <= 0 || (P & (P - 1)) || K % P) return -1;
    const int S = kPanel[v].lanes * kPanel[v].cols;
    if (P % S || ((uintptr_t)A % 16) || ((uintptr_t)x % 16)) return -1;
    int lp = 0;
    while ((1ll << lp) < P) ++lp;
    const int rows = 64 / kPanel[v].lanes;
    const int64_t blocks = (M + rows - 1) / rows;
    if (blocks >= (1ll << 31)) return -1;
    hipLaunchKernelGGL(kPanel[v].fn, dim3((unsigned)blocks), dim3(64), 0, (hipStream_t)stream, A, M, K, lp, x, y);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
}
