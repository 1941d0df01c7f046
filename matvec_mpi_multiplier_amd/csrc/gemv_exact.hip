// Bit-exact fp64 GEMV for gfx950: the reference's own arithmetic at HBM speed.
//
// multiply_std_rowwise (reference src/matr_utils.c:86-96) computes every row as
//     sum = 0; for j in 0..K-1: sum = round(sum + round(A[i][j] * x[j]))
// — a strictly sequential chain, a rounded multiply then a rounded add (no FMA: gcc on x86-64
// does not contract), and multiply_colwise (src/multiplier_colwise.c:107-122) does the same on a
// strip (scale in place = the rounded product, then the left-to-right row sum from 0.0). The
// tree-summed kernels in gemv.hip match that to ~1e-15; the kernels here reproduce it bit for
// bit, so y (and the `%.17g` y file) is identical to the reference's.
//
// A sequential chain cannot be split over lanes, so one lane owns one row for the whole of K.
// Reading A that way directly (64 lanes -> 64 rows per load instruction) would defeat
// coalescing; instead each one-wave workgroup owns RW consecutive rows (16, 32 or 64) and streams
// them through LDS in tiles of RW rows x 2T columns:
//   load  : RW*T/64 `global_load_lds_dwordx4` per tile (LDS-DMA, no VGPRs, nt): instruction i
//           fills rows [i*64/T, +64/T) of the tile, every row segment a contiguous 16*T bytes;
//   read  : lane l takes row l's 16-B chunks in column order with `ds_read_b128`;
//   swizzle: a lane-linear LDS image would put chunk k of all 64 rows in the same bank group,
//           so the source address of LDS slot s in row r is chunk s ^ (r & 15) and the read of
//           chunk k goes to slot k ^ (l & 15) — the same involution on both sides, conflict-free
//           over every ds_read_b128 lane group (rule 21 of the HIP guide);
//   x     : wave-uniform; gemv_seq reads it through the scalar cache into SGPRs (v_mul_f64
//           operands), gemv_seq_x — the forms the dispatch uses — carries each tile's x segment
//           in the same LDS ring and reads it back as a broadcast, so its latency stays off the
//           sequential chain;
//   pipeline: NB tile buffers per wave, NB-1 tiles' loads in flight behind the one being summed,
//           retired with a counted `s_waitcnt vmcnt(RW*T/64*(NB-1))` (hipcc does not track
//           LDS-DMA completion: it emits no wait before a ds_read of a DMA'd buffer).
// With RW < 64 the upper lanes repeat rows and store nothing (more waves for few rows).
// Rows past M re-read row M-1 (never stored); the column tail K % 2T and any A that is not
// 16-B aligned with an even lda take per-lane 8-B loads in the same column order.
// Everywhere but line-aligned tall shapes (>= 32768 rows, lda a multiple of 16, 2048 < K <
// 65536) the chain-hopping forms (gemv_seq_hop, below) take over: L lanes share a row, the data
// arrives by plain coalesced loads into VGPRs, and the running sum hops from lane to lane by
// DPP, still in column order.
#include <atomic>

#include <stdio.h>

#include "common.h"
#include "lds_dma.h"

// hipcc contracts a*b + c into an FMA by default (-ffp-contract=fast); the reference rounds the
// product first. Off for this whole file (the Makefile also passes -ffp-contract=off for it).
#pragma clang fp contract(off)

namespace mvg {

typedef double dbl2x __attribute__((ext_vector_type(2)));

// The reference's step: a rounded product, then a rounded add (never fused: plain operators
// under the pragma above; HIP's __dmul_rn/__dadd_rn are defined where contraction is on, and
// the backend fuses them after inlining).
__device__ __forceinline__ double seq_step(double sum, double a, double x) {
    const double p = a * x;
    return sum + p;
}

template <int RW, int T, int NB>
__global__ __launch_bounds__(64) void gemv_seq(const double* __restrict__ A, int64_t lda,
                                               const double* __restrict__ x,
                                               double* __restrict__ y, int64_t M, int64_t K) {
    static_assert(RW == 16 || RW == 32 || RW == 64, "rows per wave");
    static_assert(T >= 16 && T <= 64 && (T & (T - 1)) == 0, "tile width: 16..64 chunks");
    constexpr int kRows = 64 / T;          // rows one LDS-DMA instruction fills (1 KiB)
    constexpr int kInst = RW / kRows;      // LDS-DMA instructions per tile
    static_assert(kInst * kRows == RW, "a tile is whole instructions");
    static_assert(NB >= 2 && kInst * (NB - 1) <= 63, "loads in flight must fit the vmcnt counter");
    constexpr int kCols = 2 * T;           // columns per tile
    constexpr int kRowBytes = 16 * T;      // LDS row stride
    constexpr int kTileBytes = RW * kRowBytes;
    __shared__ __attribute__((aligned(16))) unsigned char lds[NB * kTileBytes];

    const int lane = threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.x * RW;
    const int64_t ntiles = K / kCols;

    // load side: instruction i, lane -> tile row i*kRows + lane/T (clamped to the last row),
    // LDS slot lane%T, which holds the row's chunk slot ^ (row & 15). Addresses are a
    // wave-uniform base (this tile's columns of row r0, in SGPRs) plus a 32-bit per-lane byte
    // offset (the caller guarantees 64 rows of lda fit 32 bits).
    uint32_t off[kInst];
#pragma unroll
    for (int i = 0; i < kInst; ++i) {
        const int row = i * kRows + lane / T;
        const int64_t rr = r0 + row < M ? row : M - 1 - r0;
        off[i] = (uint32_t)((rr * lda + 2 * ((lane % T) ^ (row & 15))) * (int64_t)sizeof(double));
    }
    const unsigned char* const a0 = reinterpret_cast<const unsigned char*>(A + r0 * lda);
    auto issue = [&](int64_t t, int b) {
        const unsigned char* base = a0 + t * kCols * (int64_t)sizeof(double);
#pragma unroll
        for (int i = 0; i < kInst; ++i)
            __builtin_amdgcn_global_load_lds((gbl_void_t)(base + off[i]),
                                             (lds_void_t)(lds + b * kTileBytes + i * 1024), 16, 0,
                                             2 /* nt */);
    };

    // compute side: lane l sums tile row l % RW (with RW < 64 the upper lanes repeat rows and
    // store nothing); row r's chunk k sits at slot k ^ (r & 15): base_r ^ (k << 4)
    const int myr = lane % RW;
    double sum = 0.0;
    const uint32_t my_row = (uint32_t)(myr * kRowBytes + ((myr & 15) << 4));
    auto consume = [&](int64_t t, int b) {
        const double* xt = x + t * kCols;
        const unsigned char* tile = lds + b * kTileBytes;
        // groups of 16 chunks: the group's LDS reads issue together, then its 32 steps
#pragma unroll
        for (int g = 0; g < T; g += 16) {
            dbl2x a[16];
#pragma unroll
            for (int k = 0; k < 16; ++k)
                a[k] = *reinterpret_cast<const dbl2x*>(tile + (my_row ^ (uint32_t)((g + k) << 4)));
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                sum = seq_step(sum, a[k].x, xt[2 * (g + k)]);
                sum = seq_step(sum, a[k].y, xt[2 * (g + k) + 1]);
            }
        }
    };

    for (int p = 0; p < NB - 1; ++p)
        if (p < ntiles) issue(p, p);
    for (int64_t t = 0; t < ntiles; ++t) {
        const int64_t tn = t + NB - 1;
        if (tn < ntiles) {
            // buffer tn % NB was summed in iteration t-1; its ds_reads have returned (their
            // values fed the adds), the wait only keeps the order explicit
            wait_lgkmcnt0();
            issue(tn, (int)(tn % NB));
            wait_vmcnt<kInst*(NB - 1)>();
        } else {
            wait_vmcnt<0>();
        }
        consume(t, (int)(t % NB));
    }
    // column tail, same order
    int64_t rr = r0 + myr;
    rr = rr < M ? rr : M - 1;
    const double* arow = A + rr * lda;
    for (int64_t j = ntiles * kCols; j < K; ++j) sum = seq_step(sum, arow[j], x[j]);
    if (lane < RW && r0 + lane < M) y[r0 + lane] = sum;
}

// x through the LDS ring as well: each tile buffer carries the tile's x segment (one more
// LDS-DMA instruction per tile, 1 KiB), read back with wave-uniform ds_read_b128 (a broadcast),
// so x arrives with the tile instead of through scalar loads issued at the point of use (whose
// L2 latency sat on the sequential chain). The LDS reads of chunk group g + 1 are issued before
// the sums of group g (two register sets of G chunks), so the chain waits on neither.
template <int RW, int T, int NB, int G>
__global__ __launch_bounds__(64) void gemv_seq_x(const double* __restrict__ A, int64_t lda,
                                                 const double* __restrict__ x,
                                                 double* __restrict__ y, int64_t M, int64_t K) {
    static_assert(RW == 16 || RW == 32 || RW == 64, "rows per wave");
    static_assert(T >= 16 && T <= 64 && (T & (T - 1)) == 0, "tile width: 16..64 chunks");
    static_assert(G >= 4 && T % G == 0, "chunk groups");
    constexpr int kRows = 64 / T;
    constexpr int kInst = RW / kRows + 1;  // + the x segment
    static_assert(RW % kRows == 0, "a tile is whole instructions");
    static_assert(NB >= 2 && kInst * (NB - 1) <= 63, "loads in flight must fit the vmcnt counter");
    constexpr int kCols = 2 * T;
    constexpr int kRowBytes = 16 * T;
    constexpr int kTileBytes = RW * kRowBytes;
    constexpr int kBufBytes = kTileBytes + 1024;  // tile + x segment (lanes past T repeat chunk T-1)
    __shared__ __attribute__((aligned(16))) unsigned char lds[NB * kBufBytes];

    const int lane = threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.x * RW;
    const int64_t ntiles = K / kCols;
    uint32_t off[kInst - 1];
#pragma unroll
    for (int i = 0; i < kInst - 1; ++i) {
        const int row = i * kRows + lane / T;
        const int64_t rr = r0 + row < M ? row : M - 1 - r0;
        off[i] = (uint32_t)((rr * lda + 2 * ((lane % T) ^ (row & 15))) * (int64_t)sizeof(double));
    }
    const uint32_t xoff = (uint32_t)(2 * (lane < T ? lane : T - 1) * sizeof(double));
    const unsigned char* const a0 = reinterpret_cast<const unsigned char*>(A + r0 * lda);
    const unsigned char* const x0 = reinterpret_cast<const unsigned char*>(x);
    auto issue = [&](int64_t t, int b) {
        const int64_t colb = t * kCols * (int64_t)sizeof(double);
#pragma unroll
        for (int i = 0; i < kInst - 1; ++i)
            __builtin_amdgcn_global_load_lds((gbl_void_t)(a0 + colb + off[i]),
                                             (lds_void_t)(lds + b * kBufBytes + i * 1024), 16, 0, 2 /* nt */);
        __builtin_amdgcn_global_load_lds((gbl_void_t)(x0 + colb + xoff), (lds_void_t)(lds + b * kBufBytes + kTileBytes),
                                         16, 0, 0);
    };

    const int myr = lane % RW;
    double sum = 0.0;
    const uint32_t my_row = (uint32_t)(myr * kRowBytes + ((myr & 15) << 4));
    auto consume = [&](int b) {
        const unsigned char* tile = lds + b * kBufBytes;
        const unsigned char* xs = tile + kTileBytes;
        dbl2x a[2][G], xv[2][G];
        auto read = [&](int g, dbl2x (&ad)[G], dbl2x (&xd)[G]) {
#pragma unroll
            for (int k = 0; k < G; ++k) {
                ad[k] = *reinterpret_cast<const dbl2x*>(tile + (my_row ^ (uint32_t)((g + k) << 4)));
                xd[k] = *reinterpret_cast<const dbl2x*>(xs + (g + k) * 16);
            }
        };
        read(0, a[0], xv[0]);
#pragma unroll
        for (int g = 0; g < T; g += G) {
            const int cur = (g / G) & 1;
            if (g + G < T) read(g + G, a[cur ^ 1], xv[cur ^ 1]);
#pragma unroll
            for (int k = 0; k < G; ++k) {
                sum = seq_step(sum, a[cur][k].x, xv[cur][k].x);
                sum = seq_step(sum, a[cur][k].y, xv[cur][k].y);
            }
        }
    };

    for (int p = 0; p < NB - 1; ++p)
        if (p < ntiles) issue(p, p);
    for (int64_t t = 0; t < ntiles; ++t) {
        const int64_t tn = t + NB - 1;
        if (tn < ntiles) {
            wait_lgkmcnt0();
            issue(tn, (int)(tn % NB));
            wait_vmcnt<kInst*(NB - 1)>();
        } else {
            wait_vmcnt<0>();
        }
        consume((int)(t % NB));
    }
    int64_t rr = r0 + myr;
    rr = rr < M ? rr : M - 1;
    const double* arow = A + rr * lda;
    for (int64_t j = ntiles * kCols; j < K; ++j) sum = seq_step(sum, arow[j], x[j]);
    if (lane < RW && r0 + lane < M) y[r0 + lane] = sum;
}

// ------------------------------------------------------------------ chain hopping across lanes
// The LDS forms above give every row one lane for the whole of K, so a wave advances one
// element of each of its rows per step; where few rows exist (the reference's own R x 60000 and
// 600^2 ... 10200^2 shapes) few waves run and each one's step rate — an add, a multiply, the LDS
// reads and their waits — is the whole story. Here L lanes share a row instead: a segment of
// L*W columns is one set of plain coalesced 16-B loads into VGPRs (lane c of the row's group
// holds W consecutive columns), every lane forms its W products at once, and the chain walks the
// group — lane c adds its W products in order, then the running sum hops to lane c+1 by DPP
// (row_shr:1; wave_shr:1 beyond 16 lanes). Odd segments place the columns the other way round
// (lane L-1-c holds the c-th W) and hop backwards, so each segment starts where the previous
// one ended and the chain stays in column order without a wrap-around move. All lanes execute
// every add; only the lane holding the chain adds its own products to the real sum, the others
// carry garbage that the next hop overwrites. Per column: one dependent add plus 1/W of a hop.
// U segments are in flight per wave (the compiler counts plain loads itself).
template <int L, bool FWD>
__device__ __forceinline__ double hop(double v) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    constexpr int kCtrl = L <= 16 ? (FWD ? 0x111 : 0x101) : (FWD ? 0x138 : 0x130);
    const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)b, kCtrl, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), kCtrl, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// One segment of the chain: lane t of the group adds its W products at step t, then hands over.
// Every lane executes every add (switching the non-holders off in the exec mask, an eighth of the
// VALU work at L = 8, measured no faster: round 3, profiles/r03/sweep_exact_masked.jsonl).
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

// A lane's W consecutive doubles of a segment: 16-B loads, or (B8) 8-B loads, which need
// neither a 16-B aligned A or x nor an even lda (an odd-width column strip, an offset view).
template <int V, bool B8, bool NT>
__device__ __forceinline__ void load_run(const double* p, dbl2x (&d)[V]) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
        if constexpr (B8 && NT)
            d[v] = dbl2x{__builtin_nontemporal_load(p + 2 * v), __builtin_nontemporal_load(p + 2 * v + 1)};
        else if constexpr (B8)
            d[v] = dbl2x{p[2 * v], p[2 * v + 1]};
        else if constexpr (NT)
            d[v] = __builtin_nontemporal_load(reinterpret_cast<const dbl2x*>(p) + v);
        else
            d[v] = reinterpret_cast<const dbl2x*>(p)[v];
    }
}

// A segment whose columns outside [lo, hi) contribute 0 x 0 = +0.0 products: adding +0.0 leaves
// the running sum unchanged bit for bit (it is never -0.0: it starts at +0.0 and
// round-to-nearest gives +0.0 for every exact cancellation). cb: this lane's first column.
template <int L, int W>
__device__ __forceinline__ double hop_masked_segment(double sum, const double* __restrict__ arow,
                                                     const double* __restrict__ x, int64_t cb, int64_t lo,
                                                     int64_t hi, bool fwd) {
    dbl2x ta[W / 2], tx[W / 2];
#pragma unroll
    for (int v = 0; v < W / 2; ++v) {
        const int64_t j0 = cb + 2 * v, j1 = j0 + 1;
        const bool in0 = j0 >= lo && j0 < hi, in1 = j1 >= lo && j1 < hi;
        ta[v] = dbl2x{in0 ? arow[j0] : 0.0, in1 ? arow[j1] : 0.0};
        tx[v] = dbl2x{in0 ? x[j0] : 0.0, in1 ? x[j1] : 0.0};
    }
    return fwd ? hop_segment<L, W, true>(sum, ta, tx) : hop_segment<L, W, false>(sum, ta, tx);
}

// every row of A starts on a 128-B line: A on a line and lda a multiple of 16 doubles
__device__ __forceinline__ bool lines_aligned(const double* A, int64_t lda) {
    return (((uintptr_t)A & 127u) == 0) && (lda % 16 == 0);
}

// Segment g of a row runs forward (lane 0 -> L-1) when g is even. A row's segments: a head
// (g = 0) ending at the row's first 128-B boundary, so that every main segment's loads start on
// a cache line — a row that starts mid-line would make each 128-B piece touch two lines
// (16384 x 16386: 373 us against 314 us at 16384^2, sweep_exact13_lines.jsonl) — then nseg
// main segments, the same count for every row of the wave, then one or two tail segments for
// what is left. Head and tails are masked segments (zeros outside the row's columns).
// NW waves per workgroup (wave w of workgroup b owns rows [(b * NW + w) * R, +R)): with NW > 1 and
// a launch-time LDS reservation, the dispatcher places the same number of waves on every CU.
template <int L, int W, int U, bool B8 = false, int NW = 1>
__global__ __launch_bounds__(64 * NW) void gemv_seq_hop(const double* __restrict__ A, int64_t lda,
                                                        const double* __restrict__ x,
                                                        double* __restrict__ y, int64_t M, int64_t K) {
    static_assert(L == 1 || L == 2 || L == 4 || L == 8 || L == 16 || L == 32 || L == 64, "lanes per row");
    static_assert(W % 2 == 0 && U % 2 == 0, "whole 16-B pieces; segment pairs per unrolled step");
    constexpr int R = 64 / L;  // rows per wave
    constexpr int S = L * W;   // columns per segment
    constexpr int V = W / 2;   // 16-B pieces per lane per segment
    static_assert(S >= 16, "the head (up to 15 columns) fits one segment");
    const int lane = threadIdx.x & 63;
    const int c = lane % L;
    const int64_t row = ((int64_t)blockIdx.x * NW + (threadIdx.x >> 6)) * R + lane / L;
    const int64_t rr = row < M ? row : M - 1;
    const double* arow = A + rr * lda;
    const int off[2] = {c * W, (L - 1 - c) * W};  // even / odd segment
    double sum = 0.0;
    int64_t nseg = 0, ntail = 0;
    if (K > 0) {
        // head: columns [0, h) with h the distance to the row's next 128-B boundary (0 ... 15)
        const int64_t h = (int64_t)(((128u - ((uintptr_t)arow & 127u)) & 127u) >> 3);
        sum = hop_masked_segment<L, W>(sum, arow, x, h - S + off[0], 0, h < K ? h : K, true);
        // every row has >= nseg * S columns past its head; when every row starts on a line (A on
        // a line, lda a multiple of 16: h = 0 throughout) that is K / S, and a row of whole
        // segments (config 5's 512 columns) needs no masked tail, whose loads would not be in
        // flight ahead of the chain
        nseg = lines_aligned(A, lda) ? K / S : K >= 15 ? (K - 15) / S : 0;
        ntail = (K - nseg * S + S - 1) / S;            // what any row has left: 0, 1 or 2 segments (0: line-aligned rows of whole segments)
        const double* ar = arow + h;
        const double* xr = x + h;
        if (nseg > 0) {
            dbl2x a[U][V], xv[U][V];
#pragma unroll
            for (int i = 0; i < U; ++i) {
                const int64_t sg = i < nseg ? i : nseg - 1;
                load_run<V, B8, true>(ar + sg * S + off[(i + 1) & 1], a[i]);
                load_run<V, true, false>(xr + sg * S + off[(i + 1) & 1], xv[i]);
                __builtin_amdgcn_sched_barrier(0);  // same load order as the loop's refills
            }
            // Whole groups of U segments, one basic block: slot i is summed, then refilled U
            // segments ahead; the scheduling barriers keep the loads in slot order, so the
            // compiler's vmcnt waits retire exactly the slot about to be summed. Main segment i
            // is the row's segment i + 1 (after the head).
            // (strict <: a group whose refills would all lie past the row's last segment is left
            // to the remainder below instead of re-reading that segment U times)
            int64_t base = 0;
            for (; base + U < nseg; base += U) {
#pragma unroll
                for (int i = 0; i < U; ++i) {
                    sum = (i & 1) ? hop_segment<L, W, true>(sum, a[i], xv[i]) : hop_segment<L, W, false>(sum, a[i], xv[i]);
                    __builtin_amdgcn_sched_barrier(0);
                    const int64_t sg = base + i + U < nseg ? base + i + U : nseg - 1;
                    load_run<V, B8, true>(ar + sg * S + off[(i + 1) & 1], a[i]);
                    load_run<V, true, false>(xr + sg * S + off[(i + 1) & 1], xv[i]);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            // the last nseg - base <= U segments are already in slots 0 .. nseg - base - 1 (base is even)
#pragma unroll
            for (int i = 0; i < U; ++i)
                if (base + i < nseg)
                    sum = (i & 1) ? hop_segment<L, W, true>(sum, a[i], xv[i]) : hop_segment<L, W, false>(sum, a[i], xv[i]);
        }
        for (int64_t t = 0; t < ntail; ++t) {
            const int64_t g = 1 + nseg + t;  // the row's segment index
            sum = hop_masked_segment<L, W>(sum, arow, x, h + (nseg + t) * S + off[g & 1], h, K, (g & 1) == 0);
        }
    }
    // the chain ends in lane L-1 after an odd number of segments, in lane 0 otherwise
    const int holder = (K > 0 && ((1 + nseg + ntail) & 1)) ? L - 1 : 0;
    if (c == holder && row < M) y[row] = sum;
}

// gemv_seq_hop with x staged in LDS once per workgroup of NW waves (short rows, K <= kXlMaxK):
// the main segments read their x pieces from LDS (all row groups of a wave read the same 16 B per
// lane group: broadcasts) instead of re-reading x through L1 beside the A stream, so the vector
// memory pipeline carries A alone. Same chain, same order, same bits as gemv_seq_hop<L, W, U, true>.
template <int L, int W, int U, int NW>
__global__ __launch_bounds__(64 * NW) void gemv_seq_hop_xl(const double* __restrict__ A, int64_t lda,
                                                           const double* __restrict__ x,
                                                           double* __restrict__ y, int64_t M, int64_t K) {
    static_assert(L == 4 || L == 8 || L == 16, "lanes per row");
    static_assert(W % 2 == 0 && U % 2 == 0, "whole 16-B pieces; segment pairs per unrolled step");
    extern __shared__ double xl[];  // K doubles
    constexpr int R = 64 / L;
    constexpr int S = L * W;
    constexpr int V = W / 2;
    static_assert(S >= 16, "the head (up to 15 columns) fits one segment");
    for (int64_t j = threadIdx.x; j < K; j += 64 * NW) xl[j] = x[j];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int c = lane % L;
    const int64_t row = ((int64_t)blockIdx.x * NW + (threadIdx.x >> 6)) * R + lane / L;
    const int64_t rr = row < M ? row : M - 1;
    const double* arow = A + rr * lda;
    const int off[2] = {c * W, (L - 1 - c) * W};
    double sum = 0.0;
    int64_t nseg = 0, ntail = 0;
    if (K > 0) {
        const int64_t h = (int64_t)(((128u - ((uintptr_t)arow & 127u)) & 127u) >> 3);
        sum = hop_masked_segment<L, W>(sum, arow, x, h - S + off[0], 0, h < K ? h : K, true);
        nseg = lines_aligned(A, lda) ? K / S : K >= 15 ? (K - 15) / S : 0;
        ntail = (K - nseg * S + S - 1) / S;  // 0, 1 or 2 tail segments, as in gemv_seq_hop
        const double* ar = arow + h;
        const double* xr = xl + h;
        auto xload = [&](const double* p, dbl2x (&d)[V]) {
#pragma unroll
            for (int v = 0; v < V; ++v) d[v] = dbl2x{p[2 * v], p[2 * v + 1]};
        };
        if (nseg > 0) {
            dbl2x a[U][V], xv[U][V];
#pragma unroll
            for (int i = 0; i < U; ++i) {
                const int64_t sg = i < nseg ? i : nseg - 1;
                load_run<V, true, true>(ar + sg * S + off[(i + 1) & 1], a[i]);
                xload(xr + sg * S + off[(i + 1) & 1], xv[i]);
                __builtin_amdgcn_sched_barrier(0);
            }
            int64_t base = 0;
            for (; base + U < nseg; base += U) {
#pragma unroll
                for (int i = 0; i < U; ++i) {
                    sum = (i & 1) ? hop_segment<L, W, true>(sum, a[i], xv[i]) : hop_segment<L, W, false>(sum, a[i], xv[i]);
                    __builtin_amdgcn_sched_barrier(0);
                    const int64_t sg = base + i + U < nseg ? base + i + U : nseg - 1;
                    load_run<V, true, true>(ar + sg * S + off[(i + 1) & 1], a[i]);
                    xload(xr + sg * S + off[(i + 1) & 1], xv[i]);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
#pragma unroll
            for (int i = 0; i < U; ++i)
                if (base + i < nseg)
                    sum = (i & 1) ? hop_segment<L, W, true>(sum, a[i], xv[i]) : hop_segment<L, W, false>(sum, a[i], xv[i]);
        }
        for (int64_t t = 0; t < ntail; ++t) {
            const int64_t g = 1 + nseg + t;
            sum = hop_masked_segment<L, W>(sum, arow, x, h + (nseg + t) * S + off[g & 1], h, K, (g & 1) == 0);
        }
    }
    const int holder = (K > 0 && ((1 + nseg + ntail) & 1)) ? L - 1 : 0;
    if (c == holder && row < M) y[row] = sum;
}
constexpr int64_t kXlMaxK = 8192;  // x in LDS: up to 64 KiB per workgroup

// ------------------------------------------------------------------ column-panel layout
// Every exact form streams all M rows at once — a row's chain (>= 2.5 ns per column) is too slow
// for the tree kernel's sliding window of a thousand rows — so at any moment it reads M scattered
// pieces of a row-major A, one per row: the access pattern of a plain streaming read of
// thousands of separate ranges, and the same rate (16384^2: exact 312 us, streaming read 309,
// tree 295; profiles/r02/sweep_exact15_stream_cal.jsonl). With A in column panels — panel p =
// columns [pP, pP + P) of every row, rows P doubles apart, panels pstride >= M*P doubles apart —
// the same all-rows-at-once chain order reads one contiguous M*P*8-byte region at a time: a
// sliding window again, over panels (16384^2: 299 us at P = 256; 65536 x 32768: 2385 against
// 2466; profiles/r02/panel_probe_*.jsonl). The engine keeps such a copy of its shard in exact
// mode (engine.cpp). The arithmetic and its order are those of gemv_seq_hop, so y is the same
// bit for bit. P is a power of two and a multiple of the segment (L*W columns), so no segment
// straddles two panels; K % (L*W) columns end in one masked segment. Ap 16-B aligned with
// P*8 a multiple of 128 B puts every segment on a cache line (no head segment).
// (one-wave workgroups: unlike the row-major hop form's, their placement costs nothing
// measurable — 299-302 us at 16384^2 in every process state; as 8-wave workgroups one per CU,
// 304-309, round 4, profiles/r04/r4j)
template <int L, int W, int U>
__global__ __launch_bounds__(64) void gemv_seq_hop_panel(const double* __restrict__ Ap, int64_t pstride, int lp,
                                                         const double* __restrict__ x,
                                                         double* __restrict__ y, int64_t M, int64_t K) {
    static_assert(L == 8 || L == 16, "lanes per row");
    static_assert(W % 2 == 0 && U % 2 == 0, "whole 16-B pieces; segment pairs per unrolled step");
    constexpr int R = 64 / L;  // rows per wave
    constexpr int S = L * W;   // columns per segment
    constexpr int V = W / 2;   // 16-B pieces per lane per segment
    const int lane = threadIdx.x;
    const int c = lane % L;
    const int64_t row = (int64_t)blockIdx.x * R + lane / L;
    const int64_t rr = row < M ? row : M - 1;
    const int64_t pmask = (1ll << lp) - 1;
    const double* arow = Ap + (rr << lp);
    const int off[2] = {c * W, (L - 1 - c) * W};  // even / odd segment
    // segment g of this row (columns [gS, gS + S)): panel gS >> lp, offset gS & (P - 1) in it
    auto seg = [&](int64_t g) { return arow + ((g * S) >> lp) * pstride + ((g * S) & pmask); };
    const int64_t nseg = K / S;
    const int64_t tail = K - nseg * S;
    double sum = 0.0;
    if (nseg > 0) {
        dbl2x a[U][V], xv[U][V];
#pragma unroll
        for (int i = 0; i < U; ++i) {
            const int64_t g = i < nseg ? i : nseg - 1;
            load_run<V, false, true>(seg(g) + off[i & 1], a[i]);
            load_run<V, false, false>(x + g * S + off[i & 1], xv[i]);
            __builtin_amdgcn_sched_barrier(0);
        }
        // as in gemv_seq_hop: slot i is summed, then refilled U segments ahead, loads kept in
        // slot order so the counted vmcnt waits retire exactly the slot about to be summed;
        // segment g runs forward when g is even (base is a multiple of U, U even)
        int64_t base = 0;
        for (; base + U < nseg; base += U) {
#pragma unroll
            for (int i = 0; i < U; ++i) {
                sum = (i & 1) ? hop_segment<L, W, false>(sum, a[i], xv[i]) : hop_segment<L, W, true>(sum, a[i], xv[i]);
                __builtin_amdgcn_sched_barrier(0);
                const int64_t g = base + i + U < nseg ? base + i + U : nseg - 1;
                load_run<V, false, true>(seg(g) + off[i & 1], a[i]);
                load_run<V, false, false>(x + g * S + off[i & 1], xv[i]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int i = 0; i < U; ++i)
            if (base + i < nseg)
                sum = (i & 1) ? hop_segment<L, W, false>(sum, a[i], xv[i]) : hop_segment<L, W, true>(sum, a[i], xv[i]);
    }
    if (tail > 0) {
        // the last K % S columns: a masked segment over the panel's columns (zeros outside K);
        // hop_masked_segment indexes by column, so hand it the segment's base shifted back by gS
        const int64_t g = nseg;
        sum = hop_masked_segment<L, W>(sum, seg(g) - g * S, x, g * S + off[g & 1], 0, K, (g & 1) == 0);
    }
    const int holder = ((nseg + (tail > 0 ? 1 : 0)) & 1) ? L - 1 : 0;
    if (c == holder && row < M) y[row] = sum;
}

// Row-major rows [0, m) of A (lda) -> the same rows of the panel layout (rows P doubles apart,
// panels pstride apart). One workgroup per row: 64-lane runs of consecutive elements on both
// sides (2 KiB per panel row at P = 256). V16: 16-B pairs (A 16-B aligned, lda even; P, pstride
// and the pair's column even, so a pair never straddles two panels and lands 16-B aligned),
// else 8-B elements (any lda and alignment). HBM-bound: 16 bytes moved per element.
template <bool V16>
__global__ __launch_bounds__(256) void panel_relayout_kernel(const double* __restrict__ A, int64_t lda, int64_t m,
                                                             int64_t k, double* __restrict__ Ap, int64_t pstride,
                                                             int lp) {
    const int64_t pmask = (1ll << lp) - 1;
    for (int64_t r = blockIdx.x; r < m; r += gridDim.x) {
        const double* src = A + r * lda;
        double* dst = Ap + (r << lp);
        if constexpr (V16) {
            const dbl2x* src2 = reinterpret_cast<const dbl2x*>(src);
            for (int64_t q = threadIdx.x; q < k / 2; q += 256) {
                const int64_t j = 2 * q;
                *reinterpret_cast<dbl2x*>(dst + (j >> lp) * pstride + (j & pmask)) = __builtin_nontemporal_load(src2 + q);
            }
            if ((k & 1) && threadIdx.x == 0) dst[((k - 1) >> lp) * pstride + ((k - 1) & pmask)] = src[k - 1];
        } else {
            for (int64_t j = threadIdx.x; j < k; j += 256)
                dst[(j >> lp) * pstride + (j & pmask)] = __builtin_nontemporal_load(src + j);
        }
    }
}

// Any alignment, any lda: lane = row, 8-B loads walking the row (uncoalesced; small or odd
// shapes only).
__global__ __launch_bounds__(64) void gemv_seq_scalar(const double* __restrict__ A, int64_t lda,
                                                      const double* __restrict__ x,
                                                      double* __restrict__ y, int64_t M, int64_t K) {
    const int64_t row = (int64_t)blockIdx.x * 64 + threadIdx.x;
    const int64_t rr = row < M ? row : M - 1;
    const double* arow = A + rr * lda;
    double sum = 0.0;
    int64_t j = 0;
    for (; j + 4 <= K; j += 4) {
        const double a0 = arow[j], a1 = arow[j + 1], a2 = arow[j + 2], a3 = arow[j + 3];
        sum = seq_step(sum, a0, x[j]);
        sum = seq_step(sum, a1, x[j + 1]);
        sum = seq_step(sum, a2, x[j + 2]);
        sum = seq_step(sum, a3, x[j + 3]);
    }
    for (; j < K; ++j) sum = seq_step(sum, arow[j], x[j]);
    if (row < M) y[row] = sum;
}

// ------------------------------------------------------------------ exact combines
// MPI_Reduce(SUM, root 0) as the reference's MPICH 3.3.2 runs it for a commutative op
// (colwise.c:124; MPIR_Reduce_intra_auto): with n * 8 > 2048 bytes and n >= pof2 (the largest
// power of two <= P) reduce-scatter + gather — ranks 2i, 2i+1 (i < rem = P - pof2) fold into new
// rank i, rank r >= 2 rem becomes new rank r - rem, and the recursive halving sums the pof2 new
// ranks as a binomial tree — otherwise a binomial tree over all P ranks in rank order,
// ((p0 + p1) + (p2 + p3)) + .... parts[r*n + i] = rank r's partial; `fold` = rem (0: binomial).
// Overwrites parts; y[i] = the root's result.
__global__ void combine_mpich(double* __restrict__ parts, int P, int fold, int64_t n, double* __restrict__ y) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        for (int f = 0; f < fold; ++f) parts[2 * f * n + i] = parts[2 * f * n + i] + parts[(2 * f + 1) * n + i];
        const int m = P - fold;  // ranks left in the tree; new rank k lives in real rank k < fold ? 2k : k + fold
        for (int mask = 1; mask < m; mask <<= 1)
            for (int k = 0; k + mask < m; k += 2 * mask) {
                const int a = k < fold ? 2 * k : k + fold;
                const int b = k + mask < fold ? 2 * (k + mask) : k + mask + fold;
                parts[a * n + i] = parts[a * n + i] + parts[b * n + i];
            }
        y[i] = parts[i];
    }
}

// rem = P - pof2 when MPICH takes its reduce-scatter + gather algorithm for n doubles, else 0
int mpich_reduce_fold(int P, int64_t n) {
    int pof2 = 1;
    while (pof2 * 2 <= P) pof2 *= 2;
    return (n * 8 > 2048 && n >= pof2) ? P - pof2 : 0;
}

// gather_local_results (blockwise.c:150-207): y starts at 0 and every block's partial of the
// grid row is added in rank order (the root's own first; the reference takes the others in
// MPI_ANY_SOURCE arrival order, which for two grid columns gives the same sum). parts[r*lr + j]
// = rank r's partial; y[gi*lr + j] = ((0 + p[gi*gc]) + p[gi*gc + 1]) + ...
__global__ void combine_grid_rows(const double* __restrict__ parts, int gr, int gc, int64_t lr,
                                  double* __restrict__ y) {
    const int64_t n = (int64_t)gr * lr;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t gi = idx / lr, j = idx % lr;
        double s = 0.0;
        for (int c = 0; c < gc; ++c) s = s + parts[(gi * gc + c) * lr + j];
        y[idx] = s;
    }
}

int launch_combine_mpich_reduce(double* parts, int P, int64_t n, double* y, hipStream_t s) {
    if (n <= 0) return MVG_OK;
    const int64_t blocks = (n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096;
    hipLaunchKernelGGL(combine_mpich, dim3((unsigned)blocks), dim3(256), 0, s, parts, P, mpich_reduce_fold(P, n), n,
                       y);
    MVG_HIP(hipGetLastError());
    return MVG_OK;
}

int launch_combine_grid_rows(const double* parts, int gr, int gc, int64_t lr, double* y, hipStream_t s) {
    const int64_t n = (int64_t)gr * lr;
    if (n <= 0) return MVG_OK;
    const int64_t blocks = (n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096;
    hipLaunchKernelGGL(combine_grid_rows, dim3((unsigned)blocks), dim3(256), 0, s, parts, gr, gc, lr, y);
    MVG_HIP(hipGetLastError());
    return MVG_OK;
}

// ------------------------------------------------------------------ variant table
typedef void (*seq_fn)(const double*, int64_t, const double*, double*, int64_t, int64_t);
struct SeqVariant {
    const char* name;
    seq_fn fn;
    int needs;  // operand requirements: kAnyOperands, kVec16 or kVec16Lda23 (below)
    int rows;   // rows per workgroup
    int waves = 1;       // waves per workgroup
    bool xlds = false;   // x staged in LDS (K doubles of dynamic LDS; K <= kXlMaxK)
    int lds_reserve = 0;  // dynamic LDS bytes reserved (unused by the kernel): workgroups per CU cap
};

// kVec16: 16-B loads, so 16-B aligned A and x and an even lda; kVec16Lda23: also 32-bit
// per-lane LDS-DMA offsets over 64 rows of lda (lda < 2^23)
constexpr int kAnyOperands = 0, kVec16 = 1, kVec16Lda23 = 2;
#define SEQ(RW, T, NB) {"seq_r" #RW "_t" #T "_b" #NB, gemv_seq<RW, T, NB>, kVec16Lda23, RW}
#define HOP(L, W, U) {"hop_l" #L "_w" #W "_u" #U, gemv_seq_hop<L, W, U>, kVec16, 64 / L}
#define HOP8(L, W, U) {"hop8_l" #L "_w" #W "_u" #U, gemv_seq_hop<L, W, U, true>, kAnyOperands, 64 / L}
// NW waves per workgroup and an LDS reservation that lets only 160 / KB of them on a CU: the
// same count of long-lived waves on every CU
#define HOP8E(L, W, U, NW, KB) \
    {"hop8e_l" #L "_w" #W "_u" #U "_n" #NW, gemv_seq_hop<L, W, U, true, NW>, kAnyOperands, NW * 64 / L, NW, false, KB * 1024}
#define HOPXL(L, W, U, NW) \
    {"hopxl_l" #L "_w" #W "_u" #U "_n" #NW, gemv_seq_hop_xl<L, W, U, NW>, kAnyOperands, NW * 64 / L, NW, true}
static constexpr SeqVariant kSeqVariants[] = {
    {"auto", nullptr, kAnyOperands, 64},  // 0
    {"seq_scalar", gemv_seq_scalar, kAnyOperands, 64},
    // x through the scalar cache (the first form; kept for comparison)
    SEQ(64, 16, 2),   // LDS per wave: NB x RW x 16T bytes; 32 KiB
    SEQ(64, 32, 2),   // 64 KiB
    SEQ(32, 32, 2),   // 32 KiB
    SEQ(32, 64, 2),   // 64 KiB
    SEQ(16, 64, 2),   // 32 KiB
    // x through the LDS ring, LDS reads one chunk group ahead of the sums
    {"seqx_r32_t64_b2_g8", gemv_seq_x<32, 64, 2, 8>, kVec16Lda23, 32},
    {"seqx_r32_t64_b2_g16", gemv_seq_x<32, 64, 2, 16>, kVec16Lda23, 32},
    {"seqx_r64_t16_b2_g8", gemv_seq_x<64, 16, 2, 8>, kVec16Lda23, 64},
    {"seqx_r64_t32_b2_g8", gemv_seq_x<64, 32, 2, 8>, kVec16Lda23, 64},
    {"seqx_r16_t64_b2_g8", gemv_seq_x<16, 64, 2, 8>, kVec16Lda23, 16},
    {"seqx_r16_t32_b4_g8", gemv_seq_x<16, 32, 4, 8>, kVec16Lda23, 16},
    // L lanes per row, the chain hopping across them (registers, no LDS)
    HOP(64, 8, 4),
    HOP(32, 8, 4),
    HOP(32, 4, 8),
    HOP(16, 8, 4),
    HOP(16, 4, 8),
    HOP(16, 2, 16),
    HOP(8, 8, 4),
    HOP(8, 4, 8),
    HOP(8, 2, 16),
    HOP(8, 2, 24),
    HOP(4, 4, 8),
    // the same with 8-B loads: any alignment, any lda
    HOP8(8, 2, 16),
    HOP8(8, 2, 24),
    HOP8(8, 4, 8),
    HOP8(16, 2, 16),
    HOP8(16, 4, 8),
    HOP8(16, 8, 4),
    HOP8(32, 8, 4),
    // the same waves placed evenly: one 8-wave workgroup per CU, or two 4-wave ones
    HOP8E(8, 2, 16, 8, 96),
    HOP8E(8, 2, 16, 4, 64),
    // x staged in LDS once per workgroup of NW waves (short rows)
    HOPXL(8, 2, 16, 4),
    HOPXL(8, 2, 8, 4),
    HOPXL(4, 4, 8, 4),
    HOPXL(8, 2, 16, 2),
};
constexpr int kNumSeqVariants = (int)(sizeof(kSeqVariants) / sizeof(kSeqVariants[0]));

static bool operands_ok(int needs, int64_t lda, bool aligned) {
    if (needs == kAnyOperands) return true;
    if (!aligned || lda % 2 != 0) return false;
    return needs == kVec16 || lda < (1ll << 23);
}

template <typename T, size_t N>
constexpr int seq_id(const T (&table)[N], const char* name) {
    for (size_t i = 0; i < N; ++i) {
        const char *a = table[i].name, *b = name;
        while (*a && *a == *b) ++a, ++b;
        if (*a == *b) return (int)i;
    }
    return -1;
}
constexpr int kSeqScalar = seq_id(kSeqVariants, "seq_scalar");
constexpr int kSeqManyRows = seq_id(kSeqVariants, "seqx_r64_t16_b2_g8");
constexpr int kHopRows = seq_id(kSeqVariants, "hop8_l8_w2_u16");
constexpr int kHopLongRows = seq_id(kSeqVariants, "hop8_l8_w2_u24");
constexpr int kHopWide = seq_id(kSeqVariants, "hop8_l16_w4_u8");
constexpr int kHopWidest = seq_id(kSeqVariants, "hop8_l16_w8_u4");
constexpr int kHopFewRows = seq_id(kSeqVariants, "hop8_l32_w8_u4");
constexpr int kHopEven = seq_id(kSeqVariants, "hop8e_l8_w2_u16_n8");
static_assert(kHopEven > 0 && kSeqVariants[kHopEven].needs == kAnyOperands, "the evenly placed pick takes any operands");
static_assert(kSeqScalar > 0 && kSeqVariants[kSeqScalar].needs == kAnyOperands, "8-B exact fallback");
static_assert(kSeqManyRows > 0 && kHopRows > 0 && kHopLongRows > 0 && kHopWide > 0 && kHopWidest > 0 &&
                  kHopFewRows > 0,
              "exact dispatch names a missing variant");
static_assert(kSeqVariants[kHopRows].needs == kAnyOperands && kSeqVariants[kHopLongRows].needs == kAnyOperands &&
                  kSeqVariants[kHopWide].needs == kAnyOperands && kSeqVariants[kHopWidest].needs == kAnyOperands &&
                  kSeqVariants[kHopFewRows].needs == kAnyOperands,
              "the chain-hopping picks take any operands");

// From the round-2 MI355X sweeps (tools/sweep_exact.py -> profiles/r02/sweep_exact*.jsonl; the
// dispatch below from sweep_exact13_lines.jsonl, 31 shapes: the BASELINE configs' shards, the
// reference's own sizes, odd widths and rows that start mid-line). The LDS forms only where
// they still win: >= 32768 rows whose every row starts on a 128-B line (A on a line, lda a
// multiple of 16) with 2048 < K < 65536 — 64-row waves of 256-B row segments (the strips and
// blocks of configs 3 and 4: 622 against 663 us, 2461 against 2490). Everything else takes the
// chain-hopping forms, with 8-B loads (they equal the 16-B ones on aligned data and take any
// lda): 8 lanes x 16 B per row from 6144 rows (or K <= 8192; 24 segments in flight from
// K = 65536: 131072^2 19.8 against 20.4 ms, 2.9 %, profiles/r03/sweep_exact_u16_u24_big.jsonl;
// level at 65536^2), 16 lanes x 32 B for 2048 .. 6143 rows (x 64 B below 4096 rows with K >= 32768),
// 32 lanes x 64 B for fewer rows with K > 4096, where the chain dominates (the reference's
// R x 60000: 1200 rows in 203 us, 679 with the LDS forms), 16 x 32 B for short ones. On rows
// that start mid-line they beat the tree form itself (16384 x 16386: 305 us against 315);
// config 5's shards and 4,194,304 x 512 run at 0.96-1.0 of the tree form's speed.
// short rows (K <= 768) go out in launches of at most 1 GiB of A (mvg_gemv_exact_variant below)
constexpr int64_t kShortRowK = 768;
constexpr int64_t kShortRowLaunchBytes = 1ll << 30;
constexpr int64_t kMinPieceRows = 65536;
constexpr int kMi355xCUs = 256;  // when no device answers (host-only callers, tests)
//
// Evenly placed 8-lane forms (round 4, profiles/r04/r4g, r4h): the 8-lane hop forms' one-wave
// workgroups all stay resident for the whole launch, and how the dispatcher spreads them over the
// CUs depends on the process's hardware-queue state — with two more used HIP streams in the
// process (the engine's, torch's) the same launch took 335 us at 16384^2 against 312 alone. The
// same waves as one 8-wave workgroup per CU (an LDS reservation admits one per CU) take 310-314 us
// in every state, and 0.4-1.6 % less than the one-wave form in a fresh process (16384^2,
// 16384 x 16383, 32768 x 16384). They are taken where whole rounds of one workgroup per CU cover
// the rows (64-row workgroups a multiple of the CU count: the BASELINE configs' 16384-row
// multiples) and K < 65536; a partial last round costs a whole round (24576 x 16384: 541 against
// 470 us), and at 131072^2 the 24-segment one-wave form stays 2 % ahead (19.64 against 20.03 ms).
// Test hooks (mvg_debug_*, include/matvec_gpu.h): a CU count standing in for the device's, and
// an LDS reservation for the evenly placed form that a runtime must refuse (above the CU's
// 160 KiB) to drive the refusal fallback below.
static std::atomic<int> g_cu_override{0};
static std::atomic<int64_t> g_even_lds_override{0};
// Per device: the runtime refused the evenly placed form's LDS reservation once; the dispatch
// then keeps to the one-wave forms on that device (no failing launch per call).
static std::atomic<int> g_even_refused[64];

static int current_device() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
        (void)hipGetLastError();
        return -1;
    }
    return dev;
}

static int device_cu_count() {
    static std::atomic<int> cached[64];
    if (const int o = g_cu_override.load(std::memory_order_relaxed); o > 0) return o;
    const int dev = current_device();
    if (dev < 0) return kMi355xCUs;
    int n = cached[dev].load(std::memory_order_relaxed);
    if (n > 0) return n;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        n = kMi355xCUs;
    }
    cached[dev].store(n, std::memory_order_relaxed);
    return n;
}

static bool even_refused() {
    const int dev = current_device();
    return dev >= 0 && g_even_refused[dev].load(std::memory_order_relaxed) != 0;
}

// The errors with which the runtime turns down a launch's resources before dispatching it: the
// LDS request above the CU's (hipErrorInvalidValue on ROCm 7, profiles/r05/p5a/lds_refusal.txt),
// a workgroup shape or resource set it cannot place. Anything else is reported, never retried.
static bool launch_refused(hipError_t e) {
    return e == hipErrorInvalidValue || e == hipErrorInvalidConfiguration || e == hipErrorLaunchOutOfResources;
}

// A refusal error counts as the LDS refusal only when the request is above what the device
// grants one workgroup (hipDeviceAttributeMaxSharedMemoryPerBlock: 160 KiB on gfx950); any other
// failure with the same code is this launch's error and is reported. Unknown limit: taken as the
// refusal (the one-wave form then computes the same sums).
static bool lds_refusal_confirmed(hipError_t e, size_t lds) {
    if (!launch_refused(e)) return false;
    const int dev = current_device();
    int max_lds = 0;
    if (dev < 0 || hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess ||
        max_lds <= 0) {
        (void)hipGetLastError();
        return true;
    }
    return lds > (size_t)max_lds;
}

static int pick_seq_variant(int64_t lda, int64_t M, int64_t K, bool aligned, bool lines) {
    if (lines && operands_ok(kVec16Lda23, lda, aligned) && M >= 32768 && K > 2048 && K < 65536)
        return kSeqManyRows;
    if (M >= 6144 && K > kShortRowK && K < 65536 && !even_refused()) {
        const int64_t wgs = (M + 63) / 64, cus = device_cu_count();
        if (wgs >= cus && wgs % cus == 0) return kHopEven;
    }
    if (M >= 6144) return K >= 65536 ? kHopLongRows : kHopRows;
    if (M >= 2048) return K <= 8192 ? kHopRows : M < 4096 && K >= 32768 ? kHopWidest : kHopWide;
    return K <= 4096 ? kHopWide : kHopFewRows;
}

// Panel-layout forms (gemv_seq_hop_panel). From profiles/r02/panel_probe_*.jsonl: P = 256
// (P = 128 within 1 %; 64, 512 and 1024 2-8 % slower, 16 and 4096 well behind), 8 lanes x 16 B
// per row, 8 segments in flight.
typedef void (*panel_fn)(const double*, int64_t, int, const double*, double*, int64_t, int64_t);
struct PanelVariant {
    const char* name;
    panel_fn fn;
    int rows;  // rows per one-wave workgroup
    int seg;   // columns per segment (P must be a multiple)
};
#define PANEL(L, W, U) {"panel_l" #L "_w" #W "_u" #U, gemv_seq_hop_panel<L, W, U>, 64 / L, L * W}
static constexpr PanelVariant kPanelVariants[] = {
    {"auto", nullptr, 8, 16},  // 0
    PANEL(8, 2, 8),
    PANEL(8, 2, 16),
    PANEL(8, 2, 24),
    PANEL(16, 2, 16),
};
#undef PANEL
constexpr int kNumPanelVariants = (int)(sizeof(kPanelVariants) / sizeof(kPanelVariants[0]));
constexpr int kPanelRows = seq_id(kPanelVariants, "panel_l8_w2_u8");
static_assert(kPanelRows > 0, "panel dispatch names a missing variant");
constexpr int64_t kPanelWidth = 256;


// one form for every shape: 24 segments in flight gained only 1-2 % from 32768 rows (round 2),
// inside the box-to-box spread, so round 3 dropped that threshold
static int pick_panel_variant(int64_t) { return kPanelRows; }

}  // namespace mvg

using namespace mvg;

extern "C" {

int mvg_gemv_exact_variant_count(void) { return kNumSeqVariants; }

const char* mvg_gemv_exact_variant_name(int v) {
    if (v < 0 || v >= kNumSeqVariants) return "invalid";
    return kSeqVariants[v].name;
}

int mvg_gemv_exact_auto_variant(int64_t lda, int64_t m, int64_t k) {
    return pick_seq_variant(lda, m, k, true, lda % 16 == 0);
}

int mvg_gemv_exact_variant(const double* A, int64_t lda, const double* x, double* y, int64_t m, int64_t k,
                           int variant, void* stream) {
    if (m < 0 || k < 0) return fail(MVG_E_INVALID, "mvg_gemv_exact: negative size");
    if (variant < 0 || variant >= kNumSeqVariants || (variant > 0 && !kSeqVariants[variant].fn))
        return fail(MVG_E_INVALID, "mvg_gemv_exact: bad variant");
    if (m == 0) return MVG_OK;
    if (!y) return fail(MVG_E_INVALID, "mvg_gemv_exact: null y");
    hipStream_t s = (hipStream_t)stream;
    if (k > 0) {
        if (!A || !x) return fail(MVG_E_INVALID, "mvg_gemv_exact: null A or x");
        if (lda < k) return fail(MVG_E_INVALID, "mvg_gemv_exact: lda < k");
    }
    // An error the caller's last HIP call left pending is that call's: reported here as it is
    // (this call fails, nothing launched), before any HIP call of ours (the dispatch's device
    // queries included) could replace it, and never mistaken for a refusal of the launch below.
    if (int rc = take_pending_error("mvg_gemv_exact"); rc != MVG_OK) return rc;
    const bool aligned = ((uintptr_t)A % 16 == 0) && ((uintptr_t)x % 16 == 0);
    const bool lines = (uintptr_t)A % 128 == 0 && lda % 16 == 0;  // every row starts on a 128-B line
    const int v = variant == 0 ? pick_seq_variant(lda, m, k, aligned, lines) : variant;
    if (!operands_ok(kSeqVariants[v].needs, lda, aligned))
        return fail(MVG_E_INVALID, kSeqVariants[v].needs == kVec16
                                       ? "mvg_gemv_exact: 16-B variant needs 16-B aligned A, x and an even lda"
                                       : "mvg_gemv_exact: LDS-DMA variant needs 16-B aligned A, x and an even lda < 2^23");
    const SeqVariant& var = kSeqVariants[v];
    if (var.xlds && k > kXlMaxK) return fail(MVG_E_INVALID, "mvg_gemv_exact: x-in-LDS variant needs k <= 8192");
    // k == 0 runs the kernel too: every row's sum stays 0 (the reference's `sum = 0`)
    // grid-size cap: fewer than 2^32 threads per launch
    int64_t max_rows = ((1ll << 32) / (64 * var.waves) - 1) * var.rows;
    // short rows (K <= 768): at most 1 GiB of A per launch, as the tree form's one-row waves
    // (gemv.hip): config 5's 16 GiB in 2.46 ms instead of 2.58, its 2 GiB shard 316 against
    // 318 us (round 3, profiles/r03/sublaunch/)
    // (1 GiB of the bytes read, k per row, never under 65536 rows: a view's wider lda does not
    // shrink the pieces below what fills the chip)
    if (k > 0 && k <= kShortRowK) {
        int64_t cap = kShortRowLaunchBytes / (k * (int64_t)sizeof(double));
        if (cap < kMinPieceRows) cap = kMinPieceRows;
        cap = cap / var.rows * var.rows;
        if (cap < max_rows) max_rows = cap;
    }
    size_t lds = var.xlds ? (size_t)k * sizeof(double) : (size_t)var.lds_reserve;
    if (v == kHopEven)
        if (const int64_t o = g_even_lds_override.load(std::memory_order_relaxed); o > 0) lds = (size_t)o;
    for (int64_t r0 = 0; r0 < m; r0 += max_rows) {
        const int64_t mm = m - r0 < max_rows ? m - r0 : max_rows;
        const int rw = var.rows;
        hipLaunchKernelGGL(var.fn, dim3((unsigned)((mm + rw - 1) / rw)), dim3(64 * var.waves), lds, s,
                           A ? A + r0 * lda : A, lda, x, y + r0, mm, k);
        const hipError_t e = hipGetLastError();
        // A runtime that turns down the evenly placed form's LDS reservation (the first launch of
        // the call, nothing of it dispatched) gets the same sums from the one-wave form, and the
        // dispatch keeps to the one-wave forms on this device from then on.
        if (e != hipSuccess && variant == 0 && v == kHopEven && r0 == 0 && lds_refusal_confirmed(e, lds)) {
            const int dev = current_device();
            if (dev >= 0 && g_even_refused[dev].exchange(1, std::memory_order_relaxed) == 0)
                fprintf(stderr, "matvec_gpu: device %d refused %zu B of LDS for the exact kernel's evenly placed form "
                                "(%s); the exact dispatch keeps to the one-wave forms on it\n",
                        dev, lds, hipGetErrorString(e));
            return mvg_gemv_exact_variant(A, lda, x, y, m, k, kHopRows, stream);
        }
        MVG_HIP(e);
    }
    return MVG_OK;
}

int mvg_gemv_exact_even_refused(int device) {
    if (device < 0 || device >= 64) return fail(MVG_E_INVALID, "mvg_gemv_exact_even_refused: bad device");
    return g_even_refused[device].load(std::memory_order_relaxed) != 0;
}

int mvg_debug_set_cu_count(int n) {
    if (n < 0) return fail(MVG_E_INVALID, "mvg_debug_set_cu_count: negative count");
    g_cu_override.store(n, std::memory_order_relaxed);
    return MVG_OK;
}

int mvg_debug_set_exact_even_lds(int64_t bytes) {
    if (bytes < 0) return fail(MVG_E_INVALID, "mvg_debug_set_exact_even_lds: negative size");
    g_even_lds_override.store(bytes, std::memory_order_relaxed);
    for (auto& f : g_even_refused) f.store(0, std::memory_order_relaxed);
    return MVG_OK;
}

int mvg_gemv_exact(const double* A, int64_t lda, const double* x, double* y, int64_t m, int64_t k,
                   void* stream) {
    return mvg_gemv_exact_variant(A, lda, x, y, m, k, 0, stream);
}

// ---- column-panel layout (gemv_seq_hop_panel; the engine's exact mode)
int64_t mvg_exact_panel_width(int64_t m, int64_t k) {
    // where the panels beat the row-major exact dispatch (profiles/r02/panel_probe_product*.jsonl,
    // 15 shapes, and the bench's configs): the 8-lane hop forms' domain (>= 6144 rows), at least
    // 8 panels and 128 MiB (6144 x 2048 ran 4 % slower on panels), not the few-row long-row
    // corner (8192 x 16384: 3 % slower; its 1024 waves are one per SIMD), and at most 16 GiB:
    // 65536^2 (32 GiB) was 1.5 % faster on one box and 2 % slower on another, 131072^2 (128 GiB,
    // config 4 on one GPU) 3 % slower; in between 1.3-18 % faster
    if (m < 6144 || k < 2048 || m * k < (1ll << 24) || m * k > (1ll << 31)) return 0;
    if (m <= 8192 && k > 8192) return 0;
    return kPanelWidth;
}

int mvg_gemv_exact_panel_variant_count(void) { return kNumPanelVariants; }

const char* mvg_gemv_exact_panel_variant_name(int v) {
    if (v < 0 || v >= kNumPanelVariants) return "invalid";
    return kPanelVariants[v].name;
}

int mvg_gemv_exact_panel_auto_variant(int64_t m, int64_t k) {
    (void)k;
    return pick_panel_variant(m);
}

static int panel_log2(int64_t P) {
    int lp = 0;
    while ((1ll << lp) < P) ++lp;
    return (1ll << lp) == P ? lp : -1;
}

int mvg_panel_relayout(const double* A, int64_t lda, int64_t m, int64_t k, double* Ap, int64_t pstride, int64_t P,
                       void* stream) {
    const int lp = P > 0 ? panel_log2(P) : -1;
    if (m < 0 || k < 0 || lp < 0 || lda < k) return fail(MVG_E_INVALID, "mvg_panel_relayout: bad shape or panel width");
    if (m == 0 || k == 0) return MVG_OK;
    if (!A || !Ap) return fail(MVG_E_INVALID, "mvg_panel_relayout: null pointer");
    if (pstride < m * P && (k + P - 1) / P > 1) return fail(MVG_E_INVALID, "mvg_panel_relayout: pstride < m * P");
    if (int rc = take_pending_error("mvg_panel_relayout"); rc != MVG_OK) return rc;
    const int64_t blocks = m < (1ll << 20) ? m : (1ll << 20);
    const bool v16 = (uintptr_t)A % 16 == 0 && (uintptr_t)Ap % 16 == 0 && lda % 2 == 0 && P % 2 == 0 && pstride % 2 == 0;
    if (v16)
        hipLaunchKernelGGL(panel_relayout_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, A,
                           lda, m, k, Ap, pstride, lp);
    else
        hipLaunchKernelGGL(panel_relayout_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, A,
                           lda, m, k, Ap, pstride, lp);
    MVG_HIP(hipGetLastError());
    return MVG_OK;
}

int mvg_gemv_exact_panels(const double* Ap, int64_t pstride, int64_t P, const double* x, double* y, int64_t m,
                          int64_t k, int variant, void* stream) {
    if (m < 0 || k < 0) return fail(MVG_E_INVALID, "mvg_gemv_exact_panels: negative size");
    if (variant < 0 || variant >= kNumPanelVariants) return fail(MVG_E_INVALID, "mvg_gemv_exact_panels: bad variant");
    if (m == 0) return MVG_OK;
    if (!y) return fail(MVG_E_INVALID, "mvg_gemv_exact_panels: null y");
    const int v = variant == 0 ? pick_panel_variant(m) : variant;
    const int lp = P > 0 ? panel_log2(P) : -1;
    if (lp < 0 || P % kPanelVariants[v].seg != 0)
        return fail(MVG_E_INVALID, "mvg_gemv_exact_panels: P must be a power of two and a multiple of the segment");
    if (k > 0) {
        if (!Ap || !x) return fail(MVG_E_INVALID, "mvg_gemv_exact_panels: null A or x");
        if ((uintptr_t)Ap % 16 || (uintptr_t)x % 16)
            return fail(MVG_E_INVALID, "mvg_gemv_exact_panels: A and x must be 16-B aligned");
        if (pstride < m * P && (k + P - 1) / P > 1) return fail(MVG_E_INVALID, "mvg_gemv_exact_panels: pstride < m * P");
    }
    const int rw = kPanelVariants[v].rows;
    const int64_t blocks = (m + rw - 1) / rw;
    if (blocks >= (1ll << 31)) return fail(MVG_E_INVALID, "mvg_gemv_exact_panels: too many rows for one launch");
    if (int rc = take_pending_error("mvg_gemv_exact_panels"); rc != MVG_OK) return rc;
    hipLaunchKernelGGL(kPanelVariants[v].fn, dim3((unsigned)blocks), dim3(64), 0, (hipStream_t)stream, Ap, pstride, lp,
                       x, y, m, k);
    MVG_HIP(hipGetLastError());
    return MVG_OK;
}

}  // extern "C"
