// fp64 row-major GEMV for gfx950 (MI355X) — the hot kernel of all three multipliers.
//
// Replaces multiply_std_rowwise (reference src/matr_utils.c:86-96) and the strip product of
// multiply_colwise (src/multiplier_colwise.c:105-122, which is the same y = A_s * x_s done as
// scale-in-place then row-sum). Arithmetic intensity is 2 flop / 8 B, so the roofline is HBM
// bandwidth; there is nothing for MFMA to do here.
//
// Mapping: a wave64 is split into G = 64/LPR lane groups of LPR lanes. Each group owns RPG
// rows and walks them left to right together, each lane loading 16 B (two fp64, one
// global_load_dwordx4) per row per sub-step, UNR sub-steps per iteration, so one lane keeps
// RPG*UNR 16-B loads of A in flight plus UNR loads of x (x is shared by the G*RPG rows of
// the wave: x traffic is 1/(G*RPG) of A traffic and is served by L1/L2). Per-lane partial
// sums are FMAs in a fixed order, reduced across the group with xor-shuffles (DPP/permute),
// so the result is deterministic run to run. LPR = 64 serves long rows (K >= ~1024),
// LPR = 16/8 serves short rows (the 4,194,304 x 512 tall-skinny config) without idle lanes.
//
// A row stride (lda) that is odd, or a base 8 bytes off a 16-B boundary, still takes the 16-B
// kernels: their loads promise only 8-B alignment (dbl2u below) and compile to the same
// global_load_dwordx4, which gfx950 serves unaligned. Only a base off an 8-B boundary falls back
// to the scalar variants (8 B per lane, still coalesced).
#include "common.h"
#include "lds_dma.h"

#include <map>
#include <mutex>
#include <utility>

namespace mvg {

typedef double dbl2 __attribute__((ext_vector_type(2)));
// the same pair as a load type promising only 8-B alignment: still one global_load_dwordx4
// (gfx950 serves unaligned vector loads), so the 16-B kernels also run on an odd lda or a view
// 8 bytes off a 16-B boundary, with no 16-B alignment assumed anywhere in the address code
typedef double dbl2u __attribute__((ext_vector_type(2), aligned(8)));

template <bool NT>
__device__ __forceinline__ dbl2 load2(const double* p) {
    if constexpr (NT) {
        return __builtin_nontemporal_load(reinterpret_cast<const dbl2u*>(p));
    } else {
        return *reinterpret_cast<const dbl2u*>(p);
    }
}

template <bool NT>
__device__ __forceinline__ double load1(const double* p) {
    if constexpr (NT) {
        return __builtin_nontemporal_load(p);
    } else {
        return *p;
    }
}

template <int LPR>
__device__ __forceinline__ double group_sum(double v) {
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// One DPP lane permutation of an fp64 value (two 32-bit v_mov_b32_dpp): a VALU op, no LDS
// round trip, unlike the ds_bpermute_b32 pair __shfl_xor compiles to.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), CTRL, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, lane);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), lane);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// Sum over each group of LPR lanes with DPP: quad xor 1, quad xor 2, row half-mirror (8 lanes),
// row mirror (16 lanes) — after each step every lane of the span holds the same value, since
// fp64 addition is commutative (a + b == b + a bit for bit) — then one xor-16 shuffle for
// 32-lane groups, or the four 16-lane row sums read as scalars for the whole wave.
// Fixed order throughout: deterministic, and the same value in every lane of a group (lane 0
// of the group stores it; for LPR = 64 the result is wave-uniform).
template <int LPR>
__device__ __forceinline__ double group_sum_dpp(double v) {
    static_assert(LPR == 8 || LPR == 16 || LPR == 32 || LPR == 64, "DPP group size");
    v += dpp_d<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_d<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp_d<0x141>(v);  // row_half_mirror
    if constexpr (LPR >= 16) v += dpp_d<0x140>(v);  // row_mirror
    if constexpr (LPR == 32) v += __shfl_xor(v, 16, 64);
    if constexpr (LPR == 64)
        v = (readlane_d(v, 0) + readlane_d(v, 16)) + (readlane_d(v, 32) + readlane_d(v, 48));
    return v;
}

constexpr int kBlock = 256;  // 4 waves

// Options of the 16-B kernel (template bit mask).
constexpr int kPipe = 1;     // software pipeline: chunk i+1's loads issue before chunk i's FMAs
constexpr int kStagger = 2;  // each wave starts at its own column chunk and wraps around, so the
                             // waves in flight read spread-out columns instead of all the same one
constexpr int kDpp = 4;      // cross-lane sums with DPP (group_sum_dpp) instead of ds_bpermute

template <int RPG, int UNR, bool NT>
__device__ __forceinline__ void load_chunk(const double* const (&arow)[RPG], const double* x, int64_t base,
                                           int64_t step, dbl2 (&xv)[UNR], dbl2 (&av)[RPG][UNR]) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) xv[u] = load2<false>(x + base + u * step);
#pragma unroll
    for (int r = 0; r < RPG; ++r)
#pragma unroll
        for (int u = 0; u < UNR; ++u) av[r][u] = load2<NT>(arow[r] + base + u * step);
}

template <int RPG, int UNR>
__device__ __forceinline__ void fma_chunk(double (&acc)[RPG], const dbl2 (&xv)[UNR], const dbl2 (&av)[RPG][UNR]) {
#pragma unroll
    for (int r = 0; r < RPG; ++r)
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            acc[r] = __builtin_fma(av[r][u].x, xv[u].x, acc[r]);
            acc[r] = __builtin_fma(av[r][u].y, xv[u].y, acc[r]);
        }
}

// 16-B path (A and x 8-B aligned; fastest with an even lda and 16-B aligned A, x).
template <int LPR, int RPG, int UNR, bool NT, int OPT>
__global__ __launch_bounds__(kBlock) void gemv_vec(const double* __restrict__ A, int64_t lda,
                                                   const double* __restrict__ x,
                                                   double* __restrict__ y, int64_t M,
                                                   int64_t K) {
    constexpr int G = 64 / LPR;
    const int lane = threadIdx.x & 63;
    const int g = lane / LPR;
    const int gl = lane % LPR;
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const int64_t row0 = (wave * G + g) * RPG;

    const double* arow[RPG];
#pragma unroll
    for (int r = 0; r < RPG; ++r) {
        int64_t rr = row0 + r;
        rr = rr < M ? rr : M - 1;  // clamp: out-of-range rows re-read a valid row, never stored
        arow[r] = A + rr * lda;
    }
    double acc[RPG];
#pragma unroll
    for (int r = 0; r < RPG; ++r) acc[r] = 0.0;

    constexpr int64_t kStep = 2 * LPR;        // columns one group covers per sub-step
    constexpr int64_t kChunk = kStep * UNR;   // columns per iteration
    const int64_t nch = K / kChunk;
    const int64_t kmain = nch * kChunk;
    const int64_t c0 = 2 * gl;
    int64_t start = 0;
    if constexpr ((OPT & kStagger) != 0) start = nch > 0 ? (wave * 5) % nch : 0;
    auto chunk_base = [&](int64_t i) {
        int64_t c = start + i;
        if (c >= nch) c -= nch;
        return c * kChunk + c0;
    };

    if constexpr ((OPT & kPipe) != 0) {
        if (nch > 0) {
            dbl2 xa[UNR], xb[UNR];
            dbl2 aa[RPG][UNR], ab[RPG][UNR];
            load_chunk<RPG, UNR, NT>(arow, x, chunk_base(0), kStep, xa, aa);
            int64_t i = 1;
            for (; i + 1 < nch; i += 2) {
                load_chunk<RPG, UNR, NT>(arow, x, chunk_base(i), kStep, xb, ab);
                fma_chunk<RPG, UNR>(acc, xa, aa);
                load_chunk<RPG, UNR, NT>(arow, x, chunk_base(i + 1), kStep, xa, aa);
                fma_chunk<RPG, UNR>(acc, xb, ab);
            }
            if (i < nch) {
                load_chunk<RPG, UNR, NT>(arow, x, chunk_base(i), kStep, xb, ab);
                fma_chunk<RPG, UNR>(acc, xa, aa);
                fma_chunk<RPG, UNR>(acc, xb, ab);
            } else {
                fma_chunk<RPG, UNR>(acc, xa, aa);
            }
        }
    } else {
        for (int64_t i = 0; i < nch; ++i) {
            dbl2 xv[UNR];
            dbl2 av[RPG][UNR];
            load_chunk<RPG, UNR, NT>(arow, x, chunk_base(i), kStep, xv, av);
            fma_chunk<RPG, UNR>(acc, xv, av);
        }
    }
    // column tail: whole pairs, then a possible last odd column
    for (int64_t c = kmain + c0; c < K; c += kStep) {
        if (c + 1 < K) {
            const dbl2 xv = load2<false>(x + c);
#pragma unroll
            for (int r = 0; r < RPG; ++r) {
                const dbl2 a = load2<NT>(arow[r] + c);
                acc[r] = __builtin_fma(a.x, xv.x, acc[r]);
                acc[r] = __builtin_fma(a.y, xv.y, acc[r]);
            }
        } else {
            const double xs = x[c];
#pragma unroll
            for (int r = 0; r < RPG; ++r) acc[r] = __builtin_fma(arow[r][c], xs, acc[r]);
        }
    }
#pragma unroll
    for (int r = 0; r < RPG; ++r) {
        const double s = (OPT & kDpp) != 0 ? group_sum_dpp<LPR>(acc[r]) : group_sum<LPR>(acc[r]);
        if (gl == 0 && row0 + r < M) y[row0 + r] = s;
    }
}

// Row-per-workgroup 16-B path: workgroup b (NW waves) owns rows [b*RPB, +RPB); wave w takes
// column chunks w, w+NW, w+2NW, ... of every such row (a chunk = 64 lanes x UNR x 16 B), so the
// workgroup sweeps its rows front to back and consecutive workgroups - which the dispatcher
// keeps resident together - read consecutive memory: the chip streams a sliding window of A
// instead of thousands of scattered row positions. Per-wave partial sums meet in LDS and are
// added in wave order (fixed, deterministic). Pipelined: chunk i+NW's loads issue before
// chunk i's FMAs.
// XCD-aware order: the dispatcher deals workgroups round-robin over the 8 XCDs, so without a
// remap XCD k streams rows {b : b % 8 == k}; with it, XCD k streams one contiguous row range.
// Bijective for any grid size (the guide's remap for nwg % 8 != 0). Speed only, never
// correctness.
__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t nwg) {
    const int64_t q = nwg / 8, r = nwg % 8, xcd = b % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
}

// Chunked XCD order: XCD k takes runs of Q consecutive workgroups, the 8 XCDs' runs side by
// side, so each XCD still streams contiguous memory while all of them stay inside one sliding
// window (the full-range remap above puts the XCDs' streams R/8 rows apart, a power-of-two
// distance for power-of-two shapes). Identity on the tail that does not fill 8*Q.
template <int Q>
__device__ __forceinline__ int64_t xcd_chunk_remap(int64_t b, int64_t nwg) {
    const int64_t full = nwg / (8 * Q) * (8 * Q);
    if (b >= full) return b;
    const int64_t xcd = b % 8, j = b / 8;
    return ((j / Q) * 8 + xcd) * Q + j % Q;
}

template <int NW, int RPB, int UNR, bool NT, int XCD = 0>
__global__ __launch_bounds__(NW * 64) void gemv_rowblock(const double* __restrict__ A, int64_t lda,
                                                         const double* __restrict__ x,
                                                         double* __restrict__ y, int64_t M,
                                                         int64_t K) {
    __shared__ double part[NW][RPB];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    int64_t bid = blockIdx.x;
    if constexpr (XCD == 1) bid = xcd_remap(bid, gridDim.x);
    if constexpr (XCD > 1) bid = xcd_chunk_remap<XCD>(bid, gridDim.x);
    const int64_t row0 = bid * RPB;
    const double* arow[RPB];
#pragma unroll
    for (int r = 0; r < RPB; ++r) {
        int64_t rr = row0 + r;
        rr = rr < M ? rr : M - 1;
        arow[r] = A + rr * lda;
    }
    double acc[RPB];
#pragma unroll
    for (int r = 0; r < RPB; ++r) acc[r] = 0.0;

    constexpr int64_t kStep = 128;            // columns per wave per sub-step (64 lanes x 2)
    constexpr int64_t kChunk = kStep * UNR;
    const int64_t nch = K / kChunk;
    const int64_t c0 = 2 * lane;
    int64_t i = w;
    if (i < nch) {
        dbl2 xa[UNR], xb[UNR];
        dbl2 aa[RPB][UNR], ab[RPB][UNR];
        load_chunk<RPB, UNR, NT>(arow, x, i * kChunk + c0, kStep, xa, aa);
        for (; i + NW < nch; i += 2 * NW) {
            load_chunk<RPB, UNR, NT>(arow, x, (i + NW) * kChunk + c0, kStep, xb, ab);
            fma_chunk<RPB, UNR>(acc, xa, aa);
            if (i + 2 * NW < nch) {
                load_chunk<RPB, UNR, NT>(arow, x, (i + 2 * NW) * kChunk + c0, kStep, xa, aa);
                fma_chunk<RPB, UNR>(acc, xb, ab);
            } else {
                fma_chunk<RPB, UNR>(acc, xb, ab);
                i = nch;  // both buffers consumed
                break;
            }
        }
        if (i < nch) fma_chunk<RPB, UNR>(acc, xa, aa);
    }
    // column tail (K % kChunk), spread over the whole workgroup
    for (int64_t c = nch * kChunk + 2 * (int64_t)threadIdx.x; c < K; c += 2 * NW * 64) {
        if (c + 1 < K) {
            const dbl2 xv = load2<false>(x + c);
#pragma unroll
            for (int r = 0; r < RPB; ++r) {
                const dbl2 a = load2<NT>(arow[r] + c);
                acc[r] = __builtin_fma(a.x, xv.x, acc[r]);
                acc[r] = __builtin_fma(a.y, xv.y, acc[r]);
            }
        } else {
            const double xs = x[c];
#pragma unroll
            for (int r = 0; r < RPB; ++r) acc[r] = __builtin_fma(arow[r][c], xs, acc[r]);
        }
    }
#pragma unroll
    for (int r = 0; r < RPB; ++r) {
        const double s = group_sum_dpp<64>(acc[r]);
        if (lane == 0) part[w][r] = s;
    }
    __syncthreads();
    if (threadIdx.x < RPB && row0 + threadIdx.x < M) {
        double s = 0.0;
#pragma unroll
        for (int v = 0; v < NW; ++v) s += part[v][threadIdx.x];
        y[row0 + threadIdx.x] = s;
    }
}

// Row-per-workgroup form for rows that do not start on 128-B lines (an lda that is not a
// multiple of 16 — the reference's 4200 and 10200, every odd width — or a view off a line):
// there each 1-KiB wave load spans 9 cache lines instead of 8 (7 % more L2 requests at
// 16384 x 16386, profiles/r02/pmc_exact_gemv_seq_hop_final_16384x16386.json). Rows r and r + p
// with p = 16 >> min(ctz(lda), 4) start at the same offset within a line (p * lda * 8 is a
// multiple of 128), so a workgroup takes that pair: both rows first add their h columns up to
// the next line (h the same for both, 0 ... 15 columns, lanes 0 .. h-1 of wave 0), then stream
// line-aligned chunks against x shifted by the same h — x stays one load for both rows, as in
// gemv_rowblock. Workgroup b of a block of 2p rows takes rows (b mod p, b mod p + p): the pairs
// of a block cover it, consecutive workgroups still read neighbouring rows.
template <int NW, int UNR, bool NT, int XCD = 0>
__global__ __launch_bounds__(NW * 64) void gemv_rowblock_lines(const double* __restrict__ A, int64_t lda,
                                                               const double* __restrict__ x,
                                                               double* __restrict__ y, int64_t M,
                                                               int64_t K) {
    constexpr int RPB = 2;
    __shared__ double part[NW][RPB];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    int64_t bid = blockIdx.x;
    if constexpr (XCD == 1) bid = xcd_remap(bid, gridDim.x);
    const int tz = lda == 0 ? 4 : __builtin_ctzll((unsigned long long)lda);
    const int64_t p = 16 >> (tz < 4 ? tz : 4);
    const int64_t row_of[RPB] = {bid / p * 2 * p + bid % p, bid / p * 2 * p + bid % p + p};
    const double* arow[RPB];
#pragma unroll
    for (int r = 0; r < RPB; ++r) arow[r] = A + (row_of[r] < M ? row_of[r] : M - 1) * lda;
    int64_t h = (int64_t)(((128u - ((uintptr_t)arow[0] & 127u)) & 127u) >> 3);
    h = h < K ? h : K;
    double acc[RPB];
#pragma unroll
    for (int r = 0; r < RPB; ++r) acc[r] = threadIdx.x < h ? arow[r][threadIdx.x] * x[threadIdx.x] : 0.0;
#pragma unroll
    for (int r = 0; r < RPB; ++r) arow[r] += h;
    const double* xs = x + h;
    const int64_t Kh = K - h;

    constexpr int64_t kStep = 128;
    constexpr int64_t kChunk = kStep * UNR;
    const int64_t nch = Kh / kChunk;
    const int64_t c0 = 2 * lane;
    int64_t i = w;
    if (i < nch) {
        dbl2 xa[UNR], xb[UNR];
        dbl2 aa[RPB][UNR], ab[RPB][UNR];
        load_chunk<RPB, UNR, NT>(arow, xs, i * kChunk + c0, kStep, xa, aa);
        for (; i + NW < nch; i += 2 * NW) {
            load_chunk<RPB, UNR, NT>(arow, xs, (i + NW) * kChunk + c0, kStep, xb, ab);
            fma_chunk<RPB, UNR>(acc, xa, aa);
            if (i + 2 * NW < nch) {
                load_chunk<RPB, UNR, NT>(arow, xs, (i + 2 * NW) * kChunk + c0, kStep, xa, aa);
                fma_chunk<RPB, UNR>(acc, xb, ab);
            } else {
                fma_chunk<RPB, UNR>(acc, xb, ab);
                i = nch;
                break;
            }
        }
        if (i < nch) fma_chunk<RPB, UNR>(acc, xa, aa);
    }
    for (int64_t c = nch * kChunk + 2 * (int64_t)threadIdx.x; c < Kh; c += 2 * NW * 64) {
        if (c + 1 < Kh) {
            const dbl2 xv = load2<false>(xs + c);
#pragma unroll
            for (int r = 0; r < RPB; ++r) {
                const dbl2 a = load2<NT>(arow[r] + c);
                acc[r] = __builtin_fma(a.x, xv.x, acc[r]);
                acc[r] = __builtin_fma(a.y, xv.y, acc[r]);
            }
        } else {
            const double xv = xs[c];
#pragma unroll
            for (int r = 0; r < RPB; ++r) acc[r] = __builtin_fma(arow[r][c], xv, acc[r]);
        }
    }
#pragma unroll
    for (int r = 0; r < RPB; ++r) {
        const double s = group_sum_dpp<64>(acc[r]);
        if (lane == 0) part[w][r] = s;
    }
    __syncthreads();
    if (threadIdx.x < RPB && row_of[threadIdx.x] < M) {
        double s = 0.0;
#pragma unroll
        for (int v = 0; v < NW; ++v) s += part[v][threadIdx.x];
        y[row_of[threadIdx.x]] = s;
    }
}

// Split-K for short, wide problems (few rows, so too few row workgroups to fill 256 CUs):
// workgroup b takes row block b / S and K-range b % S of width ks (a multiple of the chunk), so
// consecutive workgroups still read consecutive memory; the partial sums go to
// partial[row * S + s] and gemv_splitk_reduce adds them in s order (deterministic).
template <int NW, int RPB, int UNR, bool NT>
__global__ __launch_bounds__(NW * 64) void gemv_rowblock_split(const double* __restrict__ A,
                                                               int64_t lda,
                                                               const double* __restrict__ x,
                                                               double* __restrict__ partial,
                                                               int64_t M, int64_t Kfull, int64_t ks,
                                                               int64_t S) {
    __shared__ double part[NW][RPB];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int64_t rb = (int64_t)blockIdx.x / S;
    const int64_t sp = (int64_t)blockIdx.x % S;
    const int64_t k0 = sp * ks;
    const int64_t K = (k0 + ks < Kfull ? k0 + ks : Kfull) - k0;  // this workgroup's K-range
    const int64_t row0 = rb * RPB;
    A += k0;
    x += k0;
    const double* arow[RPB];
#pragma unroll
    for (int r = 0; r < RPB; ++r) {
        int64_t rr = row0 + r;
        rr = rr < M ? rr : M - 1;
        arow[r] = A + rr * lda;
    }
    double acc[RPB];
#pragma unroll
    for (int r = 0; r < RPB; ++r) acc[r] = 0.0;

    constexpr int64_t kStep = 128;            // columns per wave per sub-step (64 lanes x 2)
    constexpr int64_t kChunk = kStep * UNR;
    const int64_t nch = K / kChunk;
    const int64_t c0 = 2 * lane;
    int64_t i = w;
    if (i < nch) {
        dbl2 xa[UNR], xb[UNR];
        dbl2 aa[RPB][UNR], ab[RPB][UNR];
        load_chunk<RPB, UNR, NT>(arow, x, i * kChunk + c0, kStep, xa, aa);
        for (; i + NW < nch; i += 2 * NW) {
            load_chunk<RPB, UNR, NT>(arow, x, (i + NW) * kChunk + c0, kStep, xb, ab);
            fma_chunk<RPB, UNR>(acc, xa, aa);
            if (i + 2 * NW < nch) {
                load_chunk<RPB, UNR, NT>(arow, x, (i + 2 * NW) * kChunk + c0, kStep, xa, aa);
                fma_chunk<RPB, UNR>(acc, xb, ab);
            } else {
                fma_chunk<RPB, UNR>(acc, xb, ab);
                i = nch;  // both buffers consumed
                break;
            }
        }
        if (i < nch) fma_chunk<RPB, UNR>(acc, xa, aa);
    }
    // column tail (K % kChunk), spread over the whole workgroup
    for (int64_t c = nch * kChunk + 2 * (int64_t)threadIdx.x; c < K; c += 2 * NW * 64) {
        if (c + 1 < K) {
            const dbl2 xv = load2<false>(x + c);
#pragma unroll
            for (int r = 0; r < RPB; ++r) {
                const dbl2 a = load2<NT>(arow[r] + c);
                acc[r] = __builtin_fma(a.x, xv.x, acc[r]);
                acc[r] = __builtin_fma(a.y, xv.y, acc[r]);
            }
        } else {
            const double xs = x[c];
#pragma unroll
            for (int r = 0; r < RPB; ++r) acc[r] = __builtin_fma(arow[r][c], xs, acc[r]);
        }
    }
#pragma unroll
    for (int r = 0; r < RPB; ++r) {
        const double s = group_sum_dpp<64>(acc[r]);
        if (lane == 0) part[w][r] = s;
    }
    __syncthreads();
    if (threadIdx.x < RPB && row0 + threadIdx.x < M) {
        double s = 0.0;
#pragma unroll
        for (int v = 0; v < NW; ++v) s += part[v][threadIdx.x];
        partial[(row0 + threadIdx.x) * S + sp] = s;
    }
}

__global__ void gemv_splitk_reduce(const double* __restrict__ partial, int64_t S,
                                   double* __restrict__ y, int64_t M) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < M;
         r += (int64_t)gridDim.x * blockDim.x) {
        const double* p = partial + r * S;
        double s = 0.0;
        for (int64_t j = 0; j < S; ++j) s += p[j];
        y[r] = s;
    }
}

// 8-B path: any lda, any 8-B alignment.
template <int LPR, int RPG, int UNR, bool NT>
__global__ __launch_bounds__(kBlock) void gemv_scalar(const double* __restrict__ A, int64_t lda,
                                                      const double* __restrict__ x,
                                                      double* __restrict__ y, int64_t M,
                                                      int64_t K) {
    constexpr int G = 64 / LPR;
    const int lane = threadIdx.x & 63;
    const int g = lane / LPR;
    const int gl = lane % LPR;
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const int64_t row0 = (wave * G + g) * RPG;

    const double* arow[RPG];
#pragma unroll
    for (int r = 0; r < RPG; ++r) {
        int64_t rr = row0 + r;
        rr = rr < M ? rr : M - 1;
        arow[r] = A + rr * lda;
    }
    double acc[RPG];
#pragma unroll
    for (int r = 0; r < RPG; ++r) acc[r] = 0.0;

    constexpr int64_t kStep = LPR;
    constexpr int64_t kChunk = kStep * UNR;
    const int64_t kmain = (K / kChunk) * kChunk;
    for (int64_t base = gl; base < kmain; base += kChunk) {
        double xv[UNR];
        double av[RPG][UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) xv[u] = x[base + u * kStep];
#pragma unroll
        for (int r = 0; r < RPG; ++r)
#pragma unroll
            for (int u = 0; u < UNR; ++u) av[r][u] = load1<NT>(arow[r] + base + u * kStep);
#pragma unroll
        for (int r = 0; r < RPG; ++r)
#pragma unroll
            for (int u = 0; u < UNR; ++u) acc[r] = __builtin_fma(av[r][u], xv[u], acc[r]);
    }
    for (int64_t c = kmain + gl; c < K; c += kStep) {
        const double xs = x[c];
#pragma unroll
        for (int r = 0; r < RPG; ++r) acc[r] = __builtin_fma(arow[r][c], xs, acc[r]);
    }
#pragma unroll
    for (int r = 0; r < RPG; ++r) {
        const double s = group_sum<LPR>(acc[r]);
        if (gl == 0 && row0 + r < M) y[row0 + r] = s;
    }
}

// ------------------------------------------------------------------ variant table
typedef void (*gemv_fn)(const double*, int64_t, const double*, double*, int64_t, int64_t);

typedef void (*gemv_split_fn)(const double*, int64_t, const double*, double*, int64_t, int64_t,
                              int64_t, int64_t);


struct Variant {
    const char* name;
    gemv_fn fn;
    int rows_per_block;  // rows one workgroup covers
    bool vec;            // needs 16-B alignment + even lda
    int threads;         // workgroup size
    gemv_split_fn split = nullptr;  // split-K form (row-per-workgroup variants only)
    int chunk = 0;                  // columns per wave chunk (split width granule)
    int extra_blocks = 0;           // workgroups past ceil(m / rows): the row-pair forms' last block
};

#define VEC(LPR, RPG, UNR, NT, OPT)                                                             \
    {"vec_l" #LPR "_r" #RPG "_u" #UNR "_nt" #NT "_o" #OPT, gemv_vec<LPR, RPG, UNR, NT, OPT>, \
     (kBlock / 64) * (64 / LPR) * RPG, true, kBlock}
#define SCL(LPR, RPG, UNR, NT)                                                              \
    {"scl_l" #LPR "_r" #RPG "_u" #UNR "_nt" #NT, gemv_scalar<LPR, RPG, UNR, NT>,            \
     (kBlock / 64) * (64 / LPR) * RPG, false, kBlock}
#define RWB(NW, RPB, UNR)                                                                  \
    {"rowblk_w" #NW "_r" #RPB "_u" #UNR, gemv_rowblock<NW, RPB, UNR, true>, RPB, true, NW * 64}
#define RWS(NW, RPB, UNR)                                                                  \
    {"rowblk_w" #NW "_r" #RPB "_u" #UNR "_splitk", nullptr, RPB, true, NW * 64,                \
     gemv_rowblock_split<NW, RPB, UNR, true>, 128 * UNR}
#define RWX(NW, RPB, UNR)                                                                  \
    {"rowblk_w" #NW "_r" #RPB "_u" #UNR "_xcd", gemv_rowblock<NW, RPB, UNR, true, 1>, RPB, true, NW * 64}
#define RWL(NW, UNR, XCD)                                                                  \
    {"rowlines_w" #NW "_u" #UNR "_x" #XCD, gemv_rowblock_lines<NW, UNR, true, XCD>, 2, true, NW * 64, \
     nullptr, 0, 16}
#define RWQ(NW, RPB, UNR, Q)                                                               \
    {"rowblk_w" #NW "_r" #RPB "_u" #UNR "_xq" #Q, gemv_rowblock<NW, RPB, UNR, true, Q>, RPB, true, NW * 64}

static constexpr Variant kVariants[] = {
    {"auto", nullptr, 0, false},   // 0
    VEC(64, 4, 4, 0, 0),           // 1
    VEC(64, 4, 4, 1, 0),           // 2
    VEC(64, 2, 8, 1, 0),           // 3
    VEC(64, 8, 2, 1, 0),           // 4
    VEC(64, 1, 8, 1, 0),           // 5
    VEC(32, 2, 4, 1, 0),           // 6
    VEC(16, 2, 4, 1, 0),           // 7
    VEC(8, 2, 4, 1, 0),            // 8
    SCL(64, 4, 4, 1),              // 9
    SCL(16, 2, 4, 1),              // 10
    VEC(64, 4, 4, 1, 1),           // 11 pipelined
    VEC(64, 2, 4, 1, 1),           // 12
    VEC(64, 4, 4, 1, 2),           // 13 staggered
    VEC(64, 2, 8, 1, 2),           // 14
    VEC(64, 2, 4, 1, 3),           // 15 both
    VEC(64, 4, 2, 1, 3),           // 16
    VEC(32, 2, 4, 1, 2),           // 17
    VEC(32, 2, 2, 1, 3),           // 18
    VEC(64, 1, 4, 1, 1),           // 19
    VEC(64, 1, 8, 1, 2),           // 20
    RWB(4, 1, 4),                  // 21 row per workgroup
    RWB(8, 1, 4),                  // 22
    RWB(16, 1, 4),                 // 23
    RWB(8, 2, 4),                  // 24
    RWB(8, 1, 2),                  // 25
    RWB(16, 1, 2),                 // 26
    RWB(4, 2, 4),                  // 27
    RWB(8, 2, 2),                  // 28
    RWB(8, 4, 2),                  // 29
    RWB(4, 4, 2),                  // 30
    RWB(16, 2, 4),                 // 31
    RWB(4, 2, 8),                  // 32
    RWB(2, 2, 4),                  // 33
    RWB(2, 4, 4),                  // 34
    RWB(4, 4, 4),                  // 35
    VEC(64, 2, 4, 1, 0),           // 36 short rows: 2 rows per wave, unpipelined
    VEC(32, 1, 4, 1, 1),           // 37 two 512-col rows per wave, pipelined
    VEC(32, 2, 4, 1, 1),           // 38
    VEC(64, 1, 2, 1, 1),           // 39
    VEC(16, 1, 4, 1, 0),           // 40
    RWX(4, 2, 8),                  // 41 XCD-remapped
    RWX(8, 2, 4),                  // 42
    RWB(8, 2, 8),                  // 43
    RWB(4, 3, 8),                  // 44
    RWX(4, 1, 8),                  // 45
    RWB(4, 1, 8),                  // 46
    RWS(4, 2, 8),                  // 47 split-K
    RWS(4, 2, 4),                  // 48
    RWS(4, 1, 8),                  // 49
    RWS(8, 1, 4),                  // 50
    RWS(4, 1, 4),                  // 51
    RWQ(4, 2, 8, 16),              // 52 chunked XCD order
    RWQ(4, 2, 8, 64),              // 53
    RWQ(4, 2, 8, 256),             // 54
    RWQ(8, 2, 4, 64),              // 55
    RWQ(4, 2, 8, 4),               // 56
    VEC(64, 1, 4, 1, 5),           // 57 DPP cross-lane sums (kDpp)
    VEC(64, 1, 8, 1, 4),           // 58
    VEC(64, 2, 4, 1, 7),           // 59
    VEC(64, 4, 4, 1, 5),           // 60
    VEC(32, 1, 4, 1, 5),           // 61
    VEC(32, 2, 4, 1, 4),           // 62
    VEC(16, 1, 4, 1, 4),           // 63
    VEC(16, 2, 4, 1, 4),           // 64
    VEC(8, 2, 4, 1, 4),            // 65
    RWL(4, 8, 0),                  // 66 rows off the 128-B lines: line-aligned row pairs
    RWL(4, 8, 1),                  // 67
    RWL(8, 4, 0),                  // 68
    RWL(2, 4, 0),                  // 69
};
constexpr int kNumVariants = (int)(sizeof(kVariants) / sizeof(kVariants[0]));

// Variants are addressed by name, resolved at compile time: inserting or removing a table
// entry cannot send a shape to the wrong kernel (a missing name fails the build).
constexpr bool name_eq(const char* a, const char* b) {
    while (*a && *a == *b) ++a, ++b;
    return *a == *b;
}
template <typename T, size_t N>
constexpr int variant_id(const T (&table)[N], const char* name) {
    for (size_t i = 0; i < N; ++i)
        if (name_eq(table[i].name, name)) return (int)i;
    return -1;
}
constexpr int kScalarLong = variant_id(kVariants, "scl_l64_r4_u4_nt1");   // 8-B path, K >= 256
constexpr int kScalarShort = variant_id(kVariants, "scl_l16_r2_u4_nt1");  // 8-B path, K < 256
constexpr int kSplitK = variant_id(kVariants, "rowblk_w4_r2_u4_splitk");
constexpr int kRowLong = variant_id(kVariants, "rowblk_w4_r2_u8");
constexpr int kRowMid = variant_id(kVariants, "rowblk_w8_r2_u4");
constexpr int kRowSmall = variant_id(kVariants, "rowblk_w2_r2_u4");
constexpr int kVecTwoRows = variant_id(kVariants, "vec_l64_r2_u4_nt1_o7");
constexpr int kVecFourRows = variant_id(kVariants, "vec_l64_r4_u4_nt1_o5");
constexpr int kVecOneRow = variant_id(kVariants, "vec_l64_r1_u4_nt1_o5");
constexpr int kRowLongOdd = variant_id(kVariants, "rowblk_w4_r2_u8_xcd");
constexpr int kRowLines = variant_id(kVariants, "rowlines_w8_u4_x0");
constexpr int kVecFourRowsOdd = variant_id(kVariants, "vec_l64_r4_u4_nt1_o0");
static_assert(kScalarLong > 0 && !kVariants[kScalarLong].vec, "8-B fallback must not need 16-B loads");
static_assert(kScalarShort > 0 && !kVariants[kScalarShort].vec, "8-B fallback must not need 16-B loads");
static_assert(kSplitK > 0 && kVariants[kSplitK].split != nullptr, "split-K variant");
static_assert(kRowLong > 0 && kRowMid > 0 && kRowSmall > 0 && kVecTwoRows > 0 && kVecFourRows > 0 &&
                  kVecOneRow > 0 && kRowLongOdd > 0 && kVecFourRowsOdd > 0 && kRowLines > 0,
              "dispatch names a variant missing from kVariants");

constexpr int64_t kSplitTarget = 1024;  // workgroups a split launch aims for (4 per CU)

// Shape-adaptive choice, from the round-1 MI355X sweeps (profiles/r01/variant_sweep*.jsonl).
// Long rows (K >= 8192), by the number of 2-row workgroups nrb = M/2:
//   nrb < 700            split-K, 4 waves x 2 rows x 512-col chunks (two-pass): 120 x 60000 in
//                        13 us instead of 28, 1200 x 60000 at 6.5 TB/s instead of 5.9
//   K >= 16384           4 waves x 2 rows x 1024-col chunks (218 VGPR, 8 x 16 B in flight per
//                        row per lane)
//   8192 <= K < 16384    8 waves x 2 rows x 512-col chunks
// Workgroup order: the plain one. The XCD-contiguous order (each XCD streams one row range) won
// only 0.7-1.8 % on aligned tall shapes with the 8 ranges < 2 GiB apart (round 2,
// variant_sweep25/27/28_*.jsonl), flipped sign across allocations at 2 GiB apart and lost 5-7 %
// from 4 GiB apart: inside the +-5 % box-to-box spread, so round 3 dropped it for aligned rows.
// Shorter rows (768 < K < 8192), by the size of A (variant_sweep14_grid.jsonl: 42 shapes
// 1024..65536 x 1024..12288, the reference's test.sh squares among them):
//   A < 1 GiB         row-per-workgroup again: 2 waves x 2 rows x 512-col chunks, or 8 waves for
//                     6144 <= K with >= 700 workgroups (within 1.024x of the best variant on
//                     average over those shapes, worst 1.08x; the wave-owns-rows forms below
//                     were up to 1.57x slower there: 4200^2 29 -> 23.6 us, 1800^2 7.3 -> 5.5 us)
//   A >= 1 GiB, 4096 <= K   8 waves x 2 rows (variant_sweep26_midk_tall.jsonl, 13 shapes:
//                     131072 x 6144 906 -> 862 us, 524288 x 4096 2373 -> 2314; at K = 2048 the
//                     wave-owns-rows form stays 6 % ahead)
//   A >= 1 GiB, 1536 < K    wave-owns-2-rows, pipelined + staggered start column
//   A >= 1 GiB, K <= 1536   wave-owns-4-rows, pipelined
//   K <= 768          one row per wave (the whole row is one chunk: 524288 short waves stream
//                     consecutive memory, config 5's shard)
// The wave-owns-rows picks finish with DPP sums (kDpp, round 2): within +-0.3 % of the
// ds_bpermute forms on every swept shape (profiles/r02/variant_sweep_dpp.jsonl) — the
// reduction was never the limit — and they keep the LDS unit out of the epilogue.
// An odd lda or a view 8 bytes off a 16-B boundary (round 2: the 16-B kernels read through
// unaligned vector loads, variant_sweep21_odd.jsonl over 8 odd-width shapes): split-K for few
// long rows, else the XCD-remapped long-row form (rows alternate between 16-B aligned and not,
// and per-XCD contiguous streams win there: 16384 x 16383 307 us, 65536 x 8191 609 us, against
// 329 / 652 for the 8-B kernel); the 2-wave row form for 768 < K < 4096, wave-owns-4-rows for
// short rows. Only operands off an 8-B boundary keep the 8-B kernels.
// Rows that do not start on 128-B lines (lines == false: an lda not a multiple of 16 or A off
// a line), long (K >= 6144) and many (M >= 4096): the line-aligned row-pair form
// (gemv_rowblock_lines; variant_sweep23_lines.jsonl: 16384 x 16386 300 against 313 us,
// 16384 x 16383 300 / 307, 10200^2 120 / 123, 7800^2 70.5 / 72.1, 65536 x 8191 599 / 609).
static int pick_variant(int64_t lda, int64_t M, int64_t K, bool aligned, bool aligned8, bool lines) {
    if (!lines && aligned8 && K >= 6144 && M >= 4096) return kRowLines;
    const bool vec = aligned && (lda % 2 == 0);
    if (!vec) {
        if (!aligned8) return K >= 256 ? kScalarLong : kScalarShort;
        if (K >= 4096) return (M + 1) / 2 < 700 ? kSplitK : kRowLongOdd;
        return K > 768 ? kRowSmall : kVecFourRowsOdd;
    }
    const int64_t nrb = (M + 1) / 2;
    if (K >= 8192) {
        if (nrb < 700) return kSplitK;
        return K >= 16384 ? kRowLong : kRowMid;
    }
    if (K > 768 && M * K < (int64_t)(1ll << 27)) return K >= 6144 && nrb >= 700 ? kRowMid : kRowSmall;
    if (K >= 4096) return kRowMid;
    if (K > 1536) return kVecTwoRows;
    if (K > 768) return kVecFourRows;
    return kVecOneRow;
}

// Split-K workspace: one fp64 buffer per (device, stream), grown on demand (growth frees the
// old buffer, which hipFree synchronises); a split launch is not graph-capturable on first use.
static std::mutex g_ws_mu;
static std::map<std::pair<int, hipStream_t>, std::pair<double*, size_t>> g_ws;

static int workspace(hipStream_t s, size_t n, double** out) {
    int dev = 0;
    MVG_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_ws_mu);
    auto& e = g_ws[{dev, s}];
    if (e.second < n) {
        if (e.first) MVG_HIP(hipFree(e.first));
        e = {nullptr, 0};
        MVG_HIP(hipMalloc((void**)&e.first, n * sizeof(double)));
        e.second = n;
    }
    *out = e.first;
    return MVG_OK;
}

// Number of K-ranges for a split launch: enough workgroups to fill the chip, each wave keeping
// at least one whole chunk; `force` keeps >= 2 whenever K allows (explicit split variants).
static int64_t split_count(const Variant& var, int64_t M, int64_t K, bool force) {
    const int64_t nrb = (M + var.rows_per_block - 1) / var.rows_per_block;
    const int64_t nw = var.threads / 64;
    int64_t smax = K / (nw * var.chunk);
    if (smax < 1) smax = 1;
    int64_t S = (kSplitTarget + nrb - 1) / nrb;
    if (force && S < 2) S = 2;
    return S < smax ? S : smax;
}

// HIP caps a launch at gridDim.x * blockDim.x < 2^32 threads: very tall problems run as
// several launches over consecutive row ranges (each range is an independent GEMV).
constexpr int64_t kOneRowLaunchBytes = 1ll << 30;
constexpr int64_t kMinPieceRows = 65536;
static int launch(int v, const double* A, int64_t lda, const double* x, double* y, int64_t M,
                  int64_t K, hipStream_t s, bool force_split) {
    const Variant& var = kVariants[v];
    const int64_t max_blocks = (1ll << 31) / var.threads;
    if (var.split) {
        int64_t S = split_count(var, M, K, force_split);
        const int64_t ks = ((K + S - 1) / S + var.chunk - 1) / var.chunk * var.chunk;
        S = (K + ks - 1) / ks;
        const int64_t nrb = (M + var.rows_per_block - 1) / var.rows_per_block;
        if (nrb * S > max_blocks) return fail(MVG_E_INVALID, "mvg_gemv: split-K grid too large");
        double* partial = nullptr;
        int rc = workspace(s, (size_t)(M * S), &partial);
        if (rc != MVG_OK) return rc;
        hipLaunchKernelGGL(var.split, dim3((unsigned)(nrb * S)), dim3(var.threads), 0, s, A, lda, x, partial, M,
                           K, ks, S);
        MVG_HIP(hipGetLastError());
        const int64_t rblocks = (M + 255) / 256 < 4096 ? (M + 255) / 256 : 4096;
        hipLaunchKernelGGL(gemv_splitk_reduce, dim3((unsigned)rblocks), dim3(256), 0, s, partial, S, y, M);
        MVG_HIP(hipGetLastError());
        return MVG_OK;
    }
    int64_t max_rows = max_blocks * var.rows_per_block;
    // One row per wave (short rows): at most 1 GiB of A per launch. A longer launch of this
    // form streams at one of two rates depending on where the buffer landed (config 5's 16 GiB:
    // 2.37-2.38 ms or 2.50-2.53 ms, the slow placement in most bench runs); 1 GiB launches run at
    // 2.34-2.36 ms on either (2.39-2.40 on some boxes' fast buffers: the extra launch boundaries),
    // and the 2 GiB shard at 292 instead of 301-310 us (round 3, profiles/r03/sublaunch/).
    // (1 GiB of the bytes read, k per row — a view's wider lda does not shrink the pieces — and
    // never under 65536 rows, so a launch still fills the chip)
    if (v == kVecOneRow) {
        int64_t cap = kOneRowLaunchBytes / (K * (int64_t)sizeof(double));
        if (cap < kMinPieceRows) cap = kMinPieceRows;
        cap = cap / var.rows_per_block * var.rows_per_block;
        if (cap < max_rows) max_rows = cap;
    }
    for (int64_t r0 = 0; r0 < M; r0 += max_rows) {
        const int64_t m = M - r0 < max_rows ? M - r0 : max_rows;
        // row-pair forms: a last block of 2p rows with r < 2p rows left needs min(p, r) pairs,
        // more than ceil(r / 2); up to p = 16 spare workgroups cover it (theirs are rows >= m:
        // clamped loads, no store)
        const int64_t blocks = (m + var.rows_per_block - 1) / var.rows_per_block + var.extra_blocks;
        hipLaunchKernelGGL(var.fn, dim3((unsigned)blocks), dim3(var.threads), 0, s, A + r0 * lda, lda, x,
                           y + r0, m, K);
        MVG_HIP(hipGetLastError());
    }
    return MVG_OK;
}

// ------------------------------------------------------------------ several x per pass
// Y[:, v] = A X[:, v] for v < nv: A is streamed once for NV vectors. X and Y
// are column-major (vector v at X + v*ldx, Y + v*ldy); vectors v >= nv alias vector 0 and are
// never stored. Per lane: the A pairs of its rows and the x pairs of all NV vectors for the same
// columns, FMAs in a fixed order, then fixed-order reductions (deterministic). The x reads
// (NV per A read shared by the rows of a lane) are L2 hits: A's HBM stream is the roofline.
template <int RPG, int NV, int UNR>
__device__ __forceinline__ void mload(const double* const (&arow)[RPG], const double* const (&xv)[NV],
                                      int64_t base, int64_t step, dbl2 (&xa)[NV][UNR], dbl2 (&aa)[RPG][UNR]) {
#pragma unroll
    for (int r = 0; r < RPG; ++r)
#pragma unroll
        for (int u = 0; u < UNR; ++u) aa[r][u] = load2<true>(arow[r] + base + u * step);
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
        for (int u = 0; u < UNR; ++u) xa[v][u] = load2<false>(xv[v] + base + u * step);
}

template <int RPG, int NV, int UNR>
__device__ __forceinline__ void mfma(double (&acc)[RPG][NV], const dbl2 (&xa)[NV][UNR], const dbl2 (&aa)[RPG][UNR]) {
#pragma unroll
    for (int r = 0; r < RPG; ++r)
#pragma unroll
        for (int v = 0; v < NV; ++v)
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                acc[r][v] = __builtin_fma(aa[r][u].x, xa[v][u].x, acc[r][v]);
                acc[r][v] = __builtin_fma(aa[r][u].y, xa[v][u].y, acc[r][v]);
            }
}

template <int RPG, int NV>
__device__ __forceinline__ void mtail(double (&acc)[RPG][NV], const double* const (&arow)[RPG],
                                      const double* const (&xv)[NV], int64_t c, int64_t K) {
    if (c + 1 < K) {
        dbl2 xx[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) xx[v] = load2<false>(xv[v] + c);
#pragma unroll
        for (int r = 0; r < RPG; ++r) {
            const dbl2 a = load2<true>(arow[r] + c);
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                acc[r][v] = __builtin_fma(a.x, xx[v].x, acc[r][v]);
                acc[r][v] = __builtin_fma(a.y, xx[v].y, acc[r][v]);
            }
        }
    } else {
#pragma unroll
        for (int r = 0; r < RPG; ++r)
#pragma unroll
            for (int v = 0; v < NV; ++v) acc[r][v] = __builtin_fma(arow[r][c], xv[v][c], acc[r][v]);
    }
}

// Wave-group form (short and mid rows): a wave64 is split into 64/LPR groups of LPR lanes; each
// group owns RPG rows and walks them left to right, UNR 16-B pairs per lane per chunk, chunk
// i+1's loads issued before chunk i's FMAs. The groups of a wave read the same x addresses (one
// fetch per wave instruction), so x costs NV/(RPG*64/LPR) of A's cache-line traffic.
template <int LPR, int RPG, int NV, int UNR>
__global__ __launch_bounds__(kBlock) void gemv_mvec(const double* __restrict__ A, int64_t lda,
                                                    const double* __restrict__ X, int64_t ldx,
                                                    double* __restrict__ Y, int64_t ldy, int64_t M,
                                                    int64_t K, int nv) {
    constexpr int G = 64 / LPR;
    const int lane = threadIdx.x & 63;
    const int g = lane / LPR;
    const int gl = lane % LPR;
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const int64_t row0 = (wave * G + g) * RPG;
    const double* arow[RPG];
#pragma unroll
    for (int r = 0; r < RPG; ++r) {
        int64_t rr = row0 + r;
        rr = rr < M ? rr : M - 1;
        arow[r] = A + rr * lda;
    }
    const double* xv[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) xv[v] = X + (v < nv ? v : 0) * ldx;
    double acc[RPG][NV];
#pragma unroll
    for (int r = 0; r < RPG; ++r)
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[r][v] = 0.0;

    constexpr int64_t kStep = 2 * LPR;
    constexpr int64_t kChunk = kStep * UNR;
    const int64_t nch = K / kChunk;
    const int64_t c0 = 2 * gl;
    if (nch > 0) {
        dbl2 xa[NV][UNR], xb[NV][UNR];
        dbl2 aa[RPG][UNR], ab[RPG][UNR];
        mload<RPG, NV, UNR>(arow, xv, c0, kStep, xa, aa);
        int64_t i = 1;
        for (; i + 1 < nch; i += 2) {
            mload<RPG, NV, UNR>(arow, xv, i * kChunk + c0, kStep, xb, ab);
            mfma<RPG, NV, UNR>(acc, xa, aa);
            mload<RPG, NV, UNR>(arow, xv, (i + 1) * kChunk + c0, kStep, xa, aa);
            mfma<RPG, NV, UNR>(acc, xb, ab);
        }
        if (i < nch) {
            mload<RPG, NV, UNR>(arow, xv, i * kChunk + c0, kStep, xb, ab);
            mfma<RPG, NV, UNR>(acc, xa, aa);
            mfma<RPG, NV, UNR>(acc, xb, ab);
        } else {
            mfma<RPG, NV, UNR>(acc, xa, aa);
        }
    }
    for (int64_t c = nch * kChunk + c0; c < K; c += kStep) mtail<RPG, NV>(acc, arow, xv, c, K);
#pragma unroll
    for (int r = 0; r < RPG; ++r)
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const double s = group_sum<LPR>(acc[r][v]);
            if (gl == 0 && row0 + r < M && v < nv) Y[v * ldy + row0 + r] = s;
        }
}

// Workgroup form (long rows): workgroup b (NW waves) owns rows [b*RPB, +RPB); wave w takes
// column chunks w, w+NW, ... of them (the single-vector gemv_rowblock stream), pipelined; the
// per-wave sums meet in LDS and are added in wave order.
template <int NW, int RPB, int NV, int UNR>
__global__ __launch_bounds__(NW * 64) void gemv_mrow(const double* __restrict__ A, int64_t lda,
                                                     const double* __restrict__ X, int64_t ldx,
                                                     double* __restrict__ Y, int64_t ldy, int64_t M,
                                                     int64_t K, int nv) {
    __shared__ double part[NW][RPB][NV];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int64_t row0 = (int64_t)blockIdx.x * RPB;
    const double* arow[RPB];
#pragma unroll
    for (int r = 0; r < RPB; ++r) {
        int64_t rr = row0 + r;
        rr = rr < M ? rr : M - 1;
        arow[r] = A + rr * lda;
    }
    const double* xv[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) xv[v] = X + (v < nv ? v : 0) * ldx;
    double acc[RPB][NV];
#pragma unroll
    for (int r = 0; r < RPB; ++r)
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[r][v] = 0.0;

    constexpr int64_t kStep = 128;
    constexpr int64_t kChunk = kStep * UNR;
    const int64_t nch = K / kChunk;
    const int64_t c0 = 2 * lane;
    int64_t i = w;
    if (i < nch) {
        dbl2 xa[NV][UNR], xb[NV][UNR];
        dbl2 aa[RPB][UNR], ab[RPB][UNR];
        mload<RPB, NV, UNR>(arow, xv, i * kChunk + c0, kStep, xa, aa);
        for (; i + NW < nch; i += 2 * NW) {
            mload<RPB, NV, UNR>(arow, xv, (i + NW) * kChunk + c0, kStep, xb, ab);
            mfma<RPB, NV, UNR>(acc, xa, aa);
            if (i + 2 * NW < nch) {
                mload<RPB, NV, UNR>(arow, xv, (i + 2 * NW) * kChunk + c0, kStep, xa, aa);
                mfma<RPB, NV, UNR>(acc, xb, ab);
            } else {
                mfma<RPB, NV, UNR>(acc, xb, ab);
                i = nch;
                break;
            }
        }
        if (i < nch) mfma<RPB, NV, UNR>(acc, xa, aa);
    }
    for (int64_t c = nch * kChunk + 2 * (int64_t)threadIdx.x; c < K; c += 2 * NW * 64)
        mtail<RPB, NV>(acc, arow, xv, c, K);
#pragma unroll
    for (int r = 0; r < RPB; ++r)
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const double s = group_sum<64>(acc[r][v]);
            if (lane == 0) part[w][r][v] = s;
        }
    __syncthreads();
    for (int t = threadIdx.x; t < RPB * NV; t += NW * 64) {
        const int r = t / NV, v = t % NV;
        if (row0 + r < M && v < nv) {
            double s = 0.0;
#pragma unroll
            for (int q = 0; q < NW; ++q) s += part[q][r][v];
            Y[v * ldy + row0 + r] = s;
        }
    }
}

// LDS form (mid and long rows, nv >= 2): the mvec/mrow forms hold every vector's x pairs in
// registers next to A's, double-buffered, which leaves room for only 4-8 KiB of A in flight per
// wave at nv = 8. Here the 4 waves of a workgroup (RPW rows each) walk the same column chunks
// (128 * UNR columns) in lockstep; the chunk's x for all NV vectors is loaded once per workgroup
// (one dbl2 of it per thread per 256), parked in a double-buffered LDS tile, and read back by
// every wave with conflict-free ds_read_b128 right before its FMAs. Registers go to A: chunk
// i + 1's A and x loads are issued before chunk i's FMAs; one barrier per chunk. The column tail
// (K % chunk) reads x from global; per-lane FMAs in a fixed order, fixed-order reductions.
template <int RPW, int NV, int UNR>
__global__ __launch_bounds__(kBlock) void gemv_mlds(const double* __restrict__ A, int64_t lda,
                                                    const double* __restrict__ X, int64_t ldx,
                                                    double* __restrict__ Y, int64_t ldy, int64_t M,
                                                    int64_t K, int nv) {
    constexpr int NW = kBlock / 64;
    constexpr int CH2 = 64 * UNR;                 // dbl2 per vector per chunk
    constexpr int XP = NV * CH2 / kBlock;         // x dbl2 each thread stages per chunk
    static_assert(XP >= 1 && NV * CH2 % kBlock == 0, "x chunk must split over the workgroup");
    __shared__ dbl2 xs[2][NV][CH2];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int64_t row0 = (int64_t)blockIdx.x * (NW * RPW) + w * RPW;
    const double* arow[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        int64_t rr = row0 + r;
        rr = rr < M ? rr : M - 1;
        arow[r] = A + rr * lda;
    }
    const double* xv[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) xv[v] = X + (v < nv ? v : 0) * ldx;
    // the x pairs this thread stages: flat index j = threadIdx.x + kBlock * q over [NV][CH2]
    const double* xsrc[XP];
#pragma unroll
    for (int q = 0; q < XP; ++q) {
        const int j = threadIdx.x + kBlock * q;
        xsrc[q] = xv[j / CH2] + 2 * (j % CH2);
    }
    double acc[RPW][NV];
#pragma unroll
    for (int r = 0; r < RPW; ++r)
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[r][v] = 0.0;

    constexpr int64_t kChunk = 128 * UNR;
    const int64_t nch = K / kChunk;
    const int64_t c0 = 2 * lane;
    auto xload = [&](dbl2 (&xr)[XP], int64_t i) {
#pragma unroll
        for (int q = 0; q < XP; ++q) xr[q] = load2<false>(xsrc[q] + i * kChunk);
    };
    auto xstore = [&](int b, const dbl2 (&xr)[XP]) {
#pragma unroll
        for (int q = 0; q < XP; ++q) {
            const int j = threadIdx.x + kBlock * q;
            xs[b][j / CH2][j % CH2] = xr[q];
        }
    };
    auto aload = [&](dbl2 (&aa)[RPW][UNR], int64_t i) {
#pragma unroll
        for (int r = 0; r < RPW; ++r)
#pragma unroll
            for (int u = 0; u < UNR; ++u) aa[r][u] = load2<true>(arow[r] + i * kChunk + c0 + 128 * u);
    };
    auto compute = [&](int b, const dbl2 (&aa)[RPW][UNR]) {
#pragma unroll
        for (int u = 0; u < UNR; ++u)
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                const dbl2 xx = xs[b][v][lane + 64 * u];
#pragma unroll
                for (int r = 0; r < RPW; ++r) {
                    acc[r][v] = __builtin_fma(aa[r][u].x, xx.x, acc[r][v]);
                    acc[r][v] = __builtin_fma(aa[r][u].y, xx.y, acc[r][v]);
                }
            }
    };
    if (nch > 0) {
        dbl2 aa[RPW][UNR], ab[RPW][UNR];
        dbl2 xr[XP];
        xload(xr, 0);
        aload(aa, 0);
        xstore(0, xr);
        __syncthreads();
        int64_t i = 0;  // always even at the top: chunk i sits in aa / xs[0]
        for (; i + 1 < nch; i += 2) {
            xload(xr, i + 1);
            aload(ab, i + 1);
            compute(0, aa);
            xstore(1, xr);
            __syncthreads();
            if (i + 2 < nch) {
                xload(xr, i + 2);
                aload(aa, i + 2);
                compute(1, ab);
                xstore(0, xr);
                __syncthreads();
            } else {
                compute(1, ab);
                i = nch;  // both consumed
                break;
            }
        }
        if (i < nch) compute(0, aa);
    }
    for (int64_t c = nch * kChunk + c0; c < K; c += 128) mtail<RPW, NV>(acc, arow, xv, c, K);
#pragma unroll
    for (int r = 0; r < RPW; ++r)
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const double s = group_sum<64>(acc[r][v]);
            if (lane == 0 && row0 + r < M && v < nv) Y[v * ldy + row0 + r] = s;
        }
}

// x-resident form (short rows, several vectors): the workgroup stages x for all NV vectors in
// LDS once per 1024-column tile — for K <= 1024 that is all of x, once, behind one barrier —
// and its lane groups (LPR lanes, RPG rows each, as in gemv_mvec) walk their rows reading x
// back with ds_read_b128, so the registers hold A (UNR steps double-buffered) and accumulators
// only, and the vector-memory pipe carries A alone.
template <int LPR, int RPG, int NV, int UNR>
__global__ __launch_bounds__(kBlock) void gemv_mxres(const double* __restrict__ A, int64_t lda,
                                                     const double* __restrict__ X, int64_t ldx,
                                                     double* __restrict__ Y, int64_t ldy, int64_t M,
                                                     int64_t K, int nv) {
    constexpr int TK = 1024;  // columns per x tile
    constexpr int G = 64 / LPR;
    __shared__ dbl2 xs[NV][TK / 2];
    const int lane = threadIdx.x & 63;
    const int g = lane / LPR;
    const int gl = lane % LPR;
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const int64_t row0 = (wave * G + g) * RPG;
    const double* arow[RPG];
#pragma unroll
    for (int r = 0; r < RPG; ++r) {
        int64_t rr = row0 + r;
        rr = rr < M ? rr : M - 1;
        arow[r] = A + rr * lda;
    }
    double acc[RPG][NV];
#pragma unroll
    for (int r = 0; r < RPG; ++r)
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[r][v] = 0.0;
    constexpr int64_t kStep = 2 * LPR;  // columns per step of a lane group
    constexpr int64_t kChunk = kStep * UNR;
    auto compute = [&](const dbl2 (&aa)[RPG][UNR], int pbase) {  // pbase: this lane's pair index in the tile
#pragma unroll
        for (int u = 0; u < UNR; ++u)
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                const dbl2 xx = xs[v][pbase + LPR * u];
#pragma unroll
                for (int r = 0; r < RPG; ++r) {
                    acc[r][v] = __builtin_fma(aa[r][u].x, xx.x, acc[r][v]);
                    acc[r][v] = __builtin_fma(aa[r][u].y, xx.y, acc[r][v]);
                }
            }
    };
    auto aload = [&](dbl2 (&aa)[RPG][UNR], int64_t c) {
#pragma unroll
        for (int r = 0; r < RPG; ++r)
#pragma unroll
            for (int u = 0; u < UNR; ++u) aa[r][u] = load2<true>(arow[r] + c + kStep * u);
    };
    for (int64_t t0 = 0; t0 < K; t0 += TK) {
        const int64_t t1 = K - t0 < TK ? K : t0 + TK;
        if (t0 > 0) __syncthreads();  // every wave is done with the previous tile
        for (int j = threadIdx.x; j < NV * (TK / 2); j += kBlock) {
            const int v = j / (TK / 2), pp = j % (TK / 2);
            const int64_t c = t0 + 2 * pp;
            const double* xv = X + (v < nv ? v : 0) * ldx;
            dbl2 val = {0.0, 0.0};
            if (c + 1 < t1) val = load2<false>(xv + c);
            else if (c < t1) val.x = xv[c];
            xs[v][pp] = val;
        }
        __syncthreads();
        const int64_t nch = (t1 - t0) / kChunk;  // whole chunks in the tile
        if (nch > 0) {
            dbl2 aa[RPG][UNR], ab[RPG][UNR];
            aload(aa, t0 + 2 * gl);
            int64_t i = 0;
            for (; i + 1 < nch; i += 2) {
                aload(ab, t0 + (i + 1) * kChunk + 2 * gl);
                compute(aa, (int)(i * kChunk / 2) + gl);
                if (i + 2 < nch) {
                    aload(aa, t0 + (i + 2) * kChunk + 2 * gl);
                    compute(ab, (int)((i + 1) * kChunk / 2) + gl);
                } else {
                    compute(ab, (int)((i + 1) * kChunk / 2) + gl);
                    i = nch;
                    break;
                }
            }
            if (i < nch) compute(aa, (int)(i * kChunk / 2) + gl);
        }
        // tile tail: pairs past the whole chunks, then an odd last column (x zero-padded in LDS)
        for (int64_t c = t0 + nch * kChunk + 2 * gl; c < t1; c += kStep) {
            const int pp = (int)((c - t0) / 2);
#pragma unroll
            for (int r = 0; r < RPG; ++r) {
                dbl2 a;
                if (c + 1 < t1) {
                    a = load2<true>(arow[r] + c);
                } else {
                    a.x = arow[r][c];
                    a.y = 0.0;
                }
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    const dbl2 xx = xs[v][pp];
                    acc[r][v] = __builtin_fma(a.x, xx.x, acc[r][v]);
                    acc[r][v] = __builtin_fma(a.y, xx.y, acc[r][v]);
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < RPG; ++r)
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const double sum = group_sum<LPR>(acc[r][v]);
            if (gl == 0 && row0 + r < M && v < nv) Y[v * ldy + row0 + r] = sum;
        }
}

// A through LDS by DMA (mid and long rows, nv >= 2). The register forms above keep A's loads in
// flight in VGPRs next to RPG x NV accumulators, which at nv = 8 leaves room for too little A
// (r01: 5.6 TB/s of A at 16384^2 against 7.0 for one vector). Here A never passes through
// VGPRs on its way in: workgroup b owns rows [16*RQ*b, +16*RQ) and its NW waves split the column
// tiles (wave w takes tiles w, w + NW, ...: the workgroup sweeps its rows' columns in order, a
// sliding window over A as in gemv_rowblock). A tile is 16*RQ rows x 2T columns, loaded with
// `global_load_lds_dwordx4` (nt) into a per-wave ring of NB buffers together with the tile's x
// segment for all NV vectors (linear, [v][chunk]); NB-1 tiles in flight behind the one summed.
//   swizzle: LDS slot s of row r holds the row's 16-B chunk s ^ (r & 15), so the compute reads
//            below are conflict-free over every ds_read_b128 lane group;
//   compute: lane (i = l & 15, g = l >> 4) takes chunk 4s + g of rows i + 16q (q < RQ) at step s
//            (one ds_read_b128 per row) and the same chunk of each vector's x (a 4-address
//            broadcast), and adds its 2*RQ*NV FMAs into acc[q][v];
//   reduce : over g (xor 16, 32), then over the waves in wave order through LDS — fixed order,
//            deterministic. The column tail (K % 2T) is summed from global memory.
// Needs 16-B aligned A and X with even lda and ldx, 16*RQ rows of lda and NV rows of ldx within
// 32-bit byte offsets (host-checked: dma_ok).
template <int RQ, int T, int NB, int NW, int NV, int ROT>
__global__ __launch_bounds__(NW * 64) void gemv_mdma(const double* __restrict__ A, int64_t lda,
                                                     const double* __restrict__ X, int64_t ldx,
                                                     double* __restrict__ Y, int64_t ldy, int64_t M,
                                                     int64_t K, int nv) {
    static_assert(T == 16 || T == 32 || T == 64, "tile width: 16, 32 or 64 chunks of 16 B");
    constexpr int RB = 16 * RQ;                   // rows per workgroup
    constexpr int kRows = 64 / T;                 // rows one DMA instruction fills (1 KiB)
    constexpr int kInst = RB / kRows;             // A instructions per tile
    constexpr int kXInst = (NV * T + 63) / 64;    // x instructions per tile
    constexpr int kPer = kInst + kXInst;
    static_assert(kPer * (NB - 1) <= 63, "loads in flight must fit the vmcnt counter");
    constexpr int kCols = 2 * T;
    constexpr int kRowBytes = 16 * T;
    constexpr int kTileBytes = RB * kRowBytes;
    constexpr int kBufBytes = kTileBytes + kXInst * 1024;
    static_assert(NB * kBufBytes >= RQ * NV * 16 * (int)sizeof(double), "partials fit the ring");
    __shared__ __attribute__((aligned(16))) unsigned char lds[NW][NB * kBufBytes];

    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int64_t r0 = (int64_t)blockIdx.x * RB;
    const int64_t ntiles = K / kCols;
    unsigned char* const ring = lds[w];

    // DMA side: A instruction j, lane -> tile row j*kRows + lane/T (rows past M re-read the
    // last row), LDS slot lane%T; x instruction j, lane -> flat [v][chunk] index 64j + lane
    // (vectors past nv re-read vector 0, indices past NV*T land in the padding).
    uint32_t aoff[kInst], xoff[kXInst];
#pragma unroll
    for (int j = 0; j < kInst; ++j) {
        const int row = j * kRows + lane / T;
        const int64_t rr = r0 + row < M ? row : M - 1 - r0;
        aoff[j] = (uint32_t)((rr * lda + 2 * ((lane % T) ^ (row & 15))) * (int64_t)sizeof(double));
    }
#pragma unroll
    for (int j = 0; j < kXInst; ++j) {
        int q = 64 * j + lane;
        q = q < NV * T ? q : NV * T - 1;
        const int v = q / T;
        xoff[j] = (uint32_t)(((v < nv ? v : 0) * ldx + 2 * (q % T)) * (int64_t)sizeof(double));
    }
    const unsigned char* const a0 = reinterpret_cast<const unsigned char*>(A + r0 * lda);
    const unsigned char* const x0 = reinterpret_cast<const unsigned char*>(X);
    // ROT > 0: workgroup b starts at tile b*ROT (mod ntiles) and wraps around, so workgroups in
    // flight read different columns (rows a power-of-two stride apart otherwise hit the same
    // HBM channels at the same time)
    const int64_t rot = ROT > 0 && ntiles > 0 ? ((int64_t)blockIdx.x * ROT) % ntiles : 0;
    auto issue = [&](int64_t t, int b) {
        t += rot;
        if (t >= ntiles) t -= ntiles;
        const int64_t colb = t * kCols * (int64_t)sizeof(double);
        unsigned char* buf = ring + b * kBufBytes;
#pragma unroll
        for (int j = 0; j < kInst; ++j)
            __builtin_amdgcn_global_load_lds((gbl_void_t)(a0 + colb + aoff[j]), (lds_void_t)(buf + j * 1024),
                                             16, 0, 2 /* nt */);
#pragma unroll
        for (int j = 0; j < kXInst; ++j)
            __builtin_amdgcn_global_load_lds((gbl_void_t)(x0 + colb + xoff[j]),
                                             (lds_void_t)(buf + kTileBytes + j * 1024), 16, 0, 0);
    };

    const int i = lane & 15;
    const int g = lane >> 4;
    double acc[RQ][NV];
#pragma unroll
    for (int q = 0; q < RQ; ++q)
#pragma unroll
        for (int v = 0; v < NV; ++v) acc[q][v] = 0.0;
    auto consume = [&](int b) {
        const unsigned char* buf = ring + b * kBufBytes;
#pragma unroll
        for (int s = 0; s < T / 4; ++s) {
            const int c = 4 * s + g;
            dbl2 a[RQ], xx[NV];
#pragma unroll
            for (int q = 0; q < RQ; ++q)
                a[q] = *reinterpret_cast<const dbl2*>(buf + (i + 16 * q) * kRowBytes + 16 * (c ^ i));
#pragma unroll
            for (int v = 0; v < NV; ++v)
                xx[v] = *reinterpret_cast<const dbl2*>(buf + kTileBytes + 16 * (v * T + c));
#pragma unroll
            for (int q = 0; q < RQ; ++q)
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    acc[q][v] = __builtin_fma(a[q].x, xx[v].x, acc[q][v]);
                    acc[q][v] = __builtin_fma(a[q].y, xx[v].y, acc[q][v]);
                }
        }
    };

    const int64_t nt = ntiles > w ? (ntiles - w + NW - 1) / NW : 0;  // this wave's tiles
#pragma unroll
    for (int p = 0; p < NB - 1; ++p)
        if (p < nt) issue(w + (int64_t)NW * p, p);
    for (int64_t u = 0; u < nt; ++u) {
        const int64_t un = u + NB - 1;
        if (un < nt) {
            // buffer un % NB was summed in iteration u-1; its ds_reads have returned (their
            // values fed the FMAs), the wait only keeps the order explicit
            wait_lgkmcnt0();
            issue(w + (int64_t)NW * un, (int)(un % NB));
            wait_vmcnt<kPer*(NB - 1)>();
        } else {
            wait_vmcnt<0>();
        }
        consume((int)(u % NB));
    }

    // column tail: column c of rows i + 16q, columns spread over the waves and the four g lanes
    for (int64_t c = ntiles * kCols + 4 * w + g; c < K; c += 4 * NW) {
#pragma unroll
        for (int q = 0; q < RQ; ++q) {
            const int64_t rr = r0 + i + 16 * q < M ? r0 + i + 16 * q : M - 1;
            const double a = A[rr * lda + c];
#pragma unroll
            for (int v = 0; v < NV; ++v) acc[q][v] = __builtin_fma(a, X[(v < nv ? v : 0) * ldx + c], acc[q][v]);
        }
    }

#pragma unroll
    for (int q = 0; q < RQ; ++q)
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            acc[q][v] += __shfl_xor(acc[q][v], 16, 64);
            acc[q][v] += __shfl_xor(acc[q][v], 32, 64);
        }
    if constexpr (NW == 1) {
#pragma unroll
        for (int q = 0; q < RQ; ++q)
#pragma unroll
            for (int v = 0; v < NV; ++v)
                if (g == 0 && r0 + i + 16 * q < M && v < nv) Y[v * ldy + r0 + i + 16 * q] = acc[q][v];
    } else {
        // partials [q][v][i] in the wave's own ring (all its DMA retired and its reads consumed)
        wait_vmcnt<0>();
        wait_lgkmcnt0();
        double* part = reinterpret_cast<double*>(ring);
        if (g == 0) {
#pragma unroll
            for (int q = 0; q < RQ; ++q)
#pragma unroll
                for (int v = 0; v < NV; ++v) part[(q * NV + v) * 16 + i] = acc[q][v];
        }
        __syncthreads();
        for (int t = threadIdx.x; t < RQ * NV * 16; t += NW * 64) {
            const int ii = t % 16, v = (t / 16) % NV, q = t / (16 * NV);
            const int64_t row = r0 + ii + 16 * q;
            if (row < M && v < nv) {
                double s = 0.0;
#pragma unroll
                for (int ww = 0; ww < NW; ++ww) s += reinterpret_cast<const double*>(lds[ww])[t];
                Y[v * ldy + row] = s;
            }
        }
    }
}

// Sixteen vectors per pass on the matrix cores: gemv_mdma's tiles and workgroup shape, with the
// sums done by v_mfma_f64_16x16x4_f64 — a 16-row x 16-vector tile of Y per RQ row group, 4 f64
// accumulators per lane instead of 16 x RQ, and one ds_read_b128 of x per step instead of one
// per vector. fp64 MFMA has the fp64 VALU's peak on MI355X, so this pays only when all 16
// columns carry vectors: nv = 9..16 in one pass over A instead of two.
//   operands (step s, chunk c = 4s + g of the tile): lane (i = l & 15, g = l >> 4) holds row i's
//            pair A[i][2c], A[i][2c+1] and lane (j = l & 15, g) vector j's pair x_j[2c], x_j[2c+1];
//            the .x halves make one MFMA and the .y halves the next — k index g of each MFMA is
//            column 8s + 2g (+1) for both operands, a fixed permutation of the tile's columns;
//   x image: LDS slot (v, s) of the tile's x segment holds vector v's chunk s ^ (v & 15), the
//            same XOR as A's rows, so the B reads are conflict-free too;
//   result : lane (j, g) holds Y rows g + 4r (r < 4) of vector j in register r (gfx950's f64
//            MFMA layout); the column tail (K % 2T) goes through the same MFMAs from global memory,
//            4 columns a step, zero past K; partials meet in LDS in wave order.
typedef double dbl4 __attribute__((ext_vector_type(4)));

template <int RQ, int T, int NB, int NW, int ROT>
__global__ __launch_bounds__(NW * 64) void gemv_mdma16(const double* __restrict__ A, int64_t lda,
                                                       const double* __restrict__ X, int64_t ldx,
                                                       double* __restrict__ Y, int64_t ldy, int64_t M,
                                                       int64_t K, int nv) {
    static_assert(T == 16 || T == 32, "tile width: 16 or 32 chunks of 16 B");
    constexpr int NV = 16;
    constexpr int RB = 16 * RQ;
    constexpr int kRows = 64 / T;
    constexpr int kInst = RB / kRows;
    constexpr int kXInst = NV * T / 64;
    constexpr int kPer = kInst + kXInst;
    static_assert(kPer * (NB - 1) <= 63, "loads in flight must fit the vmcnt counter");
    constexpr int kCols = 2 * T;
    constexpr int kRowBytes = 16 * T;
    constexpr int kTileBytes = RB * kRowBytes;
    constexpr int kBufBytes = kTileBytes + kXInst * 1024;
    static_assert(NB * kBufBytes >= RQ * 4 * 64 * (int)sizeof(double), "partials fit the ring");
    __shared__ __attribute__((aligned(16))) unsigned char lds[NW][NB * kBufBytes];

    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int64_t r0 = (int64_t)blockIdx.x * RB;
    const int64_t ntiles = K / kCols;
    unsigned char* const ring = lds[w];

    uint32_t aoff[kInst], xoff[kXInst];
#pragma unroll
    for (int j = 0; j < kInst; ++j) {
        const int row = j * kRows + lane / T;
        const int64_t rr = r0 + row < M ? row : M - 1 - r0;
        aoff[j] = (uint32_t)((rr * lda + 2 * ((lane % T) ^ (row & 15))) * (int64_t)sizeof(double));
    }
#pragma unroll
    for (int j = 0; j < kXInst; ++j) {
        const int q = 64 * j + lane;  // LDS slot: vector q / T, slot q % T
        const int v = q / T;
        const int c = (q % T) ^ (v & 15);
        xoff[j] = (uint32_t)(((v < nv ? v : 0) * ldx + 2 * c) * (int64_t)sizeof(double));
    }
    const unsigned char* const a0 = reinterpret_cast<const unsigned char*>(A + r0 * lda);
    const unsigned char* const x0 = reinterpret_cast<const unsigned char*>(X);
    const int64_t rot = ROT > 0 && ntiles > 0 ? ((int64_t)blockIdx.x * ROT) % ntiles : 0;
    auto issue = [&](int64_t t, int b) {
        t += rot;
        if (t >= ntiles) t -= ntiles;
        const int64_t colb = t * kCols * (int64_t)sizeof(double);
        unsigned char* buf = ring + b * kBufBytes;
#pragma unroll
        for (int j = 0; j < kInst; ++j)
            __builtin_amdgcn_global_load_lds((gbl_void_t)(a0 + colb + aoff[j]), (lds_void_t)(buf + j * 1024),
                                             16, 0, 2 /* nt */);
#pragma unroll
        for (int j = 0; j < kXInst; ++j)
            __builtin_amdgcn_global_load_lds((gbl_void_t)(x0 + colb + xoff[j]),
                                             (lds_void_t)(buf + kTileBytes + j * 1024), 16, 0, 0);
    };

    const int i = lane & 15;  // A row / x vector of this lane's operands
    const int g = lane >> 4;  // k index
    dbl4 acc[RQ];
#pragma unroll
    for (int q = 0; q < RQ; ++q) acc[q] = dbl4{0.0, 0.0, 0.0, 0.0};
    auto consume = [&](int b) {
        const unsigned char* buf = ring + b * kBufBytes;
#pragma unroll
        for (int s = 0; s < T / 4; ++s) {
            const int c = 4 * s + g;
            const uint32_t sw = 16 * (uint32_t)(c ^ i);
            const dbl2 xb = *reinterpret_cast<const dbl2*>(buf + kTileBytes + i * kRowBytes + sw);
#pragma unroll
            for (int q = 0; q < RQ; ++q) {
                const dbl2 a = *reinterpret_cast<const dbl2*>(buf + (i + 16 * q) * kRowBytes + sw);
                acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a.x, xb.x, acc[q], 0, 0, 0);
                acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a.y, xb.y, acc[q], 0, 0, 0);
            }
        }
    };

    const int64_t nt = ntiles > w ? (ntiles - w + NW - 1) / NW : 0;
#pragma unroll
    for (int p = 0; p < NB - 1; ++p)
        if (p < nt) issue(w + (int64_t)NW * p, p);
    for (int64_t u = 0; u < nt; ++u) {
        const int64_t un = u + NB - 1;
        if (un < nt) {
            wait_lgkmcnt0();
            issue(w + (int64_t)NW * un, (int)(un % NB));
            wait_vmcnt<kPer*(NB - 1)>();
        } else {
            wait_vmcnt<0>();
        }
        consume((int)(u % NB));
    }

    // column tail through the same MFMAs: 4 columns a step (k index g), zero past K
    {
        const double* xj = X + (i < nv ? i : 0) * ldx;
        for (int64_t c0 = ntiles * kCols + 4 * w; c0 < K; c0 += 4 * NW) {
            const int64_t c = c0 + g;
            const double xv = c < K ? xj[c] : 0.0;
#pragma unroll
            for (int q = 0; q < RQ; ++q) {
                const int64_t rr = r0 + i + 16 * q < M ? r0 + i + 16 * q : M - 1;
                const double a = c < K ? A[rr * lda + c] : 0.0;
                acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, xv, acc[q], 0, 0, 0);
            }
        }
    }

    // lane (j, g) register r: Y row 16q + g + 4r of vector j
    if constexpr (NW == 1) {
#pragma unroll
        for (int q = 0; q < RQ; ++q)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t row = r0 + 16 * q + g + 4 * r;
                if (row < M && i < nv) Y[i * ldy + row] = acc[q][r];
            }
    } else {
        wait_vmcnt<0>();
        wait_lgkmcnt0();
        double* part = reinterpret_cast<double*>(ring);
#pragma unroll
        for (int q = 0; q < RQ; ++q)
#pragma unroll
            for (int r = 0; r < 4; ++r) part[(q * 4 + r) * 64 + lane] = acc[q][r];
        __syncthreads();
        for (int t = threadIdx.x; t < RQ * 4 * 64; t += NW * 64) {
            const int l = t % 64, r = (t / 64) % 4, q = t / 256;
            const int64_t row = r0 + 16 * q + (l >> 4) + 4 * r;
            if (row < M && (l & 15) < nv) {
                double s = 0.0;
#pragma unroll
                for (int ww = 0; ww < NW; ++ww) s += reinterpret_cast<const double*>(lds[ww])[t];
                Y[(l & 15) * ldy + row] = s;
            }
        }
    }
}

// host side of the DMA forms' address limits: rows_per_block rows of A and nvec rows of X in
// 32-bit offsets
inline bool dma_ok(int rows_per_block, int64_t lda, int64_t ldx, int nvec = 8) {
    return (int64_t)rows_per_block * lda * (int64_t)sizeof(double) < (1ll << 31) &&
           nvec * ldx * (int64_t)sizeof(double) < (1ll << 31);
}

typedef void (*gemv_multi_fn)(const double*, int64_t, const double*, int64_t, double*, int64_t, int64_t,
                              int64_t, int);

struct MultiVariant {
    const char* name;
    gemv_multi_fn fn[3];  // NV = 2, 4, 8
    int rows_per_block;
    int block;
    bool dma = false;     // gemv_mdma / gemv_mdma16: 32-bit DMA offsets (dma_ok)
    gemv_multi_fn fn16 = nullptr;  // gemv_mdma16: up to 16 vectors per pass (fn[] unused)
};

#define MVEC(LPR, RPG, UNR)                                                                              \
    {"mvec_l" #LPR "_r" #RPG "_u" #UNR,                                                                  \
     {gemv_mvec<LPR, RPG, 2, UNR>, gemv_mvec<LPR, RPG, 4, UNR>, gemv_mvec<LPR, RPG, 8, UNR>},            \
     (kBlock / 64) * (64 / LPR) * RPG, kBlock}
#define MROW(NW, RPB, UNR)                                                                               \
    {"mrow_w" #NW "_r" #RPB "_u" #UNR,                                                                   \
     {gemv_mrow<NW, RPB, 2, UNR>, gemv_mrow<NW, RPB, 4, UNR>, gemv_mrow<NW, RPB, 8, UNR>}, RPB, NW * 64}

#define MLDS(RPW, UNR)                                                                                   \
    {"mlds_r" #RPW "_u" #UNR,                                                                            \
     {gemv_mlds<RPW, 2, (UNR > 1 ? UNR : 2)>, gemv_mlds<RPW, 4, UNR>, gemv_mlds<RPW, 8, UNR>},           \
     (kBlock / 64) * RPW, kBlock}

#define MXR(LPR, RPG, UNR)                                                                               \
    {"mxres_l" #LPR "_r" #RPG "_u" #UNR,                                                                 \
     {gemv_mxres<LPR, RPG, 2, UNR>, gemv_mxres<LPR, RPG, 4, UNR>, gemv_mxres<LPR, RPG, 8, UNR>},         \
     (kBlock / 64) * (64 / LPR) * RPG, kBlock}

#define MDMA(RQ, T, NB, NW)                                                                              \
    {"mdma_r" #RQ "_t" #T "_b" #NB "_w" #NW,                                                             \
     {gemv_mdma<RQ, T, NB, NW, 2, 0>, gemv_mdma<RQ, T, NB, NW, 4, 0>, gemv_mdma<RQ, T, NB, NW, 8, 0>},   \
     16 * RQ, NW * 64, true}
#define MDMAS(RQ, T, NB, NW, ROT)                                                                        \
    {"mdma_r" #RQ "_t" #T "_b" #NB "_w" #NW "_s" #ROT,                                                   \
     {gemv_mdma<RQ, T, NB, NW, 2, ROT>, gemv_mdma<RQ, T, NB, NW, 4, ROT>,                                \
      gemv_mdma<RQ, T, NB, NW, 8, ROT>},                                                                 \
     16 * RQ, NW * 64, true}

#define M16(RQ, T, NB, NW, ROT)                                                                          \
    {"m16_r" #RQ "_t" #T "_b" #NB "_w" #NW "_s" #ROT, {nullptr, nullptr, nullptr}, 16 * RQ, NW * 64, true, \
     gemv_mdma16<RQ, T, NB, NW, ROT>}

static constexpr MultiVariant kMultiVariants[] = {
    {"auto", {nullptr, nullptr, nullptr}, 0, 0},  // 0
    MVEC(16, 1, 1),                               // 1
    MVEC(16, 2, 1),                               // 2
    MVEC(16, 1, 2),                               // 3
    MVEC(32, 1, 1),                               // 4
    MVEC(32, 2, 1),                               // 5
    MVEC(64, 1, 1),                               // 6
    MVEC(64, 2, 1),                               // 7
    MVEC(64, 1, 2),                               // 8
    MROW(4, 2, 1),                                // 9
    MROW(4, 2, 2),                                // 10
    MROW(4, 4, 1),                                // 11
    MROW(8, 2, 1),                                // 12
    MROW(8, 1, 2),                                // 13
    MROW(4, 1, 2),                                // 14
    MVEC(16, 4, 1),                               // 15
    MVEC(32, 4, 1),                               // 16
    MVEC(64, 4, 1),                               // 17
    MVEC(16, 3, 1),                               // 18
    MVEC(32, 3, 1),                               // 19
    MROW(4, 8, 1),                                // 20
    MROW(2, 4, 1),                                // 21
    MLDS(2, 2),                                   // 22
    MLDS(2, 4),                                   // 23
    MLDS(4, 2),                                   // 24
    MLDS(4, 4),                                   // 25
    MLDS(8, 2),                                   // 26
    MLDS(1, 4),                                   // 27
    MLDS(8, 1),                                   // 28
    MXR(16, 4, 1),                                // 29 x resident in LDS
    MXR(16, 4, 2),                                // 30
    MXR(32, 4, 1),                                // 31
    MXR(16, 2, 2),                                // 32
    MXR(64, 2, 2),                                // 33
    MXR(32, 2, 2),                                // 34
    MXR(16, 8, 1),                                // 35
    MDMA(2, 16, 3, 2),                            // 36 A through LDS by DMA
    MDMA(2, 16, 4, 2),                            // 37
    MDMA(2, 16, 2, 4),                            // 38
    MDMA(1, 16, 2, 4),                            // 39
    MDMA(4, 16, 2, 1),                            // 40
    MDMA(2, 32, 2, 2),                            // 41
    MDMA(1, 16, 3, 8),                            // 42
    MDMAS(2, 16, 2, 4, 1),                        // 43 rotated starts
    MDMAS(2, 16, 2, 4, 5),                        // 44
    MDMAS(2, 16, 2, 4, 17),                       // 45
    MDMAS(1, 16, 2, 4, 5),                        // 46
    MDMAS(2, 16, 4, 2, 5),                        // 47
    MDMAS(1, 16, 3, 2, 5),                        // 48
    MDMAS(4, 16, 2, 1, 5),                        // 49
    M16(2, 16, 2, 4, 5),                          // 50 16 vectors per pass, matrix cores
    M16(2, 16, 2, 2, 5),                          // 51
    M16(2, 16, 3, 2, 5),                          // 52
    M16(4, 16, 2, 2, 5),                          // 53
    M16(4, 16, 2, 1, 5),                          // 54
    M16(1, 16, 2, 4, 5),                          // 55
    M16(2, 32, 2, 2, 5),                          // 56
    M16(1, 16, 3, 4, 5),                          // 57
};
constexpr int kNumMultiVariants = (int)(sizeof(kMultiVariants) / sizeof(kMultiVariants[0]));

// From the MI355X sweeps (tools/multi_bench.py -> profiles/r01/multi_sweep.jsonl, then
// multi_sweep2_lds.jsonl with the LDS form and multi_sweep5_xres.jsonl with the x-resident form;
// 8 shapes, K = 512 ... 65536): per (nv group, K class) the variant with the best geometric mean
// of (rate / best rate on the shape): 0.93-1.0 per class, worst single shape 0.90. (K < 6144;
// longer rows take the DMA forms, below.)
constexpr int kMx16r4u2 = variant_id(kMultiVariants, "mxres_l16_r4_u2");
constexpr int kMx16r4u1 = variant_id(kMultiVariants, "mxres_l16_r4_u1");
constexpr int kMx32r2u2 = variant_id(kMultiVariants, "mxres_l32_r2_u2");
constexpr int kMv32r2u1 = variant_id(kMultiVariants, "mvec_l32_r2_u1");
constexpr int kMv32r4u1 = variant_id(kMultiVariants, "mvec_l32_r4_u1");
constexpr int kMrow4r4u1 = variant_id(kMultiVariants, "mrow_w4_r4_u1");
constexpr int kMlds2u2 = variant_id(kMultiVariants, "mlds_r2_u2");
constexpr int kMlds8u2 = variant_id(kMultiVariants, "mlds_r8_u2");
static_assert(kMx16r4u2 > 0 && kMx16r4u1 > 0 && kMx32r2u2 > 0 && kMv32r2u1 > 0 && kMv32r4u1 > 0 &&
                  kMrow4r4u1 > 0 && kMlds2u2 > 0 && kMlds8u2 > 0,
              "multi-vector dispatch names a variant missing from kMultiVariants");

// A through LDS by DMA (gemv_mdma), workgroups starting 5 tiles apart: 32 rows x 4 waves per
// workgroup from 8192 rows — vector groups of 8 from K = 1024, of 3-4 from K = 1280, pairs from
// K = 6144 — and 16 rows x 4 waves for 4096-8191 rows of K >= 8192. From the MI355X sweeps
// (tools/multi_bench.py -> profiles/r03/multi_sweep_dma*.jsonl, 20 shapes): nv = 8 reads A at
// 6.3-7.0 TB/s where the register forms above reached 4.5-6.2 (rows a power-of-two stride apart
// need the staggered starts: 16-20 % without them), nv = 4 within 3 % of the best form or
// better, pairs level or better on the long rows; below those sizes the forms above stay.
constexpr int kMd2w4s5 = variant_id(kMultiVariants, "mdma_r2_t16_b2_w4_s5");
constexpr int kMd1w4s5 = variant_id(kMultiVariants, "mdma_r1_t16_b2_w4_s5");
static_assert(kMd2w4s5 > 0 && kMd1w4s5 > 0, "multi-vector dispatch names a missing DMA variant");

int pick_multi_dma(int64_t m, int64_t k, int nvp) {
    if (m >= 8192) return (nvp >= 8 ? k >= 1024 : nvp >= 4 ? k >= 1280 : k >= 6144) ? kMd2w4s5 : 0;
    return m >= 4096 && k >= 8192 ? kMd1w4s5 : 0;
}

// 9..16 vectors: one pass on the matrix cores (gemv_mdma16) where the DMA forms run, else two
// passes of <= 8
constexpr int kM16 = variant_id(kMultiVariants, "m16_r2_t16_b2_w4_s5");
static_assert(kM16 > 0, "multi-vector dispatch names a missing 16-vector variant");

int pick_multi16(int64_t m, int64_t k, int64_t lda, int64_t ldx) {
    return m >= 8192 && k >= 1024 && dma_ok(kMultiVariants[kM16].rows_per_block, lda, ldx, 16) ? kM16 : 0;
}

int pick_multi_variant(int64_t m, int64_t k, int nvp, int64_t lda, int64_t ldx) {
    const int d = pick_multi_dma(m, k, nvp);
    if (d > 0 && dma_ok(kMultiVariants[d].rows_per_block, lda, ldx)) return d;
    if (k <= 768) return nvp <= 4 ? kMx16r4u2 : kMx16r4u1;
    if (nvp <= 2) return k <= 1024 ? kMv32r2u1 : kMrow4r4u1;
    if (nvp <= 4) return k <= 1024 ? kMx32r2u2 : k < 6144 ? kMlds2u2 : kMlds8u2;
    return k <= 1024 ? kMx16r4u1 : k < 6144 ? kMlds2u2 : kMv32r4u1;
}

// ------------------------------------------------------------------ other kernels
__global__ void zero_kernel(double* y, int64_t m) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m;
         i += (int64_t)gridDim.x * blockDim.x)
        y[i] = 0.0;
}

__global__ __launch_bounds__(kBlock) void synth_fill_kernel(double* __restrict__ dst, int64_t ld,
                                                            int64_t m, int64_t k, int64_t row_off,
                                                            int64_t col_off, int64_t ncols,
                                                            uint64_t s0) {
    for (int64_t r = blockIdx.x; r < m; r += gridDim.x) {
        const uint64_t gbase = (uint64_t)(row_off + r) * (uint64_t)ncols + (uint64_t)col_off;
        double* d = dst + r * ld;
        for (int64_t c = threadIdx.x; c < k; c += kBlock) d[c] = synth_value(s0, gbase + c);
    }
}

// Read-only stream: HBM ceiling for a pure fp64 read with the same load shape as the GEMV
// (16 B per lane, nt, 8 loads in flight per lane). Each wave reads one contiguous segment.
__global__ __launch_bounds__(kBlock) void stream_read_kernel(const double* __restrict__ src,
                                                             int64_t n2, double* sink) {
    constexpr int UNR = 8;
    const dbl2* s = reinterpret_cast<const dbl2*>(src);
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * (kBlock / 64);
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
    if (acc.x == -1.0 && acc.y == -2.0) sink[threadIdx.x] = acc.x;  // never true for real data; keeps loads live
}

}  // namespace mvg

using namespace mvg;

extern "C" {

int mvg_gemv_variant_count(void) { return kNumVariants; }

int mvg_gemv_auto_variant(int64_t lda, int64_t m, int64_t k) {
    return pick_variant(lda, m, k, true, true, lda % 16 == 0);
}

const char* mvg_gemv_variant_name(int v) {
    if (v < 0 || v >= kNumVariants) return "invalid";
    return kVariants[v].name;
}

int mvg_gemv_variant(const double* A, int64_t lda, const double* x, double* y, int64_t m,
                     int64_t k, int variant, void* stream) {
    if (m < 0 || k < 0) return fail(MVG_E_INVALID, "mvg_gemv: negative size");
    if (variant < 0 || variant >= kNumVariants) return fail(MVG_E_INVALID, "mvg_gemv: bad variant");
    hipStream_t s = (hipStream_t)stream;
    if (m == 0) return MVG_OK;
    if (!y) return fail(MVG_E_INVALID, "mvg_gemv: null y");
    if (k > 0 && (!A || !x)) return fail(MVG_E_INVALID, "mvg_gemv: null A or x");
    if (k > 0 && lda < k) return fail(MVG_E_INVALID, "mvg_gemv: lda < k");
    if (int rc = take_pending_error("mvg_gemv"); rc != MVG_OK) return rc;  // before our first HIP call
    if (k == 0) {
        hipLaunchKernelGGL(zero_kernel, dim3((unsigned)((m + 255) / 256 < 4096 ? (m + 255) / 256 : 4096)),
                           dim3(256), 0, s, y, m);
        MVG_HIP(hipGetLastError());
        return MVG_OK;
    }
    const bool aligned = ((uintptr_t)A % 16 == 0) && ((uintptr_t)x % 16 == 0);
    const bool aligned8 = ((uintptr_t)A % 8 == 0) && ((uintptr_t)x % 8 == 0);
    const bool lines = (uintptr_t)A % 128 == 0 && lda % 16 == 0;  // every row starts on a 128-B line
    int v = variant == 0 ? pick_variant(lda, m, k, aligned, aligned8, lines) : variant;
    if (kVariants[v].vec && ((uintptr_t)A % 8 != 0 || (uintptr_t)x % 8 != 0))
        return fail(MVG_E_INVALID, "mvg_gemv: 16-B variant needs 8-B aligned A, x");
    return launch(v, A, lda, x, y, m, k, s, variant != 0);
}

int mvg_gemv(const double* A, int64_t lda, const double* x, double* y, int64_t m, int64_t k,
             void* stream) {
    return mvg_gemv_variant(A, lda, x, y, m, k, 0, stream);
}

int mvg_gemv_multi_variant_count(void) { return kNumMultiVariants; }

int mvg_gemv_multi_auto_variant(int64_t lda, int64_t ldx, int64_t m, int64_t k, int nv) {
    if (nv < 2) return 0;
    if (nv > 8) {
        const int v = pick_multi16(m, k, lda, ldx);
        if (v > 0) return v;
    }
    const int g = nv < 8 ? nv : 8;
    return pick_multi_variant(m, k, g <= 2 ? 2 : g <= 4 ? 4 : 8, lda, ldx);
}

const char* mvg_gemv_multi_variant_name(int v) {
    if (v < 0 || v >= kNumMultiVariants) return "invalid";
    return kMultiVariants[v].name;
}

int mvg_gemv_multi_variant(const double* A, int64_t lda, const double* X, int64_t ldx, double* Y,
                           int64_t ldy, int64_t m, int64_t k, int nv, int variant, void* stream) {
    if (m < 0 || k < 0 || nv < 0) return fail(MVG_E_INVALID, "mvg_gemv_multi: negative size");
    if (variant < 0 || variant >= kNumMultiVariants) return fail(MVG_E_INVALID, "mvg_gemv_multi: bad variant");
    if (m == 0 || nv == 0) return MVG_OK;
    if (!Y || ldy < m || (k > 0 && (!A || !X || lda < k || ldx < k)))
        return fail(MVG_E_INVALID, "mvg_gemv_multi: null pointer or leading dimension too small");
    if (int rc = take_pending_error("mvg_gemv_multi"); rc != MVG_OK) return rc;
    hipStream_t s = (hipStream_t)stream;
    const bool vec = ((uintptr_t)A % 16 == 0) && ((uintptr_t)X % 16 == 0) && lda % 2 == 0 && ldx % 2 == 0;
    if (!vec || k == 0) {  // odd lda/ldx or a view off 16 B (or k = 0): one vector at a time,
        // each through the single-vector dispatch (its unaligned 16-B forms, §4 "Odd widths")
        if (variant != 0) return fail(MVG_E_INVALID, "mvg_gemv_multi: variants need even lda/ldx, 16-B aligned A, X");
        for (int v = 0; v < nv; ++v) {
            int rc = mvg_gemv_variant(A, lda, X + v * ldx, Y + v * ldy, m, k, 0, stream);
            if (rc != MVG_OK) return rc;
        }
        return MVG_OK;
    }
    const bool fixed16 = variant != 0 && kMultiVariants[variant].fn16 != nullptr;
    for (int v0 = 0; v0 < nv;) {  // groups of <= 8 (or 16) vectors per pass over A
        const int rest = nv - v0;
        int v = variant, g = rest < 8 ? rest : 8;
        if (fixed16) {
            g = rest < 16 ? rest : 16;
        } else if (variant == 0 && rest > 8 && (v = pick_multi16(m, k, lda, ldx)) > 0) {
            g = rest < 16 ? rest : 16;  // 9..16 vectors: one pass on the matrix cores
        } else {
            v = variant;
        }
        const double* Xg = X + v0 * ldx;
        double* Yg = Y + v0 * ldy;
        v0 += g;
        if (g == 1 && v == 0) {  // one vector: the single-vector dispatch
            int rc = mvg_gemv_variant(A, lda, Xg, Yg, m, k, 0, stream);
            if (rc != MVG_OK) return rc;
            continue;
        }
        const int slot = g <= 2 ? 0 : g <= 4 ? 1 : 2;
        if (v == 0) v = pick_multi_variant(m, k, 2 << slot, lda, ldx);
        const MultiVariant& mv = kMultiVariants[v];
        if (mv.dma && !dma_ok(mv.rows_per_block, lda, ldx, mv.fn16 ? 16 : 8))
            return fail(MVG_E_INVALID, "mvg_gemv_multi: lda or ldx too large for the DMA variant");
        const gemv_multi_fn fn = mv.fn16 ? mv.fn16 : mv.fn[slot];
        // launches of < 2^32 threads each (the grid-size cap), row ranges in order
        const int64_t max_rows = ((1ll << 31) / mv.block) * mv.rows_per_block;
        for (int64_t r0 = 0; r0 < m; r0 += max_rows) {
            const int64_t mm = m - r0 < max_rows ? m - r0 : max_rows;
            const int64_t blocks = (mm + mv.rows_per_block - 1) / mv.rows_per_block;
            hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(mv.block), 0, s, A + r0 * lda, lda, Xg, ldx,
                               Yg + r0, ldy, mm, k, g);
            MVG_HIP(hipGetLastError());
        }
    }
    return MVG_OK;
}

int mvg_gemv_multi(const double* A, int64_t lda, const double* X, int64_t ldx, double* Y, int64_t ldy,
                   int64_t m, int64_t k, int nv, void* stream) {
    return mvg_gemv_multi_variant(A, lda, X, ldx, Y, ldy, m, k, nv, 0, stream);
}

int mvg_stream_read(const double* src, int64_t n, double* sink, void* stream) {
    if (!src || !sink || n < 0 || (n & 1) || ((uintptr_t)src % 16))
        return fail(MVG_E_INVALID, "mvg_stream_read: need even n, 16-B aligned src, sink");
    if (int rc = take_pending_error("mvg_stream_read"); rc != MVG_OK) return rc;
    hipLaunchKernelGGL(stream_read_kernel, dim3(256 * 4), dim3(kBlock), 0, (hipStream_t)stream, src,
                       n / 2, sink);
    MVG_HIP(hipGetLastError());
    return MVG_OK;
}

int mvg_synth_fill_device(double* dst, int64_t ld, int64_t m, int64_t k, int64_t row_off,
                          int64_t col_off, int64_t ncols, uint64_t seed, void* stream) {
    if (m < 0 || k < 0 || ld < k || row_off < 0 || col_off < 0 || col_off + k > ncols)
        return fail(MVG_E_INVALID, "mvg_synth_fill_device: bad shape");
    if (m == 0 || k == 0) return MVG_OK;
    if (!dst) return fail(MVG_E_INVALID, "mvg_synth_fill_device: null dst");
    if (int rc = take_pending_error("mvg_synth_fill_device"); rc != MVG_OK) return rc;
    const int64_t blocks = m < 65536 ? m : 65536;
    hipLaunchKernelGGL(synth_fill_kernel, dim3((unsigned)blocks), dim3(kBlock), 0,
                       (hipStream_t)stream, dst, ld, m, k, row_off, col_off, ncols,
                       splitmix64(seed));
    MVG_HIP(hipGetLastError());
    return MVG_OK;
}

}  // extern "C"
