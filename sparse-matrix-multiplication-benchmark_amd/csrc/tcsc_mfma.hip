// tcsc_mfma.hip -- the MFMA path for near-dense W.
//
// At 50 % density (BASELINE cfg 5) the gather walks half of W: 33.5 M
// nonzeros x 2048 rows at ~27 T adds/s = 2.5 ms, while the matrix cores
// multiply the dense W far faster in bf16.  The path keeps fp32 results
// without an fp32 MFMA (the fp32 matrix rate is the vector rate): every x is
// split exactly into three bf16 parts, x = h + m + l (truncations of x and of
// its remainders: 8 + 8 + 8 significand bits), W is exact in bf16 (0, +-1,
// or small integers for duplicate rows), so each product is exact and the
// GEMM
//     Y = [h | m | l] . [W ; W ; W]           (M x 3K) . (3K x N)
// accumulates in fp32 on the matrix cores -- k_gemm3, written here for
// gfx950: 256 x 256 tiles of 8 waves (v_mfma_f32_16x16x32_bf16), X3 (M x ldk,
// [h | m | l] per 64-k block) and W^T (N x ldw, stored once) staged into LDS
// rings by LDS-DMA with a conflict-free swizzle, each W block multiplied with
// the three parts of its X3 block in turn, bias (+ PReLU) fused into the
// store.  Only the summation order differs from the gather's: the result is
// within the fast-order bound, and bit-exact on integer-valued inputs.
//
// Rows the split cannot carry are recomputed by the gather order: a
// non-finite x would make inf*0 = NaN in columns whose W is 0 there (the
// reference never touches those products), and bf16 MFMA inputs below
// 2^-126 may be flushed.  k_split3 flags every row holding a non-finite x
// or a nonzero |x| < 2^-100 (it writes every row's flag on every call, so a
// captured graph replays correctly); k_fixup rewrites those rows from the
// plan's merged per-column CSC copy, +1 and -1 rows in ascending k (+1 first
// on a tie), then the bias, then the PReLU -- the exact arithmetic of
// k_stream's fast order (= the reference's dense.c gemm_basic order).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "tcsc_internal.h"

namespace tcsc {
namespace {

inline int grid_of(long long n, int block) {
    long long g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > 65535LL * 16) g = 65535LL * 16;
    return (int)g;
}

__device__ inline uint32_t f2u(float x) { return __float_as_uint(x); }
__device__ inline float u2f(uint32_t u) { return __uint_as_float(u); }

// x -> (h, m, l) bf16 bit patterns with h + m + l == x exactly (finite x);
// a non-finite x goes whole into h (a quiet NaN keeps its sign), m = l = 0.
// Returns whether the row needs the exact fixup.
__device__ inline bool split3(float x, uint16_t& h, uint16_t& m, uint16_t& l) {
    const uint32_t u = f2u(x);
    if ((u & 0x7f800000u) == 0x7f800000u) {  // inf or NaN
        const bool nan = (u & 0x007fffffu) != 0;
        h = (uint16_t)(nan ? ((u >> 16) | 0x0040u) : (u >> 16));
        m = l = 0;
        return true;
    }
    const uint32_t hu = u & 0xffff0000u;
    const float r = x - u2f(hu);              // exact: the low 16 bits of x
    const uint32_t mu = f2u(r) & 0xffff0000u;
    const float s = r - u2f(mu);              // exact: at most 8 significant bits left
    h = (uint16_t)(hu >> 16);
    m = (uint16_t)(mu >> 16);
    l = (uint16_t)(f2u(s) >> 16);
    return x != 0.0f && fabsf(x) < 0x1p-100f;
}

// X (M x K, pitch K) -> X3 (M x ldk bf16): [h | m | l | 0 ...] per row, one
// workgroup per row; flags[row] = 1 when the fixup must recompute the row,
// else 0 (written every call).  A thread loads kSplitU 16-B pieces before it
// splits and stores any of them: at small M (one workgroup per row, few rows)
// the row's loads then overlap instead of running as kq / 256 dependent round
// trips (M = 64, K = 8192: 11.3 us before).
constexpr int kSplitU = 8;
__global__ void __launch_bounds__(256) k_split3(const float* __restrict__ X, int M, int K, uint16_t* __restrict__ X3,
                                               int ldk, int* __restrict__ flags) {
    const int row = blockIdx.x;
    const float* src = X + (size_t)row * K;
    uint16_t* dst = X3 + (size_t)row * ldk;
    const bool vec = (K & 3) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
    bool fix = false;
    const int kq = (K + 3) / 4;
    typedef float f4 __attribute__((ext_vector_type(4)));
    typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
    if (vec) {
        for (int q0 = threadIdx.x; q0 < kq; q0 += kSplitU * blockDim.x) {
            f4 w[kSplitU];
#pragma unroll
            for (int u = 0; u < kSplitU; ++u) {
                const int q = q0 + u * blockDim.x;
                if (q < kq) w[u] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(src + 4 * q));
            }
#pragma unroll
            for (int u = 0; u < kSplitU; ++u) {
                const int q = q0 + u * blockDim.x;
                if (q >= kq) break;
                const int k0 = 4 * q;  // k0 .. k0+3 lie in one block
                uint16_t h[4], m[4], l[4];
                for (int j = 0; j < 4; ++j) fix |= split3(w[u][j], h[j], m[j], l[j]);
                *reinterpret_cast<u16x4*>(dst + x3_index(k0, 0)) = u16x4{h[0], h[1], h[2], h[3]};
                *reinterpret_cast<u16x4*>(dst + x3_index(k0, 1)) = u16x4{m[0], m[1], m[2], m[3]};
                *reinterpret_cast<u16x4*>(dst + x3_index(k0, 2)) = u16x4{l[0], l[1], l[2], l[3]};
            }
        }
    } else {
        for (int q = threadIdx.x; q < kq; q += blockDim.x) {
            const int k0 = 4 * q;
            float v[4];
            for (int j = 0; j < 4; ++j) v[j] = k0 + j < K ? src[k0 + j] : 0.0f;
            uint16_t h[4], m[4], l[4];
            for (int j = 0; j < 4; ++j) fix |= split3(v[j], h[j], m[j], l[j]);
            for (int j = 0; j < 4 && k0 + j < K; ++j) {
                dst[x3_index(k0 + j, 0)] = h[j];
                dst[x3_index(k0 + j, 1)] = m[j];
                dst[x3_index(k0 + j, 2)] = l[j];
            }
        }
    }
    // zeros past K: the last block's tail in each part, then the row pad
    const int tail0 = (mfma_nblk(K) - 1) * 3 * kMfmaBlk;
    for (int i = tail0 + threadIdx.x; i < ldk; i += blockDim.x)
        if (i >= 3 * kMfmaBlk * mfma_nblk(K) || (mfma_nblk(K) - 1) * kMfmaBlk + i % kMfmaBlk >= K) dst[i] = 0;
    fix = __syncthreads_or(fix);
    if (threadIdx.x == 0) flags[row] = fix ? 1 : 0;
}

// The +1/-1 entries of column j (rebased CSC) added into a dense fp32 image
// of W^T (ncols x K, k contiguous; atomics: a row may repeat in a column).
__global__ void k_w_scatter(const int* __restrict__ cs, const int* __restrict__ ri, int col_begin, int ncols,
                            int K, float sign, float* __restrict__ WfT) {
    const int lane = threadIdx.x & 63;
    const int j = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (j >= ncols) return;
    const int base = cs[col_begin];
    const int e0 = cs[col_begin + j] - base, e1 = cs[col_begin + j + 1] - base;
    const int* r = ri + base;
    for (int e = e0 + lane; e < e1; e += 64) atomicAdd(&WfT[(size_t)j * K + r[e]], sign);
}

// WfT (ncols x K fp32) -> WT (ncols x ldw bf16, the pad zeroed before), k
// contiguous like X3.  Values must be integers of magnitude <= 256 to be
// exact in bf16; *bad = 1 otherwise.
__global__ void k_wt_from(const float* __restrict__ WfT, int ncols, int K, uint16_t* __restrict__ WT, int ldw,
                          int* __restrict__ bad) {
    const long long n = (long long)ncols * K;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        const float w = WfT[i];
        if (fabsf(w) > 256.0f) *bad = 1;
        const long long j = i / K, k = i - j * K;
        WT[j * ldw + k] = (uint16_t)(f2u(w) >> 16);
    }
}

// dst[e] = src[base + e], base = cs[col_begin] (the column range's first entry)
__global__ void k_copy_from(const int* __restrict__ src, const int* __restrict__ cs, int col_begin, long long n,
                            int* __restrict__ dst) {
    const int base = cs[col_begin];
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        dst[i] = src[base + i];
}

// gq[g] = quads of group g: its longest column's entries over 4, rounded up
// to a multiple of 16 quads (the small-M kernel's unroll); gq[groups] = 0.
__global__ void k_group_quads(const int* __restrict__ cp, const int* __restrict__ cn, int ncols,
                              int* __restrict__ gq) {
    const int ng = csc_groups(ncols);
    for (int g = blockIdx.x * blockDim.x + threadIdx.x; g <= ng; g += gridDim.x * blockDim.x) {
        int mx = 0;
        if (g < ng)
            for (int j = g * kCscGroup; j < min(ncols, (g + 1) * kCscGroup); ++j)
                mx = max(mx, cp[j + 1] - cp[j] + cn[j + 1] - cn[j]);
        gq[g] = g < ng ? ((mx + 3) / 4 + 15) & ~15 : 0;
    }
}

// Merge each column's +1 and -1 rows (rebased lists rp / rn, offsets cp /
// cn) into one list in ascending row order -- entries 4*row for +1 rows and
// csc_neg_base(rows) + 4*row for -1 rows, a +1 entry first on a tie (k_scatter's
// rule) -- in the quad layout, padded to its group's length with 4*rows
// entries: the order in which k_stream's fast order adds a column's nonzeros.
__global__ void k_merge_csc(const int* __restrict__ cp, const int* __restrict__ cn, const int* __restrict__ rp,
                            const int* __restrict__ rn, const int* __restrict__ cq, int ncols, int rows,
                            int* __restrict__ rm) {
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < ncols; j += gridDim.x * blockDim.x) {
        const int g = j / kCscGroup;
        const int n = 4 * (cq[g + 1] - cq[g]);
        int p = cp[j], q = cn[j], i = 0;
        const int p1 = cp[j + 1], q1 = cn[j + 1];
        while (p < p1 || q < q1) {
            int e;
            if (q >= q1 || (p < p1 && rp[p] <= rn[q]))
                e = 4 * rp[p++];
            else
                e = csc_neg_base(rows) + 4 * rn[q++];
            rm[csc_entry(cq, j, i++)] = e;
        }
        for (; i < n; ++i) rm[csc_entry(cq, j, i)] = 4 * rows;
    }
}

// Output (row, j) recomputed exactly as k_stream's fast order (see the file
// comment): x rebuilt from its three parts, the column's merged rows in
// ascending k, the bias first or last, then the PReLU.
template <bool BIAS_FIRST, bool PRELU>
__device__ inline float exact_out(const uint16_t* __restrict__ X3, int K, int ldk, const int* __restrict__ cq,
                                  const int* __restrict__ rm, const float* __restrict__ Bias, int row, int j,
                                  float a) {
    const uint16_t* x3 = X3 + (size_t)row * ldk;
    auto xk = [&](int k) {
        return (u2f((uint32_t)x3[x3_index(k, 0)] << 16) + u2f((uint32_t)x3[x3_index(k, 1)] << 16)) +
               u2f((uint32_t)x3[x3_index(k, 2)] << 16);
    };
    float acc = BIAS_FIRST ? Bias[j] : 0.0f;
    const int g = j / kCscGroup, n = 4 * (cq[g + 1] - cq[g]);
    for (int i = 0; i < n; ++i) {
        const int r = rm[csc_entry(cq, j, i)];
        if (r == 4 * K) break;  // the column's padding
        const bool neg = r >= csc_neg_base(K);
        const int k = (neg ? r - csc_neg_base(K) : r) >> 2;
        acc = fmaf(xk(k), neg ? -1.0f : 1.0f, acc);
    }
    if (!BIAS_FIRST) acc += Bias[j];
    if (PRELU) acc = (acc < 0.0f) ? a * acc : acc;
    return acc;
}

// Flagged rows, after the GEMM (which wrote act(sum + bias) for every row):
// one thread per column.  A block first ORs the row flags; most calls have
// none and the kernel ends there.
template <bool BIAS_FIRST, bool PRELU>
__global__ void __launch_bounds__(256) k_fixup(const uint16_t* __restrict__ X3, int M, int K, int ldk,
                                               const int* __restrict__ cq, const int* __restrict__ rm,
                                               int ncols,
                                               const float* __restrict__ Bias, float* __restrict__ Y, int ldy, float a,
                                               const int* __restrict__ flags) {
    int any = 0;
    for (int r = threadIdx.x; r < M; r += blockDim.x) any |= flags[r];
    if (!__syncthreads_or(any)) return;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= ncols) return;
    for (int row = 0; row < M; ++row)
        if (flags[row])
            Y[(size_t)row * ldy + j] = exact_out<BIAS_FIRST, PRELU>(X3, K, ldk, cq, rm, Bias, row, j, a);
}

// ---------------------------------------------------------------------------
// k_gemm3: Y[m, n] = act(sum_k A[m, k] * Bt[n, k] + bias[n]), bf16 in, fp32
// accumulate, A = X3 (M x ldk: [h | m | l] per 64-k block), Bt = WT (N x ldw:
// W's block once).
//
// * Tile TM x TN = (WM*FI*16) x (WN*FJ*16) per workgroup of WM*WN waves; a
//   wave owns FI x FJ blocks of 16 x 16 (v_mfma_f32_16x16x32_bf16, 4 fp32
//   accumulators per lane per block).  128 x 512 with 8 waves (1 x 8, 128 x
//   64 per wave) for the large shapes; 128 x 128 with 4 waves for grids that
//   would leave CUs idle.
// * The k loop runs over sub-steps (block, part): one part of X3's 64-k
//   block against W's block.  A is staged per sub-step in a 2-slot ring, W
//   once per block in a 2-slot ring of its own, by LDS-DMA
//   (global_load_lds_dwordx4: 1 KiB per wave-instruction, no VGPRs).  The
//   GEMM is bound by that staging (L2 -> LDS, ~43 GB/s per CU): staging W once
//   per block instead of with every part moves 1/3 fewer bytes per MFMA.
// * LDS image of a slot: 1-KiB pieces of 8 rows x 64
//   k (128 B per row).  Inside a piece the 16-B granule g (8 k) of row r sits
//   at slot 8r + (g ^ r): the DMA writes the piece lane-linear (lane = slot)
//   from per-lane source addresses, and the MFMA fragment reads (lane l:
//   row l & 15 of a 16-row block, granule 4*kh + l/16) then hit 16 distinct
//   16-B slots in every ds_read_b128 lane group: conflict-free (4 LDS
//   cycles per read instead of 16-32 for a linear image).
// * Rows past M / N load the last valid row (in bounds) and are not stored.
// * Tile order: XCD-aware and bijective; an XCD's ~32 concurrent workgroups
//   take 4 row tiles x 8 column tiles, sharing A and W tiles in its L2.
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Split K (k_gemm3 PARTIAL): the slabs added in slice order, then the bias,
// then the PReLU -- k_reduce4's arithmetic, element for element -- with
// k_fixup folded in: a flagged row takes exact_out() instead, so a split call
// needs no fixup launch.  VEC: 4 columns per thread (N % 4 == 0, ldy % 4 ==
// 0, 16-B aligned slabs, bias and Y), all slices' loads in flight.
template <bool PRELU, bool VEC>
__global__ void __launch_bounds__(256) k_reduce_fix(const float* __restrict__ ws, int slices, int M, int N,
                                                    const float* __restrict__ Bias, float* __restrict__ Y, int ldy,
                                                    float a, const int* __restrict__ flags,
                                                    const uint16_t* __restrict__ X3, int K, int ldk,
                                                    const int* __restrict__ cq, const int* __restrict__ rm) {
    constexpr int W = VEC ? 4 : 1;
    const int nq = N / W;
    const long long total = (long long)M * nq;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int row = (int)(i / nq), col = W * (int)(i % nq);
        float v[W];
        if (flags[row]) {
#pragma unroll
            for (int u = 0; u < W; ++u) v[u] = exact_out<false, PRELU>(X3, K, ldk, cq, rm, Bias, row, col + u, a);
        } else {
            const size_t slab = (size_t)M * N, e = (size_t)row * N + col;
            float p[16][W];
#pragma unroll
            for (int s = 0; s < 16; ++s)
                if (s < slices) {
                    if constexpr (VEC) {
                        const f32x4 q = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(ws + s * slab + e));
#pragma unroll
                        for (int u = 0; u < 4; ++u) p[s][u] = q[u];
                    } else {
                        p[s][0] = ws[s * slab + e];
                    }
                }
#pragma unroll
            for (int u = 0; u < W; ++u) {
                float t = 0.f;
#pragma unroll
                for (int s = 0; s < 16; ++s)
                    if (s < slices) t += p[s][u];
                t += Bias[col + u];
                if (PRELU) t = (t < 0.0f) ? a * t : t;
                v[u] = t;
            }
        }
        float* dst = Y + (size_t)row * ldy + col;
        if constexpr (VEC) {
            const f32x4 o = {v[0], v[1], v[2], v[3]};
            __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(dst));
        } else {
            dst[0] = v[0];
        }
    }
}


// XCD-aware bijective renumbering of blockIdx.x (an XCD's workgroups get
// consecutive numbers), then bands of gm row tiles walked column by column:
// an XCD's ~32 concurrent workgroups take gm row tiles x 32 / gm column
// tiles, sharing those A and W tiles in its L2.
template <int TM, int TN>
__device__ __forceinline__ void gemm3_tile(int tiles_m, int tiles_n, int gm, int& m0, int& n0) {
    const int T = tiles_m * tiles_n, L = blockIdx.x;
    const int q = T >> 3, r = T & 7, x = L & 7;
    const int Lg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (L >> 3);
    const int band = Lg / (gm * tiles_n), rb = Lg - band * gm * tiles_n;
    const int g = min(gm, tiles_m - band * gm);  // the last band may be shorter
    m0 = (band * gm + rb % g) * TM;
    n0 = (rb / g) * TN;
}

// The k_gemm3 epilogue (both staging forms): Y = act(acc + bias) for the
// workgroup's tile, the raw sums parked in the LDS (LDSB bytes, free once the
// k loop has drained) and stored as whole rows.
template <int WM, int WN, int FI, int FJ, bool PRELU, bool BIAS, int LDSB>
__device__ __forceinline__ void gemm3_store(const f32x4 (&acc)[FI][FJ], char* lds, int lane, int wr, int wc, int m0,
                                            int n0, int M, int N, const float* __restrict__ bias,
                                            float* __restrict__ Y, int ldy, float a) {
    constexpr int TM = WM * FI * 16, TN = WN * FJ * 16, NW = WM * WN;
    // Epilogue: lane l holds rows 4*(l/16) + reg, column l % 16 of each 16 x 16
    // block.  Stored as is, one instruction would write 4 rows x 16 columns of
    // 4-B pieces (store-issue-bound); instead each pass of 64 tile rows is
    // parked in the (now free) LDS, row stride TN + 4 floats (the 4 row groups
    // of a block fall 16 banks apart), and read back as whole rows: 16-B
    // stores, TN / 4 lanes per row.  Same values, same bits.
    constexpr int PR = 64, SROW = TN + 4, LPR = TN / 4;  // rows per pass, staged row, lanes per row
    static_assert(PR * SROW * 4 <= LDSB && TM % PR == 0 && (64 % LPR == 0 || LPR % 64 == 0), "epilogue staging");
    // (the raw sums are parked; bias and PReLU are applied to the rows read
    // back, where a lane's 4 columns stay the same: NW * 64 is a multiple of LPR)
    static_assert((NW * 64) % LPR == 0, "a lane keeps its columns across the read-back");
    float* stg = reinterpret_cast<float*>(lds);
    const bool vec = (ldy & 3) == 0 && (reinterpret_cast<uintptr_t>(Y) & 15) == 0;
    const int c4 = 4 * (threadIdx.x % LPR), col = n0 + c4;
    f32x4 bq = f32x4{0.f, 0.f, 0.f, 0.f};
    if (BIAS)
#pragma unroll
        for (int u = 0; u < 4; ++u) bq[u] = col + u < N ? bias[col + u] : 0.0f;
#pragma unroll
    for (int p = 0; p < TM / PR; ++p) {
#pragma unroll
        for (int i = 0; i < FI; ++i) {
            if (((wr * FI + i) * 16) / PR != p) continue;  // uniform
            const int rb = (wr * FI + i) * 16 - p * PR + 4 * (lane >> 4);
#pragma unroll
            for (int j = 0; j < FJ; ++j) {
                const int c = (wc * FJ + j) * 16 + (lane & 15);
#pragma unroll
                for (int rg = 0; rg < 4; ++rg) stg[(rb + rg) * SROW + c] = acc[i][j][rg];
            }
        }
        __syncthreads();
        for (int e = threadIdx.x; e < PR * LPR; e += NW * 64) {
            const int r = e / LPR;
            const int row = m0 + p * PR + r;
            if (row >= M) continue;
            f32x4 v = *reinterpret_cast<const f32x4*>(stg + r * SROW + c4);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (BIAS) v[u] = v[u] + bq[u];
                if (PRELU) v[u] = (v[u] < 0.0f) ? a * v[u] : v[u];
            }
            float* dst = Y + (size_t)row * ldy + col;
            if (vec && col + 3 < N) {
                __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(dst));
            } else {
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (col + u < N) __builtin_nontemporal_store(v[u], dst + u);
            }
        }
        __syncthreads();  // the staging is reused by the next pass
    }
}

// PARTIAL (split-K, blockIdx.y = the slice): the workgroup walks 64-k blocks
// [y * bps, min(nblk, (y + 1) * bps)) and stores its raw fp32 sums into slab
// y of Y (M x ldy floats per slab); k_reduce4 adds the slabs in slice order,
// then the bias and the PReLU.
template <int WM, int WN, int FI, int FJ, bool PRELU, bool PARTIAL>
__global__ void __launch_bounds__(WM * WN * 64) k_gemm3(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bt,
                                                      int ldk, int ldw, int M, int N, int nblk,
                                                      const float* __restrict__ bias, float* __restrict__ Y, int ldy,
                                                      float a, int tiles_m, int tiles_n, int gm, int bps) {
    static_assert(!(PARTIAL && PRELU), "a partial slab carries raw sums");
    constexpr int TM = WM * FI * 16, TN = WN * FJ * 16, NW = WM * WN;
    constexpr int PA = TM / 8, PB = TN / 8;  // 1-KiB pieces of a slot
    constexpr int ASLOT = PA * 1024, BSLOT = PB * 1024, BOFF = 2 * ASLOT;
    constexpr int PAW = PA / NW, PBW = PB / NW;  // pieces each wave moves per A / B slot
    static_assert(PA % NW == 0 && PB % NW == 0, "whole pieces per wave");
    __shared__ __attribute__((aligned(1024))) char lds[2 * ASLOT + 2 * BSLOT];

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = wave / WN, wc = wave % WN;

    int m0, n0;
    gemm3_tile<TM, TN>(tiles_m, tiles_n, gm, m0, n0);

    // this wave's DMA pieces: a uniform base (the operand's tile) plus per-lane
    // byte offsets (rows clamped into the matrix; 32-bit: the saddr form)
    const int row_in = lane >> 3, gsel = (lane & 7) ^ row_in;
    uint32_t offa[PAW];
#pragma unroll
    for (int i = 0; i < PAW; ++i)
        offa[i] = 2u * (uint32_t)(min(8 * (wave * PAW + i) + row_in, M - 1 - m0) * ldk + 8 * gsel);
    const char* abase = reinterpret_cast<const char*>(A + (size_t)m0 * ldk);
    const char* bbase = reinterpret_cast<const char*>(Bt + (size_t)n0 * ldw);
    auto dma_a = [&](int blk, int part, int slot) {  // X3's part `part` of 64-k block `blk`
        const char* g = abase + 2 * (size_t)(kMfmaBlk * (3 * blk + part));
#pragma unroll
        for (int i = 0; i < PAW; ++i)
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(g + offa[i]),
                                             (__attribute__((address_space(3))) void*)(lds + slot * ASLOT +
                                                                                       (wave * PAW + i) * 1024),
                                             16, 0, 0);
    };
    auto dma_b = [&](int blk, int slot) {  // W's 64-k block `blk` (offsets recomputed: once per block)
        const char* g = bbase + 2 * (size_t)(kMfmaBlk * blk);
#pragma unroll
        for (int i = 0; i < PBW; ++i)
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(
                                                 g + 2u * (uint32_t)(min(8 * (wave * PBW + i) + row_in, N - 1 - n0) * ldw +
                                                                     8 * gsel)),
                                             (__attribute__((address_space(3))) void*)(lds + BOFF + slot * BSLOT +
                                                                                       (wave * PBW + i) * 1024),
                                             16, 0, 0);
    };

    // fragment read offsets inside a 16-row block (the swizzle above)
    int foff[2];
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
        foff[kh] = ((lane & 15) >> 3) * 1024 + 16 * (8 * (lane & 7) + ((4 * kh + (lane >> 4)) ^ (lane & 7)));

    f32x4 acc[FI][FJ];
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // Half-step pipeline: the fragments of the two k halves live in two
    // register sets, and the one barrier per sub-step sits between them.
    // Sub-step s (block s / 3, part s % 3; A slot s & 1, B slot block & 1):
    //   read kh 1 of s (set 1)  |  MFMAs on set 0 (kh 0 of s)
    //   wait: set 1 read, DMA of s+1 landed; barrier (every wave is done with
    //   s's A slot -- and, at a block's first part, with the previous block's
    //   B slot -- and s+1 is in LDS)
    //   DMA A of s+2 into s's slot (+ the next block's B at a first part),
    //   read kh 0 of s+1 (set 0)  |  MFMAs on set 1
    // so each wave leaves the barrier with 32 MFMAs whose operands are already
    // in registers, and the DMA issue and the next reads run under them.
    // W's fragments are the same for a block's three parts: set kh of bfr is
    // read at the block's first part and kept through its last (A's are read
    // every sub-step).
    bf16x8 af[2][FI], bfr[2][FJ];
    auto frag_a = [&](int set, int aslot, int kh) {
        const char* sa = lds + aslot * ASLOT;
#pragma unroll
        for (int i = 0; i < FI; ++i)
            af[set][i] = *reinterpret_cast<const bf16x8*>(sa + ((wr * FI + i) * 2) * 1024 + foff[kh]);
    };
    auto frag_b = [&](int set, int bslot, int kh) {
        const char* sb = lds + BOFF + bslot * BSLOT;
#pragma unroll
        for (int j = 0; j < FJ; ++j)
            bfr[set][j] = *reinterpret_cast<const bf16x8*>(sb + ((wc * FJ + j) * 2) * 1024 + foff[kh]);
    };
    auto mma = [&](int set) {
#pragma unroll
        for (int i = 0; i < FI; ++i)
#pragma unroll
            for (int j = 0; j < FJ; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[set][i], bfr[set][j], acc[i][j], 0, 0, 0);
    };

    // The order is pinned (the compiler otherwise hoists the barrier over the
    // MFMAs and issues every read and DMA piece in one burst): each half step
    // is one scheduling region, one read per MFMA pair.  The tail's DMA is
    // clamped to the last block (a harmless reload into a slot no one reads
    // again) and its extra fragment read is discarded.
    constexpr int NM = FI * FJ;
    static_assert(2 * (FI + FJ) <= NM, "one read per MFMA pair");
    auto pin = [&](auto nr_c) {  // nr reads, one per MFMA pair, then the rest of the MFMAs
        constexpr int NR = decltype(nr_c)::value;
#pragma unroll
        for (int k = 0; k < NR; ++k) {
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // MFMA (first: its operands are the older reads)
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
        }
        if constexpr (NM > 2 * NR) __builtin_amdgcn_sched_group_barrier(0x008, NM - 2 * NR, 0);
        __builtin_amdgcn_sched_barrier(0);
    };
    using with_b = std::integral_constant<int, FI + FJ>;
    using a_only = std::integral_constant<int, FI>;
    // this workgroup's 64-k blocks (the host makes every slice non-empty);
    // ring slots count from the first of them
    const int b0 = PARTIAL ? (int)blockIdx.y * bps : 0;
    const int b1 = PARTIAL ? min(nblk, b0 + bps) : nblk;
    const int last = b1 - 1;
    dma_a(b0, 0, 0);
    dma_b(b0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    dma_a(b0, 1, 1);
    frag_b(0, 0, 0);
    frag_a(0, 0, 0);
    for (int blk = b0; blk < b1; ++blk) {
        const int bs = (blk - b0) & 1;
#pragma unroll
        for (int part = 0; part < 3; ++part) {
            const int as = (blk - b0 + part) & 1;  // (3 * (blk - b0) + part) & 1
            if (part == 0) frag_b(1, bs, 1);
            frag_a(1, as, 1);
            mma(0);
            if (part == 0) pin(with_b{}); else pin(a_only{});
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            __builtin_amdgcn_sched_barrier(0);
            // A of sub-step s + 2: (blk, 2) after part 0, else (blk + 1, part - 1)
            if (part == 0) {
                dma_a(blk, 2, as);
                dma_b(min(blk + 1, last), bs ^ 1);
            } else {
                const bool tail = blk == last;  // uniform: a scalar select, no branch
                dma_a(tail ? last : blk + 1, tail ? 2 : part - 1, as);
            }
            if (part == 2) frag_b(0, bs ^ 1, 0);  // the next block's
            frag_a(0, as ^ 1, 0);
            mma(1);
            if (part == 2) pin(with_b{}); else pin(a_only{});
        }
    }
    // the tail's reloads land and every wave's last reads are done before the
    // epilogue reuses the LDS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    float* out = PARTIAL ? Y + (size_t)blockIdx.y * M * ldy : Y;
    gemm3_store<WM, WN, FI, FJ, PRELU, !PARTIAL, 2 * ASLOT + 2 * BSLOT>(acc, lds, lane, wr, wc, m0, n0, M, N, bias, out,
                                                                        ldy, a);
}

}  // namespace

hipError_t csc_prepare(const int* csp, const int* csn, const int* rip, const int* rin, int col_begin, int ncols,
                       long long n_pos, long long n_neg, int* cp, int* cn, int* crp, int* crn, int* gq, void* scan_tmp,
                       size_t scan_tmp_bytes, int* cq, hipStream_t st) {
    hipError_t e;
    if ((e = rebase_offsets(csp, col_begin, ncols, cp, st)) != hipSuccess) return e;
    if ((e = rebase_offsets(csn, col_begin, ncols, cn, st)) != hipSuccess) return e;
    if (n_pos > 0)
        hipLaunchKernelGGL(k_copy_from, dim3(grid_of(n_pos, 256)), dim3(256), 0, st, rip, csp, col_begin, n_pos, crp);
    if (n_neg > 0)
        hipLaunchKernelGGL(k_copy_from, dim3(grid_of(n_neg, 256)), dim3(256), 0, st, rin, csn, col_begin, n_neg, crn);
    const int ng = csc_groups(ncols);
    hipLaunchKernelGGL(k_group_quads, dim3(grid_of((long long)ng + 1, 256)), dim3(256), 0, st, cp, cn, ncols, gq);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return exclusive_scan_i32(gq, cq, ng + 1, scan_tmp, scan_tmp_bytes, st);
}

hipError_t csc_fill(const int* cp, const int* cn, const int* crp, const int* crn, const int* cq, int ncols, int rows,
                    int* crq, size_t crq_entries, hipStream_t st) {
    hipError_t e;
    // the guard quads (and nothing else) stay 0: row 0, read only by the look-ahead
    if ((e = hipMemsetAsync(crq, 0, crq_entries * sizeof(int), st)) != hipSuccess) return e;
    if (ncols > 0)
        hipLaunchKernelGGL(k_merge_csc, dim3(grid_of(ncols, 256)), dim3(256), 0, st, cp, cn, crp, crn, cq, ncols, rows,
                           crq);
    return hipGetLastError();
}

hipError_t mfma_build_wt(const int* csp, const int* csn, const int* rip, const int* rin, int col_begin, int rows,
                         int ncols, float* wf, uint16_t* wt, int ldw, long long n_pos, long long n_neg, int* bad,
                         hipStream_t st) {
    const long long n = (long long)rows * ncols;
    hipError_t e = hipMemsetAsync(wf, 0, (size_t)n * sizeof(float), st);
    if (e != hipSuccess) return e;
    if ((e = hipMemsetAsync(wt, 0, (size_t)ncols * ldw * sizeof(uint16_t), st)) != hipSuccess) return e;
    const int wpb = 4;  // waves (columns) per block
    if (n_pos > 0)
        hipLaunchKernelGGL(k_w_scatter, dim3((ncols + wpb - 1) / wpb), dim3(64 * wpb), 0, st, csp, rip, col_begin,
                           ncols, rows, 1.0f, wf);
    if (n_neg > 0)
        hipLaunchKernelGGL(k_w_scatter, dim3((ncols + wpb - 1) / wpb), dim3(64 * wpb), 0, st, csn, rin, col_begin,
                           ncols, rows, -1.0f, wf);
    hipLaunchKernelGGL(k_wt_from, dim3(grid_of(n, 256)), dim3(256), 0, st, wf, ncols, rows, wt, ldw, bad);
    return hipGetLastError();
}

hipError_t mfma_split_x(const float* X, int M, int K, uint16_t* x3, int ldk, int* flags, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_split3, dim3(M), dim3(256), 0, st, X, M, K, x3, ldk, flags);
    return hipGetLastError();
}

// Tile choice: 128 x 512 (8 waves) unless a grid of 256 x 256 tiles would
// leave more than half of the 256 CUs idle, then 128 x 128 (4 waves).
bool mfma_big_tiles(int M, int N) { return (long long)((M + 255) / 256) * ((N + 255) / 256) >= 128; }

// M <= 64 on a small grid: 64 x 256 tiles of 4 waves (1 x 4, 64 x 64 each),
// so no MFMA work and no A staging go to rows past M (the 128 x 128 tiles
// would spend half of both on copies of row M - 1).
bool mfma_narrow_tiles(int M, int N) { return M <= 64 && !mfma_big_tiles(M, N); }

// Workgroups of the unsplit grid: 128 x 512 tiles, 64 x 256 or 128 x 128.
long long mfma_tiles(int M, int N) {
    if (mfma_big_tiles(M, N)) return (long long)((M + 127) / 128) * ((N + 511) / 512);
    if (mfma_narrow_tiles(M, N)) return (long long)((M + 63) / 64) * ((N + 255) / 256);
    return (long long)((M + 127) / 128) * ((N + 127) / 128);
}

// Split-K of a grid with fewer tiles than it can run at once: enough slices
// of the 64-k blocks to bring it to ~512 workgroups of the small or narrow
// tiles (two fit a CU: 64 / 80 KiB of LDS, 4 waves each; ~1,024 of the
// narrow ones, whose slices are cheap to reduce: M <= 64) or ~256 of the
// large ones (one per CU), each slice at least 8 blocks, at most 16 slices (k_reduce4's limit);
// normalized so no slice is empty.  Measured (tools/crossover.py, K = N =
// 8192): M = 64 0.199 -> 0.062 ms, M = 256 0.212 -> 0.108, M = 1024 (large
// tiles, 2 slices) 0.456 -> 0.32; targets of 768 / 1024 small tiles or 512
// large ones were slower.  Narrow tiles: 1024 equals 512 at K = N = 8192 (16
// slices either way) and is 19 % faster at M = 16, K = N = 16384.  $TCSC_MFMA_WGS overrides the target (A/B; 0 =
// never split).
int mfma_split_target(bool big, bool narrow) {
    const char* e = std::getenv("TCSC_MFMA_WGS");
    return e ? std::atoi(e) : big ? 256 : narrow ? 1024 : 512;
}

int mfma_slices(int M, int N, int K) {
    if (M <= 0 || N <= 0) return 1;
    const long long tiles = mfma_tiles(M, N);
    const int nblk = mfma_nblk(K);
    const long long s =
        std::min<long long>({mfma_split_target(mfma_big_tiles(M, N), mfma_narrow_tiles(M, N)) / tiles, 16, nblk / 8});
    if (s < 2) return 1;
    const int bps = (int)((nblk + s - 1) / s);
    return (nblk + bps - 1) / bps;
}

size_t mfma_slab_bytes(int M, int N, int K) {
    const int s = mfma_slices(M, N, K);
    return s > 1 ? (size_t)s * M * N * sizeof(float) : 0;
}

template <bool PRELU>
static hipError_t launch_gemm3_t(const uint16_t* x3, int ldk, const uint16_t* wt, int ldw, int K, int nblk, int M,
                                 int N, const float* B, float* Y, int ldy, float a, float* slabs, int slices,
                                 const int* flags, const int* cq, const int* crq, hipStream_t st) {
    // bands of 4 row tiles: an XCD's 32 workgroups share 4 A tiles (staged every
    // sub-step) and 8 W tiles (once per block); 8 x 4 was 2 % slower at cfg 5
    constexpr int kGm = 4;
    if (mfma_big_tiles(M, N)) {
        // 128 x 512 tiles of 8 waves (1 x 8, 128 x 64 each): A, staged every
        // sub-step, is the narrow side (37.3 KiB staged per sub-step, 256 x 256
        // tiles: 42.7; 1.4 % faster at cfg 5).  Its LDS is the whole 160 KiB.
        const int tm = (M + 127) / 128, tn = (N + 511) / 512;
        const int gm = std::min(kGm, tm);
        if (slices <= 1)
            hipLaunchKernelGGL((k_gemm3<1, 8, 8, 4, PRELU, false>), dim3(tm * tn), dim3(512), 0, st, x3, wt, ldk, ldw,
                               M, N, nblk, B, Y, ldy, a, tm, tn, gm, nblk);
        else
            hipLaunchKernelGGL((k_gemm3<1, 8, 8, 4, false, true>), dim3(tm * tn, slices), dim3(512), 0, st, x3, wt,
                               ldk, ldw, M, N, nblk, nullptr, slabs, N, 0.0f, tm, tn, gm, (nblk + slices - 1) / slices);
    } else if (mfma_narrow_tiles(M, N)) {
        const int tn = (N + 255) / 256;
        if (slices <= 1)
            hipLaunchKernelGGL((k_gemm3<1, 4, 4, 4, PRELU, false>), dim3(tn), dim3(256), 0, st, x3, wt, ldk, ldw, M, N,
                               nblk, B, Y, ldy, a, 1, tn, 1, nblk);
        else
            hipLaunchKernelGGL((k_gemm3<1, 4, 4, 4, false, true>), dim3(tn, slices), dim3(256), 0, st, x3, wt, ldk, ldw,
                               M, N, nblk, nullptr, slabs, N, 0.0f, 1, tn, 1, (nblk + slices - 1) / slices);
    } else {
        const int tm = (M + 127) / 128, tn = (N + 127) / 128;
        const int gm = std::min(kGm, tm);
        if (slices <= 1)
            hipLaunchKernelGGL((k_gemm3<2, 2, 4, 4, PRELU, false>), dim3(tm * tn), dim3(256), 0, st, x3, wt, ldk, ldw,
                               M, N, nblk, B, Y, ldy, a, tm, tn, gm, nblk);
        else
            hipLaunchKernelGGL((k_gemm3<2, 2, 4, 4, false, true>), dim3(tm * tn, slices), dim3(256), 0, st, x3, wt,
                               ldk, ldw, M, N, nblk, nullptr, slabs, N, 0.0f, tm, tn, gm, (nblk + slices - 1) / slices);
    }
    // split K: raw partial tiles went into slabs[slice] (M x N); then
    // act(s0 + s1 + ... + b) in slice order, flagged rows exact (k_fixup's)
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess || slices <= 1) return e;
    const bool vec = N % 4 == 0 && ldy % 4 == 0 &&
                     ((reinterpret_cast<uintptr_t>(Y) | reinterpret_cast<uintptr_t>(slabs) |
                       reinterpret_cast<uintptr_t>(B)) & 15) == 0;
    const long long n = (long long)M * (vec ? N / 4 : N);
    if (vec)
        hipLaunchKernelGGL((k_reduce_fix<PRELU, true>), dim3(grid_of(n, 256)), dim3(256), 0, st, slabs, slices, M, N, B,
                           Y, ldy, a, flags, x3, K, ldk, cq, crq);
    else
        hipLaunchKernelGGL((k_reduce_fix<PRELU, false>), dim3(grid_of(n, 256)), dim3(256), 0, st, slabs, slices, M, N,
                           B, Y, ldy, a, flags, x3, K, ldk, cq, crq);
    return hipGetLastError();
}

hipError_t mfma_gemm3(const uint16_t* x3, int ldk, const uint16_t* wt, int ldw, int K, int M, int N, const float* B,
                      float* Y, int ldy, bool prelu, float a, float* slabs, size_t slab_bytes, const int* flags,
                      const int* cq, const int* crq, hipStream_t st) {
    if (M <= 0 || N <= 0) return hipSuccess;
    const int nblk = mfma_nblk(K);
    if (nblk < 1 || ldk != mfma_ldk(K) || ldw != mfma_ldw(K)) return hipErrorInvalidValue;
    const int slices = mfma_slices(M, N, K);
    if (slices > 1 && (!slabs || slab_bytes < mfma_slab_bytes(M, N, K))) return hipErrorInvalidValue;
    return prelu ? launch_gemm3_t<true>(x3, ldk, wt, ldw, K, nblk, M, N, B, Y, ldy, a, slabs, slices, flags, cq, crq,
                                        st)
                 : launch_gemm3_t<false>(x3, ldk, wt, ldw, K, nblk, M, N, B, Y, ldy, a, slabs, slices, flags, cq, crq,
                                         st);
}

hipError_t mfma_fixup(const uint16_t* x3, int M, int K, int ldk, const int* cq, const int* crq, int ncols,
                      const float* B, float* Y, int ldy, bool bias_first, bool prelu, float a, const int* flags,
                      hipStream_t st) {
    const dim3 grid((ncols + 255) / 256), block(256);
#define TCSC_FIX_ARGS x3, M, K, ldk, cq, crq, ncols, B, Y, ldy, a, flags
    if (bias_first) {
        if (prelu)
            hipLaunchKernelGGL((k_fixup<true, true>), grid, block, 0, st, TCSC_FIX_ARGS);
        else
            hipLaunchKernelGGL((k_fixup<true, false>), grid, block, 0, st, TCSC_FIX_ARGS);
    } else {
        if (prelu)
            hipLaunchKernelGGL((k_fixup<false, true>), grid, block, 0, st, TCSC_FIX_ARGS);
        else
            hipLaunchKernelGGL((k_fixup<false, false>), grid, block, 0, st, TCSC_FIX_ARGS);
    }
#undef TCSC_FIX_ARGS
    return hipGetLastError();
}

}  // namespace tcsc
