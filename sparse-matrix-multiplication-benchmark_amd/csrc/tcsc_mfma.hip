// tcsc_mfma.hip -- the MFMA path for near-dense W.
//
// At 50 % density (BASELINE cfg 5) the gather walks half of W: 33.5 M
// nonzeros x 2048 rows at ~27 T adds/s = 2.5 ms, while the matrix cores
// multiply the dense W at ~1.7 PFLOP/s in bf16.  The path keeps fp32
// results without an fp32 MFMA (0.15 PFLOP/s): every x is split exactly into
// three bf16 parts, x = h + m + l (truncations of x and of its remainders:
// 8 + 8 + 8 significand bits), W is exact in bf16 (0, +-1, or small
// integers for duplicate rows), so each product is exact and the GEMM
//     Y = [h | m | l] . [W ; W ; W]           (M x 3K) . (3K x N)
// (W stored transposed, N x 3K, so both operands run along k)
// accumulates in fp32 on the matrix cores (rocBLAS gemm_ex bf16 -> f32).
// Only the summation order differs from the gather's: the result is within
// the fast-order bound, and bit-exact on integer-valued inputs.
//
// Rows the split cannot carry are recomputed by the gather order: a
// non-finite x would make inf*0 = NaN in columns whose W is 0 there (the
// reference never touches those products), and bf16 MFMA inputs below
// 2^-126 may be flushed.  k_split3 flags every row holding a non-finite x
// or a nonzero |x| < 2^-100; k_fixup rewrites those rows from the plan's
// per-column CSC copy, +1 and -1 rows merged in ascending k (+1 first on a
// tie), bias first for tcsc_sgemm_basic, then the PReLU -- the exact
// arithmetic of k_stream's fast order.
#include <hip/hip_runtime.h>

#include <cstdint>

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

// X (M x K, pitch K) -> X3 (M x 3K bf16, pitch 3K): [h | m | l] per row.
// flags[m] = gen (and *any = gen) for a row the fixup must recompute; gen
// is new for every staging, so the flags need no clearing (a stale value
// equal to gen could only make the fixup recompute a row exactly).
__global__ void k_split3(const float* __restrict__ X, int M, int K, uint16_t* __restrict__ X3,
                         int* __restrict__ flags, int* __restrict__ any, int gen) {
    const int kq = (K + 3) / 4;
    const long long total = (long long)M * kq;
    const bool vec = (K & 3) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int row = (int)(i / kq), k0 = 4 * (int)(i % kq);
        const float* src = X + (size_t)row * K + k0;
        float v[4];
        if (vec) {
            const float4 q = *reinterpret_cast<const float4*>(src);
            v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
        } else {
            for (int j = 0; j < 4; ++j) v[j] = k0 + j < K ? src[j] : 0.0f;
        }
        uint16_t h[4], m[4], l[4];
        bool fix = false;
        for (int j = 0; j < 4; ++j) fix |= split3(v[j], h[j], m[j], l[j]);
        uint16_t* dst = X3 + (size_t)row * 3 * K + k0;
        if (vec) {
            // 8-byte stores: k0 is a multiple of 4 and K too, so all three are aligned
            typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
            *reinterpret_cast<u16x4*>(dst) = u16x4{h[0], h[1], h[2], h[3]};
            *reinterpret_cast<u16x4*>(dst + K) = u16x4{m[0], m[1], m[2], m[3]};
            *reinterpret_cast<u16x4*>(dst + 2 * (size_t)K) = u16x4{l[0], l[1], l[2], l[3]};
        } else {
            for (int j = 0; j < 4 && k0 + j < K; ++j) {
                dst[j] = h[j];
                dst[K + j] = m[j];
                dst[2 * (size_t)K + j] = l[j];
            }
        }
        if (fix) {
            flags[row] = gen;
            *any = gen;
        }
    }
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

// WfT (ncols x K fp32) -> W3T (ncols x 3K bf16): row n = [w | w | w], so both
// GEMM operands run along k (the "TN" form, ~8 % faster than W3 as 3K x
// ncols: tools/dense3_bench.cpp).  Values must be integers of magnitude
// <= 256 to be exact in bf16; *bad = 1 otherwise.
__global__ void k_w3_from(const float* __restrict__ WfT, int ncols, int K, uint16_t* __restrict__ W3T,
                          int* __restrict__ bad) {
    const long long n = (long long)ncols * K;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        const float w = WfT[i];
        if (fabsf(w) > 256.0f) *bad = 1;
        const uint16_t b = (uint16_t)(f2u(w) >> 16);
        const long long j = i / K, k = i - j * K;
        uint16_t* row = W3T + j * 3 * K;
        row[k] = b;
        row[K + k] = b;
        row[2 * K + k] = b;
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

// Output (row, j) recomputed exactly as k_stream's fast order (see the file
// comment): x rebuilt from its three parts, +1 and -1 rows merged in
// ascending k, the bias first or last, then the PReLU.
template <bool BIAS_FIRST, bool PRELU>
__device__ inline float exact_out(const uint16_t* __restrict__ X3, int K, const int* __restrict__ cp,
                                  const int* __restrict__ cn, const int* __restrict__ rp,
                                  const int* __restrict__ rn, const float* __restrict__ Bias, int row, int j,
                                  float a) {
    const uint16_t* x3 = X3 + (size_t)row * 3 * K;
    auto xk = [&](int k) {
        return (u2f((uint32_t)x3[k] << 16) + u2f((uint32_t)x3[K + k] << 16)) + u2f((uint32_t)x3[2 * K + k] << 16);
    };
    float acc = BIAS_FIRST ? Bias[j] : 0.0f;
    int p = cp[j], q = cn[j];
    const int p1 = cp[j + 1], q1 = cn[j + 1];
    while (p < p1 || q < q1) {
        if (q >= q1 || (p < p1 && rp[p] <= rn[q])) {
            acc = fmaf(xk(rp[p]), 1.0f, acc);
            ++p;
        } else {
            acc = fmaf(xk(rn[q]), -1.0f, acc);
            ++q;
        }
    }
    if (!BIAS_FIRST) acc += Bias[j];
    if (PRELU) acc = (acc < 0.0f) ? a * acc : acc;
    return acc;
}

// Flagged rows, after a GEMM that already added the bias (no PReLU).  One
// thread per column; every block walks the flag list.
template <bool BIAS_FIRST, bool PRELU>
__global__ void k_fixup(const uint16_t* __restrict__ X3, int M, int K, const int* __restrict__ cp,
                        const int* __restrict__ cn, const int* __restrict__ rp, const int* __restrict__ rn,
                        int ncols, const float* __restrict__ Bias, float* __restrict__ Y, int ldy, float a,
                        const int* __restrict__ flags, const int* __restrict__ any, int gen) {
    if (*any != gen) return;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= ncols) return;
    for (int row = 0; row < M; ++row)
        if (flags[row] == gen)
            Y[(size_t)row * ldy + j] = exact_out<BIAS_FIRST, PRELU>(X3, K, cp, cn, rp, rn, Bias, row, j, a);
}

// The epilogue after a plain GEMM, with the fixup folded in: Y = act(Y + B)
// for the rows the split carried, the exact fast-order value for the
// flagged ones.  One launch instead of two.
template <bool BIAS_FIRST, bool PRELU>
__global__ void k_epilogue_fix(float* __restrict__ Y, int M, int N, int ldy, const float* __restrict__ Bias, float a,
                               const uint16_t* __restrict__ X3, int K, const int* __restrict__ cp,
                               const int* __restrict__ cn, const int* __restrict__ rp, const int* __restrict__ rn,
                               const int* __restrict__ flags, const int* __restrict__ any, int gen) {
    const bool some = *any == gen;
    const int nq = (N + 3) / 4;
    const long long total = (long long)M * nq;
    const bool vec = (ldy & 3) == 0 && (N & 3) == 0 && ((reinterpret_cast<uintptr_t>(Y) & 15) == 0);
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int m = (int)(i / nq), n = 4 * (int)(i % nq);
        float* y = Y + (size_t)m * ldy + n;
        if (some && flags[m] == gen) {
            for (int c = 0; c < 4 && n + c < N; ++c)
                y[c] = exact_out<BIAS_FIRST, PRELU>(X3, K, cp, cn, rp, rn, Bias, m, n + c, a);
            continue;
        }
        if (vec) {
            float4 v = *reinterpret_cast<float4*>(y);
            v.x += Bias[n + 0];
            v.y += Bias[n + 1];
            v.z += Bias[n + 2];
            v.w += Bias[n + 3];
            if (PRELU) {
                v.x = (v.x < 0.0f) ? a * v.x : v.x;
                v.y = (v.y < 0.0f) ? a * v.y : v.y;
                v.z = (v.z < 0.0f) ? a * v.z : v.z;
                v.w = (v.w < 0.0f) ? a * v.w : v.w;
            }
            *reinterpret_cast<float4*>(y) = v;
        } else {
            for (int c = 0; c < 4 && n + c < N; ++c) {
                float v = y[c] + Bias[n + c];
                if (PRELU) v = (v < 0.0f) ? a * v : v;
                y[c] = v;
            }
        }
    }
}

}  // namespace

hipError_t csc_copy(const int* csp, const int* csn, const int* rip, const int* rin, int col_begin, int ncols,
                    long long n_pos, long long n_neg, int* cp, int* cn, int* crp, int* crn, hipStream_t st) {
    hipError_t e;
    if ((e = rebase_offsets(csp, col_begin, ncols, cp, st)) != hipSuccess) return e;
    if ((e = rebase_offsets(csn, col_begin, ncols, cn, st)) != hipSuccess) return e;
    if (n_pos > 0)
        hipLaunchKernelGGL(k_copy_from, dim3(grid_of(n_pos, 256)), dim3(256), 0, st, rip, csp, col_begin, n_pos, crp);
    if (n_neg > 0)
        hipLaunchKernelGGL(k_copy_from, dim3(grid_of(n_neg, 256)), dim3(256), 0, st, rin, csn, col_begin, n_neg, crn);
    return hipGetLastError();
}

hipError_t mfma_build_w3(const int* csp, const int* csn, const int* rip, const int* rin, int col_begin, int rows,
                         int ncols, float* wf, uint16_t* w3, long long n_pos, long long n_neg, int* bad,
                         hipStream_t st) {
    const long long n = (long long)rows * ncols;
    hipError_t e = hipMemsetAsync(wf, 0, (size_t)n * sizeof(float), st);
    if (e != hipSuccess) return e;
    const int wpb = 4;  // waves (columns) per block
    if (n_pos > 0)
        hipLaunchKernelGGL(k_w_scatter, dim3((ncols + wpb - 1) / wpb), dim3(64 * wpb), 0, st, csp, rip, col_begin,
                           ncols, rows, 1.0f, wf);
    if (n_neg > 0)
        hipLaunchKernelGGL(k_w_scatter, dim3((ncols + wpb - 1) / wpb), dim3(64 * wpb), 0, st, csn, rin, col_begin,
                           ncols, rows, -1.0f, wf);
    hipLaunchKernelGGL(k_w3_from, dim3(grid_of(n, 256)), dim3(256), 0, st, wf, ncols, rows, w3, bad);
    return hipGetLastError();
}

hipError_t mfma_split_x(const float* X, int M, int K, uint16_t* x3, int* flags, int* any, int gen, hipStream_t st) {
    const long long total = (long long)M * ((K + 3) / 4);
    hipLaunchKernelGGL(k_split3, dim3(grid_of(total, 256)), dim3(256), 0, st, X, M, K, x3, flags, any, gen);
    return hipGetLastError();
}

hipError_t mfma_epilogue_fix(const uint16_t* x3, int M, int K, const int* cp, const int* cn, const int* crp,
                             const int* crn, int ncols, const float* B, float* Y, int ldy, bool bias_first, bool prelu,
                             float a, const int* flags, const int* any, int gen, hipStream_t st) {
    const long long total = (long long)M * ((ncols + 3) / 4);
    const dim3 grid(grid_of(total, 256)), block(256);
#define TCSC_EPI_ARGS Y, M, ncols, ldy, B, a, x3, K, cp, cn, crp, crn, flags, any, gen
    if (bias_first) {
        if (prelu)
            hipLaunchKernelGGL((k_epilogue_fix<true, true>), grid, block, 0, st, TCSC_EPI_ARGS);
        else
            hipLaunchKernelGGL((k_epilogue_fix<true, false>), grid, block, 0, st, TCSC_EPI_ARGS);
    } else {
        if (prelu)
            hipLaunchKernelGGL((k_epilogue_fix<false, true>), grid, block, 0, st, TCSC_EPI_ARGS);
        else
            hipLaunchKernelGGL((k_epilogue_fix<false, false>), grid, block, 0, st, TCSC_EPI_ARGS);
    }
#undef TCSC_EPI_ARGS
    return hipGetLastError();
}

hipError_t mfma_fixup(const uint16_t* x3, int M, int K, const int* cp, const int* cn, const int* crp, const int* crn,
                      int ncols, const float* B, float* Y, int ldy, bool bias_first, bool prelu, float a,
                      const int* flags, const int* any, int gen, hipStream_t st) {
    const dim3 grid((ncols + 255) / 256), block(256);
    if (bias_first) {
        if (prelu)
            hipLaunchKernelGGL((k_fixup<true, true>), grid, block, 0, st, x3, M, K, cp, cn, crp, crn, ncols, B, Y, ldy,
                               a, flags, any, gen);
        else
            hipLaunchKernelGGL((k_fixup<true, false>), grid, block, 0, st, x3, M, K, cp, cn, crp, crn, ncols, B, Y,
                               ldy, a, flags, any, gen);
    } else {
        if (prelu)
            hipLaunchKernelGGL((k_fixup<false, true>), grid, block, 0, st, x3, M, K, cp, cn, crp, crn, ncols, B, Y,
                               ldy, a, flags, any, gen);
        else
            hipLaunchKernelGGL((k_fixup<false, false>), grid, block, 0, st, x3, M, K, cp, cn, crp, crn, ncols, B, Y,
                               ldy, a, flags, any, gen);
    }
    return hipGetLastError();
}

}  // namespace tcsc
