// tcsc_kernels.hip -- gfx950 (MI355X / CDNA4) kernels for the TCSC
// sparse-ternary GEMM  Y = act(X * W + b),  W in {-1,0,+1}.
//
// Replaces the CPU loops of /root/reference/sparse/tcsc.c:
//   tcsc_sgemm_basic                     tcsc.c:69-98
//   tcsc_sgemm_optimized                 tcsc.c:101-140
//   tcsc_sgemm_prelu_basic               tcsc.c:143-165
//   tcsc_sgemm_prelu_optimized_separate  tcsc.c:179-227
//   tcsc_sgemm_prelu_optimized_onthego   tcsc.c:231-275
// and tcsc_from_dense (tcsc.c:6-66) with a device builder.
//
// Design (DESIGN.md has the full derivation):
//  * lanes = rows of X.  A workgroup owns TM = 128 rows (two per lane) and
//    WAVES*CW output columns.  K is cut into chunks of TK rows; each chunk of
//    X is staged in LDS transposed, as float2 pairs xs[k][lane] =
//    (X[m0+2*lane][k0+k], X[m0+2*lane+1][k0+k]) -- one 512-B LDS row per k.
//  * Every nonzero of a column is then ONE conflict-free ds_read_b64 that all
//    64 lanes issue at the same k (the index is wave-uniform and lives in an
//    SGPR), followed by two adds/subtracts.  No multiplies, no MFMA (W is
//    ternary and 98 % sparse at the headline size: a dense product would do
//    50x the work).
//  * W is re-laid out once per tcsc_t ("plan"): the +1 and -1 lists of a
//    column are merged in ascending k and bucketed by (chunk, column), so the
//    entries a wave needs for one chunk are contiguous.  Entry encoding:
//    bits 0-15 = k - k0 (row inside the chunk), bit 31 = sign (1 = -1).
//  * Accumulators stay in VGPRs for the whole K loop; the epilogue adds the
//    bias (first or last, matching the reference variant's order) and
//    applies PReLU in registers before the single store of Y.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "tcsc_internal.h"

namespace tcsc {

// ---------------------------------------------------------------------------
// Plan building
// ---------------------------------------------------------------------------

__device__ __forceinline__ int lower_bound_i32(const int* __restrict__ a, int lo, int hi, int key) {
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (a[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// For every (chunk boundary c in [0, nch], column n): absolute position of the
// first +1 (resp. -1) entry of column n with row >= c*TK.
__global__ void k_chunk_bounds(const int* __restrict__ csp, const int* __restrict__ csn,
                               const int* __restrict__ rip, const int* __restrict__ rin,
                               int col_begin, int ncols, int nch, int tk, int K,
                               int* __restrict__ lbp, int* __restrict__ lbn) {
    const long long total = (long long)(nch + 1) * ncols;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int c = (int)(i / ncols), n = (int)(i % ncols);
        const int key = (c == nch) ? 0x7fffffff : c * tk;
        const int gn = col_begin + n;
        lbp[i] = lower_bound_i32(rip, csp[gn], csp[gn + 1], key);
        lbn[i] = lower_bound_i32(rin, csn[gn], csn[gn + 1], key);
    }
}

// cnt[c*ncols + n] = entries of column n inside chunk c.
__global__ void k_chunk_counts(const int* __restrict__ lbp, const int* __restrict__ lbn,
                               int ncols, int nch, int* __restrict__ cnt) {
    const long long total = (long long)nch * ncols;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        cnt[i] = (lbp[i + ncols] - lbp[i]) + (lbn[i + ncols] - lbn[i]);
    }
}

// Scatter the +1 (SIGN=0) or -1 (SIGN=1) entries of columns
// [col_begin, col_begin+ncols) to their merged position.  Position inside the
// (chunk, column) bucket = rank among own-sign entries of the bucket + number
// of opposite-sign entries of the bucket with a smaller row.
template <int SIGN>
__global__ void k_scatter(const int* __restrict__ cs_own, const int* __restrict__ ri_own,
                          const int* __restrict__ cs_oth, const int* __restrict__ ri_oth,
                          const int* __restrict__ lb_own, const int* __restrict__ lb_oth,
                          const int* __restrict__ cptr, int col_begin, int ncols, int tk,
                          int* __restrict__ ent) {
    const int base = cs_own[col_begin];
    const int total = cs_own[col_begin + ncols] - base;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
        const int i = base + t;
        // column: last n with cs_own[col_begin+n] <= i
        int lo = 0, hi = ncols;  // answer in [0, ncols)
        while (hi - lo > 1) {
            int mid = (lo + hi) >> 1;
            if (cs_own[col_begin + mid] <= i) lo = mid; else hi = mid;
        }
        const int n = lo, gn = col_begin + n;
        const int k = ri_own[i];
        const int c = k / tk;
        const long long b = (long long)c * ncols + n;
        const int rank_own = i - lb_own[b];
        const int rank_oth = lower_bound_i32(ri_oth, cs_oth[gn], cs_oth[gn + 1], k) - lb_oth[b];
        const int pos = cptr[b] + rank_own + rank_oth;
        ent[pos] = (k - c * tk) | (SIGN ? (int)0x80000000u : 0);
    }
}

// ---------------------------------------------------------------------------
// The gather kernel
// ---------------------------------------------------------------------------

template <int TK>
__device__ __forceinline__ void stage_x_tile(const float* __restrict__ X, int M, int K, int m0, int k0,
                                             float2* __restrict__ xs, bool vec4) {
    // Tile = 128 rows x TK k.  Work item = (row pair p, 4-wide k group q).
    // Lanes run over 16 consecutive pairs first so the transposed LDS writes
    // (xs[4q+j][p], 8 B each) from one 16-lane group hit 128 contiguous bytes.
    constexpr int NQ = TK / 4;
    constexpr int ITEMS = 64 * NQ;
    for (int it = threadIdx.x; it < ITEMS; it += blockDim.x) {
        const int p = (it & 15) | (((it >> 4) / NQ) << 4);
        const int q = (it >> 4) % NQ;
        const int r0 = m0 + 2 * p, r1 = r0 + 1;
        const int kk = k0 + 4 * q;
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
        if (vec4 && kk + 3 < K) {
            if (r0 < M) a = *reinterpret_cast<const float4*>(X + (size_t)r0 * K + kk);
            if (r1 < M) b = *reinterpret_cast<const float4*>(X + (size_t)r1 * K + kk);
        } else {
            float va[4] = {0.f, 0.f, 0.f, 0.f}, vb[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (kk + j < K) {
                    if (r0 < M) va[j] = X[(size_t)r0 * K + kk + j];
                    if (r1 < M) vb[j] = X[(size_t)r1 * K + kk + j];
                }
            }
            a = make_float4(va[0], va[1], va[2], va[3]);
            b = make_float4(vb[0], vb[1], vb[2], vb[3]);
        }
        xs[(4 * q + 0) * 64 + p] = make_float2(a.x, b.x);
        xs[(4 * q + 1) * 64 + p] = make_float2(a.y, b.y);
        xs[(4 * q + 2) * 64 + p] = make_float2(a.z, b.z);
        xs[(4 * q + 3) * 64 + p] = make_float2(a.w, b.w);
    }
}

// BIAS_FIRST: y = b; y +- x ...   (tcsc_sgemm_basic order, tcsc.c:74-96)
// otherwise:  y = 0; y +- x ...; y += b   (prelu_basic order, tcsc.c:149-161)
template <int TK, int CW, int WAVES, bool BIAS_FIRST, bool PRELU>
__global__ void __launch_bounds__(WAVES * 64)
k_tcsc_gather(const float* __restrict__ X, int M, int K,
              const int* __restrict__ ent, const int* __restrict__ cptr, int ncols,
              const float* __restrict__ Bias, float* __restrict__ Y, int ldy, float a, int vec4) {
    __shared__ float2 xs[TK * 64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int m0 = blockIdx.y * 128;
    const int nw = (blockIdx.x * WAVES + wave) * CW;  // first column of this wave
    const int nch = (K + TK - 1) / TK;
    const int nvalid = min(CW, max(ncols - nw, 0));  // wave-uniform

    float2 acc[CW];
#pragma unroll
    for (int j = 0; j < CW; ++j) {
        float b0 = 0.f;
        if (BIAS_FIRST && j < nvalid) b0 = Bias[nw + j];
        acc[j] = make_float2(b0, b0);
    }

    for (int c = 0; c < nch; ++c) {
        if (c) __syncthreads();
        stage_x_tile<TK>(X, M, K, m0, c * TK, xs, vec4 != 0);
        __syncthreads();
        if (nvalid == 0) continue;
        const int* __restrict__ cp = cptr + (size_t)c * ncols + nw;
        int p = cp[0];
#pragma unroll
        for (int j = 0; j < CW; ++j) {
            if (j < nvalid) {
                const int pe = cp[j + 1];
                for (; p < pe; ++p) {
                    const int e = ent[p];
                    const float2 x = xs[(e & 0xffff) * 64 + lane];
                    const float s = __int_as_float((e & (int)0x80000000u) | 0x3f800000);
                    acc[j].x = __builtin_fmaf(x.x, s, acc[j].x);
                    acc[j].y = __builtin_fmaf(x.y, s, acc[j].y);
                }
            }
        }
    }

    // epilogue
    const int r0 = m0 + 2 * lane, r1 = r0 + 1;
#pragma unroll
    for (int j = 0; j < CW; ++j) {
        if (j < nvalid) {
            float y0 = acc[j].x, y1 = acc[j].y;
            if (!BIAS_FIRST) {
                const float b0 = Bias[nw + j];
                y0 += b0;
                y1 += b0;
            }
            if (PRELU) {
                y0 = (y0 < 0.0f) ? a * y0 : y0;
                y1 = (y1 < 0.0f) ? a * y1 : y1;
            }
            if (r0 < M) Y[(size_t)r0 * ldy + nw + j] = y0;
            if (r1 < M) Y[(size_t)r1 * ldy + nw + j] = y1;
        }
    }
}

// ---------------------------------------------------------------------------
// Device tcsc_from_dense (bit-exact with tcsc.c:6-66): per-column counts,
// exclusive scans, then a fill that keeps rows ascending inside a column.
// ---------------------------------------------------------------------------
__global__ void k_dense_col_counts(const float* __restrict__ D, int rows, int cols,
                                   int* __restrict__ cntp, int* __restrict__ cntn) {
    // one thread per column; rows swept in order (coalesced across columns)
    for (int n = blockIdx.x * blockDim.x + threadIdx.x; n < cols; n += gridDim.x * blockDim.x) {
        int p = 0, q = 0;
        for (int i = 0; i < rows; ++i) {
            const float v = D[(size_t)i * cols + n];
            p += (v == 1.0f);
            q += (v == -1.0f);
        }
        cntp[n] = p;
        cntn[n] = q;
    }
}

__global__ void k_dense_fill(const float* __restrict__ D, int rows, int cols,
                             const int* __restrict__ csp, const int* __restrict__ csn,
                             int* __restrict__ rip, int* __restrict__ rin) {
    for (int n = blockIdx.x * blockDim.x + threadIdx.x; n < cols; n += gridDim.x * blockDim.x) {
        int p = csp[n], q = csn[n];
        for (int i = 0; i < rows; ++i) {
            const float v = D[(size_t)i * cols + n];
            if (v == 1.0f) rip[p++] = i;
            else if (v == -1.0f) rin[q++] = i;
        }
    }
}

// ---------------------------------------------------------------------------
// Host-side launchers (called from tcsc_api.cpp)
// ---------------------------------------------------------------------------

static inline int grid_for(long long n, int block) {
    long long g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > 65535LL * 16) g = 65535LL * 16;
    return (int)g;
}

hipError_t plan_build(const PlanDev& in, PlanOut& out, hipStream_t st) {
    const int ncols = in.ncols, nch = out.n_chunks, tk = out.chunk_k;
    const long long nb = (long long)(nch + 1) * ncols;
    hipError_t e;
    hipLaunchKernelGGL(k_chunk_bounds, dim3(grid_for(nb, 256)), dim3(256), 0, st, in.csp, in.csn,
                       in.rip, in.rin, in.col_begin, ncols, nch, tk, in.rows, out.lbp, out.lbn);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const long long nc = (long long)nch * ncols;
    hipLaunchKernelGGL(k_chunk_counts, dim3(grid_for(nc, 256)), dim3(256), 0, st, out.lbp, out.lbn,
                       ncols, nch, out.cnt);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // cptr[i] = exclusive sum of cnt; cnt has one trailing 0 so cptr[nc] = nnz
    size_t tmp_bytes = out.scan_tmp_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(out.scan_tmp, tmp_bytes, out.cnt, out.cptr, (int)(nc + 1), st);
    if (e != hipSuccess) return e;
    if (in.n_pos > 0) {
        hipLaunchKernelGGL(k_scatter<0>, dim3(grid_for(in.n_pos, 256)), dim3(256), 0, st, in.csp, in.rip,
                           in.csn, in.rin, out.lbp, out.lbn, out.cptr, in.col_begin, ncols, tk, out.ent);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (in.n_neg > 0) {
        hipLaunchKernelGGL(k_scatter<1>, dim3(grid_for(in.n_neg, 256)), dim3(256), 0, st, in.csn, in.rin,
                           in.csp, in.rip, out.lbn, out.lbp, out.cptr, in.col_begin, ncols, tk, out.ent);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t plan_scan_tmp_bytes(long long n, size_t* bytes) {
    *bytes = 0;
    return hipcub::DeviceScan::ExclusiveSum(nullptr, *bytes, (int*)nullptr, (int*)nullptr, (int)n,
                                            (hipStream_t)0);
}

template <int TK, int CW, int WAVES>
static hipError_t launch_gather_t(const GemmArgs& g, hipStream_t st) {
    dim3 grid((g.ncols + WAVES * CW - 1) / (WAVES * CW), (g.M + 127) / 128);
    dim3 block(WAVES * 64);
    const int vec4 = (g.K % 4 == 0) && ((reinterpret_cast<uintptr_t>(g.X) & 15) == 0);
    if (g.bias_first) {
        if (g.prelu)
            hipLaunchKernelGGL((k_tcsc_gather<TK, CW, WAVES, true, true>), grid, block, 0, st, g.X, g.M, g.K,
                               g.ent, g.cptr, g.ncols, g.B, g.Y, g.ldy, g.a, vec4);
        else
            hipLaunchKernelGGL((k_tcsc_gather<TK, CW, WAVES, true, false>), grid, block, 0, st, g.X, g.M, g.K,
                               g.ent, g.cptr, g.ncols, g.B, g.Y, g.ldy, g.a, vec4);
    } else {
        if (g.prelu)
            hipLaunchKernelGGL((k_tcsc_gather<TK, CW, WAVES, false, true>), grid, block, 0, st, g.X, g.M, g.K,
                               g.ent, g.cptr, g.ncols, g.B, g.Y, g.ldy, g.a, vec4);
        else
            hipLaunchKernelGGL((k_tcsc_gather<TK, CW, WAVES, false, false>), grid, block, 0, st, g.X, g.M, g.K,
                               g.ent, g.cptr, g.ncols, g.B, g.Y, g.ldy, g.a, vec4);
    }
    return hipGetLastError();
}

hipError_t launch_gemm(const GemmArgs& g, hipStream_t st) {
    if (g.M <= 0 || g.ncols <= 0) return hipSuccess;
    if (g.chunk_k != kChunkK) return hipErrorInvalidValue;
    return launch_gather_t<kChunkK, 16, 4>(g, st);
}

hipError_t dense_to_tcsc_counts(const float* D, int rows, int cols, int* cntp, int* cntn, hipStream_t st) {
    hipLaunchKernelGGL(k_dense_col_counts, dim3(grid_for(cols, 256)), dim3(256), 0, st, D, rows, cols, cntp,
                       cntn);
    return hipGetLastError();
}

hipError_t dense_to_tcsc_fill(const float* D, int rows, int cols, const int* csp, const int* csn, int* rip,
                              int* rin, hipStream_t st) {
    hipLaunchKernelGGL(k_dense_fill, dim3(grid_for(cols, 256)), dim3(256), 0, st, D, rows, cols, csp, csn, rip,
                       rin);
    return hipGetLastError();
}

hipError_t exclusive_scan_i32(const int* in, int* out, int n, void* tmp, size_t tmp_bytes, hipStream_t st) {
    return hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, in, out, n, st);
}

}  // namespace tcsc
