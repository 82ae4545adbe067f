// bcsr_kernels.hip -- k_bcsr, the gfx950 (MI355X / CDNA4) kernel behind the
// BCSR operator API (include/sparse/bcsr.h), replacing the CPU loops of
// /root/reference/sparse/bcsr.c:
//   bcsr_sgemm_basic        bcsr.c:141-175
//   bcsr_sgemm_prelu_basic  bcsr.c:177-218
//   bcsr_sgemm_avx          bcsr.c:222-261
//   bcsr_sgemm_prelu_avx    bcsr.c:264-312
//   bcsr_sgemm_avx2         bcsr.c:316-385
//
// The reference walks Y row by row and scatters every stored block into Y's
// columns (CSR over block rows).  Here every output element belongs to one
// lane for the whole launch, so the plan (bcsr_api.cpp) re-indexes W by block
// column: per block column, its stored blocks in the order the reference
// visits them (block row ascending, then block index, bcsr.c:156-160).  That
// is exactly the accumulation order of every element of the column, so the
// kernel replays the reference's arithmetic element by element -- bias first
// (bcsr.c:146-150), one rounded update per (block, block row i), PReLU after
// every update for the prelu variants (bcsr.c:208-209, 302-304) -- and the
// outputs are bit-identical for any float input, not only within a tolerance.
//
// Geometry: a wave owns 256 rows (4 per lane: one float4 of X^T per block
// row, coalesced 1 KiB per wave) and one strip of up to 8 output columns of
// one block column (32 accumulators per lane); the 4 waves of a workgroup
// take 4 consecutive strips, i.e. 32 adjacent output columns.  A block row's
// strip of values is wave-uniform and comes through the scalar cache.  Block
// rows go kBatch at a time, the next batch's X and values in flight during
// the current batch's updates.
// X^T rows are read from L2 (the row tile of a workgroup is shared by the
// workgroups an XCD runs at once: XCD-aware tile order).  Roofline: VALU,
// one v_fma (or v_mul + v_add, + 3 for PReLU) per stored value, row and
// column -- zeros inside a stored block included (DESIGN.md "BCSR").
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tcsc_internal.h"

namespace tcsc {
namespace {

constexpr int kBcsrRows = 256;  // rows per wave (and workgroup): 64 lanes x 4
constexpr int kBcsrWaves = 4;   // strips per workgroup
constexpr int kStrip = 8;       // output columns per strip (= the reference's 8-wide AVX rows)
constexpr int kBatch = 4;       // block rows per pipeline step

// XCD-aware tile order (speed only): launch index L runs on XCD L % 8;
// renumber so every XCD takes a contiguous range of (strip group fastest,
// row tile).  Bijective for any grid size.
__device__ __forceinline__ void bcsr_tile(int& sg, int& rt) {
    const int nsg = gridDim.x;
    const int T = nsg * gridDim.y;
    const int L = blockIdx.x + nsg * blockIdx.y;
    const int q = T >> 3, r = T & 7, x = L & 7;
    const int Lg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (L >> 3);
    sg = Lg % nsg;
    rt = Lg / nsg;
}

// One update of the reference's inner loop.  basic / prelu_basic:
// `Y[...] += X[...] * val` (bcsr.c:169, 208) -- a rounded product, then a
// rounded sum: contraction must stay off.  avx variants: _mm256_fmadd_ps
// (bcsr.c:254, 300, 370-377), one rounding.
template <bool FMA>
__device__ __forceinline__ float bcsr_update(float y, float x, float w) {
#pragma clang fp contract(off)
    if constexpr (FMA) {
        return __builtin_fmaf(x, w, y);
    } else {
        return y + x * w;
    }
}

// (v > 0) ? v : a*v after every update (bcsr.c:209; the avx form's
// _CMP_GT_OS mask + blend, bcsr.c:302-304, is the same predicate: NaN takes
// the a*v branch).  PR = 1: that select.  PR = 2, only for 0 < a <= 1:
// max(v, a*v), the same value for every v (v > 0: a*v <= v; v < 0 and
// -inf: a*v >= v; +-0: a*v = v; NaN: NaN) in two packed VALU ops per row
// pair instead of a multiply, a compare and a select per row.
template <int PR>
__device__ __forceinline__ float bcsr_act(float v, float a) {
    if constexpr (PR == 1) {
        return (v > 0.0f) ? v : a * v;
    } else if constexpr (PR == 2) {
        return __builtin_fmaxf(v, a * v);
    } else {
        return v;
    }
}

template <bool FMA, int PRELU, bool FULL>
__global__ void __launch_bounds__(kBcsrWaves * 64)
k_bcsr(const float* __restrict__ XT, int ldxt, int M, const int* __restrict__ colptr, const int2* __restrict__ ent,
       const float* __restrict__ vals, int c, int nbc, int spb, int nstrips, int N,
       const float* __restrict__ Bias, float* __restrict__ Y, int ldy, float a, int vec_store) {
    int sg, rt;
    bcsr_tile(sg, rt);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int s = sg * kBcsrWaves + wave;
    if (s >= nstrips) return;  // wave-uniform; no barrier below
    // strip s -> output columns [col0, col0 + cj) and the block list of its
    // block column; strips past the block columns cover the columns
    // [nbc*c, N) that no block touches (bias only, bcsr.c:146-150)
    const int body = nbc * spb;
    int col0, cj, e = 0, e1 = 0, j0 = 0;
    if (s < body) {
        const int bcx = s / spb;
        j0 = (s - bcx * spb) * kStrip;
        col0 = bcx * c + j0;
        cj = min(kStrip, c - j0);
        e = colptr[bcx];
        e1 = colptr[bcx + 1];
    } else {
        col0 = nbc * c + (s - body) * kStrip;
        cj = min(kStrip, N - col0);
    }
    const int m = rt * kBcsrRows + 4 * lane;

    float acc[kStrip][4];
#pragma unroll
    for (int j = 0; j < kStrip; ++j) {
        const float b = j < cj ? Bias[col0 + j] : 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[j][q] = b;
    }

    // the block column's row stream (one entry per (block, block row i):
    // X^T row and value offset), kBatch rows per step, the next batch's X^T
    // quads and values loaded before the current batch's updates
    const float* xt = XT + m;
    const int nfull = (e1 - e) / kBatch;
    float4 xa[kBatch];
    float wa[kBatch][kStrip];
    auto load_batch = [&](int t) {
#pragma unroll
        for (int u = 0; u < kBatch; ++u) {
            const int2 en = ent[t + u];
            xa[u] = *reinterpret_cast<const float4*>(xt + (size_t)en.x * ldxt);
#pragma unroll
            for (int j = 0; j < kStrip; ++j) wa[u][j] = (FULL || j < cj) ? vals[en.y + j0 + j] : 0.f;
        }
    };
    auto update_row = [&](const float4& x, const float (&w)[kStrip]) {
#pragma unroll
        for (int j = 0; j < kStrip; ++j) {
            if (FULL || j < cj) {
                acc[j][0] = bcsr_act<PRELU>(bcsr_update<FMA>(acc[j][0], x.x, w[j]), a);
                acc[j][1] = bcsr_act<PRELU>(bcsr_update<FMA>(acc[j][1], x.y, w[j]), a);
                acc[j][2] = bcsr_act<PRELU>(bcsr_update<FMA>(acc[j][2], x.z, w[j]), a);
                acc[j][3] = bcsr_act<PRELU>(bcsr_update<FMA>(acc[j][3], x.w, w[j]), a);
            }
        }
    };
    if (nfull > 0) load_batch(e);
    for (int b = 0; b < nfull; ++b) {
        float4 xc[kBatch];
        float wc[kBatch][kStrip];
#pragma unroll
        for (int u = 0; u < kBatch; ++u) {
            xc[u] = xa[u];
#pragma unroll
            for (int j = 0; j < kStrip; ++j) wc[u][j] = wa[u][j];
        }
        e += kBatch;
        if (b + 1 < nfull) load_batch(e);
#pragma unroll
        for (int u = 0; u < kBatch; ++u) update_row(xc[u], wc[u]);
    }
    for (; e < e1; ++e) {  // the last (e1 - e0) % kBatch rows
        const int2 en = ent[e];
        const float4 x = *reinterpret_cast<const float4*>(xt + (size_t)en.x * ldxt);
        float w[kStrip];
#pragma unroll
        for (int j = 0; j < kStrip; ++j) w[j] = (FULL || j < cj) ? vals[en.y + j0 + j] : 0.f;
        update_row(x, w);
    }

    // 32 contiguous bytes per row and lane; the workgroup's 4 strips fill
    // 128 contiguous bytes of each row
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int row = m + q;
        if (row >= M) break;
        float* yr = Y + (size_t)row * ldy + col0;
        if (vec_store && cj == kStrip) {
            *reinterpret_cast<float4*>(yr) = make_float4(acc[0][q], acc[1][q], acc[2][q], acc[3][q]);
            *reinterpret_cast<float4*>(yr + 4) = make_float4(acc[4][q], acc[5][q], acc[6][q], acc[7][q]);
        } else {
#pragma unroll
            for (int j = 0; j < kStrip; ++j)
                if (j < cj) yr[j] = acc[j][q];
        }
    }
}

template <bool FMA, int PRELU, bool FULL>
hipError_t launch_v(const BcsrArgs& g, int spb, int nstrips, int vec, hipStream_t st) {
    const dim3 grid((nstrips + kBcsrWaves - 1) / kBcsrWaves, (g.M + kBcsrRows - 1) / kBcsrRows);
    hipLaunchKernelGGL((k_bcsr<FMA, PRELU, FULL>), grid, dim3(kBcsrWaves * 64), 0, st, g.XT, g.ldxt, g.M, g.colptr,
                       g.ent, g.vals, g.c, g.nbc, spb, nstrips, g.N, g.B, g.Y, g.ldy, g.a, vec);
    return hipGetLastError();
}

template <bool FMA, int PRELU>
hipError_t launch_f(const BcsrArgs& g, int spb, int nstrips, int vec, hipStream_t st) {
    if (g.c % kStrip == 0) return launch_v<FMA, PRELU, true>(g, spb, nstrips, vec, st);
    return launch_v<FMA, PRELU, false>(g, spb, nstrips, vec, st);
}

}  // namespace

// g.XT must hold K x ldxt floats with ldxt >= ldxt_for(g.M) (the API layer's
// workspace); g.N >= g.nbc * g.c.
hipError_t launch_bcsr(const BcsrArgs& g, hipStream_t st) {
    if (g.M <= 0 || g.N <= 0) return hipSuccess;
    const int spb = (g.c + kStrip - 1) / kStrip;
    const long long tail = ((long long)g.N - (long long)g.nbc * g.c + kStrip - 1) / kStrip;
    const long long nstrips = (long long)g.nbc * spb + tail;
    if (nstrips <= 0) return hipSuccess;
    if (nstrips > 0x7fffffffLL || (g.M + kBcsrRows - 1) / kBcsrRows > 65535) return hipErrorInvalidValue;
    const int vec = (g.c % 4 == 0) && (g.ldy % 4 == 0) && ((reinterpret_cast<uintptr_t>(g.Y) & 15) == 0);
    const int ns = (int)nstrips;
    const int pr = !g.prelu ? 0 : (g.a > 0.f && g.a <= 1.f) ? 2 : 1;
    if (g.fma) {
        if (pr == 2) return launch_f<true, 2>(g, spb, ns, vec, st);
        return pr ? launch_f<true, 1>(g, spb, ns, vec, st) : launch_f<true, 0>(g, spb, ns, vec, st);
    }
    if (pr == 2) return launch_f<false, 2>(g, spb, ns, vec, st);
    return pr ? launch_f<false, 1>(g, spb, ns, vec, st) : launch_f<false, 0>(g, spb, ns, vec, st);
}

}  // namespace tcsc
