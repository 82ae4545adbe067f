// tcsc_small.hip -- the small-M path ("Small M").
//
// k_stream stages 256 rows of X per workgroup; with M = 1 (the reference
// harness's first cases, main.cpp:258-261) the staging, the barriers and the
// 256-row epilogue are all overhead: ~37 us for 1 x 512 x 2048.  For M <= 16
// one LANE per output column walks the column's merged row list (the plan's
// CSC copy, +1 and -1 rows in ascending k, -1 rows tagged in bit 31) and adds
// +-X[m, k] in that order, straight from L1/L2 (X is at most 16 x K floats
// here), then the bias, then the PReLU: the exact arithmetic of k_stream's
// fast order, so the outputs are bit-identical to the gather path's (K not
// split) and to the reference's dense.c gemm_basic (dense.c:64-77: y = 0,
// y += X*W over ascending k, + B; a ternary W makes every product exact).
// (Rounds 2-4 summed 64 lanes' strided partial sums and reduced them by a
// butterfly: within the bound, not in the gather's order; the reference's
// main.cpp checks tcsc_sgemm_basic against dense.c's gemm_basic with an
// absolute 1e-4, which its M = 1, K = 2048 case missed by 2e-5.)
#include <hip/hip_runtime.h>

#include "tcsc_internal.h"

namespace tcsc {
namespace {

constexpr int kBlock = kCscGroup;  // columns (lanes) per workgroup: one wave, one group of the list layout

// One lane per column; the column's sum is one dependent chain of adds in
// the merged list's order, so everything else runs off that chain:
//  * the workgroup stages X in LDS as rows of K+1 floats, the last one -0.0
//    (the exact additive identity): 8 loads per lane in flight, addresses
//    clamped instead of branched around (a load under a runtime condition
//    makes hipcc branch around it and drain vmcnt per load);
//  * the list (csc_prepare/csc_fill: entries 4*k with the -1 sign in bit 31,
//    the 64 columns of this workgroup interleaved by 16-B quads, padded to
//    the group's length with 4*K entries) is read one quad per lane and load
//    -- a coalesced 1 KiB for the wave -- 16 quads ahead of the adds, and
//    the values 3 quads ahead, for the group's whole length (a wave-uniform
//    trip count, a multiple of 16 quads);
//  * an entry is directly the byte offset of its value in an LDS row
//    (padding reads the -0.0), so an add is ds_read -> sign xor -> v_add;
//  * the look-ahead loads are pinned ahead of the adds (hipcc would sink
//    them to their first use).
template <int MB, bool BIAS_FIRST, bool PRELU>
__global__ void __launch_bounds__(kBlock)
k_small_m(const float* __restrict__ X, int M, int K, const int* __restrict__ cq, const int* __restrict__ rm,
          int ncols, const float* __restrict__ Bias, float* __restrict__ Y, int ldy, float a) {
    extern __shared__ float xs[];
    const int lane = threadIdx.x;
    for (int r = 0; r < M; ++r) {
        const float* __restrict__ xr = X + (size_t)r * K;
        float* dr = xs + r * (K + 1);
        for (int k0 = 0; k0 < K; k0 += 8 * kBlock) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = xr[min(k0 + u * kBlock + lane, K - 1)];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (k0 + u * kBlock + lane < K) dr[k0 + u * kBlock + lane] = v[u];
        }
        if (lane == 0) dr[K] = -0.0f;
    }
    __syncthreads();
    const int j = blockIdx.x * kBlock + lane;
    const bool col_ok = j < ncols;
    const float b = Bias[col_ok ? j : ncols - 1];
    float acc[MB];
#pragma unroll
    for (int r = 0; r < MB; ++r) acc[r] = BIAS_FIRST ? b : 0.0f;
    const int q0 = cq[blockIdx.x], nq = cq[blockIdx.x + 1] - q0;  // uniform; a multiple of 4
    const int4* __restrict__ lst = reinterpret_cast<const int4*>(rm) + (size_t)q0 * kBlock + lane;
    // one (entry, row) value with the entry's sign applied (rows >= M read row M-1's, unused)
    auto xval = [&](int e, int r) {
        const int rr = r < M ? r : M - 1;
        const float v = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(xs) + (e & kCscRowMask) +
                                                         rr * (K + 1) * 4);
        return __builtin_bit_cast(float, __builtin_bit_cast(unsigned, v) ^ ((unsigned)e & 0x80000000u));
    };
    // Look-ahead: entries kIR quads ahead (index ring, refilled by coalesced
    // loads), values kXD quads ahead (value ring, LDS reads); the body is
    // unrolled by kIR so every slot is a static register set.  Group lengths
    // are multiples of kIR quads; the guard quads past the last group are 0.
    constexpr int kIR = MB <= 2 ? 16 : 8, kXR = 4, kXD = 3;  // MB = 4: 8 quads keep it under 256 VGPRs
    static_assert(kIR % kXR == 0 && 16 % kIR == 0 && kXD < kXR && kIR <= kCscGuardQuads, "look-ahead geometry");
    int4 ring[kIR];
#pragma unroll
    for (int i = 0; i < kIR; ++i) ring[i] = lst[(size_t)i * kBlock];
    float xv[kXR][4][MB];
    auto load_x = [&](const int4& qv, float (&x)[4][MB]) {
#pragma unroll
        for (int r = 0; r < MB; ++r) {
            x[0][r] = xval(qv.x, r);
            x[1][r] = xval(qv.y, r);
            x[2][r] = xval(qv.z, r);
            x[3][r] = xval(qv.w, r);
        }
    };
#pragma unroll
    for (int i = 0; i < kXD; ++i) load_x(ring[i], xv[i]);
    for (int q0 = 0; q0 < nq; q0 += kIR) {
#pragma unroll
        for (int s = 0; s < kIR; ++s) {
            // values of quad q + kXD (its entries arrived kIR - kXD steps ago)
            load_x(ring[(s + kXD) % kIR], xv[(s + kXD) % kXR]);
            ring[s] = lst[(size_t)(q0 + s + kIR) * kBlock];  // quad q + kIR into the slot quad q left
            asm volatile("" ::: "memory");  // the look-ahead loads stay ahead of the adds
            // acc + x with x = +-X[m, k] (sign applied exactly) is fma(X, +-1, acc):
            // the gather's arithmetic; padding adds -0.0, which changes nothing
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int r = 0; r < MB; ++r) acc[r] = acc[r] + xv[s % kXR][i][r];
        }
    }
    if (!col_ok) return;
#pragma unroll
    for (int r = 0; r < MB; ++r) {
        if (r >= M) break;
        float v = BIAS_FIRST ? acc[r] : acc[r] + b;
        if (PRELU) v = (v < 0.0f) ? a * v : v;
        Y[(size_t)r * ldy + j] = v;
    }
}

template <int MB, bool BF, bool PR>
void launch_one(const float* X, int M, int K, const int* cq, const int* rm, int ncols, const float* B, float* Y,
                int ldy, float a, hipStream_t st) {
    static const bool attr = [] {  // LDS beyond the 64 KiB default for dynamic shared memory
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_small_m<MB, BF, PR>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)small_m_lds_bytes_max());
        return true;
    }();
    (void)attr;
    const dim3 grid((ncols + kBlock - 1) / kBlock), block(kBlock);
    hipLaunchKernelGGL((k_small_m<MB, BF, PR>), grid, block, (size_t)M * (K + 1) * sizeof(float), st, X, M, K, cq,
                       rm, ncols, B, Y, ldy, a);
}

template <int MB>
void launch_mb(const float* X, int M, int K, const int* cq, const int* rm, int ncols, const float* B, float* Y,
               int ldy, bool bias_first, bool prelu, float a, hipStream_t st) {
    if (bias_first) {
        if (prelu)
            launch_one<MB, true, true>(X, M, K, cq, rm, ncols, B, Y, ldy, a, st);
        else
            launch_one<MB, true, false>(X, M, K, cq, rm, ncols, B, Y, ldy, a, st);
    } else {
        if (prelu)
            launch_one<MB, false, true>(X, M, K, cq, rm, ncols, B, Y, ldy, a, st);
        else
            launch_one<MB, false, false>(X, M, K, cq, rm, ncols, B, Y, ldy, a, st);
    }
}

}  // namespace

hipError_t launch_small_m(const float* X, int M, int K, const int* cq, const int* crq, int ncols, const float* B,
                          float* Y, int ldy, bool bias_first, bool prelu, float a, hipStream_t st) {
    if (M <= 0 || ncols <= 0) return hipSuccess;
    if (!small_m_fits(M, K)) return hipErrorInvalidValue;
    if (M == 1)
        launch_mb<1>(X, M, K, cq, crq, ncols, B, Y, ldy, bias_first, prelu, a, st);
    else if (M <= 2)
        launch_mb<2>(X, M, K, cq, crq, ncols, B, Y, ldy, bias_first, prelu, a, st);
    else if (M <= 4)
        launch_mb<4>(X, M, K, cq, crq, ncols, B, Y, ldy, bias_first, prelu, a, st);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace tcsc
