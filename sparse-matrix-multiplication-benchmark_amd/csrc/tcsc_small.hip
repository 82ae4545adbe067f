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

constexpr int kBlock = 64;  // columns (lanes) per workgroup: one wave, spread over the CUs

// Entries of a column are read kBlk at a time (independent loads, the next
// block's issued before the current block's adds); the X values of a block
// are loaded before its adds, so only the adds are serial.
template <int MB, bool BIAS_FIRST, bool PRELU>
__global__ void __launch_bounds__(kBlock)
k_small_m(const float* __restrict__ X, int M, int K, const int* __restrict__ cp, const int* __restrict__ cn,
          const int* __restrict__ rm, int ncols, const float* __restrict__ Bias, float* __restrict__ Y, int ldy,
          float a) {
    constexpr int kBlk = MB <= 2 ? 16 : MB <= 4 ? 8 : 4;
    const int j = blockIdx.x * kBlock + threadIdx.x;
    if (j >= ncols) return;
    const float b = Bias[j];
    float acc[MB];
#pragma unroll
    for (int r = 0; r < MB; ++r) acc[r] = BIAS_FIRST ? b : 0.0f;
    int e = cp[j] + cn[j];
    const int e1 = cp[j + 1] + cn[j + 1];
    int nxt[kBlk];
#pragma unroll
    for (int i = 0; i < kBlk; ++i) nxt[i] = e + i < e1 ? rm[e + i] : 0;
    for (; e < e1; e += kBlk) {
        int cur[kBlk];
#pragma unroll
        for (int i = 0; i < kBlk; ++i) cur[i] = nxt[i];
#pragma unroll
        for (int i = 0; i < kBlk; ++i) nxt[i] = e + kBlk + i < e1 ? rm[e + kBlk + i] : 0;
        float x[kBlk][MB];
#pragma unroll
        for (int i = 0; i < kBlk; ++i) {
            const float* xp = X + (cur[i] & 0x7fffffff);
#pragma unroll
            for (int r = 0; r < MB; ++r) x[i][r] = (r < M && e + i < e1) ? xp[(size_t)r * K] : 0.0f;
        }
#pragma unroll
        for (int i = 0; i < kBlk; ++i) {
            if (e + i >= e1) break;
            const float sg = cur[i] < 0 ? -1.0f : 1.0f;
#pragma unroll
            for (int r = 0; r < MB; ++r) acc[r] = fmaf(x[i][r], sg, acc[r]);
        }
    }
#pragma unroll
    for (int r = 0; r < MB; ++r) {
        if (r >= M) break;
        float v = BIAS_FIRST ? acc[r] : acc[r] + b;
        if (PRELU) v = (v < 0.0f) ? a * v : v;
        Y[(size_t)r * ldy + j] = v;
    }
}

template <int MB>
void launch_mb(const float* X, int M, int K, const int* cp, const int* cn, const int* rm, int ncols, const float* B,
               float* Y, int ldy, bool bias_first, bool prelu, float a, hipStream_t st) {
    const dim3 grid((ncols + kBlock - 1) / kBlock), block(kBlock);
    if (bias_first) {
        if (prelu)
            hipLaunchKernelGGL((k_small_m<MB, true, true>), grid, block, 0, st, X, M, K, cp, cn, rm, ncols, B, Y, ldy,
                               a);
        else
            hipLaunchKernelGGL((k_small_m<MB, true, false>), grid, block, 0, st, X, M, K, cp, cn, rm, ncols, B, Y,
                               ldy, a);
    } else {
        if (prelu)
            hipLaunchKernelGGL((k_small_m<MB, false, true>), grid, block, 0, st, X, M, K, cp, cn, rm, ncols, B, Y,
                               ldy, a);
        else
            hipLaunchKernelGGL((k_small_m<MB, false, false>), grid, block, 0, st, X, M, K, cp, cn, rm, ncols, B, Y,
                               ldy, a);
    }
}

}  // namespace

hipError_t launch_small_m(const float* X, int M, int K, const int* cp, const int* cn, const int* crm, int ncols,
                          const float* B, float* Y, int ldy, bool bias_first, bool prelu, float a, hipStream_t st) {
    if (M <= 0 || ncols <= 0) return hipSuccess;
    if (M == 1)
        launch_mb<1>(X, M, K, cp, cn, crm, ncols, B, Y, ldy, bias_first, prelu, a, st);
    else if (M <= 2)
        launch_mb<2>(X, M, K, cp, cn, crm, ncols, B, Y, ldy, bias_first, prelu, a, st);
    else if (M <= 4)
        launch_mb<4>(X, M, K, cp, cn, crm, ncols, B, Y, ldy, bias_first, prelu, a, st);
    else if (M <= 8)
        launch_mb<8>(X, M, K, cp, cn, crm, ncols, B, Y, ldy, bias_first, prelu, a, st);
    else if (M <= 16)
        launch_mb<16>(X, M, K, cp, cn, crm, ncols, B, Y, ldy, bias_first, prelu, a, st);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace tcsc
