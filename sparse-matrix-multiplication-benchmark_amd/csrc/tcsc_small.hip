// tcsc_small.hip -- the small-M path ("Small M").
//
// k_stream stages 256 rows of X per workgroup; with M = 1 (the reference
// harness's first cases, main.cpp:258-261) the staging, the barriers and the
// 256-row epilogue are all overhead: ~37 us for 1 x 512 x 2048.  For M <= 16
// one wave per output column walks the column's +1 and -1 rows (the plan's
// CSC copy) instead, 64 entries at a time, gathering X[m, k] straight from
// L2 (X is at most 16 x K floats here), then reduces across the wave.  Per
// lane the +1 rows are added, then the -1 rows subtracted, in ascending k;
// lane 0's butterfly result is stored, so the order is fixed (deterministic)
// but not the gather's merged order: the result is held to the same fp32
// bound, and is exact on integer-valued inputs.
#include <hip/hip_runtime.h>

#include "tcsc_internal.h"

namespace tcsc {
namespace {

constexpr int kColsPerBlock = 4;  // one wave per column

template <int MB, bool BIAS_FIRST, bool PRELU>
__global__ void __launch_bounds__(64 * kColsPerBlock)
k_small_m(const float* __restrict__ X, int M, int K, const int* __restrict__ cp, const int* __restrict__ cn,
          const int* __restrict__ rp, const int* __restrict__ rn, int ncols, const float* __restrict__ Bias,
          float* __restrict__ Y, int ldy, float a) {
    const int lane = threadIdx.x & 63;
    const int j = blockIdx.x * kColsPerBlock + (threadIdx.x >> 6);
    if (j >= ncols) return;  // the whole wave
    float acc[MB];
#pragma unroll
    for (int r = 0; r < MB; ++r) acc[r] = 0.0f;
    const int p1 = cp[j + 1], q1 = cn[j + 1];
    for (int e = cp[j] + lane; e < p1; e += 64) {
        const float* x = X + rp[e];
#pragma unroll
        for (int r = 0; r < MB; ++r)
            if (r < M) acc[r] += x[(size_t)r * K];
    }
    for (int e = cn[j] + lane; e < q1; e += 64) {
        const float* x = X + rn[e];
#pragma unroll
        for (int r = 0; r < MB; ++r)
            if (r < M) acc[r] -= x[(size_t)r * K];
    }
#pragma unroll
    for (int r = 0; r < MB; ++r)
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) acc[r] += __shfl_xor(acc[r], off);
    if (lane == 0) {
        const float b = Bias[j];
#pragma unroll
        for (int r = 0; r < MB; ++r) {
            if (r >= M) break;
            float v = BIAS_FIRST ? b + acc[r] : acc[r] + b;
            if (PRELU) v = (v < 0.0f) ? a * v : v;
            Y[(size_t)r * ldy + j] = v;
        }
    }
}

template <int MB>
void launch_mb(const float* X, int M, int K, const int* cp, const int* cn, const int* crp, const int* crn, int ncols,
               const float* B, float* Y, int ldy, bool bias_first, bool prelu, float a, hipStream_t st) {
    const dim3 grid((ncols + kColsPerBlock - 1) / kColsPerBlock), block(64 * kColsPerBlock);
    if (bias_first) {
        if (prelu)
            hipLaunchKernelGGL((k_small_m<MB, true, true>), grid, block, 0, st, X, M, K, cp, cn, crp, crn, ncols, B,
                               Y, ldy, a);
        else
            hipLaunchKernelGGL((k_small_m<MB, true, false>), grid, block, 0, st, X, M, K, cp, cn, crp, crn, ncols, B,
                               Y, ldy, a);
    } else {
        if (prelu)
            hipLaunchKernelGGL((k_small_m<MB, false, true>), grid, block, 0, st, X, M, K, cp, cn, crp, crn, ncols, B,
                               Y, ldy, a);
        else
            hipLaunchKernelGGL((k_small_m<MB, false, false>), grid, block, 0, st, X, M, K, cp, cn, crp, crn, ncols, B,
                               Y, ldy, a);
    }
}

}  // namespace

hipError_t launch_small_m(const float* X, int M, int K, const int* cp, const int* cn, const int* crp, const int* crn,
                          int ncols, const float* B, float* Y, int ldy, bool bias_first, bool prelu, float a,
                          hipStream_t st) {
    if (M <= 0 || ncols <= 0) return hipSuccess;
    if (M == 1)
        launch_mb<1>(X, M, K, cp, cn, crp, crn, ncols, B, Y, ldy, bias_first, prelu, a, st);
    else if (M <= 2)
        launch_mb<2>(X, M, K, cp, cn, crp, crn, ncols, B, Y, ldy, bias_first, prelu, a, st);
    else if (M <= 4)
        launch_mb<4>(X, M, K, cp, cn, crp, crn, ncols, B, Y, ldy, bias_first, prelu, a, st);
    else if (M <= 8)
        launch_mb<8>(X, M, K, cp, cn, crp, crn, ncols, B, Y, ldy, bias_first, prelu, a, st);
    else if (M <= 16)
        launch_mb<16>(X, M, K, cp, cn, crp, crn, ncols, B, Y, ldy, bias_first, prelu, a, st);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace tcsc
