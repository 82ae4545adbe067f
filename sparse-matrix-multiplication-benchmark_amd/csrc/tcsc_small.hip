// tcsc_small.hip -- the small-M path ("Small M").
//
// k_stream stages 256 rows of X per workgroup; with M = 1 (the reference
// harness's first cases, main.cpp:258-261) the staging, the barriers and the
// 256-row epilogue are all overhead: ~37 us for 1 x 512 x 2048.  For M <= 4
// one LANE per output column walks the column's merged row list (the plan's
// CSC copy, +1 and -1 rows in ascending k) and adds +-X[m, k] in that order,
// then the bias, then the PReLU: the exact arithmetic of k_stream's fast
// order, so the outputs are bit-identical to the gather path's (K not split)
// and to the reference's dense.c gemm_basic (dense.c:64-77: y = 0, y += X*W
// over ascending k, + B; a ternary W makes every product exact).
// (Rounds 2-4 summed 64 lanes' strided partial sums and reduced them by a
// butterfly: within the bound, not in the gather's order; the reference's
// main.cpp checks tcsc_sgemm_basic against dense.c's gemm_basic with an
// absolute 1e-4, which its M = 1, K = 2048 case missed by 2e-5.)
#include <hip/hip_runtime.h>

#include "tcsc_internal.h"

namespace tcsc {
namespace {

constexpr int kBlock = kCscGroup;  // columns (lanes) per workgroup: one wave, one group of the list layout

// Look-ahead of the entry ring, in quads: one wave per CU here, so a lane can
// hold 48 quads (192 VGPRs) at M = 1, enough to cover the loads' latency.
template <int MB>
constexpr int ring_quads() {
    return MB == 1 ? 48 : (MB == 2 ? 32 : 8);
}

// One lane per column; the column's sum is one dependent chain of adds in
// the merged list's order, so everything else runs off that chain:
//  * the workgroup stages each row of X in LDS as the pair [X | -0.0 | 0.. |
//    -X | 0..] (2*Kp floats, tcsc_internal.h): an entry of the list (4k, or
//    4Kp + 4k for a -1 row, or 4K for padding) is then directly the byte
//    offset of +-X[m, k], so an add is one ds_read and one v_add (negation is
//    exact: acc + (-x) is the gather's fma(x, -1, acc)); the staging keeps 16
//    16-B loads per lane in flight, addresses clamped instead of branched
//    around (a load under a runtime condition makes hipcc branch around it
//    and drain vmcnt per load);
//  * the list (the 64 columns of this workgroup interleaved by 16-B quads,
//    padded to the group's length, a multiple of 16 quads) is read one quad
//    per lane and load -- a coalesced 1 KiB for the wave -- ring_quads()
//    quads ahead of the adds, and the values 3 quads ahead; the ring is
//    unrolled in phases of 16 quads so every slot is a static register set,
//    and the sum never runs past the group;
//  * the look-ahead loads are pinned ahead of the adds (hipcc would sink
//    them to their first use).
template <int MB, bool BIAS_FIRST, bool PRELU>
__global__ void __launch_bounds__(kBlock)
k_small_m(const float* __restrict__ X, int M, int K, const int* __restrict__ cq, const int* __restrict__ rm,
          int ncols, const float* __restrict__ Bias, float* __restrict__ Y, int ldy, float a) {
    extern __shared__ float xs[];
    const int lane = threadIdx.x;
    const int Kp = csc_half(K), S = 2 * Kp;  // floats per half / per staged row pair
    // 16-B loads, 16 per lane in flight (16 KiB per wave per round trip), where
    // X's rows are 16-B aligned; 4-B loads otherwise
    const bool vec = (K & 3) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
    for (int r = 0; r < M; ++r) {
        const float* __restrict__ xr = X + (size_t)r * K;
        float* dr = xs + (size_t)r * S;
        if (vec) {
            for (int k0 = 0; k0 < K; k0 += 16 * 4 * kBlock) {
                float4 v[16];
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    v[u] = *reinterpret_cast<const float4*>(xr + min(k0 + 4 * (u * kBlock + lane), K - 4));
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const int k = k0 + 4 * (u * kBlock + lane);
                    if (k < K) {
                        *reinterpret_cast<float4*>(dr + k) = v[u];
                        *reinterpret_cast<float4*>(dr + Kp + k) = make_float4(-v[u].x, -v[u].y, -v[u].z, -v[u].w);
                    }
                }
            }
        } else {
            for (int k0 = 0; k0 < K; k0 += 8 * kBlock) {
                float v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = xr[min(k0 + u * kBlock + lane, K - 1)];
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (k0 + u * kBlock + lane < K) {
                        dr[k0 + u * kBlock + lane] = v[u];
                        dr[Kp + k0 + u * kBlock + lane] = -v[u];
                    }
            }
        }
        if (lane == 0) dr[K] = -0.0f;  // what padding entries read: the exact additive identity
    }
    __syncthreads();
    const int j = blockIdx.x * kBlock + lane;
    const bool col_ok = j < ncols;
    const float b = Bias[col_ok ? j : ncols - 1];
    float acc[MB];
#pragma unroll
    for (int r = 0; r < MB; ++r) acc[r] = BIAS_FIRST ? b : 0.0f;
    const int q0 = cq[blockIdx.x], nq = cq[blockIdx.x + 1] - q0;  // uniform; a multiple of 16
    const int4* __restrict__ lst = reinterpret_cast<const int4*>(rm) + (size_t)q0 * kBlock + lane;
    const char* xb = reinterpret_cast<const char*>(xs);  // row pair r at byte r * S * 4
    // +-X[r, k] for an entry (rows >= M read row M-1's, unused)
    auto xval = [&](int e, int r) {
        const int rr = r < M ? r : M - 1;
        return *reinterpret_cast<const float*>(xb + e + rr * S * 4);
    };
    // entries kIR quads ahead (index ring, refilled by coalesced loads), values
    // kXD quads ahead (value ring, LDS reads); phases of kPh quads
    constexpr int kIR = ring_quads<MB>(), kPh = kIR < 16 ? kIR : 16, kXR = 4, kXD = 3;
    static_assert(kIR % kPh == 0 && 16 % kPh == 0 && kPh % kXR == 0 && kXD < kXR && kIR <= kCscGuardQuads,
                  "look-ahead geometry");
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
    for (int qb = 0; qb < nq; qb += kIR) {
#pragma unroll
        for (int ph = 0; ph < kIR / kPh; ++ph) {
            if (ph > 0 && qb + ph * kPh >= nq) break;  // uniform: the group ends on a 16-quad boundary
#pragma unroll
            for (int s = 0; s < kPh; ++s) {
                const int t = ph * kPh + s;  // compile-time after unrolling
                // values of quad q + kXD (its entries arrived kIR - kXD steps ago)
                load_x(ring[(t + kXD) % kIR], xv[(t + kXD) % kXR]);
                ring[t] = lst[(size_t)(qb + t + kIR) * kBlock];  // quad q + kIR into the slot quad q left
                asm volatile("" ::: "memory");  // the look-ahead loads stay ahead of the adds
                // padding adds -0.0, which changes nothing
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int r = 0; r < MB; ++r) acc[r] = acc[r] + xv[t % kXR][i][r];
            }
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
    hipLaunchKernelGGL((k_small_m<MB, BF, PR>), grid, block, small_m_lds_bytes(M, K), st, X, M, K, cq, rm, ncols, B,
                       Y, ldy, a);
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
