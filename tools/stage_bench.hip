// stage_bench.hip -- how fast can one 512-thread workgroup per CU stream
// 64-KiB tiles into LDS (K1's X staging)?  Tiles are contiguous 64 KiB
// blocks of a 268 MB buffer (what a pre-transposed X^T gives); `groups`
// distinct tile sequences are shared by 256/groups workgroups each.
//   reg   : 8 x global_load_dwordx4 per thread -> ds_write_b128, DEPTH tiles
//           of registers in flight (explicit rotation)
//   dma   : global_load_lds_dwordx4 (LDS-DMA, no VGPRs), NBUF LDS buffers,
//           NBUF-1 tiles in flight
// Prints per-tile time and aggregate bandwidth.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ const float4* tile_ptr(const float* X, int grp, int t, int ntile_total) {
    const size_t tile = ((size_t)grp * 1009 + t) % ntile_total;
    return reinterpret_cast<const float4*>(X) + tile * 4096;
}

template <int DEPTH>
__global__ void __launch_bounds__(512, 2) k_reg(const float* __restrict__ X, int ntiles, int groups, int ntt,
                                                float* out) {
    __shared__ float4 lds[2][4096];
    const int grp = blockIdx.x % groups;
    float4 a[8], b[8];
    float acc = 0.f;
    const float4* p = tile_ptr(X, grp, 0, ntt);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = p[threadIdx.x + 512 * i];
    if (DEPTH == 2) {
        p = tile_ptr(X, grp, 1, ntt);
#pragma unroll
        for (int i = 0; i < 8; ++i) b[i] = p[threadIdx.x + 512 * i];
    }
    for (int t = 0; t < ntiles; t += 2) {
#pragma unroll
        for (int i = 0; i < 8; ++i) lds[0][threadIdx.x + 512 * i] = a[i];
        p = tile_ptr(X, grp, t + DEPTH, ntt);
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = p[threadIdx.x + 512 * i];
        __syncthreads();
        acc += lds[0][(threadIdx.x * 7) & 4095].x;
        if (DEPTH == 2) {
#pragma unroll
            for (int i = 0; i < 8; ++i) lds[1][threadIdx.x + 512 * i] = b[i];
            p = tile_ptr(X, grp, t + 3, ntt);
#pragma unroll
            for (int i = 0; i < 8; ++i) b[i] = p[threadIdx.x + 512 * i];
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) lds[1][threadIdx.x + 512 * i] = a[i];
            p = tile_ptr(X, grp, t + 2, ntt);
#pragma unroll
            for (int i = 0; i < 8; ++i) a[i] = p[threadIdx.x + 512 * i];
        }
        __syncthreads();
        acc += lds[1][(threadIdx.x * 5) & 4095].x;
    }
    out[blockIdx.x * 512 + threadIdx.x] = acc;
}

// LDS-DMA ring of NBUF 32-KiB buffers (64 KiB tiles = 2 buffers each would
// not fit 4 deep; use 32-KiB tiles and report per 64 KiB).
template <int NBUF>
__global__ void __launch_bounds__(512, 2) k_dma(const float* __restrict__ X, int ntiles, int groups, int ntt,
                                                float* out) {
    __shared__ float4 lds[NBUF][2048];  // NBUF x 32 KiB
    const int grp = blockIdx.x % groups;
    float acc = 0.f;
    auto issue = [&](int t) {
        const float4* p = reinterpret_cast<const float4*>(X) + (((size_t)grp * 1009 + t) % (ntt * 2)) * 2048;
        float4* dst = &lds[t % NBUF][0];
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds(p + threadIdx.x + 512 * i, dst + (threadIdx.x & ~63) + 512 * i, 16, 0, 0);
    };
    for (int t = 0; t < NBUF - 1; ++t) issue(t);
    for (int t = 0; t < ntiles * 2; ++t) {
        // wait for tile t: NBUF-2 younger tiles (4 DMA each) may stay in flight
        if (NBUF == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if (NBUF == 3) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        acc += lds[t % NBUF][(threadIdx.x * 7) & 2047].x;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        issue(t + NBUF - 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    out[blockIdx.x * 512 + threadIdx.x] = acc;
}

template <class F>
float timeit(F f) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    f();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    f();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms;
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const size_t bytes = 268435456;
    const int ntt = (int)(bytes / 65536);
    float* X;
    float* out;
    CHECK(hipMalloc(&X, bytes + (1 << 20)));
    CHECK(hipMemset(X, 0, bytes));
    CHECK(hipMalloc(&out, 1 << 24));
    const int ntiles = 256, blocks = 256;
    for (int groups : {1, 4, 32, 256}) {
        auto rep = [&](const char* n, float ms) {
            printf("%-10s groups=%3d: %.3f ms  %.2f TB/s  %.2f us/64KiB-tile\n", n, groups, ms,
                   blocks * (double)ntiles * 65536.0 / ms / 1e9, ms * 1e3 / ntiles);
        };
        rep("reg d1", timeit([&] { hipLaunchKernelGGL((k_reg<1>), dim3(blocks), dim3(512), 0, 0, X, ntiles, groups, ntt, out); }));
        rep("reg d2", timeit([&] { hipLaunchKernelGGL((k_reg<2>), dim3(blocks), dim3(512), 0, 0, X, ntiles, groups, ntt, out); }));
        rep("dma 2buf", timeit([&] { hipLaunchKernelGGL((k_dma<2>), dim3(blocks), dim3(512), 0, 0, X, ntiles, groups, ntt, out); }));
        rep("dma 4buf", timeit([&] { hipLaunchKernelGGL((k_dma<4>), dim3(blocks), dim3(512), 0, 0, X, ntiles, groups, ntt, out); }));
    }
    return 0;
}
