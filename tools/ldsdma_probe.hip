// ldsdma_probe.hip -- does global_load_lds_dwordx4 with 64 per-lane source
// rows write every lane's 16 B to M0 + 16*lane?  (k_fused's transposition
// units read one X row per lane.)  For several source patterns, one wave
// DMAs 1 KiB into LDS, waits vmcnt(0), reads it back and counts the lanes
// whose 16 B differ from what a plain global load of the same address gives.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void probe(const float* __restrict__ X, int K, int pattern, int rep, int* bad) {
    __shared__ __attribute__((aligned(16))) float lds[4096];
    const int l = threadIdx.x;
    // pattern 0: contiguous (l*16 B); 1: one row per lane (row l*4, stride K);
    // 2: 8 lanes per row (row l/8, 128 B pieces); 3: one row per lane, rows l (stride K)
    unsigned off;
    switch (pattern) {
        case 0: off = 16u * l; break;
        case 1: off = (unsigned)(4 * l) * K * 4u; break;
        case 2: off = (unsigned)(l / 8) * K * 4u + 16u * (l % 8); break;
        default: off = (unsigned)l * K * 4u; break;
    }
    const char* base = reinterpret_cast<const char*>(X) + 16 * rep;
    const unsigned m0 = (unsigned)reinterpret_cast<uintptr_t>(lds);
    unsigned sv;
    asm volatile("s_mov_b32 %[sv], m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %3\n\t"
                 "s_mov_b32 m0, %[sv]\n\ts_waitcnt vmcnt(0)"
                 : [sv] "=&s"(sv)
                 : "s"(m0), "v"(off), "s"(base)
                 : "memory");
    __syncthreads();
    const float4 got = reinterpret_cast<const float4*>(lds)[l];
    const float4 want = *reinterpret_cast<const float4*>(base + off);
    if (got.x != want.x || got.y != want.y || got.z != want.z || got.w != want.w) atomicAdd(bad + l, 1);
}

int main() {
    const int K = 4096, rows = 512;
    std::vector<float> h((size_t)rows * K);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)i;
    float* d;
    int* bad;
    hipMalloc(&d, h.size() * 4);
    hipMalloc(&bad, 64 * 4);
    hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    for (int pattern = 0; pattern < 4; ++pattern) {
        hipMemset(bad, 0, 64 * 4);
        for (int rep = 0; rep < 200; ++rep) hipLaunchKernelGGL(probe, dim3(256), dim3(64), 0, 0, d, K, pattern, rep % 64, bad);
        std::vector<int> hb(64);
        hipMemcpy(hb.data(), bad, 64 * 4, hipMemcpyDeviceToHost);
        int tot = 0;
        printf("pattern %d:", pattern);
        for (int l = 0; l < 64; ++l) {
            tot += hb[l];
            if (hb[l]) printf(" l%d:%d", l, hb[l]);
        }
        printf("  total %d of %d lane-loads\n", tot, 200 * 256 * 64);
    }
    return 0;
}
