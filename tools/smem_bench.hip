// smem_bench.hip -- latency of the gather kernel's per-chunk scalar stream
// load on gfx950: 3 x s_load_dwordx16 + s_load_dwordx4 (one chunk header +
// 24 entries) followed by s_waitcnt lgkmcnt(0), per wave, timed with
// s_memtime.  Modes:
//   0  same address every iteration (scalar-cache hit), no barrier
//   1  same address, s_barrier before each load (all waves burst together)
//   2  a new address every iteration (walks a 64 MiB buffer), no barrier
//   3  new address + barrier
//   4  new address, 4 x s_load_dword instead (one per 64-B line)
// Grid: one workgroup of W waves per CU.
//   Build: hipcc --offload-arch=gfx950 -O3 -o smem_bench smem_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void k_smem(const char* buf, size_t stride_per_wave, int iters, long long* cyc, int* out) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const size_t wg = blockIdx.x;
    unsigned long long p = (unsigned long long)(buf + (wg * 16 + wave) * 256);
    const unsigned long long step = stride_per_wave;
    int acc = 0;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        if (MODE == 1 || MODE == 3) __builtin_amdgcn_s_barrier();
        int a, b, c, d;
        if (MODE == 4) {
            asm volatile(
                "s_load_dword %0, %4, 0x0\n\ts_load_dword %1, %4, 0x40\n\ts_load_dword %2, %4, 0x80\n\t"
                "s_load_dword %3, %4, 0xc0\n\ts_waitcnt lgkmcnt(0)"
                : "=s"(a), "=s"(b), "=s"(c), "=s"(d)
                : "s"(p)
                : "memory");
        } else {
            i32x16 x, y, z;
            i32x4 w;
            asm volatile(
                "s_load_dwordx16 %0, %4, 0x0\n\ts_load_dwordx16 %1, %4, 0x40\n\ts_load_dwordx16 %2, %4, 0x80\n\t"
                "s_load_dwordx4 %3, %4, 0xc0\n\ts_waitcnt lgkmcnt(0)"
                : "=s"(x), "=s"(y), "=s"(z), "=s"(w)
                : "s"(p)
                : "memory");
            a = x[0];
            b = y[3];
            c = z[5];
            d = w[1];
        }
        acc += a ^ b ^ c ^ d;
        if (MODE >= 2) p += step;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int MODE>
void run(int cus, int waves, const char* buf, long long* cyc, int* out) {
    const int iters = 512;
    // each wave walks its own 256-B slots, 4 KiB apart per iteration (new lines every time)
    const size_t stride = (size_t)cus * 16 * 256;
    hipLaunchKernelGGL((k_smem<MODE>), dim3(cus), dim3(64 * waves), 0, 0, buf, stride, iters, cyc, out);
    CHECK(hipDeviceSynchronize());
    hipLaunchKernelGGL((k_smem<MODE>), dim3(cus), dim3(64 * waves), 0, 0, buf, stride, iters, cyc, out);
    CHECK(hipDeviceSynchronize());
    long long* h = (long long*)malloc(sizeof(long long) * cus * 16);
    CHECK(hipMemcpy(h, cyc, sizeof(long long) * cus * 16, hipMemcpyDeviceToHost));
    double s = 0;
    int n = 0;
    for (int b = 0; b < cus; ++b)
        for (int w = 0; w < waves; ++w) s += (double)h[b * 16 + w], ++n;
    printf("mode %d waves/CU %2d: %7.1f cyc per load group\n", MODE, waves, s / n / iters);
    free(h);
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const size_t bytes = (size_t)cus * 16 * 256 * 520;  // iters + slack
    char* buf;
    long long* cyc;
    int* out;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMemset(buf, 1, bytes));
    CHECK(hipMalloc(&cyc, sizeof(long long) * cus * 16));
    CHECK(hipMalloc(&out, sizeof(int) * cus * 1024));
    for (int w : {1, 4, 16}) {
        run<0>(cus, w, buf, cyc, out);
        run<1>(cus, w, buf, cyc, out);
        run<2>(cus, w, buf, cyc, out);
        run<3>(cus, w, buf, cyc, out);
        run<4>(cus, w, buf, cyc, out);
    }
    return 0;
}
