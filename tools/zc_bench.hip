// zc_bench -- PCIe copies done by kernels instead of the SDMA engines: a
// "pull" kernel reads pinned host memory (zero-copy) and writes HBM, a "push"
// kernel reads HBM and writes pinned host memory; alone and concurrently on
// two streams, with WG counts 8..128, and the SDMA hipMemcpyAsync pair for
// comparison.  Development tool for the host API's band pipeline.
//   hipcc -O3 --offload-arch=gfx950 zc_bench.hip -o zc_bench
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define HIPOK(x)                                                                  \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);              \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

// grid-stride 16-B copy, 4 loads in flight per thread
__global__ void __launch_bounds__(256) k_copy(const f4* __restrict__ src, f4* __restrict__ dst, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        f4 a = __builtin_nontemporal_load(src + i), b = __builtin_nontemporal_load(src + i + stride),
           c = __builtin_nontemporal_load(src + i + 2 * stride), d = __builtin_nontemporal_load(src + i + 3 * stride);
        __builtin_nontemporal_store(a, dst + i);
        __builtin_nontemporal_store(b, dst + i + stride);
        __builtin_nontemporal_store(c, dst + i + 2 * stride);
        __builtin_nontemporal_store(d, dst + i + 3 * stride);
    }
    for (; i < n; i += stride) dst[i] = src[i];
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const size_t bytes = 256ull << 20, n = bytes / 16;
    char *hin, *hout;
    HIPOK(hipHostMalloc((void**)&hin, bytes, hipHostMallocDefault));
    HIPOK(hipHostMalloc((void**)&hout, bytes, hipHostMallocDefault));
    memset(hin, 1, bytes);
    memset(hout, 2, bytes);
    void *da, *db;
    HIPOK(hipMalloc(&da, bytes));
    HIPOK(hipMalloc(&db, bytes));
    hipStream_t s1, s2;
    HIPOK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    HIPOK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    auto gbs = [&](double t, double mult = 1) { return mult * bytes / t * 1e-9; };
    for (int rep = 0; rep < 2; ++rep) {
        double t = now();
        HIPOK(hipMemcpyAsync(da, hin, bytes, hipMemcpyHostToDevice, s1));
        HIPOK(hipMemcpyAsync(hout, db, bytes, hipMemcpyDeviceToHost, s2));
        HIPOK(hipStreamSynchronize(s1));
        HIPOK(hipStreamSynchronize(s2));
        printf("SDMA H2D || D2H: %.1f GB/s aggregate\n", gbs(now() - t, 2));
        for (int wg : {8, 16, 32, 64, 128}) {
            t = now();
            hipLaunchKernelGGL(k_copy, dim3(wg), dim3(256), 0, s1, (const f4*)hin, (f4*)da, n);
            HIPOK(hipStreamSynchronize(s1));
            const double pull = gbs(now() - t);
            t = now();
            hipLaunchKernelGGL(k_copy, dim3(wg), dim3(256), 0, s2, (const f4*)db, (f4*)hout, n);
            HIPOK(hipStreamSynchronize(s2));
            const double push = gbs(now() - t);
            t = now();
            hipLaunchKernelGGL(k_copy, dim3(wg), dim3(256), 0, s1, (const f4*)hin, (f4*)da, n);
            hipLaunchKernelGGL(k_copy, dim3(wg), dim3(256), 0, s2, (const f4*)db, (f4*)hout, n);
            HIPOK(hipStreamSynchronize(s1));
            HIPOK(hipStreamSynchronize(s2));
            printf("kernels, %3d WGs: pull %.1f, push %.1f, both %.1f GB/s aggregate\n", wg, pull, push,
                   gbs(now() - t, 2));
        }
    }
    return 0;
}
