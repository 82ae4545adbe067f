// pcie_bench -- what the host-pointer API's copies can reach on this box:
// pageable vs pinned H2D / D2H, H2D and D2H concurrently on two streams, and
// host memcpy (pageable <-> pinned staging) with 1..16 threads.
//   g++ -O2 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include pcie_bench.cpp -L/opt/rocm/lib -lamdhip64 -lpthread -o pcie_bench
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define HIPOK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const size_t bytes = 256ull << 20;
    char* pg_a = (char*)aligned_alloc(4096, bytes);
    char* pg_b = (char*)aligned_alloc(4096, bytes);
    memset(pg_a, 1, bytes);
    memset(pg_b, 2, bytes);
    char *pin_a, *pin_b;
    HIPOK(hipHostMalloc((void**)&pin_a, bytes, hipHostMallocDefault));
    HIPOK(hipHostMalloc((void**)&pin_b, bytes, hipHostMallocDefault));
    memset(pin_a, 3, bytes);
    memset(pin_b, 4, bytes);
    void *d_a, *d_b;
    HIPOK(hipMalloc(&d_a, bytes));
    HIPOK(hipMalloc(&d_b, bytes));
    hipStream_t s1, s2;
    HIPOK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    HIPOK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    auto gbs = [&](double t, double mult = 1) { return mult * bytes / t * 1e-9; };
    for (int rep = 0; rep < 2; ++rep) {
        double t = now();
        HIPOK(hipMemcpyAsync(d_a, pg_a, bytes, hipMemcpyHostToDevice, s1));
        HIPOK(hipStreamSynchronize(s1));
        printf("pageable H2D %.1f GB/s\n", gbs(now() - t));
        t = now();
        HIPOK(hipMemcpyAsync(pg_b, d_a, bytes, hipMemcpyDeviceToHost, s1));
        HIPOK(hipStreamSynchronize(s1));
        printf("pageable D2H %.1f GB/s\n", gbs(now() - t));
        t = now();
        HIPOK(hipMemcpyAsync(d_a, pin_a, bytes, hipMemcpyHostToDevice, s1));
        HIPOK(hipStreamSynchronize(s1));
        printf("pinned H2D %.1f GB/s\n", gbs(now() - t));
        t = now();
        HIPOK(hipMemcpyAsync(pin_b, d_b, bytes, hipMemcpyDeviceToHost, s1));
        HIPOK(hipStreamSynchronize(s1));
        printf("pinned D2H %.1f GB/s\n", gbs(now() - t));
        t = now();
        HIPOK(hipMemcpyAsync(d_a, pin_a, bytes, hipMemcpyHostToDevice, s1));
        HIPOK(hipMemcpyAsync(pin_b, d_b, bytes, hipMemcpyDeviceToHost, s2));
        HIPOK(hipStreamSynchronize(s1));
        HIPOK(hipStreamSynchronize(s2));
        printf("pinned H2D || D2H: %.1f GB/s aggregate\n", gbs(now() - t, 2));
        t = now();
        HIPOK(hipMemcpyAsync(d_a, pg_a, bytes, hipMemcpyHostToDevice, s1));
        HIPOK(hipMemcpyAsync(pg_b, d_b, bytes, hipMemcpyDeviceToHost, s2));
        HIPOK(hipStreamSynchronize(s1));
        HIPOK(hipStreamSynchronize(s2));
        printf("pageable H2D || D2H: %.1f GB/s aggregate\n", gbs(now() - t, 2));
        for (int nt : {1, 2, 4, 8, 16}) {
            t = now();
            std::vector<std::thread> th;
            for (int i = 0; i < nt; ++i)
                th.emplace_back([&, i] {
                    const size_t a = bytes * i / nt, b = bytes * (i + 1) / nt;
                    memcpy(pin_a + a, pg_a + a, b - a);
                });
            for (auto& x : th) x.join();
            printf("host memcpy pageable->pinned, %2d threads: %.1f GB/s\n", nt, gbs(now() - t));
        }
    }
    return 0;
}
