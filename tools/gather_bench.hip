// gather_bench.hip -- the generated gather loop of k_stream (csrc/gather_asm.inc)
// in isolation on gfx950: 16 waves per CU, each running one chunk stream of N
// entries over and over against a resident LDS chunk.  Prints cycles per
// entry per SIMD.  What it separates (DESIGN.md "Which roof binds"):
//   barrier 0/1   an s_barrier before every call (the kernel's chunk sync)
//   mode 0        nothing else: the gather's own issue cost
//   mode 1        after every call, scalar-load the next stream from new
//                 lines (scalar-cache misses, as the kernel's chunk streams)
//   mode 2        the same from the same lines every time (scalar-cache hits)
//   mode 3        a 16-dword scalar prefetch issued BEFORE every call and
//                 waited after it: what an SMEM load in flight costs the
//                 gather's lgkmcnt-counted LDS pipeline
//   mode 4..6     skewed work: wave w gets n * f[w / 4] entries (same mean),
//                 f = {1.3, 1.1, 0.9, 0.7} / {0.7, 0.9, 1.1, 1.3} /
//                 {1.15, 1.05, 0.95, 0.85}: do older waves (the SIMD arbiter
//                 favours them) finish with the younger ones if they get more?
//   Build: hipcc --offload-arch=gfx950 -O3 -I../sparse-matrix-multiplication-benchmark_amd/csrc -o gather_bench gather_bench.hip
//   Run:   ./gather_bench [N entries per stream (<= 30 for modes 1-3)] [barrier 0/1] [mode]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gather_asm.inc"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef float f32x32 __attribute__((ext_vector_type(32)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(4))) const i32x16 const_i32x16;
typedef int sbuf_tail_t __attribute__((ext_vector_type(TCSC_SBUF_TAIL ? TCSC_SBUF_TAIL : 4)));
typedef __attribute__((address_space(4))) const sbuf_tail_t const_sbuf_tail;

constexpr int kWaves = 16;
constexpr int kRows = 147;    // 3 ring buffers of 49 rows
constexpr int kSlots = 64;    // modes 1-3: stream copies per wave, 64 ints (256 B) apart

template <bool BAR>
__global__ void __launch_bounds__(kWaves * 64, kWaves / 4) k_gather(const int* stream, int stream_ints, int iters,
                                                                     int mode, long long* cyc, float* out) {
    __shared__ __attribute__((aligned(16))) float lds[kRows * 256];
    for (int i = threadIdx.x; i < kRows * 256; i += blockDim.x) lds[i] = (float)(i & 7);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int* mine = stream + (size_t)(blockIdx.x * kWaves + wave) * stream_ints;
    f32x32 acc[TCSC_ACC_VECS];
    for (int v = 0; v < TCSC_ACC_VECS; ++v)
        for (int i = 0; i < 32; ++i) acc[v][i] = 0.f;
    i32x16 sb[TCSC_SBUF_VECS];
    sbuf_tail_t sbt;
    const_i32x16* q = reinterpret_cast<const_i32x16*>(reinterpret_cast<uintptr_t>(mine));
    for (int i = 0; i < TCSC_SBUF_VECS; ++i) sb[i] = q[i];
#if TCSC_SBUF_TAIL
    sbt = *reinterpret_cast<const_sbuf_tail*>(reinterpret_cast<uintptr_t>(mine + 16 * TCSC_SBUF_VECS));
#endif
    const int nb0 = sb[0][0];
    const unsigned long long ptr0 = reinterpret_cast<unsigned long long>(mine);
    const unsigned mask = 0x3ffu, lane16 = lane * 16u;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (BAR) __builtin_amdgcn_s_barrier();
        i32x16 pf;
        if (mode == 3) {
            unsigned long long a = reinterpret_cast<unsigned long long>(mine + (size_t)((it + 1) % kSlots) * 64);
            asm volatile("" : "+s"(a));
            asm volatile("s_load_dwordx16 %0, %1, 0x0" : "=&s"(pf) : "s"(a) : "memory");
        }
        sb[0][0] = nb0;  // the loop counts the header's nb down in place
        sb[0][3] = 0;    // and advances the reload offset
        unsigned long long ptr = ptr0;
        asm volatile(TCSC_GATHER_ASM
                     : TCSC_ACC_OPERANDS(acc), TCSC_SBUF_OPERANDS(sb, sbt), TCSC_PTR_OPERAND(ptr)
                     : [lane] "v"(lane16), [mask] "v"(mask)
                     : TCSC_GATHER_CLOBBERS);
        if (mode == 3) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            acc[0][0] += __builtin_bit_cast(float, pf[1] & 0);
        } else if (mode == 1 || mode == 2) {
            unsigned long long a = reinterpret_cast<unsigned long long>(
                mode == 1 ? mine + (size_t)(it % kSlots) * 64 : mine);
            asm volatile("" : "+s"(a));
            const_i32x16* q2 = reinterpret_cast<const_i32x16*>(a);
            for (int i = 0; i < TCSC_SBUF_VECS; ++i) sb[i] = q2[i];
#if TCSC_SBUF_TAIL
            sbt = *reinterpret_cast<const_sbuf_tail*>(a + 64 * TCSC_SBUF_VECS);
#endif
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
    for (int v = 0; v < TCSC_ACC_VECS; ++v)
        for (int i = 0; i < 32; ++i) s += acc[v][i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (lane == 0) cyc[blockIdx.x * kWaves + wave] = t1 - t0;
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 16;
    const int bar = argc > 2 ? atoi(argv[2]) : 0;
    const int mode = argc > 3 ? atoi(argv[3]) : 0;
    if (mode >= 1 && mode <= 3 && n > 30) {
        printf("modes 1-3 keep streams of at most 30 entries\n");
        return 1;
    }
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    // per wave: header {nb, rem, next = 0, 0} + entries (+ slack for the
    // scalar buffer), or kSlots copies 64 ints apart for the reload modes
    const bool slots = mode >= 1 && mode <= 3;
    const int ints = slots ? kSlots * 64 : 4 + 2 * (2 * n + 64);
    const int ne = slots ? 30 : 2 * n + 64;
    std::vector<int> h((size_t)cus * kWaves * ints, 0);
    srand(1);
    for (int w = 0; w < cus * kWaves; ++w) {
        int* s = h.data() + (size_t)w * ints;
        static const float skew[3][4] = {{1.3f, 1.1f, 0.9f, 0.7f}, {0.7f, 0.9f, 1.1f, 1.3f}, {1.15f, 1.05f, 0.95f, 0.85f}};
        const int nw = mode >= 4 ? (int)(n * skew[mode - 4][(w % kWaves) / 4] + 0.5f) : n;
        s[0] = nw / TCSC_GEN_BATCH;
        s[1] = nw % TCSC_GEN_BATCH;
        for (int j = 0; j < ne; ++j) {
            const int row = rand() % kRows, slot = rand() % TCSC_GEN_CW;
            s[4 + 2 * j] = (rand() & 1) ? 0x3f800000 : (int)0xbf800000;
            s[4 + 2 * j + 1] = (row << 10) | (4 * slot);
        }
        if (slots)
            for (int k = 1; k < kSlots; ++k)
                for (int i = 0; i < 64; ++i) s[k * 64 + i] = s[i];
    }
    int* d;
    long long* cyc;
    float* out;
    CHECK(hipMalloc(&d, h.size() * sizeof(int)));
    CHECK(hipMemcpy(d, h.data(), h.size() * sizeof(int), hipMemcpyHostToDevice));
    CHECK(hipMalloc(&cyc, sizeof(long long) * cus * kWaves));
    CHECK(hipMalloc(&out, sizeof(float) * cus * kWaves * 64));
    const int iters = 2000;
    for (int rep = 0; rep < 2; ++rep) {
        if (bar)
            hipLaunchKernelGGL(k_gather<true>, dim3(cus), dim3(kWaves * 64), 0, 0, d, ints, iters, mode, cyc, out);
        else
            hipLaunchKernelGGL(k_gather<false>, dim3(cus), dim3(kWaves * 64), 0, 0, d, ints, iters, mode, cyc, out);
        CHECK(hipDeviceSynchronize());
    }
    std::vector<long long> c(cus * kWaves);
    CHECK(hipMemcpy(c.data(), cyc, c.size() * sizeof(long long), hipMemcpyDeviceToHost));
    double mx = 0, avg = 0;
    for (long long v : c) {
        avg += (double)v;
        mx = mx > (double)v ? mx : (double)v;
    }
    avg /= c.size();
    // per SIMD: kWaves/4 waves share it
    printf("mode=%d n=%d barrier=%d: %.1f cyc per call per wave; %.2f cyc per entry per SIMD (max wave %.1f)\n", mode,
           n, bar, avg / iters, avg / iters / n / (kWaves / 4), mx / iters);
    return 0;
}
