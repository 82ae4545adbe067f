// ubench.hip -- primitive-rate microbenchmarks on gfx950 that decide the
// gather kernel's structure (DESIGN.md "Measured primitive rates").
//   salu   : independent s_add_u32 chains, all waves busy -> SALU issue rate per CU
//   valu   : independent v_add_f32 chains -> VALU rate per CU
//   lds64  : uniform-offset ds_read_b64 "gathers" (512 B per wave-instr) + v_pk_add_f32
//   lds128 : same with ds_read_b128 (1 KiB per wave-instr)
//   mix_s  : lds64 + S extra SALU ops per read (interference)
//   smem   : s_load_dwordx8 of the index stream + lds64 (the v0 inner structure, batched)
// Build: hipcc --offload-arch=gfx950 -O3 -o ubench ubench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void k_salu(int iters, int* out) {
    int a = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), b = a + 1, c = a + 2, d = a + 3;
    int e = a + 4, f = a + 5, g = a + 6, h = a + 7;
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "s_mul_i32 %0, %0, 3\n s_mul_i32 %1, %1, 3\n s_mul_i32 %2, %2, 3\n s_mul_i32 %3, %3, 3\n"
            "s_mul_i32 %4, %4, 3\n s_mul_i32 %5, %5, 3\n s_mul_i32 %6, %6, 3\n s_mul_i32 %7, %7, 3\n"
            "s_mul_i32 %0, %0, 3\n s_mul_i32 %1, %1, 3\n s_mul_i32 %2, %2, 3\n s_mul_i32 %3, %3, 3\n"
            "s_mul_i32 %4, %4, 3\n s_mul_i32 %5, %5, 3\n s_mul_i32 %6, %6, 3\n s_mul_i32 %7, %7, 3\n"
            : "+s"(a), "+s"(b), "+s"(c), "+s"(d), "+s"(e), "+s"(f), "+s"(g), "+s"(h));
    }
    if (threadIdx.x == 0) out[blockIdx.x] = a + b + c + d + e + f + g + h;
}

__global__ void k_valu(int iters, float* out) {
    float a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3, e = a + 4, f = a + 5, g = a + 6, h = a + 7;
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "v_add_f32 %0, 1.0, %0\n v_add_f32 %1, 1.0, %1\n v_add_f32 %2, 1.0, %2\n v_add_f32 %3, 1.0, %3\n"
            "v_add_f32 %4, 1.0, %4\n v_add_f32 %5, 1.0, %5\n v_add_f32 %6, 1.0, %6\n v_add_f32 %7, 1.0, %7\n"
            "v_add_f32 %0, 1.0, %0\n v_add_f32 %1, 1.0, %1\n v_add_f32 %2, 1.0, %2\n v_add_f32 %3, 1.0, %3\n"
            "v_add_f32 %4, 1.0, %4\n v_add_f32 %5, 1.0, %5\n v_add_f32 %6, 1.0, %6\n v_add_f32 %7, 1.0, %7\n"
            : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d + e + f + g + h;
}

// LDS "gather": each iteration reads 8 uniform rows (offsets from a small
// SGPR table) of a [k][64 lanes] float2 tile and accumulates with v_pk_add.
template <int MODE, int SALU_EXTRA, int TILE_F4 = 8192>
__global__ void __launch_bounds__(256) k_lds(int iters, const int* __restrict__ offs, float* out) {
    __shared__ float4 tile[TILE_F4];
    for (int i = threadIdx.x; i < TILE_F4; i += blockDim.x) tile[i] = make_float4(i, i + 1, i + 2, i + 3);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    int o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = __builtin_amdgcn_readfirstlane(offs[j]);
    float2 acc0 = make_float2(0, 0), acc1 = acc0;
    float4 b0 = make_float4(0, 0, 0, 0), b1 = b0;
    int s0 = __builtin_amdgcn_readfirstlane(threadIdx.x), s1 = s0 + 1, s2 = s0 + 2, s3 = s0 + 3, s4 = s0 + 4, s5 = s0 + 5, s6 = s0 + 6, s7 = s0 + 7;
    const unsigned base = (MODE == 0 ? 8u : 16u) * lane;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const unsigned addr = base + (unsigned)(o[j] + (i & 7) * 1024);
            if (MODE == 0) {
                float2 x = *reinterpret_cast<const float2*>(reinterpret_cast<const char*>(tile) + addr);
                if (j & 1) { acc1.x += x.x; acc1.y += x.y; } else { acc0.x += x.x; acc0.y += x.y; }
            } else {
                float4 x = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(tile) + addr);
                if (j & 1) { b1.x += x.x; b1.y += x.y; b1.z += x.z; b1.w += x.w; }
                else { b0.x += x.x; b0.y += x.y; b0.z += x.z; b0.w += x.w; }
            }
            if (SALU_EXTRA >= 1) asm volatile("s_mul_i32 %0, %0, 3" : "+s"(s0));
            if (SALU_EXTRA >= 2) asm volatile("s_mul_i32 %0, %0, 5" : "+s"(s1));
            if (SALU_EXTRA >= 4) asm volatile("s_mul_i32 %0, %0, 7\n s_mul_i32 %1, %1, 9" : "+s"(s2), "+s"(s3));
            if (SALU_EXTRA >= 8) asm volatile("s_mul_i32 %0, %0, 7\n s_mul_i32 %1, %1, 9\n s_mul_i32 %2, %2, 7\n s_mul_i32 %3, %3, 9" : "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc0.x + acc0.y + acc1.x + acc1.y + b0.x + b0.y + b0.z + b0.w +
                                                  b1.x + b1.y + b1.z + b1.w + (float)(s0 + s1 + s2 + s3 + s4 + s5 + s6 + s7);
}

// Index stream through SMEM: per iteration load 8 entries (s_load_dwordx8
// from a uniform pointer), then 8 gathers; PREFETCH loads the next batch first.
template <int PREFETCH>
__global__ void __launch_bounds__(256) k_smem(int iters, const int* __restrict__ ent, int nent, float* out) {
    __shared__ float2 tile[16384];  // 128 KiB
    for (int i = threadIdx.x; i < 16384; i += blockDim.x) tile[i] = make_float2(i, i + 1);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float2 acc = make_float2(0, 0);
    int p = (w * 64) & (nent - 1);
    for (int i = 0; i < iters; ++i) {
        const int* q = ent + p;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int e = q[j];
            float2 x = tile[(e & 255) * 64 + lane];
            acc.x += x.x;
            acc.y += x.y;
        }
        p = (p + 8) & (nent - 1);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc.x + acc.y;
}

template <class F>
float time_kernel(F f, int reps = 5) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    f();
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(a));
        f();
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    return best;
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int CUs = prop.multiProcessorCount;
    printf("device %s CUs %d clock %d kHz\n", prop.gcnArchName, CUs, prop.clockRate);
    int* iout;
    float* fout;
    int* offs;
    int* ent;
    const int NENT = 1 << 20;
    CHECK(hipMalloc(&iout, 1 << 24));
    CHECK(hipMalloc(&fout, 1 << 26));
    CHECK(hipMalloc(&offs, 64));
    CHECK(hipMalloc(&ent, NENT * 4));
    std::vector<int> ho = {0, 512 * 7, 512 * 3, 512 * 9, 512 * 1, 512 * 12, 512 * 5, 512 * 2};
    CHECK(hipMemcpy(offs, ho.data(), 32, hipMemcpyHostToDevice));
    std::vector<int> he(NENT);
    for (int i = 0; i < NENT; ++i) he[i] = (i * 2654435761u) >> 24;
    CHECK(hipMemcpy(ent, he.data(), NENT * 4, hipMemcpyHostToDevice));

    const char* only = getenv("UB_ONLY");
    if (!only || only[0] == 's')
    for (int wpb : {4, 8, 16}) {
        for (int bpc : {1, 2}) {
            int blocks = CUs * bpc, iters = 16384;
            float ms = time_kernel([&] { hipLaunchKernelGGL(k_salu, dim3(blocks), dim3(64 * wpb), 0, 0, iters, iout); });
            double ops = (double)blocks * wpb * iters * 16;
            printf("salu  waves/CU=%2d : %.3f ms  %.3f SALU instr/clk/CU (at 2.4GHz)\n", wpb * bpc, ms,
                   ops / (ms * 1e-3) / CUs / 2.4e9);
        }
    }
    for (int wpb : {4, 8, 16}) {
        int blocks = CUs * 2, iters = 16384;
        float ms = time_kernel([&] { hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(64 * wpb), 0, 0, iters, fout); });
        double ops = (double)blocks * wpb * iters * 16;
        printf("valu  waves/CU=%2d : %.3f ms  %.3f wave-VALU/clk/CU = %.1f T lane-adds/s\n", wpb * 2, ms,
               ops / (ms * 1e-3) / CUs / 2.4e9, ops * 64 / (ms * 1e-3) / 1e12);
    }
    auto run_lds = [&](auto kern, const char* name, int bytes_per_read, int bpc = 1) {
        int blocks = CUs * bpc, iters = 8192 / bpc;
        float ms = time_kernel([&] { hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, iters, offs, fout); });
        double reads = (double)blocks * 4 * iters * 8;
        printf("%-14s: %.3f ms  %.1f B/clk/CU (at 2.4GHz), %.2f T fp32/s chip\n", name, ms,
               reads * 64 * bytes_per_read / (ms * 1e-3) / CUs / 2.4e9, reads * 64 * bytes_per_read / 4 / (ms * 1e-3) / 1e12);
    };
    run_lds(k_lds<0, 0>, "lds64", 8);
    run_lds(k_lds<0, 1>, "lds64+1salu", 8);
    run_lds(k_lds<0, 2>, "lds64+2salu", 8);
    run_lds(k_lds<0, 4>, "lds64+4salu", 8);
    run_lds(k_lds<0, 8>, "lds64+8salu", 8);
    run_lds(k_lds<1, 0>, "lds128", 16);
    run_lds(k_lds<1, 2>, "lds128+2salu", 16);
    run_lds(k_lds<1, 4>, "lds128+4salu", 16);
    run_lds(k_lds<0, 0, 2048>, "lds64 16w", 8, 4);
    run_lds(k_lds<0, 1, 2048>, "lds64+1s 16w", 8, 4);
    run_lds(k_lds<0, 2, 2048>, "lds64+2s 16w", 8, 4);
    run_lds(k_lds<0, 4, 2048>, "lds64+4s 16w", 8, 4);
    run_lds(k_lds<1, 0, 2048>, "lds128 16w", 16, 4);
    run_lds(k_lds<1, 2, 2048>, "lds128+2s 16w", 16, 4);
    run_lds(k_lds<1, 4, 2048>, "lds128+4s 16w", 16, 4);
    run_lds(k_lds<0, 0, 1024>, "lds64 32w", 8, 8);
    run_lds(k_lds<0, 2, 1024>, "lds64+2s 32w", 8, 8);
    run_lds(k_lds<1, 0, 1024>, "lds128 32w", 16, 8);
    run_lds(k_lds<1, 4, 1024>, "lds128+4s 32w", 16, 8);
    auto run_smem = [&](auto kern, const char* name) {
        int blocks = CUs, iters = 8192;
        float ms = time_kernel([&] { hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, iters, ent, NENT, fout); });
        double reads = (double)blocks * 4 * iters * 8;
        printf("%-14s: %.3f ms  %.1f B/clk/CU\n", name, ms, reads * 512 / (ms * 1e-3) / CUs / 2.4e9);
    };
    run_smem(k_smem<0>, "smem8+lds64");
    printf("done\n");
    return 0;
}
