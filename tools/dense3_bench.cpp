// dense3_bench -- how fast is Y = X*W (X fp32 split into three bf16 parts,
// W ternary, exact in bf16) as ONE rocBLAS bf16 GEMM with fp32 accumulation,
// against the fp32 SGEMM of the dense baseline?  Decides whether near-dense W
// (cfg 5, 50 %) should go to a dense MFMA path.  Timing only (inputs zero).
//   g++ -O2 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include dense3_bench.cpp -L/opt/rocm/lib -lrocblas -lamdhip64 -o dense3_bench
//   ./dense3_bench M K N
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define HIPOK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
#define RBOK(x) do { rocblas_status s = (x); if (s != rocblas_status_success) { printf("rocBLAS %s @%d\n", rocblas_status_to_string(s), __LINE__); exit(1);} } while (0)

template <class F>
float time_ms(F f, int reps) {
    hipEvent_t a, b;
    HIPOK(hipEventCreate(&a));
    HIPOK(hipEventCreate(&b));
    f();
    f();
    HIPOK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) f();
    HIPOK(hipEventRecord(b, 0));
    HIPOK(hipEventSynchronize(b));
    float ms;
    HIPOK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const int M = argc > 1 ? atoi(argv[1]) : 2048, K = argc > 2 ? atoi(argv[2]) : 8192, N = argc > 3 ? atoi(argv[3]) : 8192;
    rocblas_handle h;
    RBOK(rocblas_create_handle(&h));
    void *A, *B, *C, *A32, *B32;
    HIPOK(hipMalloc(&A, (size_t)M * 3 * K * 2));
    HIPOK(hipMalloc(&B, (size_t)3 * K * N * 2));
    HIPOK(hipMalloc(&C, (size_t)M * N * 4));
    HIPOK(hipMalloc(&A32, (size_t)M * K * 4));
    HIPOK(hipMalloc(&B32, (size_t)K * N * 4));
    {   // realistic operands (zeros run the matrix cores at lower power): X parts
        // ~U[-1,1) bf16, W ternary at 50 %
        std::vector<uint16_t> h((size_t)3 * K * N);
        unsigned long long s = 88172645463325252ull;
        auto rnd = [&] { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
        for (auto& v : h) { const unsigned r = rnd() & 3; v = r == 0 ? 0x3f80 : r == 1 ? 0xbf80 : 0; }
        HIPOK(hipMemcpy(B, h.data(), h.size() * 2, hipMemcpyHostToDevice));
        h.resize((size_t)M * 3 * K);
        for (auto& v : h) { float f = (float)((rnd() >> 11) * (1.0 / 9007199254740992.0)) * 2 - 1; unsigned u; memcpy(&u, &f, 4); v = u >> 16; }
        HIPOK(hipMemcpy(A, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    }
    HIPOK(hipMemset(A32, 0, (size_t)M * K * 4));
    HIPOK(hipMemset(B32, 0, (size_t)K * N * 4));
    const float one = 1.f, zero = 0.f;
    // row-major Y[M][N] = X3[M][3K] * W3[3K][N]  <=>  column-major Y^T = W3^T X3^T
    for (int parts = 1; parts <= 3; ++parts) {
        const int KK = parts * K;
        const float ms = time_ms([&] {
            RBOK(rocblas_gemm_ex(h, rocblas_operation_none, rocblas_operation_none, N, M, KK, &one, B,
                                 rocblas_datatype_bf16_r, N, A, rocblas_datatype_bf16_r, KK, &zero, C,
                                 rocblas_datatype_f32_r, N, C, rocblas_datatype_f32_r, N, rocblas_datatype_f32_r,
                                 rocblas_gemm_algo_standard, 0, 0));
        }, 10);
        printf("NN bf16 x%d (K'=%d) -> f32: %.3f ms  (%.0f TFLOP/s)\n", parts, KK, ms, 2.0 * M * KK * (double)N / ms * 1e-9);
        // TN: W stored N x K' (k contiguous), both operands K-contiguous
        const float ms2 = time_ms([&] {
            RBOK(rocblas_gemm_ex(h, rocblas_operation_transpose, rocblas_operation_none, N, M, KK, &one, B,
                                 rocblas_datatype_bf16_r, KK, A, rocblas_datatype_bf16_r, KK, &zero, C,
                                 rocblas_datatype_f32_r, N, C, rocblas_datatype_f32_r, N, rocblas_datatype_f32_r,
                                 rocblas_gemm_algo_standard, 0, 0));
        }, 10);
        printf("TN bf16 x%d (K'=%d) -> f32: %.3f ms  (%.0f TFLOP/s)\n", parts, KK, ms2, 2.0 * M * KK * (double)N / ms2 * 1e-9);
    }
    const float ms32 = time_ms([&] {
        RBOK(rocblas_sgemm(h, rocblas_operation_none, rocblas_operation_none, N, M, K, &one, (float*)B32, N,
                           (float*)A32, K, &zero, (float*)C, N));
    }, 10);
    printf("fp32 sgemm: %.3f ms (%.0f TFLOP/s)\n", ms32, 2.0 * M * K * (double)N / ms32 * 1e-9);
    return 0;
}
