// hblt_bench -- the MFMA path's GEMM (Y = X3 . W3, bf16 in, fp32 out, both
// operands k-contiguous) through hipBLASLt: every algorithm the heuristic
// offers, timed, against rocBLAS gemm_ex's pick.  Also the BIAS epilogue
// (would fold k_bias_act into the GEMM for the non-PReLU variants).
//   g++ -O2 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include hblt_bench.cpp -L/opt/rocm/lib -lhipblaslt -lrocblas -lamdhip64 -o hblt_bench
//   ./hblt_bench M K N        (K = the original K; the GEMM runs over 3K)
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <rocblas/rocblas.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define HIPOK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
#define LTOK(x) do { hipblasStatus_t s = (x); if (s != HIPBLAS_STATUS_SUCCESS) { printf("hipBLASLt %d @%d\n", (int)s, __LINE__); exit(1);} } while (0)

template <class F>
float time_ms(F f, int reps) {
    hipEvent_t a, b;
    HIPOK(hipEventCreate(&a));
    HIPOK(hipEventCreate(&b));
    f();
    f();
    HIPOK(hipDeviceSynchronize());
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
    const int KK = 3 * K;
    void *A, *B, *C, *bias, *ws;
    const size_t wsb = 256ull << 20;
    HIPOK(hipMalloc(&A, (size_t)N * KK * 2));   // W3T: N x 3K, k contiguous
    HIPOK(hipMalloc(&B, (size_t)M * KK * 2));   // X3: M x 3K, k contiguous
    HIPOK(hipMalloc(&C, (size_t)M * N * 4));
    HIPOK(hipMalloc(&bias, (size_t)N * 4));
    HIPOK(hipMalloc(&ws, wsb));
    {
        std::vector<uint16_t> h((size_t)N * KK);
        unsigned long long s = 88172645463325252ull;
        auto rnd = [&] { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
        for (auto& v : h) { const unsigned r = rnd() & 3; v = r == 0 ? 0x3f80 : r == 1 ? 0xbf80 : 0; }
        HIPOK(hipMemcpy(A, h.data(), h.size() * 2, hipMemcpyHostToDevice));
        h.resize((size_t)M * KK);
        for (auto& v : h) { float f = (float)((rnd() >> 11) * (1.0 / 9007199254740992.0)) * 2 - 1; unsigned u; memcpy(&u, &f, 4); v = u >> 16; }
        HIPOK(hipMemcpy(B, h.data(), h.size() * 2, hipMemcpyHostToDevice));
        HIPOK(hipMemset(bias, 0, (size_t)N * 4));
    }
    const double flop = 2.0 * M * (double)KK * N;
    // rocBLAS (what the library calls today)
    {
        rocblas_handle h;
        rocblas_create_handle(&h);
        const float one = 1.f, zero = 0.f;
        const float ms = time_ms([&] {
            rocblas_gemm_ex(h, rocblas_operation_transpose, rocblas_operation_none, N, M, KK, &one, A,
                            rocblas_datatype_bf16_r, KK, B, rocblas_datatype_bf16_r, KK, &zero, C, rocblas_datatype_f32_r,
                            N, C, rocblas_datatype_f32_r, N, rocblas_datatype_f32_r, rocblas_gemm_algo_standard, 0, 0);
        }, 20);
        printf("rocBLAS gemm_ex TN: %.3f ms (%.0f TFLOP/s)\n", ms, flop / ms * 1e-9);
    }
    hipblasLtHandle_t lt;
    LTOK(hipblasLtCreate(&lt));
    for (int epi = 0; epi < 2; ++epi) {
        hipblasLtMatmulDesc_t desc;
        LTOK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
        hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
        LTOK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof ta));
        LTOK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof tb));
        if (epi) {
            hipblasLtEpilogue_t e = HIPBLASLT_EPILOGUE_BIAS;
            LTOK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof e));
            LTOK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof bias));
            hipDataType bt = HIP_R_32F;
            LTOK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof bt));
        }
        hipblasLtMatrixLayout_t la, lb, lc;
        LTOK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, KK, N, KK));  // op T -> N x KK
        LTOK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, KK, M, KK));
        LTOK(hipblasLtMatrixLayoutCreate(&lc, HIP_R_32F, N, M, N));
        hipblasLtMatmulPreference_t pref;
        LTOK(hipblasLtMatmulPreferenceCreate(&pref));
        uint64_t wmax = wsb;
        LTOK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wmax, sizeof wmax));
        hipblasLtMatmulHeuristicResult_t res[32];
        int n = 0;
        LTOK(hipblasLtMatmulAlgoGetHeuristic(lt, desc, la, lb, lc, lc, pref, 32, res, &n));
        const float one = 1.f, zero = 0.f;
        float best = 1e30f;
        for (int i = 0; i < n; ++i) {
            if (res[i].state != HIPBLAS_STATUS_SUCCESS) continue;
            const float ms = time_ms([&] {
                hipblasLtMatmul(lt, desc, &one, A, la, B, lb, &zero, C, lc, C, lc, &res[i].algo, ws, wsb, 0);
            }, 10);
            if (ms < best) best = ms;
            printf("  %s algo %2d: %.3f ms (%.0f TFLOP/s) ws %zu\n", epi ? "bias" : "plain", i, ms, flop / ms * 1e-9,
                   (size_t)res[i].workspaceSize);
        }
        printf("hipBLASLt %s: %d algos, best %.3f ms (%.0f TFLOP/s)\n", epi ? "BIAS epilogue" : "plain", n, best,
               flop / best * 1e-9);
    }
    return 0;
}
