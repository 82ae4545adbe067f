/*
 * sparse_gemm.h -- C ABI behind the SparseGEMM.h drop-in.
 *
 * The reference's second API is the header-only template library
 * /root/reference/SparseGEMM.h, driven by SparseGEMM.cpp.  Its entry points
 * take raw arrays instead of a tcsc_t.  include/SparseGEMM.h keeps those
 * templates and the SparseFormat class with the same names and parameter
 * types; for T = float their bodies call the functions below, which run on
 * the same gfx950 kernels as sparse/tcsc.h.
 *
 *   tcsc_sparse_format      <- SparseFormat::SparseFormat(int*, int K, int N)   SparseGEMM.h:20-39
 *   tcsc_sparse_gemm        <- sparseGEMM<float>(X, cs+, cs-, ri+, ri-, b, Y, M, N, K)  SparseGEMM.h:104-119
 *   tcsc_sparse_gemm_prelu  <- sparseGEMM_PReLU<float>(..., M, N, K, a)        SparseGEMM.h:151-168
 *   tcsc_dense_gemm         <- GEMM<float>(X, W, b, Y, M, N, K)                 SparseGEMM.h:121-133
 *   tcsc_dense_gemm_prelu   <- GEMM_PReLU<float>(X, W, b, Y, M, N, K, a)        SparseGEMM.h:135-149
 *
 * Semantics kept from the reference:
 *   - X is M x K, Y is M x N, W (dense) is K x N, all row-major; b has N
 *     entries; the argument order is (M, N, K) (SparseGEMM.cpp:109).
 *   - Column n of the sparse W is rows row_index_pos[col_start_pos[n] ..
 *     col_start_pos[n+1]) with +1 and row_index_neg[...] with -1.
 *   - sparseGEMM: y = 0 + sum(+1 rows) - sum(-1 rows), Y = y + b.  The PReLU
 *     form then applies (y < 0) ? a*y : y (SparseGEMM.h:165), the predicate of
 *     tcsc.c:162: -0.0 and NaN pass through.
 *   - Y is fully overwritten.  The functions return nothing (the reference's
 *     templates have no error channel); errors go to stderr and
 *     tcsc_gpu_last_error(), then abort unless TCSC_ON_ERROR=continue, as
 *     for the sparse/tcsc.h entry points.
 *
 * Underneath: the host arrays are uploaded once and cached per col_start_pos
 * address, with the same content fingerprint as the tcsc_t cache (a changed
 * array gets a fresh plan); the last 8 distinct matrices stay cached.  X and
 * b go host->device per call and Y comes back.  Summation order: the fast
 * order by default (float results within the bound of DESIGN.md §5, integer
 * inputs bit-exact); TCSC_ORDER=reference reproduces SparseGEMM.h's loops
 * bit for bit (the tcsc_sgemm_prelu_basic chains).  GEMM / GEMM_PReLU are
 * the dense fp32 rocBLAS product plus the bias/PReLU epilogue
 * (tcsc_gpu_dense_sgemm).
 */
#ifndef TCSC_AMD_SPARSE_GEMM_H
#define TCSC_AMD_SPARSE_GEMM_H

#ifdef __cplusplus
extern "C" {
#endif

/* int K x N row-major matrix -> the four TCSC arrays.  First call with
 * row_index_pos/neg NULL: writes col_start_pos/neg (N+1 each) and *n_pos,
 * *n_neg.  Second call with the row arrays sized n_pos / n_neg fills them.
 * Returns 0, or TCSC_E_ARG (1) on a bad argument or > 2^31-1 entries. */
int tcsc_sparse_format(const int *matrix, int K, int N, int *col_start_pos, int *col_start_neg,
                       int *row_index_pos, int *row_index_neg, int *n_pos, int *n_neg);

void tcsc_sparse_gemm(const float *X, const int *col_start_pos, const int *col_start_neg,
                      const int *row_index_pos, const int *row_index_neg, const float *b, float *Y,
                      int M, int N, int K);

void tcsc_sparse_gemm_prelu(const float *X, const int *col_start_pos, const int *col_start_neg,
                            const int *row_index_pos, const int *row_index_neg, const float *b,
                            float *Y, int M, int N, int K, float a);

void tcsc_dense_gemm(const float *X, const float *W, const float *b, float *Y, int M, int N, int K);

void tcsc_dense_gemm_prelu(const float *X, const float *W, const float *b, float *Y, int M, int N,
                           int K, float a);

#ifdef __cplusplus
}
#endif

#endif /* TCSC_AMD_SPARSE_GEMM_H */
