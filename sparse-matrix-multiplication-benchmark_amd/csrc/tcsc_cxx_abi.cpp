// tcsc_cxx_abi.cpp -- C++-mangled aliases of the drop-in API.
//
// The reference is compiled with g++, so its .c files are C++ and the
// harness's objects reference C++-mangled names (SURVEY.md §8b "Linkage";
// /root/reference/sparse/tcsc.h:19-48 and dense/dense.h:8-21 declare them
// without extern "C").  Exporting these names lets the reference's own
// main.cpp, compiled against ITS headers, link against libtcsc_amd.so in
// place of sparse/tcsc.c + dense/dense.c ("link-level
// drop-in").  Each alias forwards to the C entry point of the same name.
// The mangled strings are the g++ (Itanium ABI) names of the reference's
// prototypes: tcsc_t is a typedef'd anonymous struct, so it mangles as
// "6tcsc_t"; dense_t is float*.
#include "../../include/dense/dense.h"
#include "../../include/sparse/bcsr.h"
#include "../../include/sparse/tcsc.h"

#define TCSC_EXPORT __attribute__((visibility("default")))

TCSC_EXPORT tcsc_t* cxx_tcsc_from_dense(float* d, int rows, int cols) __asm__("_Z15tcsc_from_densePfii");
TCSC_EXPORT tcsc_t* cxx_tcsc_from_dense(float* d, int rows, int cols) { return tcsc_from_dense(d, rows, cols); }

TCSC_EXPORT void cxx_tcsc_sgemm_basic(float* X, const tcsc_t* W, float* B, float* Y, int M, int N, int K) __asm__(
    "_Z16tcsc_sgemm_basicPfPK6tcsc_tS_S_iii");
TCSC_EXPORT void cxx_tcsc_sgemm_basic(float* X, const tcsc_t* W, float* B, float* Y, int M, int N, int K) {
    tcsc_sgemm_basic(X, W, B, Y, M, N, K);
}

TCSC_EXPORT void cxx_tcsc_sgemm_optimized(float* X, const tcsc_t* W, float* B, float* Y, int M, int N,
                                          int K) __asm__("_Z20tcsc_sgemm_optimizedPfPK6tcsc_tS_S_iii");
TCSC_EXPORT void cxx_tcsc_sgemm_optimized(float* X, const tcsc_t* W, float* B, float* Y, int M, int N, int K) {
    tcsc_sgemm_optimized(X, W, B, Y, M, N, K);
}

TCSC_EXPORT void cxx_tcsc_sgemm_prelu_basic(float* X, const tcsc_t* W, float* B, float a, float* Y, int M, int N,
                                            int K) __asm__("_Z22tcsc_sgemm_prelu_basicPfPK6tcsc_tS_fS_iii");
TCSC_EXPORT void cxx_tcsc_sgemm_prelu_basic(float* X, const tcsc_t* W, float* B, float a, float* Y, int M, int N,
                                            int K) {
    tcsc_sgemm_prelu_basic(X, W, B, a, Y, M, N, K);
}

TCSC_EXPORT void cxx_tcsc_sgemm_prelu_sep(float* X, const tcsc_t* W, float* B, float a, float* Y, int M, int N,
                                          int K) __asm__("_Z35tcsc_sgemm_prelu_optimized_separatePfPK6tcsc_tS_fS_iii");
TCSC_EXPORT void cxx_tcsc_sgemm_prelu_sep(float* X, const tcsc_t* W, float* B, float a, float* Y, int M, int N,
                                          int K) {
    tcsc_sgemm_prelu_optimized_separate(X, W, B, a, Y, M, N, K);
}

TCSC_EXPORT void cxx_tcsc_sgemm_prelu_otg(float* X, const tcsc_t* W, float* B, float a, float* Y, int M, int N,
                                          int K) __asm__("_Z34tcsc_sgemm_prelu_optimized_onthegoPfPK6tcsc_tS_fS_iii");
TCSC_EXPORT void cxx_tcsc_sgemm_prelu_otg(float* X, const tcsc_t* W, float* B, float a, float* Y, int M, int N,
                                          int K) {
    tcsc_sgemm_prelu_optimized_onthego(X, W, B, a, Y, M, N, K);
}

TCSC_EXPORT void cxx_tcsc_free(tcsc_t* W) __asm__("_Z9tcsc_freeP6tcsc_t");
TCSC_EXPORT void cxx_tcsc_free(tcsc_t* W) { tcsc_free(W); }

TCSC_EXPORT float* cxx_init_rand_dense(int rows, int cols) __asm__("_Z15init_rand_denseii");
TCSC_EXPORT float* cxx_init_rand_dense(int rows, int cols) { return init_rand_dense(rows, cols); }

TCSC_EXPORT float* cxx_init_rand_sparse(int rows, int cols, int nz) __asm__("_Z16init_rand_sparseiii");
TCSC_EXPORT float* cxx_init_rand_sparse(int rows, int cols, int nz) { return init_rand_sparse(rows, cols, nz); }

TCSC_EXPORT float* cxx_dense_random(int rows, int cols) __asm__("_Z12dense_randomii");
TCSC_EXPORT float* cxx_dense_random(int rows, int cols) { return dense_random(rows, cols); }

TCSC_EXPORT bool cxx_compare(float* r, float* t, int rows, int cols) __asm__("_Z7comparePfS_ii");
TCSC_EXPORT bool cxx_compare(float* r, float* t, int rows, int cols) { return compare(r, t, rows, cols); }

TCSC_EXPORT void cxx_gemm_basic(float* X, float* W, float* B, float* Y, int M, int N, int K) __asm__(
    "_Z10gemm_basicPfS_S_S_iii");
TCSC_EXPORT void cxx_gemm_basic(float* X, float* W, float* B, float* Y, int M, int N, int K) {
    gemm_basic(X, W, B, Y, M, N, K);
}

TCSC_EXPORT void cxx_gemm_prelu_basic(float* X, float* W, float* B, float a, float* Y, int M, int N, int K) __asm__(
    "_Z16gemm_prelu_basicPfS_S_fS_iii");
TCSC_EXPORT void cxx_gemm_prelu_basic(float* X, float* W, float* B, float a, float* Y, int M, int N, int K) {
    gemm_prelu_basic(X, W, B, a, Y, M, N, K);
}

// BCSR (reference sparse/bcsr.h:14-39): bcsr_t is a typedef'd anonymous
// struct passed by value ("6bcsr_t"); its top-level const/__restrict do not
// mangle.  These let the reference's test/test_bcsr.cpp link unchanged.
TCSC_EXPORT bcsr_t* cxx_bcsr_from_dense(float* d, int rows, int cols, int r, int c) __asm__("_Z15bcsr_from_densePfiiii");
TCSC_EXPORT bcsr_t* cxx_bcsr_from_dense(float* d, int rows, int cols, int r, int c) {
    return bcsr_from_dense(d, rows, cols, r, c);
}

TCSC_EXPORT void cxx_bcsr_sgemm_basic(float* X, bcsr_t W, float* B, float* Y, int M, int N, int K) __asm__(
    "_Z16bcsr_sgemm_basicPf6bcsr_tS_S_iii");
TCSC_EXPORT void cxx_bcsr_sgemm_basic(float* X, bcsr_t W, float* B, float* Y, int M, int N, int K) {
    bcsr_sgemm_basic(X, W, B, Y, M, N, K);
}

TCSC_EXPORT void cxx_bcsr_sgemm_prelu_basic(float* X, bcsr_t W, float* B, float a, float* Y, int M, int N,
                                            int K) __asm__("_Z22bcsr_sgemm_prelu_basicPf6bcsr_tS_fS_iii");
TCSC_EXPORT void cxx_bcsr_sgemm_prelu_basic(float* X, bcsr_t W, float* B, float a, float* Y, int M, int N, int K) {
    bcsr_sgemm_prelu_basic(X, W, B, a, Y, M, N, K);
}

TCSC_EXPORT void cxx_bcsr_sgemm_avx(float* X, bcsr_t W, float* B, float* Y, int M, int N, int K) __asm__(
    "_Z14bcsr_sgemm_avxPf6bcsr_tS_S_iii");
TCSC_EXPORT void cxx_bcsr_sgemm_avx(float* X, bcsr_t W, float* B, float* Y, int M, int N, int K) {
    bcsr_sgemm_avx(X, W, B, Y, M, N, K);
}

TCSC_EXPORT void cxx_bcsr_sgemm_prelu_avx(float* X, bcsr_t W, float* B, float a, float* Y, int M, int N,
                                          int K) __asm__("_Z20bcsr_sgemm_prelu_avxPf6bcsr_tS_fS_iii");
TCSC_EXPORT void cxx_bcsr_sgemm_prelu_avx(float* X, bcsr_t W, float* B, float a, float* Y, int M, int N, int K) {
    bcsr_sgemm_prelu_avx(X, W, B, a, Y, M, N, K);
}

TCSC_EXPORT void cxx_bcsr_sgemm_avx2(float* X, bcsr_t W, float* B, float* Y, int M, int N, int K) __asm__(
    "_Z15bcsr_sgemm_avx2Pf6bcsr_tS_S_iii");
TCSC_EXPORT void cxx_bcsr_sgemm_avx2(float* X, bcsr_t W, float* B, float* Y, int M, int N, int K) {
    bcsr_sgemm_avx2(X, W, B, Y, M, N, K);
}
