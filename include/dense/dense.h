/*
 * dense/dense.h -- drop-in dense helpers for the TCSC benchmark harness.
 *
 * Source-compatible with the reference's dense/dense.h (dense/dense.h:5-25):
 * same typedefs (`dense_elem_t`, `dense_t`), same function names, same
 * argument order (X, W, B, [a,] Y, M, N, K).  Differences, all deliberate:
 *   - valid C *and* C++ (the reference includes <cstdbool>, dense/dense.h:3,
 *     which makes the header C++-only);
 *   - every prototype has C linkage, so the harness links against the
 *     shared library libtcsc_amd.so whatever language it is compiled in;
 *   - gemm_prelu_basic is declared AND defined here (the reference declares
 *     it at dense/dense.h:22-25 but never defines it, dense/dense.c:82-85).
 *
 * The generators keep the reference's distributions (dense/utils.h:9-16 and
 * :36-68) but draw from a seeded SplitMix64 stream instead of
 * std::random_device, so runs are reproducible; see tcsc_set_seed().
 */
#ifndef TCSC_AMD_DENSE_H
#define TCSC_AMD_DENSE_H

#ifdef __cplusplus
extern "C" {
#else
#include <stdbool.h>
#endif

typedef float dense_elem_t;
typedef dense_elem_t *dense_t;

/* U[-1,1) matrix, rows*cols, 32-byte aligned (dense/dense.c:10-19). */
dense_t dense_random(int rows, int cols);
dense_t init_rand_dense(int rows, int cols);

/* Ternary matrix: P(+1)=P(-1)=1/(2*non_zero), P(0)=1-1/non_zero
 * (dense/dense.c:28-37, dense/utils.h:36-68). */
dense_t init_rand_sparse(int rows, int cols, int non_zero);

/* |result-target| <= 1e-4 everywhere; prints the first mismatch
 * (dense/dense.c:42-59). */
bool compare(const dense_t result, const dense_t target, int rows, int cols);

/* Naive dense Y = X*W + B (dense/dense.c:64-77). */
void gemm_basic(const dense_t X, const dense_t W, const dense_t B, dense_t Y,
                int M, int N, int K);

/* Naive dense Y = PReLU(X*W + B) with the reference's PReLU predicate
 * (v < 0 ? a*v : v, sparse/tcsc.c:162). */
void gemm_prelu_basic(const dense_t X, const dense_t W, const dense_t B,
                      float a, dense_t Y, int M, int N, int K);

/* Re-seed the generators above (default seed 0x7C5C0000). */
void tcsc_set_seed(unsigned long long seed);

#ifdef __cplusplus
}
#endif

#endif /* TCSC_AMD_DENSE_H */
