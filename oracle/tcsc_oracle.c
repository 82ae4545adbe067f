/*
 * tcsc_oracle.c -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the
 * reference's TCSC hot path, used as the parity checker for the gfx950
 * kernels and as bench.py's `cpu_baseline` ("port").  Nothing in the
 * product (sparse-matrix-multiplication-benchmark_amd/) links or calls this
 * file; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may.
 *
 * Parity status: PINNED.  Every function below is checked bit-for-bit
 * against the reference's own sources compiled from /root/reference into
 * oracle/_ref/libtcsc_ref.so (recipe: oracle/Makefile) on the fixtures in
 * tests/golden/ (generator: tests/golden/gen_golden.py).
 *
 * Each function follows the loop nest AND the floating-point summation
 * order of the reference line it cites; the file must be compiled without
 * -ffast-math and with -ffp-contract=off (oracle/Makefile) so the order is
 * the one written.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* ---------------------------------------------------------------------- */
/* Format builder: sparse/tcsc.c:6-66                                      */
/* ---------------------------------------------------------------------- */

/* Counting pass (tcsc.c:10-19): row-major sweep, exact float compares. */
void oracle_tcsc_count(const float *dense, int rows, int cols, int *n_pos,
                       int *n_neg) {
    int p = 0, q = 0;
    for (int i = 0; i < rows; ++i)
        for (int j = 0; j < cols; ++j) {
            float v = dense[(size_t)i * cols + j];
            if (v == 1.0f)
                ++p;
            else if (v == -1.0f)
                ++q;
        }
    *n_pos = p;
    *n_neg = q;
}

/* Fill pass (tcsc.c:45-63): column-major sweep, rows ascending. */
void oracle_tcsc_fill(const float *dense, int rows, int cols, int *col_start_pos,
                      int *col_start_neg, int *row_index_pos,
                      int *row_index_neg) {
    int p = 0, q = 0;
    for (int j = 0; j < cols; ++j) {
        col_start_pos[j] = p;
        col_start_neg[j] = q;
        for (int i = 0; i < rows; ++i) {
            float v = dense[(size_t)i * cols + j];
            if (v == 1.0f)
                row_index_pos[p++] = i;
            else if (v == -1.0f)
                row_index_neg[q++] = i;
        }
    }
    col_start_pos[cols] = p;
    col_start_neg[cols] = q;
}

/* Same output as oracle_tcsc_fill, two row-major passes (count, then fill
 * through per-column cursors).  Test infrastructure for full-size inputs
 * (the column-strided reference order takes seconds at K=N=16384); pinned
 * equal to oracle_tcsc_fill by tests/test_oracle.py. */
void oracle_tcsc_fill_rowmajor(const float *dense, int rows, int cols, int *col_start_pos,
                               int *col_start_neg, int *row_index_pos,
                               int *row_index_neg) {
    int *cp = (int *)calloc((size_t)cols + 1, sizeof(int));
    int *cn = (int *)calloc((size_t)cols + 1, sizeof(int));
    for (int i = 0; i < rows; ++i)
        for (int j = 0; j < cols; ++j) {
            float v = dense[(size_t)i * cols + j];
            cp[j] += (v == 1.0f);
            cn[j] += (v == -1.0f);
        }
    int p = 0, q = 0;
    for (int j = 0; j < cols; ++j) {
        col_start_pos[j] = p;
        col_start_neg[j] = q;
        p += cp[j];
        q += cn[j];
        cp[j] = col_start_pos[j];
        cn[j] = col_start_neg[j];
    }
    col_start_pos[cols] = p;
    col_start_neg[cols] = q;
    for (int i = 0; i < rows; ++i)
        for (int j = 0; j < cols; ++j) {
            float v = dense[(size_t)i * cols + j];
            if (v == 1.0f)
                row_index_pos[cp[j]++] = i;
            else if (v == -1.0f)
                row_index_neg[cn[j]++] = i;
        }
    free(cp);
    free(cn);
}

/* Integer-matrix builder of the original spec, SparseFormat
 * (SparseGEMM.h:20-39): thresholds >= 1 / <= -1 instead of exact compares. */
void oracle_sparseformat_fill(const int *matrix, int K, int N, int *col_start_pos,
                              int *col_start_neg, int *row_index_pos,
                              int *row_index_neg, int *n_pos, int *n_neg) {
    int p = 0, q = 0;
    for (int n = 0; n < N; ++n) {
        col_start_pos[n] = p;
        col_start_neg[n] = q;
        for (int k = 0; k < K; ++k) {
            int v = matrix[(size_t)k * N + n];
            if (v >= 1)
                row_index_pos[p++] = k;
            else if (v <= -1)
                row_index_neg[q++] = k;
        }
    }
    col_start_pos[N] = p;
    col_start_neg[N] = q;
    *n_pos = p;
    *n_neg = q;
}

/* ---------------------------------------------------------------------- */
/* Kernels.  Argument order is the reference's (M, N, K); the TCSC arrays   */
/* are passed unpacked (ctypes-friendly).                                  */
/* ---------------------------------------------------------------------- */

#define PRELU(v, a) (((v) < 0.0f) ? (a) * (v) : (v)) /* tcsc.c:162,224,272 */

/* tcsc_sgemm_basic, tcsc.c:69-98: Y=B, then per (m,n): y=Y; y+=P...; y-=Q... */
void oracle_sgemm_basic(const float *X, const int *csp, const int *csn,
                        const int *rip, const int *rin, const float *B,
                        float *Y, int M, int N, int K) {
    for (int m = 0; m < M; ++m)
        for (int n = 0; n < N; ++n)
            Y[(size_t)m * N + n] = B[n];
    for (int m = 0; m < M; ++m) {
        const float *x = X + (size_t)m * K;
        for (int n = 0; n < N; ++n) {
            float y = Y[(size_t)m * N + n];
            for (int k = csp[n]; k < csp[n + 1]; ++k) y += x[rip[k]];
            for (int k = csn[n]; k < csn[n + 1]; ++k) y -= x[rin[k]];
            Y[(size_t)m * N + n] = y;
        }
    }
}

/* tcsc_sgemm_optimized, tcsc.c:101-140: Y=B; per n: per m Y+=(0+P...);
 * per m Y-=(0+Q...). */
static void optimized_core(const float *X, const int *csp, const int *csn,
                           const int *rip, const int *rin, const float *B,
                           float *Y, int M, int N, int K, int prelu_otg,
                           float a) {
    for (int m = 0; m < M; ++m)
        for (int n = 0; n < N; ++n)
            Y[(size_t)m * N + n] = B[n];
    for (int n = 0; n < N; ++n) {
        for (int m = 0; m < M; ++m) {
            float acc = 0.0f;
            for (int k = csp[n]; k < csp[n + 1]; ++k) acc += X[(size_t)m * K + rip[k]];
            Y[(size_t)m * N + n] += acc;
        }
        for (int m = 0; m < M; ++m) {
            float acc = 0.0f;
            for (int k = csn[n]; k < csn[n + 1]; ++k) acc += X[(size_t)m * K + rin[k]];
            Y[(size_t)m * N + n] -= acc;
            if (prelu_otg) { /* tcsc.c:269-272 */
                float v = Y[(size_t)m * N + n];
                Y[(size_t)m * N + n] = PRELU(v, a);
            }
        }
    }
}

void oracle_sgemm_optimized(const float *X, const int *csp, const int *csn,
                            const int *rip, const int *rin, const float *B,
                            float *Y, int M, int N, int K) {
    optimized_core(X, csp, csn, rip, rin, B, Y, M, N, K, 0, 0.0f);
}

/* tcsc_sgemm_prelu_basic, tcsc.c:143-165: y=0; +P; -Q; y+=B[n]; PReLU. */
void oracle_sgemm_prelu_basic(const float *X, const int *csp, const int *csn,
                              const int *rip, const int *rin, const float *B,
                              float a, float *Y, int M, int N, int K) {
    for (int m = 0; m < M; ++m) {
        const float *x = X + (size_t)m * K;
        for (int n = 0; n < N; ++n) {
            float y = 0.0f;
            for (int k = csp[n]; k < csp[n + 1]; ++k) y += x[rip[k]];
            for (int k = csn[n]; k < csn[n + 1]; ++k) y -= x[rin[k]];
            y += B[n];
            Y[(size_t)m * N + n] = PRELU(y, a);
        }
    }
}

/* tcsc_sgemm_prelu_optimized_separate, tcsc.c:179-227: optimized, then a
 * separate PReLU pass. */
void oracle_sgemm_prelu_separate(const float *X, const int *csp, const int *csn,
                                 const int *rip, const int *rin, const float *B,
                                 float a, float *Y, int M, int N, int K) {
    optimized_core(X, csp, csn, rip, rin, B, Y, M, N, K, 0, 0.0f);
    for (size_t i = 0; i < (size_t)M * N; ++i) Y[i] = PRELU(Y[i], a);
}

/* tcsc_sgemm_prelu_optimized_onthego, tcsc.c:231-275. */
void oracle_sgemm_prelu_onthego(const float *X, const int *csp, const int *csn,
                                const int *rip, const int *rin, const float *B,
                                float a, float *Y, int M, int N, int K) {
    optimized_core(X, csp, csn, rip, rin, B, Y, M, N, K, 1, a);
}

/* sparseGEMM / sparseGEMM_PReLU, SparseGEMM.h:104-119,151-168: the
 * prelu_basic order (y=0; +P; -Q; +b), OpenMP over m.  This is the
 * multi-core CPU baseline; `threads` <= 0 keeps the OpenMP default.
 * prelu != 0 applies PReLU(a). */
void oracle_sparse_gemm_omp(const float *X, const int *csp, const int *csn,
                            const int *rip, const int *rin, const float *B,
                            float *Y, int M, int N, int K, int prelu, float a,
                            int threads) {
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(static)
#endif
    for (int m = 0; m < M; ++m) {
        const float *x = X + (size_t)m * K;
        for (int n = 0; n < N; ++n) {
            float y = 0.0f;
            for (int k = csp[n]; k < csp[n + 1]; ++k) y += x[rip[k]];
            for (int k = csn[n]; k < csn[n + 1]; ++k) y -= x[rin[k]];
            y = y + B[n];
            Y[(size_t)m * N + n] = prelu ? PRELU(y, a) : y;
        }
    }
}

int oracle_omp_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* gemm_basic, dense/dense.c:64-77: y=0; y += X*W over k; Y = y + B[n]. */
void oracle_gemm_basic(const float *X, const float *W, const float *B, float *Y,
                       int M, int N, int K) {
    for (int m = 0; m < M; m++)
        for (int n = 0; n < N; n++) {
            float y = 0.0f;
            for (int k = 0; k < K; k++) y += X[(size_t)m * K + k] * W[(size_t)k * N + n];
            Y[(size_t)m * N + n] = y + B[n];
        }
}

/* ---------------------------------------------------------------------- */
/* Exact reference for the tolerance test (not a reference function).       */
/* For each (m, n): y64 = b + sum_P x - sum_Q x in double, and the error     */
/* scale s = |b| + sum_{P u Q} |x| that bounds any fp32 summation order.     */
/* Rows are taken from `rows` (n_rows of them) so full-size problems can be  */
/* checked on a sample.                                                     */
/* ---------------------------------------------------------------------- */
void oracle_sgemm_f64_rows(const float *X, const int *csp, const int *csn,
                           const int *rip, const int *rin, const float *B,
                           const int *rows, int n_rows, double *Y64,
                           double *S64, int N, int K) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int r = 0; r < n_rows; ++r) {
        const float *x = X + (size_t)rows[r] * K;
        for (int n = 0; n < N; ++n) {
            double y = (double)B[n], s = fabs((double)B[n]);
            for (int k = csp[n]; k < csp[n + 1]; ++k) {
                y += (double)x[rip[k]];
                s += fabs((double)x[rip[k]]);
            }
            for (int k = csn[n]; k < csn[n + 1]; ++k) {
                y -= (double)x[rin[k]];
                s += fabs((double)x[rin[k]]);
            }
            Y64[(size_t)r * N + n] = y;
            S64[(size_t)r * N + n] = s;
        }
    }
}

/* ---------------------------------------------------------------------- */
/* Input generators (shared by tests, fixtures and bench).  SplitMix64 so   */
/* the stream is identical in C, numpy and on every host.                   */
/* Distributions follow dense/utils.h:9-16 (U[-1,1)) and :36-68 (ternary    */
/* with P(+1)=P(-1)=(1-s)/2).                                               */
/* ---------------------------------------------------------------------- */
static inline uint64_t splitmix64(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* x_i = 2*u - 1, u = top 24 bits / 2^24: exactly representable, in [-1,1). */
void oracle_fill_uniform(float *out, size_t n, uint64_t seed) {
    uint64_t s = seed;
    for (size_t i = 0; i < n; ++i) {
        uint32_t u = (uint32_t)(splitmix64(&s) >> 40);
        out[i] = (float)u * (1.0f / 8388608.0f) - 1.0f;
    }
}

/* Integer-valued floats in [-range, range] (SparseGEMM.h:42-51 style). */
void oracle_fill_int(float *out, size_t n, uint64_t seed, int range) {
    uint64_t s = seed;
    uint64_t span = (uint64_t)(2 * range + 1);
    for (size_t i = 0; i < n; ++i) out[i] = (float)((int64_t)(splitmix64(&s) % span) - range);
}

/* Ternary: density d = P(nonzero); u uniform in [0,1): u < d/2 -> +1,
 * u < d -> -1, else 0. */
void oracle_fill_ternary(float *out, size_t n, uint64_t seed, double density) {
    uint64_t s = seed;
    const double half = density * 0.5;
    for (size_t i = 0; i < n; ++i) {
        double u = (double)(splitmix64(&s) >> 11) * (1.0 / 9007199254740992.0);
        out[i] = (u < half) ? 1.0f : (u < density ? -1.0f : 0.0f);
    }
}
