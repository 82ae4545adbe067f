/*
 * ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.  C-linkage wrappers around the
 * UNMODIFIED reference sources so Python (ctypes) can call them.  Built by
 * oracle/Makefile into oracle/_ref/libtcsc_ref.so together with
 *   /root/reference/sparse/tcsc.c   (compiled in place, as C++, like the
 *   /root/reference/dense/dense.c    reference's own build does)
 * Nothing from /root/reference is copied: the headers are included by
 * absolute path and the sources are compiled where they lie.
 *
 * The reference symbols are C++-mangled (it is built with g++,
 * SURVEY.md §8b), hence this shim.
 */
#include "/root/reference/sparse/tcsc.h"
#include "/root/reference/SparseGEMM.h"

extern "C" {

/* tcsc_from_dense (tcsc.c:6-66), copied out into caller arrays. */
int ref_tcsc_from_dense(const float *dense, int rows, int cols, int *csp,
                        int *csn, int *rip, int *rin, int *n_pos, int *n_neg,
                        int query_only) {
    tcsc_t *t = tcsc_from_dense(const_cast<float *>(dense), rows, cols);
    if (!t) return -1;
    *n_pos = t->n_elem_pos;
    *n_neg = t->n_elem_neg;
    if (!query_only) {
        for (int j = 0; j <= cols; ++j) {
            csp[j] = t->col_start_pos[j];
            csn[j] = t->col_start_neg[j];
        }
        for (int i = 0; i < t->n_elem_pos; ++i) rip[i] = t->row_index_pos[i];
        for (int i = 0; i < t->n_elem_neg; ++i) rin[i] = t->row_index_neg[i];
    }
    tcsc_free(t);
    return 0;
}

static tcsc_t wrap(int K, int N, int *csp, int *csn, int *rip, int *rin) {
    tcsc_t t;
    t.rows = K;
    t.cols = N;
    t.n_elem_pos = csp[N];
    t.n_elem_neg = csn[N];
    t.col_start_pos = csp;
    t.col_start_neg = csn;
    t.row_index_pos = rip;
    t.row_index_neg = rin;
    return t;
}

/* variant: 0 basic, 1 optimized, 2 prelu_basic, 3 prelu_separate,
 * 4 prelu_onthego (the five tcsc_sgemm_* of tcsc.h:21-46). */
void ref_tcsc_sgemm(int variant, float *X, int *csp, int *csn, int *rip,
                    int *rin, float *B, float a, float *Y, int M, int N,
                    int K) {
    tcsc_t t = wrap(K, N, csp, csn, rip, rin);
    switch (variant) {
    case 0: tcsc_sgemm_basic(X, &t, B, Y, M, N, K); break;
    case 1: tcsc_sgemm_optimized(X, &t, B, Y, M, N, K); break;
    case 2: tcsc_sgemm_prelu_basic(X, &t, B, a, Y, M, N, K); break;
    case 3: tcsc_sgemm_prelu_optimized_separate(X, &t, B, a, Y, M, N, K); break;
    case 4: tcsc_sgemm_prelu_optimized_onthego(X, &t, B, a, Y, M, N, K); break;
    default: break;
    }
}

/* gemm_basic (dense/dense.c:64-77). */
void ref_gemm_basic(float *X, float *W, float *B, float *Y, int M, int N, int K) {
    gemm_basic(X, W, B, Y, M, N, K);
}

/* compare (dense/dense.c:42-59): 1 = equal within 1e-4. */
int ref_compare(float *res, float *tar, int rows, int cols) {
    return compare(res, tar, rows, cols) ? 1 : 0;
}

/* SparseFormat (SparseGEMM.h:13-40) on an int matrix. */
void ref_sparseformat(int *matrix, int K, int N, int *csp, int *csn, int *rip,
                      int *rin, int *n_pos, int *n_neg) {
    SparseFormat f(matrix, K, N);
    for (int j = 0; j <= N; ++j) {
        csp[j] = f.col_start_pos[j];
        csn[j] = f.col_start_neg[j];
    }
    for (size_t i = 0; i < f.row_index_pos.size(); ++i) rip[i] = f.row_index_pos[i];
    for (size_t i = 0; i < f.row_index_neg.size(); ++i) rin[i] = f.row_index_neg[i];
    *n_pos = (int)f.row_index_pos.size();
    *n_neg = (int)f.row_index_neg.size();
}

/* sparseGEMM / sparseGEMM_PReLU (SparseGEMM.h:104-119,151-168). */
void ref_sparse_gemm(float *X, int *csp, int *csn, int *rip, int *rin, float *B,
                     float *Y, int M, int N, int K, int prelu, float a) {
    if (prelu)
        sparseGEMM_PReLU<float>(X, csp, csn, rip, rin, B, Y, M, N, K, a);
    else
        sparseGEMM<float>(X, csp, csn, rip, rin, B, Y, M, N, K);
}

/* GEMM_PReLU (SparseGEMM.h:135-149) -- the only dense PReLU oracle the
 * reference defines. */
void ref_gemm_prelu(float *X, float *W, float *B, float *Y, int M, int N, int K,
                    float a) {
    GEMM_PReLU<float>(X, W, B, Y, M, N, K, a);
}

} /* extern "C" */
