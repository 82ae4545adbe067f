/*
 * ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.  C-linkage wrappers around the
 * UNMODIFIED reference sources so Python (ctypes) can call them.  Built by
 * oracle/Makefile into oracle/_ref/libtcsc_ref.so together with
 *   /root/reference/sparse/tcsc.c   (compiled in place, as C++, like the
 *   /root/reference/dense/dense.c    reference's own build does)
 *   /root/reference/sparse/bcsr.c   (-mavx2 -mfma: it uses AVX2/FMA intrinsics)
 * Nothing from /root/reference is copied: the headers are included by
 * absolute path and the sources are compiled where they lie.
 *
 * The reference symbols are C++-mangled (it is built with g++,
 * SURVEY.md §8b), hence this shim.
 */
#include "/root/reference/sparse/tcsc.h"
#include "/root/reference/sparse/bcsr.h"
#include "/root/reference/SparseGEMM.h"

#include <cstdlib>
#include <cstring>

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

/* bcsr_from_dense (bcsr.c:19-139), copied out.  The reference writes
 * b_row_start only for non-empty block rows plus the final k
 * (bcsr.c:114-117,137) and leaves the rest of its br+1 entries
 * uninitialised: *written = that count; the rest is returned as k.  The
 * count is derived from the dense input with the reference's predicate
 * (bcsr.c:62). */
int ref_bcsr_from_dense(const float *dense, int rows, int cols, int r, int c, int *rs, int *ci, float *vals,
                        int *k, int *written, int query_only) {
    bcsr_t *W = bcsr_from_dense(const_cast<float *>(dense), rows, cols, r, c);
    if (!W) return -1;
    int ne = 0;
    for (int a = 0; a < W->br; ++a) {
        int any = 0;
        for (int i = 0; i < r && !any; ++i)
            for (int j = 0; j < W->bc * c && !any; ++j) {
                float v = dense[(size_t)(a * r + i) * cols + j];
                any = (v == -1.0 || v == 1.0);
            }
        ne += any;
    }
    *k = W->k;
    *written = ne + 1;
    if (!query_only) {
        for (int i = 0; i <= W->br; ++i) rs[i] = i <= ne ? W->b_row_start[i] : W->k;
        for (int i = 0; i < W->k; ++i) ci[i] = W->b_col_idx[i];
        std::memcpy(vals, W->b_values, (size_t)W->k * r * c * sizeof(float));
    }
    free(W->b_values);
    free(W->b_row_start);
    free(W->b_col_idx);
    free(W);
    return 0;
}

static void *aligned32(size_t bytes) {
    void *p = nullptr;
    if (posix_memalign(&p, 32, (bytes + 31) / 32 * 32 + 32) != 0) return nullptr;
    std::memset(p, 0, (bytes + 31) / 32 * 32 + 32);
    return p;
}

/* variant: 0 basic, 1 prelu_basic, 2 avx, 3 prelu_avx, 4 avx2 (bcsr.h:16-39).
 * The avx variants use aligned 8-float loads/stores of B, Y and the values
 * (bcsr.c:229-230, 250-256): every buffer handed to them is a 32-B aligned
 * copy padded to whole 8-float groups (they are only called with N % 8 == 0
 * and c == 8 here, so the padding is never read into a result). */
void ref_bcsr_sgemm(int variant, float *X, int r, int c, int nbr, int nbc, int k, int *rs, int *ci, float *vals,
                    float *B, float a, float *Y, int M, int N, int K) {
    bcsr_t W;
    W.r = r;
    W.c = c;
    W.br = nbr;
    W.bc = nbc;
    W.k = k;
    W.b_row_start = static_cast<int *>(aligned32((size_t)(nbr + 1) * sizeof(int)));
    W.b_col_idx = static_cast<int *>(aligned32((size_t)k * sizeof(int)));
    W.b_values = static_cast<float *>(aligned32((size_t)k * r * c * sizeof(float)));
    std::memcpy(W.b_row_start, rs, (size_t)(nbr + 1) * sizeof(int));
    std::memcpy(W.b_col_idx, ci, (size_t)k * sizeof(int));
    std::memcpy(W.b_values, vals, (size_t)k * r * c * sizeof(float));
    float *Bp = static_cast<float *>(aligned32((size_t)N * sizeof(float)));
    float *Yp = static_cast<float *>(aligned32((size_t)M * N * sizeof(float)));
    std::memcpy(Bp, B, (size_t)N * sizeof(float));
    switch (variant) {
    case 0: bcsr_sgemm_basic(X, W, Bp, Yp, M, N, K); break;
    case 1: bcsr_sgemm_prelu_basic(X, W, Bp, a, Yp, M, N, K); break;
    case 2: bcsr_sgemm_avx(X, W, Bp, Yp, M, N, K); break;
    case 3: bcsr_sgemm_prelu_avx(X, W, Bp, a, Yp, M, N, K); break;
    case 4: bcsr_sgemm_avx2(X, W, Bp, Yp, M, N, K); break;
    default: break;
    }
    std::memcpy(Y, Yp, (size_t)M * N * sizeof(float));
    free(W.b_row_start);
    free(W.b_col_idx);
    free(W.b_values);
    free(Bp);
    free(Yp);
}

} /* extern "C" */
