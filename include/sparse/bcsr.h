/*
 * sparse/bcsr.h -- BCSR operator API, source- and
 * link-compatible with the reference's sparse/bcsr.h:1-39.  DESIGN.md "BCSR"
 * has the semantics kept from sparse/bcsr.c and what runs on the GPU.
 */
#ifndef TCSC_AMD_BCSR_H
#define TCSC_AMD_BCSR_H

#include "../dense/dense.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef float bcsr_elem_t;

/* sparse/bcsr.h:7-12, same field order and types */
typedef struct {
    int r, c;             /* block rows / block columns (elements)           */
    int br, bc;           /* rows / r and cols / c (blocks)                  */
    int k;                /* stored blocks                                   */
    int *b_row_start;     /* br+1 entries                                    */
    int *b_col_idx;       /* k block-column indices                          */
    bcsr_elem_t *b_values;/* k * r * c values, block-major, row-major inside */
} bcsr_t;

/* bcsr.c:19-139.  NULL for r < 1, c < 1 or allocation failure. */
bcsr_t *bcsr_from_dense(dense_t dense, int rows, int cols, int r, int c);

/* bcsr.c:141-175 */
void bcsr_sgemm_basic(const dense_t X, const bcsr_t W, const dense_t B,
                      dense_t Y, int M, int N, int K);

/* bcsr.c:177-218 */
void bcsr_sgemm_prelu_basic(const dense_t X, const bcsr_t W, const dense_t B,
                            float a, dense_t Y, int M, int N, int K);

/* bcsr.c:222-261 (needs c == 8) */
void bcsr_sgemm_avx(const dense_t X, const bcsr_t W, const dense_t B,
                    dense_t Y, int M, int N, int K);

/* bcsr.c:264-312 (needs c == 8) */
void bcsr_sgemm_prelu_avx(const dense_t X, const bcsr_t W, const dense_t B,
                          float a, dense_t Y, int M, int N, int K);

/* bcsr.c:316-385 (needs r == c == 8) */
void bcsr_sgemm_avx2(const dense_t X, const bcsr_t W, const dense_t B,
                     dense_t Y, int M, int N, int K);

/* Extension: frees the three arrays and the struct. */
void bcsr_free(bcsr_t *W);

#ifdef __cplusplus
}
#endif

#endif /* TCSC_AMD_BCSR_H */
