/*
 * sparse/tcsc.h -- drop-in replacement for the reference's TCSC operator API.
 *
 * Replaces /root/reference/sparse/tcsc.h (whole file) and the CPU bodies in
 * /root/reference/sparse/tcsc.c.  Every entry point keeps the reference's
 * name, argument order and meaning, so the reference's main.cpp compiles
 * against this header unchanged and links against libtcsc_amd.so:
 *
 *   tcsc_t                                  <- sparse/tcsc.h:6-17 (same field order/types)
 *   tcsc_from_dense                          <- sparse/tcsc.h:19, tcsc.c:6-66
 *   tcsc_sgemm_basic                         <- sparse/tcsc.h:21-24, tcsc.c:69-98
 *   tcsc_sgemm_optimized                     <- sparse/tcsc.h:26-29, tcsc.c:101-140
 *   tcsc_sgemm_prelu_basic                   <- sparse/tcsc.h:31-34, tcsc.c:143-165
 *   tcsc_sgemm_prelu_optimized_separate      <- sparse/tcsc.h:36-40, tcsc.c:179-227
 *   tcsc_sgemm_prelu_optimized_onthego       <- sparse/tcsc.h:42-46, tcsc.c:231-275
 *   tcsc_free                                <- sparse/tcsc.h:48, tcsc.c:167-175
 *
 * Semantics kept from the reference:
 *   - X is M x K row-major, Y is M x N row-major, B has N entries; the
 *     argument order is (M, N, K) (main.cpp:314).
 *   - W is K x N ternary; col_start_* have cols+1 entries and the row indices
 *     inside a column are ascending (tcsc.c:48-60).
 *   - Y is fully overwritten; the kernels return nothing (no error channel in
 *     the signature).
 *
 * What changes underneath: the five tcsc_sgemm_* entry points run the
 * hand-written gfx950 (MI355X) HIP kernels.  W is uploaded once per tcsc_t
 * and cached on every GPU used (the cache entry dies in tcsc_free); X and B
 * are copied host->device per call and Y is copied back.  With more than one
 * GPU visible the output columns are split into contiguous blocks, one per
 * GPU, with no collective: every GPU receives X, and its block is copied
 * straight into its columns of Y (TCSC_SHARD_AXIS=rows splits the rows of
 * X and Y instead, each GPU holding a plan of the whole W).
 * HIP failures are reported on stderr and through tcsc_gpu_last_error()
 * (include/tcsc_gpu.h) and then abort the process unless
 * TCSC_ON_ERROR=continue is set.
 */
#ifndef TCSC_AMD_TCSC_H
#define TCSC_AMD_TCSC_H

#include "../dense/dense.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int rows, cols;       /* K and N */
    int n_elem_pos;       /* number of +1 entries */
    int n_elem_neg;       /* number of -1 entries */
    int *col_start_pos;   /* cols+1 offsets into row_index_pos */
    int *col_start_neg;   /* cols+1 offsets into row_index_neg */
    int *row_index_pos;   /* n_elem_pos row indices, ascending per column */
    int *row_index_neg;   /* n_elem_neg row indices, ascending per column */
} tcsc_t;

/* Dense row-major rows x cols float matrix -> TCSC.  Only values that compare
 * equal to +1.0f / -1.0f are stored, everything else counts as zero
 * (tcsc.c:14-17,54-58).  Returns NULL on allocation failure. */
tcsc_t *tcsc_from_dense(dense_t dense, int rows, int cols);

void tcsc_sgemm_basic(const dense_t X, const tcsc_t *W, const dense_t B,
                      dense_t Y, int M, int N, int K);

void tcsc_sgemm_optimized(const dense_t X, const tcsc_t *W, const dense_t B,
                          dense_t Y, int M, int N, int K);

void tcsc_sgemm_prelu_basic(const dense_t X, const tcsc_t *W, const dense_t B,
                            float a, dense_t Y, int M, int N, int K);

void tcsc_sgemm_prelu_optimized_separate(const dense_t X, const tcsc_t *W,
                                         const dense_t B, float a, dense_t Y,
                                         int M, int N, int K);

void tcsc_sgemm_prelu_optimized_onthego(const dense_t X, const tcsc_t *W,
                                        const dense_t B, float a, dense_t Y,
                                        int M, int N, int K);

void tcsc_free(tcsc_t *W);

#ifdef __cplusplus
}
#endif

#endif /* TCSC_AMD_TCSC_H */
