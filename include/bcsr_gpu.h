/*
 * bcsr_gpu.h -- device-pointer API of the BCSR path (the counterpart of
 * tcsc_gpu.h for sparse/bcsr.h).  Plain C ABI; streams are `void*`
 * (hipStream_t, NULL = null stream); status codes and the error message are
 * the ones of tcsc_gpu.h (TCSC_OK, ..., tcsc_gpu_last_error()).
 *
 * A plan is the device image of one bcsr_t, re-indexed by block column: for
 * every block column, the stored blocks in the order the reference visits
 * them (block row ascending, then block index: bcsr.c:156-160), which is the
 * accumulation order of every output element of that column.
 */
#ifndef TCSC_AMD_BCSR_GPU_H
#define TCSC_AMD_BCSR_GPU_H

#include <stddef.h>
#include "sparse/bcsr.h"
#include "tcsc_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Which reference entry point a launch stands in for. */
enum bcsr_variant {
    BCSR_VARIANT_BASIC = 0,        /* bcsr_sgemm_basic        bcsr.c:141 */
    BCSR_VARIANT_PRELU_BASIC = 1,  /* bcsr_sgemm_prelu_basic  bcsr.c:177 */
    BCSR_VARIANT_AVX = 2,          /* bcsr_sgemm_avx          bcsr.c:222 (c == 8) */
    BCSR_VARIANT_PRELU_AVX = 3,    /* bcsr_sgemm_prelu_avx    bcsr.c:264 (c == 8) */
    BCSR_VARIANT_AVX2 = 4          /* bcsr_sgemm_avx2         bcsr.c:316 (r == c == 8) */
};

typedef struct bcsr_gpu_plan bcsr_gpu_plan;

/* Upload W to `device` and build the plan (host-side re-indexing, then the
 * copies on `stream`; returns after they completed).  TCSC_E_ARG when W's
 * arrays index outside W (block index >= k or block column >= bc). */
int bcsr_gpu_plan_create(const bcsr_t *W, int device, void *stream, bcsr_gpu_plan **out);

/* Blocks visited per output column group, summed over block columns
 * (== W.k for a well-formed W), and the HBM the plan holds. */
int bcsr_gpu_plan_stats(const bcsr_gpu_plan *plan, long long *block_visits, size_t *device_bytes);

/* Allocate the workspace (X^T, K x M rounded up to 256) for launches of up
 * to max_M rows of a K-column X; bcsr_gpu_sgemm grows it itself otherwise
 * (that call then allocates and synchronises). */
int bcsr_gpu_plan_reserve(bcsr_gpu_plan *plan, int max_M, int K);
void bcsr_gpu_plan_destroy(bcsr_gpu_plan *plan);

/* Y = the reference variant's result for X (M x K row-major), B (N floats),
 * Y (M rows of pitch ldy >= N).  Needs N >= W.bc*W.c and K >= W.br*W.r
 * (the reference's indexing, bcsr.c:169).  Asynchronous on `stream`. */
int bcsr_gpu_sgemm(const bcsr_gpu_plan *plan, const float *dX, const float *dB, float *dY,
                   int M, int N, int K, int ldy, int variant, float a, void *stream);

/* The two halves of bcsr_gpu_sgemm: stage X^T (k_transpose), then run the
 * block kernel (k_bcsr) on the staged X^T of the same M and K. */
int bcsr_gpu_prepare_x(const bcsr_gpu_plan *plan, const float *dX, int M, int K, void *stream);
int bcsr_gpu_sgemm_prepared(const bcsr_gpu_plan *plan, const float *dB, float *dY, int M, int N, int K,
                            int ldy, int variant, float a, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* TCSC_AMD_BCSR_GPU_H */
