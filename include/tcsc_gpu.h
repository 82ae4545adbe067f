/*
 * tcsc_gpu.h -- device-pointer extension of the TCSC drop-in API.
 *
 * The reference's API (sparse/tcsc.h:19-48) only takes host pointers and is
 * synchronous, so a call through it always pays PCIe transfers.  These entry
 * points expose the same computation on device-resident buffers, on a caller
 * supplied HIP stream, so that kernel-only throughput can be measured and so
 * that one process per GPU (torch.distributed ranks, MPI ranks, ...) can run
 * its own column shard.  Plain C ABI: no HIP or torch types in the
 * signatures; streams are passed as `void*` (a hipStream_t, NULL = the
 * device's null stream).
 *
 * A plan is the device-side image of (a column range of) one tcsc_t,
 * re-laid out for the gfx950 gather kernel ("Data layout in
 * HBM").  Building a plan is the only place W's index arrays cross PCIe.
 */
#ifndef TCSC_AMD_TCSC_GPU_H
#define TCSC_AMD_TCSC_GPU_H

#include <stddef.h>
#include "sparse/tcsc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Which reference entry point a launch stands in for.  The GPU computes all
 * of them with one kernel family; the variant only selects the epilogue
 * (PReLU or not).  See DESIGN.md "Numerics" for the summation order. */
enum tcsc_variant {
    TCSC_VARIANT_BASIC = 0,            /* tcsc_sgemm_basic                    tcsc.c:69  */
    TCSC_VARIANT_OPTIMIZED = 1,        /* tcsc_sgemm_optimized                tcsc.c:101 */
    TCSC_VARIANT_PRELU_BASIC = 2,      /* tcsc_sgemm_prelu_basic              tcsc.c:143 */
    TCSC_VARIANT_PRELU_SEPARATE = 3,   /* tcsc_sgemm_prelu_optimized_separate tcsc.c:179 */
    TCSC_VARIANT_PRELU_ONTHEGO = 4,    /* tcsc_sgemm_prelu_optimized_onthego  tcsc.c:231 */
    TCSC_VARIANT_SPARSE_GEMM = 5       /* sparseGEMM<float>          SparseGEMM.h:104-119:
                                          y = 0 + sum(+1 rows) - sum(-1 rows); Y = y + b.
                                          sparseGEMM_PReLU<float> (SparseGEMM.h:151-168)
                                          is TCSC_VARIANT_PRELU_BASIC: the same order
                                          as tcsc.c:143-165, the same predicate     */
};

/* Status codes (0 = success).  HIP errors are passed through as
 * TCSC_E_HIP; the message is in tcsc_gpu_last_error(). */
enum tcsc_status {
    TCSC_OK = 0,
    TCSC_E_ARG = 1,      /* bad argument (shape mismatch, NULL, range)   */
    TCSC_E_HIP = 2,      /* a HIP runtime call failed                     */
    TCSC_E_NOMEM = 3,    /* host or device allocation failed              */
    TCSC_E_NODEV = 4     /* no usable gfx950 device                       */
};

/* Summation order of the gather.  FAST (default): each output column adds
 * its +1 and -1 rows merged in ascending k; the five variants then agree with
 * the reference within the fp32 bound of DESIGN.md "Numerics" and bit for bit
 * on integer-valued inputs.  REFERENCE: the order of each reference variant
 * (tcsc.c:84-93 for basic, :149-161 prelu_basic, :113-137 the optimized
 * family), so float outputs are bit-identical to the reference compiled with
 * IEEE semantics, at about twice the kernel time (K is walked once per
 * sign).  Chosen per plan at creation time (tcsc_gpu_set_order, or
 * TCSC_ORDER=reference in the environment). */
enum tcsc_order {
    TCSC_ORDER_FAST = 0,
    TCSC_ORDER_REFERENCE = 1
};

typedef struct tcsc_gpu_plan tcsc_gpu_plan;

typedef struct {
    int device;          /* HIP device ordinal the plan lives on          */
    int rows;            /* K                                             */
    int cols;            /* columns in this plan (col_end - col_begin)    */
    int col_begin;       /* first column of W covered                     */
    long long nnz;       /* +1 and -1 entries in the covered columns      */
    long long n_pos, n_neg;
    int chunk_k;         /* K rows per LDS chunk used by the kernel       */
    int n_chunks;        /* ceil(K / chunk_k)                             */
    size_t device_bytes; /* HBM held by the plan                          */
    int order;           /* enum tcsc_order the plan was built for        */
    int mfma_min_M;      /* > 0: the plan holds the MFMA image of W (denser
                            W, see tcsc_gpu_sgemm) and launches with
                            M >= mfma_min_M may use it (the cost model;
                            tcsc_gpu_launch_info says which path a given
                            M takes); 0: gather only                      */
} tcsc_gpu_plan_info;

/* Number of HIP devices visible (0 when there is no GPU). */
int tcsc_gpu_device_count(void);

/* Summation order for plans created from now on, including the plans the
 * host-pointer API (sparse/tcsc.h) builds for its cache (a cached tcsc_t is
 * rebuilt when the order changes).  Process-wide; default from $TCSC_ORDER. */
void tcsc_gpu_set_order(int order);
int tcsc_gpu_get_order(void);

/* Upload columns [col_begin, col_end) of W to `device` and build the plan.
 * W is read on the host; `stream` orders the uploads and the build kernels.
 * The call returns after the plan is complete (it synchronises `stream`). */
int tcsc_gpu_plan_create(const tcsc_t *W, int col_begin, int col_end,
                         int device, void *stream, tcsc_gpu_plan **out);

/* Same, from raw TCSC arrays that already live on `device` (the layout of
 * tcsc_t: col_start_* have cols+1 entries, absolute offsets).  Nothing
 * crosses PCIe. */
int tcsc_gpu_plan_create_device(int rows, int cols,
                                const int *d_col_start_pos,
                                const int *d_col_start_neg,
                                const int *d_row_index_pos,
                                const int *d_row_index_neg,
                                int col_begin, int col_end, int device,
                                void *stream, tcsc_gpu_plan **out);

int tcsc_gpu_plan_get_info(const tcsc_gpu_plan *plan, tcsc_gpu_plan_info *info);

/* Which kernels a tcsc_gpu_sgemm of M rows on this plan runs (with X 16-B
 * aligned, the plan's reserved workspace and the current environment):
 *   TCSC_PATH_GATHER k_transpose + k_stream (+ k_reduce, or the in-launch
 *                    combine: tcsc_gpu_launch_combine)
 *   TCSC_PATH_MFMA   k_split3 + k_gemm3 + k_fixup, or with K split
 *                    k_split3 + k_gemm3 + k_reduce_fix (the slabs and the
 *                    fixup in one kernel), denser W (the cost model)
 *   TCSC_PATH_SMALL  k_small_m, M <= 4 (X and -X fit the LDS)
 * and *slices = the K split (1 = none): the gather's, or the MFMA GEMM's on
 * grids of few 128 x 128 tiles (M <= 256 at N = 8192: partial sums of whole
 * 64-k blocks, added in slice order). */
enum tcsc_path {
    TCSC_PATH_GATHER = 0,
    TCSC_PATH_FUSED = 1, /* retired (round 5): the persistent k_fused left the library; never returned */
    TCSC_PATH_MFMA = 2,
    TCSC_PATH_SMALL = 3
};
int tcsc_gpu_launch_info(const tcsc_gpu_plan *plan, int M, int *path, int *slices);

/* For TCSC_PATH_GATHER with a K split, where the split-K slabs are combined
 * (N % 4 == 0 and the plan's reserved workspace needed for either in-launch
 * form; TCSC_COMBINE=0 turns both off, =1 lifts the band form's size rule):
 *   4  inside the k_stream launch, pairwise in split halves (exactly 2
 *      slices, the grid fits the chip at one workgroup per CU: each slice
 *      stores half its partial and finalizes the other half)
 *   3  inside the k_stream launch, pairwise (exactly 2 slices: the tile's
 *      first slice to finish stores its slab, the second combines; any grid)
 *   2  inside the k_stream launch, by row bands (>= 3 slices, the grid fits
 *      the chip at one workgroup per CU, >= 64 workgroups)
 *   0  by k_reduce after it, or nothing is split.
 * Y and bias are assumed 16-B aligned with ldy = N; otherwise the launch
 * uses k_reduce. */
int tcsc_gpu_launch_combine(const tcsc_gpu_plan *plan, int M, int *in_launch);

/* Allocate the plan's workspace for launches of up to `max_M` rows: X^T
 * (K x max_M rounded up to 256 floats; the kernel streams X^T rows into LDS)
 * plus, where the gather's cost model or the MFMA GEMM's grid splits K over
 * workgroups, the fp32 partial slabs combined in a fixed order.  Optional: tcsc_gpu_sgemm grows the
 * workspace itself on the first call with a larger M (that call then
 * allocates and synchronises the device); reserving up front keeps every
 * sgemm call allocation-free.  Not thread-safe against concurrent launches
 * of the same plan. */
int tcsc_gpu_plan_reserve(tcsc_gpu_plan *plan, int max_M);
void tcsc_gpu_plan_destroy(tcsc_gpu_plan *plan);

/* Y[m, j] = act(B[j] + sum_{k in P(j)} X[m,k] - sum_{k in Q(j)} X[m,k])
 * for m < M and the plan's columns j < cols.
 *   dX : M x K row-major device array (K = plan rows), 4-byte aligned
 *   dB : `cols` floats (the plan's slice of the bias)
 *   dY : M rows with pitch `ldy` floats (ldy >= cols); columns beyond
 *        `cols` are not touched
 *   act: PReLU(v) = (v < 0 ? a*v : v) for the PRELU variants, identity
 *        otherwise.
 *   M  : any; the gather path runs more than 2^22 rows as several
 *        launches (offsets are 64-bit, so M*K may exceed 2^31).
 * Asynchronous on `stream`; once the workspace covers M (see
 * tcsc_gpu_plan_reserve) no allocation and no synchronisation (safe to
 * capture in a hipGraph).
 * Denser W (density >= 0.055, see tcsc_gpu_plan_info.mfma_min_M): launches
 * with M >= mfma_min_M run the MFMA path where a per-launch cost model says
 * it beats the gather (measured crossover ~0.08 at M >= 2048, ~0.04-0.1 at
 * M <= 256 for K = N = 8192, lower for smaller K and N) -- X
 * split exactly into three bf16 parts (k_split3) and one bf16 GEMM with fp32
 * accumulation against the plan's bf16 image of W on the matrix cores
 * (k_gemm3, the library's own gfx950 kernel, bias and PReLU fused in its
 * store; a grid with fewer tiles than the chip runs at once splits K into
 * slices of whole 64-k blocks whose partial sums k_reduce_fix adds in slice
 * order with the bias and PReLU), then the exact fixup of
 * rows holding non-finite or tiny values (k_fixup) -- with the same accuracy
 * bounds as the gather.  It allocates nothing per launch and
 * keeps no state between launches, so graph replays with new X are exact.
 * $TCSC_PATH=gather|mfma at plan creation disables / forces the path (the
 * image is never built for K of ~2.8 M rows or more: k_gemm3's staging
 * offsets are 32-bit; the gather serves those plans).
 * Thread safety: concurrent launches of ONE plan (on any streams) share its
 * workspace and are not supported; different plans are independent. */
int tcsc_gpu_sgemm(const tcsc_gpu_plan *plan, const float *dX, const float *dB,
                   float *dY, int M, int ldy, int variant, float a,
                   void *stream);

/* The two halves of tcsc_gpu_sgemm, for callers that time them apart or
 * reuse one staging of X for several launches of the same plan:
 * tcsc_gpu_prepare_x writes X (M x K) transposed into the plan's workspace
 * (kernel k_transpose); tcsc_gpu_sgemm_prepared then runs the gather
 * (k_stream, plus k_reduce when K is split) on that staged X for the same
 * M.  Same stream semantics as tcsc_gpu_sgemm. */
int tcsc_gpu_prepare_x(const tcsc_gpu_plan *plan, const float *dX, int M, void *stream);
int tcsc_gpu_sgemm_prepared(const tcsc_gpu_plan *plan, const float *dB, float *dY, int M, int ldy,
                            int variant, float a, void *stream);

/* Device-side tcsc_from_dense: dense K x N row-major float matrix on the
 * device -> TCSC arrays on the device, bit-exact with the reference builder
 * (tcsc.c:6-66).  Two calls: first with the four output pointers NULL to
 * get n_pos / n_neg (col_start arrays are still written), then with the
 * index arrays allocated.  The matrix must not change between the two calls
 * of a pair (the second call reuses the first call's per-tile counts when it
 * follows it directly with the same matrix, shape and col_start arrays; the
 * index arrays are never written past the counted sizes either way).
 * Synchronises `stream`. */
int tcsc_gpu_from_dense(const float *d_dense, int rows, int cols,
                        int *d_col_start_pos, int *d_col_start_neg,
                        int *d_row_index_pos, int *d_row_index_neg,
                        int *n_pos, int *n_neg, void *stream);

/* Dense baseline, the device counterpart of the
 * reference's gemm_basic (dense/dense.c:64-77) that the harness times for
 * its "TCSC vs Dense" line (main.cpp:379-391):
 *   Y[m, n] = act(sum_k X[m,k] * W[k,n] + B[n])
 * with W the DENSE K x N row-major float matrix (the ternary W before
 * tcsc_from_dense), computed as an fp32 rocBLAS SGEMM plus a bias/PReLU
 * epilogue kernel.  act as in tcsc_gpu_sgemm (PReLU for the PRELU
 * variants).  dX: M x K row-major; dY: M rows of pitch ldy >= N.
 * Asynchronous on `stream`. */
int tcsc_gpu_dense_sgemm(const float *dX, const float *dW, const float *dB,
                         float *dY, int M, int N, int K, int ldy, int variant,
                         float a, void *stream);

/* Message for the last failing call on this thread ("" if none). */
const char *tcsc_gpu_last_error(void);

/* Drop every device copy the host-pointer API cached (all tcsc_t's). */
void tcsc_gpu_cache_clear(void);

/* Number of GPUs the host-pointer API (sparse/tcsc.h) spreads columns over:
 * min(visible devices, $TCSC_NUM_GPUS if set).  `tcsc_gpu_set_num_shards`
 * overrides the count of column blocks (blocks are dealt round-robin over
 * the devices; >devices is allowed and is how the multi-block path is
 * exercised on a single GPU). 0 restores the default. */
int tcsc_gpu_num_shards(void);
void tcsc_gpu_set_num_shards(int shards);

/* The host-pointer API (sparse/tcsc.h, include/sparse_gemm.h) runs in EXACT
 * mode by default: every call sums each output in dense.c gemm_basic's order
 * (y = 0; y += X*W over ascending k; y += B; then the PReLU for the PReLU
 * variants) -- the fast order with K never split, never the MFMA path -- so
 * its outputs equal the reference harness's own oracle bit for bit
 * (main.cpp:307-366 checks tcsc_sgemm_basic / _optimized against it with an
 * absolute 1e-4).  $TCSC_HOST_FAST=1 (read per call) lets host calls take the
 * device API's fastest paths instead (MFMA, split K): within the fp32 bound
 * of the exact sums, not bit-equal to gemm_basic. */

/* Diagnostic build flags of the loaded library: 0 for the product build;
 * bits 1 TCSC_ABLATION, 2 TCSC_NODMA, 4 TCSC_STAMPS, 8 TCSC_TRACE (timing-only
 * builds of tools/ab.mk whose outputs are wrong by design). */
int tcsc_gpu_build_flags(void);

#ifdef __cplusplus
}
#endif

#endif /* TCSC_AMD_TCSC_GPU_H */
