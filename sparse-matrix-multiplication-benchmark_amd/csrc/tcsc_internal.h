// tcsc_internal.h -- shared between the kernels (tcsc_kernels.hip) and the
// C-ABI layer (tcsc_api.cpp).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace tcsc {

// ---- geometry of the gather kernel (DESIGN.md "Kernel K1") ---------------
constexpr int kTM = 256;                 // rows per workgroup: 64 lanes x 4 rows (ds_read_b128)
#ifndef TCSC_TK
#define TCSC_TK 48
#endif
#ifndef TCSC_NBUF
#define TCSC_NBUF 3
#endif
constexpr int kTK = TCSC_TK;             // K rows per LDS chunk
constexpr int kNBuf = TCSC_NBUF;         // LDS tile ring: chunk c in buffer c % kNBuf, kNBuf-1 chunks in flight
constexpr int kRowBytes = kTM * 4;       // one LDS row = X[m0..m0+255][k], 1 KiB
constexpr int kBufRows = kTK + 1;        // + one row of -0.0 that padding entries point at
// Gather geometry (tools/gen_gather_asm.py generates the matching loop):
#ifndef TCSC_WAVES
#define TCSC_WAVES 16
#endif
#ifndef TCSC_CW
#define TCSC_CW 16
#endif
#ifndef TCSC_BATCH
#define TCSC_BATCH 4
#endif
constexpr int kWaves = TCSC_WAVES;       // waves per workgroup (1 workgroup per CU; kWaves/4 per SIMD)
constexpr int kCW = TCSC_CW;             // most output columns of one wave (4*kCW accumulator VGPRs)
constexpr int kBatch = TCSC_BATCH;       // stream entries per batch (pipeline step, stream padding)
constexpr int kWavesPerSimd = kWaves / 4;
static_assert(kWaves % 4 == 0 && kWaves <= 16, "whole waves per SIMD");

// Output columns per wave, by the wave's age rank on its SIMD (waves 4r ..
// 4r+3 have rank r; one wave of every rank runs on each SIMD).  The SIMD's
// instruction arbiter favours older waves: with equal shares the youngest
// rank finishes its gather last (tools/stamps.py: gather cycles per chunk
// 835 / 967 / 1330 / 1600 by rank at cfg 4).  Unequal shares were measured
// slower in either direction (make lib/wid/libtcsc_amd_wd<A>_<B>_<C>_<D>.so,
// DESIGN.md §4), so the default is equal.  Multiples of 4 (16-B epilogue
// stores), at most kCW.
#ifndef TCSC_WIDTHS
#define TCSC_WIDTHS 16, 16, 16, 16
#endif
struct ColLayout {
    int w[kWavesPerSimd];
};
constexpr ColLayout kRankCols{{TCSC_WIDTHS}};
__host__ __device__ constexpr int wave_cols(int w) { return kRankCols.w[w >> 2]; }
__host__ __device__ constexpr int wave_col0(int w) {
    int s = 0;
    for (int r = 0; r < (w >> 2); ++r) s += 4 * kRankCols.w[r];
    return s + (w & 3) * kRankCols.w[w >> 2];
}
constexpr int wg_cols() {
    int s = 0;
    for (int r = 0; r < kWavesPerSimd; ++r) s += 4 * kRankCols.w[r];
    return s;
}
constexpr int kWgCols = wg_cols();  // columns of one workgroup (column block)
constexpr bool widths_ok() {
    for (int r = 0; r < kWavesPerSimd; ++r)
        if (kRankCols.w[r] <= 0 || kRankCols.w[r] > kCW || kRankCols.w[r] % 4) return false;
    return true;
}
static_assert(widths_ok(), "TCSC_WIDTHS: one width per rank, multiples of 4, at most TCSC_CW");
// Wave-column group g = column block g / kWaves, wave g % kWaves.
__host__ __device__ constexpr int group_col0(int g) { return (g / kWaves) * kWgCols + wave_col0(g % kWaves); }
__host__ __device__ constexpr int group_cols(int g) { return wave_cols(g % kWaves); }
// groups with at least one of ncols columns (group_col0 ascends with g)
__host__ __device__ constexpr int groups_for(int ncols) {
    int g = (ncols / kWgCols) * kWaves;
    while (group_col0(g) < ncols) ++g;
    return g;
}
// L2 prefetch of the entry streams: after every chunk each
// wave touches `lines` 128-B lines of its own stream starting `dist` bytes
// past the next chunk's header (one global_load_lds_dword into a 256-B
// scratch per wave after the ring: it writes no VGPR and no SGPR, and counts
// in vmcnt, not lgkmcnt, so the gather's counted LDS waits stay exact).  The
// launcher picks dist and lines from the plan's stream bytes per chunk
// (pf_stream_params).  TCSC_PF_S=0 builds without it.
#ifndef TCSC_PF_S
#define TCSC_PF_S 1
#endif
constexpr bool kPfS = TCSC_PF_S != 0;
constexpr int kPfWindow = 1792;  // dist + 128 * lines at most (bytes)
// entries allocated past the last stream (empty chain + block loads + the stream prefetch window)
constexpr int kEntGuard = kPfS ? kPfWindow / 8 + 8 : 64;
static_assert(kEntGuard <= 256, "k_fill_headers writes the guard with one block");
constexpr int kHdr = 2;                  // header entries ahead of every (group, chunk) stream
constexpr int kRingBytes = kNBuf * kBufRows * kRowBytes;  // 147 KiB
constexpr int kPfScratch = kPfS ? kWaves * 256 : 0;  // prefetch landing area, 256 B per wave
// the epilogue parks 64 rows x (kCW*4 + 16) B per wave at least
// the epilogue's staging (64 rows) + the row-band combine's own band (64 rows) + its flag words
constexpr int kEpiMinBytes = kWaves * 64 * (kCW * 4 + 16) + 64 * kRowBytes + 16;
constexpr int kLdsBytes = (kRingBytes + kPfScratch) > kEpiMinBytes ? (kRingBytes + kPfScratch) : kEpiMinBytes;
// Staging: waves 0..kDmaWaves-1 move a chunk, kDmaPerWave 1-KiB rows each,
// right after the chunk loop's barrier (TCSC_DMA_EARLY=1) or after their
// gather (0).  The SIMD arbiter favours older waves (tools/trace.py: waves
// 0-3 finish their gathers first, 12-15 last), so the DMA issue (~100 cycles
// per row) goes to the oldest waves, which have slack at the barrier.
// Round 1 measured the first half of the waves, issuing after the gather,
// 2.5 % faster than all 16.  Since round 3's stream prefetch, the DMA is issued
// by the first 4 waves, early: DMA(c+2) starts right after chunk c's barrier
// and so gets one more gather of lead time (tools/ab.sh, 3 rounds alternating:
// k_stream 1.160-1.162 -> 1.145-1.148 ms, step 1.245-1.253 -> 1.222-1.236 ms).
#ifndef TCSC_DMA_WAVES
#define TCSC_DMA_WAVES (TCSC_WAVES / 4)
#endif
#ifndef TCSC_DMA_EARLY
#define TCSC_DMA_EARLY 1
#endif
constexpr int kDmaWaves = TCSC_DMA_WAVES;
constexpr bool kDmaEarly = TCSC_DMA_EARLY != 0;
constexpr int kDmaPerWave = kTK / kDmaWaves;              // 1-KiB LDS-DMA rows per DMA wave and chunk
static_assert(kDmaWaves <= kWaves && kTK % kDmaWaves == 0, "each DMA wave moves the same number of rows");
static_assert(kLdsBytes <= 160 * 1024, "LDS");
static_assert(kNBuf >= 2 && kNBuf <= 5, "ring of 2 (DMA(c+1) before gather(c)) or n >= 3 (DMA(c+n-1) after it)");

// Stream layout (v4).  Group-major: the streams of one wave-column group
// follow each other chunk by chunk, each behind a header of kHdr entries
// {nb, rem}, {byte distance to the next header, 0}, so a wave walks its
// chain with one scalar add per chunk and reads its counts from the same
// scalar loads that bring the entries (no stream table in the loop).
// sptr[g*n_chunks + c] = entry index of the header of (g, c).
// Entry (8 bytes): word0 = +1.0f or -1.0f (bit pattern), word1 =
// (lds_row << 10) | (4*slot); lds_row = (chunk%3)*kBufRows + (k - chunk*kTK)
// or the pad row; slot = column inside the wave (0..kCW-1).
static_assert(4 * kCW <= 255, "slot index must fit the 8-bit gpr_idx field");
static_assert(64 * 16 <= 1024, "lane byte offset (16*lane) must fit the 10 low address bits");

// Input TCSC arrays (device pointers, absolute offsets as in tcsc_t) and the
// column range a plan covers.
struct PlanDev {
    int rows = 0;  // K
    int ncols = 0;
    int col_begin = 0;
    long long n_pos = 0, n_neg = 0;  // entries inside the column range
    const int* csp = nullptr;
    const int* csn = nullptr;
    const int* rip = nullptr;
    const int* rin = nullptr;
};

// Plan arrays (device).  Everything but ent/sptr is build-time scratch.
struct PlanOut {
    int n_chunks = 0;
    int n_groups = 0;          // groups_for(ncols) wave-column groups
    long long n_entries = 0;   // stream entries incl. padding
    int2* ent = nullptr;       // n_entries (+kBatch) entries
    int* sptr = nullptr;       // n_groups*n_chunks + 1 header positions (entries), group-major
    int* lbp = nullptr;
    int* lbn = nullptr;
    int* cnt = nullptr;
    int* cptr = nullptr;
    int* gcnt = nullptr;
    void* scan_tmp = nullptr;
    size_t scan_tmp_bytes = 0;
};

// ---- the in-launch split-K combine's tile words (k_stream OUT 2) ----------
// Per tile (row tile x column block) of a launch: {arrivals, done,
// claims[Z]}, zeroed when the block is allocated and reset to zero by the
// tile's last workgroup to finish, so every launch (and graph replay) finds
// them at zero.  A launch that returns an error marks the block dirty and
// the next launch on the plan re-zeroes it first (tcsc_api.cpp).
constexpr int kCombineTiles = 4096;
constexpr int kCombineWords = 32;  // per tile: 2 + Z (Z <= 16) used
constexpr size_t kCombineBytes = (size_t)kCombineTiles * kCombineWords * 4;

struct GemmArgs {
    const float* X = nullptr;
    float* XT = nullptr;       // K x ldxt workspace: X transposed (ldxt = M rounded up to kTM)
    int M = 0, K = 0;
    const int2* ent = nullptr;
    const int* sptr = nullptr;
    long long n_entries = 0;   // the empty chain of idle waves starts here
    // summation order (k_stream ORDER): 0 merged (ent = the plan); 1, 2 the
    // reference's orders (ent = the +1-only plan, ent2 = the -1-only plan)
    int order = 0;
    const int2* ent2 = nullptr;
    const int* sptr2 = nullptr;
    long long n_entries2 = 0;
    int n_groups = 0;
    int ncols = 0;
    long long nnz = 0;
    const float* B = nullptr;
    float* Y = nullptr;
    int ldy = 0;
    float a = 0.f;
    bool bias_first = false;
    bool prelu = false;
    float* ws = nullptr;       // split-K partial slabs (may be null: no split)
    size_t ws_bytes = 0;
    int force_slices = 0;      // 0 = cost model
    int stage = 0;             // 0: transpose + gather, 1: transpose only, 2: gather only (X^T prepared)
    int num_cus = 0;           // CUs of the device (the in-launch combine needs the grid resident)
    unsigned* ccnt = nullptr;  // the split-K combine's tile words (kCombineBytes), null = k_reduce4
    int combine_giveup = 0;    // test knob (TCSC_COMBINE_GIVEUP=1): every slice but the last arrival gives up at once
};

// Plan building
hipError_t plan_scan_tmp_bytes(long long n, size_t* bytes);
hipError_t plan_counts(const PlanDev& in, PlanOut& out, hipStream_t st);    // -> cptr, gcnt
hipError_t plan_fill(const PlanDev& in, PlanOut& out, hipStream_t st);      // -> sptr, ent
// Launch
int choose_slices(int M, int ncols, int K, long long nnz, int n_groups, size_t ws_bytes, int force);
// where the split-K slabs of a gather launch are combined: 0 by k_reduce4
// after it, 2 inside k_stream by row bands (combine_tile: >= 3 slices, the
// grid resident at once), 3 inside k_stream pairwise (exactly 2 slices), 4
// pairwise in split halves (2 slices, the grid resident at once)
int combine_mode(int slices, long long wgs, long long tiles, long long slab_floats, int num_cus, bool have_words,
                 bool vec);
int normalized_slices(int K, int slices);  // the K split launch_gemm actually runs
// stream prefetch of a plan of n_entries entries over n_groups x n_chunks
// streams: *dist bytes ahead, *lines 128-B lines (TCSC_PF_DIST / TCSC_PF_LINES override)
void pf_stream_params(long long n_entries, int n_groups, int n_chunks, int* dist, int* lines);
size_t workspace_bytes(int M, int ncols, int slices);
size_t xt_bytes(int M, int K);
hipError_t launch_gemm(const GemmArgs& g, hipStream_t st);
// tcsc_from_dense on the device
// tile counts cp/cn ([row tile][col], dense_tile_rows(rows) rows per tile)
// turned into per-column tile offsets in place; column totals into totp/totn
// (cols + 1 entries, the last 0)
int dense_tile_rows(int rows);
hipError_t dense_to_tcsc_counts(const float* D, int rows, int cols, int* cp, int* cn, int* totp, int* totn,
                                hipStream_t st);
// row indices from the tile offsets op/on and col_start csp/csn
hipError_t dense_to_tcsc_fill(const float* D, int rows, int cols, const int* csp, const int* csn, const int* op,
                              const int* on, int* rip, int* rin, hipStream_t st);
// Y[m, n] = act(Y[m, n] + B[n]) in place (the dense baseline's epilogue)
hipError_t launch_bias_act(float* Y, int M, int N, int ldy, const float* B, bool prelu, float a, hipStream_t st);
hipError_t exclusive_scan_i32(const int* in, int* out, int n, void* tmp, size_t tmp_bytes, hipStream_t st);
// Plan-build input checks on device TCSC arrays (tcsc_gpu_plan_create_device):
// atomically ORs 1 into *d_flag for a bad col_start or a row outside
// [0, rows), 2 for a column whose rows do not ascend.
hipError_t check_index_device(const int* cs, const int* ri, int col_begin, int ncols, int rows, int n_total,
                              int* d_flag, hipStream_t st);
// out[j] = cs[col_begin + j] - cs[col_begin] for j in [0, ncols]
hipError_t rebase_offsets(const int* cs, int col_begin, int ncols, int* out, hipStream_t st);
// per-column ascending sort of row indices (segments off[j] .. off[j+1])
hipError_t sort_columns_tmp_bytes(int n, int ncols, size_t* bytes);
hipError_t sort_columns(const int* in, int* out, int n, int ncols, const int* off, void* tmp, size_t tmp_bytes,
                        hipStream_t st);
// X (M x K) -> XT (K x ldxt), rows m >= M zero; ldxt = ldxt_for(M) (M rounded up to kTM)
int ldxt_for(int M);
hipError_t launch_transpose(const float* X, int M, int K, float* XT, int ldxt, hipStream_t st);

// ---- per-column CSC copy of a plan's range (small-M path, MFMA fixup) ------
// The merged list: each column's +1 and -1 rows in ascending order (the fast
// order's), one entry per nonzero: 4*k for a +1 row, 4*Kp + 4*k for a -1 row
// (Kp = K + 1 rounded up to a multiple of 4), padded with 4*K entries (K = the
// plan's rows, < 2^28).  An entry is the byte offset of +X[k] or -X[k] in a
// staged row pair [X | -0.0 | 0.. | -X | 0..] of 2*Kp floats (the small-M
// kernel's LDS rows, both halves 16-B aligned; padding reads the -0.0).  Columns go in
// groups of kCscGroup (a small-M workgroup's lanes), interleaved by 16-B
// quads: quad q of column j = g*kCscGroup + l sits at int4 index
// (cq[g] + q) * kCscGroup + l, so the group's quad q is one contiguous 1 KiB.
// Group g has cq[g+1] - cq[g] quads (its longest column's, rounded up to a
// multiple of 16: the small-M kernel's unroll); shorter columns are padded.
// The array ends with kCscGuardQuads quads of zeros per lane (the small-M
// kernel's look-ahead reads that far past a group).
// Built in two calls (the host reads cq[ngroups] in between to size crq)
// from the rebased per-sign lists in the scratch cp/cn (ncols+1), crp/crn.
constexpr int kCscGroup = 64;
constexpr int kCscGuardQuads = 48;
__host__ __device__ inline int csc_half(int K) { return (K + 4) & ~3; }     // Kp: floats per half of a row pair
__host__ __device__ inline int csc_neg_base(int K) { return 4 * csc_half(K); }  // a -1 row's offset: -X[k] at 4Kp + 4k
__host__ __device__ inline int csc_groups(int ncols) { return (ncols + kCscGroup - 1) / kCscGroup; }
inline size_t csc_quad_entries(long long quads) { return (size_t)(quads + kCscGuardQuads) * kCscGroup * 4; }
// cp, cn, crp, crn and the group quad offsets cq (groups+1) from the column range
hipError_t csc_prepare(const int* csp, const int* csn, const int* rip, const int* rin, int col_begin, int ncols,
                       long long n_pos, long long n_neg, int* cp, int* cn, int* crp, int* crn, int* gq, void* scan_tmp,
                       size_t scan_tmp_bytes, int* cq, hipStream_t st);
// crq (csc_quad_entries(cq[groups]) ints) from them
hipError_t csc_fill(const int* cp, const int* cn, const int* crp, const int* crn, const int* cq, int ncols, int rows,
                    int* crq, size_t crq_entries, hipStream_t st);
// column j's entry list in the quad layout: entry i at crq[csc_entry(cq, j, i)]
__host__ __device__ inline size_t csc_entry(const int* cq, int j, int i) {
    const int g = j / kCscGroup, l = j % kCscGroup;
    return ((size_t)(cq[g] + i / 4) * kCscGroup + l) * 4 + (i & 3);
}

// ---- MFMA path for near-dense W (tcsc_mfma.hip) ------------
// X3 rows are ldk = mfma_ldk(K) bf16 long, in blocks of kMfmaBlk = 64 k (one
// GEMM k step): [h | m | l] of block 0, of block 1, ..., zeros past K.  Each
// part of a block is 128 B, one cache line, so the GEMM stages it in whole
// lines.  W is stored once (WT, ncols x ldw = mfma_ldw(K)): the GEMM stages a
// block of W once and multiplies it with the block's three parts in turn.
// The accumulation runs k-major (h, m, l of a block, then the next block):
// its fp32 rounding error is about half that of a part-major [h | m | l]
// image (the accumulator is not carried across K three times).
constexpr int kMfmaBlk = 64;
__host__ __device__ inline int mfma_nblk(int K) { return (K + kMfmaBlk - 1) / kMfmaBlk; }
__host__ __device__ inline int mfma_ldk(int K) { return 3 * kMfmaBlk * mfma_nblk(K); }
__host__ __device__ inline int mfma_ldw(int K) { return kMfmaBlk * mfma_nblk(K); }
__host__ __device__ inline int x3_index(int k, int part) {
    return (k / kMfmaBlk) * (3 * kMfmaBlk) + part * kMfmaBlk + k % kMfmaBlk;
}
// Build: wf (ncols x rows fp32 scratch) <- the +1/-1 entries of columns
// [col_begin, col_begin+ncols) (absolute offsets), transposed; wt <- W^T in
// bf16 (ncols x ldw, zeros past rows).  *bad = 1 if a weight is not exact in
// bf16.
hipError_t mfma_build_wt(const int* csp, const int* csn, const int* rip, const int* rin, int col_begin, int rows,
                         int ncols, float* wf, uint16_t* wt, int ldw, long long n_pos, long long n_neg, int* bad,
                         hipStream_t st);
// ---- small-M path (tcsc_small.hip) ----------------------------
// X is staged in LDS as M row pairs [X | -0.0 | 0.. | -X | 0..] of 2*Kp
// floats: the path applies only where that fits (at most 160 KiB; K < 20,477
// at M = 1).
constexpr size_t small_m_lds_bytes_max() { return 160 * 1024; }
inline size_t small_m_lds_bytes(int M, int K) { return (size_t)M * 2 * (size_t)csc_half(K) * 4; }
inline bool small_m_fits(int M, int K) { return M >= 1 && M <= 4 && small_m_lds_bytes(M, K) <= small_m_lds_bytes_max(); }
// Y[m, j] = act(sum over column j's merged rows of +-X[m,k], ascending k,
// then + B[j]) for m < M <= 4: one lane per column over the merged CSC copy,
// the fast order's exact arithmetic (bit-identical to k_stream unsplit).
hipError_t launch_small_m(const float* X, int M, int K, const int* cq, const int* crq, int ncols, const float* B,
                          float* Y, int ldy, bool bias_first, bool prelu, float a, hipStream_t st);
// X (M x K) -> x3 (M x ldk bf16, [h | m | l | 0..]); flags[m] = 1 for the
// rows the fixup recomputes, 0 otherwise (every row, every call).
hipError_t mfma_split_x(const float* X, int M, int K, uint16_t* x3, int ldk, int* flags, hipStream_t st);
// k_gemm3: Y = act(sum over blocks and parts of x3 . wt^T + B) on the matrix
// cores (bias after the sum); K gives the block count.  Grids of small tiles
// that would leave CUs idle split K into mfma_slices() slices of whole 64-k
// blocks: raw partial sums into `slabs` (mfma_slab_bytes(): slices x M x N
// floats), added in slice order with the bias and PReLU (k_reduce4's adds)
// by k_reduce_fix, which also writes the rows `flags` marks exactly (the
// fixup, from the CSC copy cq / crq): a split call needs no mfma_fixup.
bool mfma_big_tiles(int M, int N);
bool mfma_narrow_tiles(int M, int N);
long long mfma_tiles(int M, int N);
int mfma_slices(int M, int N, int K);
size_t mfma_slab_bytes(int M, int N, int K);
hipError_t mfma_gemm3(const uint16_t* x3, int ldk, const uint16_t* wt, int ldw, int K, int M, int N, const float* B,
                      float* Y, int ldy, bool prelu, float a, float* slabs, size_t slab_bytes, const int* flags,
                      const int* cq, const int* crq, hipStream_t st);

// Rewrites the flagged rows in k_stream's fast order (no-op when none is).
hipError_t mfma_fixup(const uint16_t* x3, int M, int K, int ldk, const int* cq, const int* crq, int ncols,
                      const float* B, float* Y, int ldy, bool bias_first, bool prelu, float a, const int* flags,
                      hipStream_t st);

// Error channel shared by every entry point of the library (tcsc_api.cpp):
// the message behind tcsc_gpu_last_error(), and the host API's policy
// (stderr + abort unless TCSC_ON_ERROR=continue).
void set_error_msg(const char* msg);
const char* error_msg();
void report_status(int rc);

// ---- BCSR (bcsr_kernels.hip / bcsr_api.cpp) --------------------------------
struct BcsrArgs {
    const float* XT = nullptr;  // K x ldxt (X^T)
    int ldxt = 0, M = 0, N = 0, ldy = 0;
    const int* colptr = nullptr;  // nbc + 1
    const int2* ent = nullptr;    // per block column, per (block, block row): {X row, value offset}
    const float* vals = nullptr;
    int r = 1, c = 1, nbc = 0;
    const float* B = nullptr;
    float* Y = nullptr;
    float a = 0.f;
    bool fma = false;    // fused multiply-add (avx variants, or exact ternary products)
    bool prelu = false;  // PReLU after every update (bcsr.c:208-209)
};
hipError_t launch_bcsr(const BcsrArgs& g, hipStream_t st);

}  // namespace tcsc
