/*
 * bcsr_oracle.c -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the
 * reference's BCSR path (/root/reference/sparse/bcsr.c), the parity checker
 * of the gfx950 kernel k_bcsr.  Linked into oracle/liboracle.so next to
 * tcsc_oracle.c; nothing in the product links or calls it (tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg only).
 *
 * Parity status: PINNED.  Every function is checked bit-for-bit against the
 * reference's bcsr.c compiled from /root/reference into
 * oracle/_ref/libtcsc_ref.so (oracle/Makefile `ref`) on the fixtures in
 * tests/golden/bcsr/ (generator: tests/golden/gen_golden_bcsr.py).
 *
 * Compiled with -ffp-contract=off (oracle/Makefile): bcsr_sgemm_basic's
 * `Y += X * val` stays a rounded product plus a rounded sum, as written; the
 * avx variants' _mm256_fmadd_ps is fmaf().
 */
#include <math.h>
#include <stddef.h>

/* bcsr.c:53-63: a block is stored when any value compares equal to +-1. */
static int block_has_pm1(const float *d, int cols, int brow, int bcol, int r, int c) {
    for (int i = 0; i < r; ++i)
        for (int j = 0; j < c; ++j) {
            float v = d[(size_t)(brow * r + i) * cols + (size_t)bcol * c + j];
            if (v == -1.0f || v == 1.0f) return 1;
        }
    return 0;
}

/* Counting pass (bcsr.c:40-72): stored blocks and non-empty block rows. */
void oracle_bcsr_count(const float *dense, int rows, int cols, int r, int c, int *k, int *nonempty_rows) {
    int br = rows / r, bc = cols / c, n = 0, ne = 0;
    for (int a = 0; a < br; ++a) {
        int any = 0;
        for (int b = 0; b < bc; ++b)
            if (block_has_pm1(dense, cols, a, b, r, c)) {
                ++n;
                any = 1;
            }
        ne += any;
    }
    *k = n;
    *nonempty_rows = ne;
}

/* Fill pass (bcsr.c:99-137): blocks numbered block-row-major; b_row_start
 * gets the first block of every NON-EMPTY block row (bcsr.c:114-117) then k
 * (bcsr.c:137).  The reference leaves b_row_start[ne+1 .. br] uninitialised;
 * they are k here (the convention of include/sparse/bcsr.h). */
void oracle_bcsr_fill(const float *dense, int rows, int cols, int r, int c, int *b_row_start, int *b_col_idx,
                      float *b_values) {
    int br = rows / r, bc = cols / c, blk = 0, w = 0;
    for (int a = 0; a < br; ++a) {
        int first = 1;
        for (int b = 0; b < bc; ++b) {
            if (!block_has_pm1(dense, cols, a, b, r, c)) continue;
            if (first) {
                b_row_start[w++] = blk;
                first = 0;
            }
            b_col_idx[blk] = b;
            for (int i = 0; i < r; ++i)
                for (int j = 0; j < c; ++j)
                    b_values[(size_t)blk * r * c + (size_t)i * c + j] =
                        dense[(size_t)(a * r + i) * cols + (size_t)b * c + j];
            ++blk;
        }
    }
    for (int i = w; i <= br; ++i) b_row_start[i] = blk;
}

/* variant 0 bcsr_sgemm_basic        (bcsr.c:141-175)
 *         1 bcsr_sgemm_prelu_basic  (bcsr.c:177-218)
 *         2 bcsr_sgemm_avx          (bcsr.c:222-261, c == 8)
 *         3 bcsr_sgemm_prelu_avx    (bcsr.c:264-312, c == 8)
 *         4 bcsr_sgemm_avx2         (bcsr.c:316-385, r == c == 8)
 * Per output element all five run the same sequence: Y = B, then for every
 * visited block (block row ascending, bi ascending: bcsr.c:157-160) and its
 * rows i ascending one update y = y + x*v (fmaf for 2-4), PReLU
 * (y > 0 ? y : a*y) after each update for 1 and 3 (bcsr.c:208-209,
 * 302-304; _CMP_GT_OS is false for NaN like the scalar compare). */
void oracle_bcsr_sgemm(int variant, const float *X, int r, int c, int nbr, const int *b_row_start,
                       const int *b_col_idx, const float *b_values, const float *B, float a, float *Y, int M, int N,
                       int K) {
    const int fma = variant >= 2, prelu = (variant == 1 || variant == 3);
    for (int m = 0; m < M; ++m)
        for (int n = 0; n < N; ++n) Y[(size_t)m * N + n] = B[n];
    for (int m = 0; m < M; ++m)
        for (int b = 0; b < nbr; ++b)
            for (int bi = b_row_start[b]; bi < b_row_start[b + 1]; ++bi) {
                const int bcol = b_col_idx[bi];
                for (int i = 0; i < r; ++i) {
                    const float x = X[(size_t)m * K + (size_t)b * r + i];
                    for (int j = 0; j < c; ++j) {
                        const float v = b_values[(size_t)bi * r * c + (size_t)i * c + j];
                        float *y = &Y[(size_t)m * N + (size_t)bcol * c + j];
                        float t = fma ? fmaf(x, v, *y) : *y + x * v;
                        if (prelu) t = (t > 0) ? t : a * t;
                        *y = t;
                    }
                }
            }
}
