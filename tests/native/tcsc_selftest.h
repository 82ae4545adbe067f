/* tcsc_selftest.h -- host-side self-test hooks of libtcsc_amd.so (test-only:
 * exported only by the sanitizer builds, which compile the host sources with
 * -DTCSC_SELFTEST: `make -C sparse-matrix-multiplication-benchmark_amd asan
 * tsan`; tests/test_sanitizers.py runs tests/native/host_selftest.cpp against
 * them).  No GPU needed.
 *   tcsc_selftest_fingerprint: the host API's plan-cache fingerprint of W
 *     summed on its worker pool (the path host_sgemm overlaps with a call)
 *     against the same hash summed serially; returns 0 when they agree.
 *   tcsc_selftest_copy2d: `rows` rows of `row_bytes` from src (pitch sp)
 *     to dst (pitch dp) on device `dev`'s copy pool for direction `side`
 *     (0 in, 1 out) -- the pinned-staging copies of the band pipeline. */
#ifndef TCSC_AMD_SELFTEST_H
#define TCSC_AMD_SELFTEST_H
#include <stddef.h>

#include "../../include/sparse/tcsc.h"

#ifdef __cplusplus
extern "C" {
#endif
int tcsc_selftest_fingerprint(const tcsc_t *W);
int tcsc_selftest_copy2d(void *dst, size_t dp, const void *src, size_t sp,
                         size_t row_bytes, size_t rows, int dev, int side);
#ifdef __cplusplus
}
#endif
#endif /* TCSC_AMD_SELFTEST_H */
