// host_selftest.cpp -- the host-side code of libtcsc_amd.so under
// AddressSanitizer / ThreadSanitizer (SURVEY.md §5 "Race detection /
// sanitizers: -fsanitize=address for host code").  No GPU needed: the
// format builders, the dense helpers, the worker pools of the host API (the
// fingerprint pool and the per-device copy pools, from several threads at
// once) and the no-device error path of the drop-in calls.  Built by
// `make -C sparse-matrix-multiplication-benchmark_amd asan tsan`; run by
// tests/test_sanitizers.py.  Exit status 0 = every check passed (a
// sanitizer report makes the sanitizer runtime exit non-zero).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/sparse/tcsc.h"
#include "../../include/tcsc_gpu.h"
#include "../../include/sparse_gemm.h"
#include "tcsc_selftest.h"

static int g_fail = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                   \
        }                                                               \
    } while (0)

static unsigned long long g_s = 0x1234567;
static unsigned rnd() {
    g_s = g_s * 6364136223846793005ULL + 1442695040888963407ULL;
    return (unsigned)(g_s >> 33);
}

// tcsc_from_dense against a direct per-column scan (tcsc.c:6-66 semantics)
static void check_from_dense(int K, int N, int nz) {
    std::vector<float> d((size_t)K * N + 1);
    for (size_t i = 0; i < (size_t)K * N; ++i) {
        const unsigned r = rnd() % (2 * nz);
        d[i] = r == 0 ? 1.0f : r == 1 ? -1.0f : (r == 2 ? 0.5f : 0.0f);  // non-ternary values count as 0
    }
    tcsc_t* W = tcsc_from_dense(d.data(), K, N);
    CHECK(W != nullptr);
    if (!W) return;
    CHECK(W->rows == K && W->cols == N);
    int p = 0, q = 0;
    for (int n = 0; n < N; ++n) {
        CHECK(W->col_start_pos[n] == p && W->col_start_neg[n] == q);
        for (int k = 0; k < K; ++k) {
            const float v = d[(size_t)k * N + n];
            if (v == 1.0f) CHECK(W->row_index_pos[p++] == k);
            else if (v == -1.0f) CHECK(W->row_index_neg[q++] == k);
        }
    }
    CHECK(W->col_start_pos[N] == p && W->col_start_neg[N] == q);
    CHECK(W->n_elem_pos == p && W->n_elem_neg == q);
    CHECK(tcsc_selftest_fingerprint(W) == 0);
    tcsc_free(W);
}

static void check_sparse_format(int K, int N) {
    std::vector<int> m((size_t)K * N + 1);
    for (size_t i = 0; i < (size_t)K * N; ++i) m[i] = (int)(rnd() % 7) - 3;
    int np = 0, nn = 0;
    std::vector<int> csp(N + 1), csn(N + 1);
    CHECK(tcsc_sparse_format(m.data(), K, N, csp.data(), csn.data(), nullptr, nullptr, &np, &nn) == 0);
    std::vector<int> rip(np + 1), rin(nn + 1);
    CHECK(tcsc_sparse_format(m.data(), K, N, csp.data(), csn.data(), rip.data(), rin.data(), &np, &nn) == 0);
    int p = 0, q = 0;
    for (int n = 0; n < N; ++n)
        for (int k = 0; k < K; ++k) {
            const int v = m[(size_t)k * N + n];
            if (v >= 1) CHECK(rip[p++] == k);
            else if (v <= -1) CHECK(rin[q++] == k);
        }
    CHECK(p == np && q == nn);
}

// the per-device copy pools (both directions) and the fingerprint pool,
// driven from several threads at once as the host API's per-device threads do
static void pools_concurrently(int threads) {
    std::vector<float> d((size_t)2048 * 512);
    for (auto& v : d) {
        const unsigned r = rnd() % 40;
        v = r == 0 ? 1.0f : r == 1 ? -1.0f : 0.0f;
    }
    tcsc_t* W = tcsc_from_dense(d.data(), 2048, 512);  // ~52 K nonzeros ... grown below
    std::vector<float> big((size_t)4096 * 1024);
    for (auto& v : big) {
        const unsigned r = rnd() % 20;
        v = r == 0 ? 1.0f : r == 1 ? -1.0f : 0.0f;
    }
    tcsc_t* W2 = tcsc_from_dense(big.data(), 4096, 1024);  // ~420 K nonzeros: the pooled path
    CHECK(W && W2 && W2->n_elem_pos + W2->n_elem_neg > (1 << 16));
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            const size_t rows = 300 + 37 * t, rb = 4000 + 12 * t, sp = rb + 64, dp = rb + 128;
            std::vector<char> src(rows * sp), dst(rows * dp, 0);
            for (size_t i = 0; i < src.size(); ++i) src[i] = (char)(i * 31 + t);
            for (int it = 0; it < 20; ++it) {
                CHECK(tcsc_selftest_copy2d(dst.data(), dp, src.data(), sp, rb, rows, t % 4, it & 1) == 0);
                CHECK(tcsc_selftest_fingerprint(it & 1 ? W2 : W) == 0);
            }
            for (size_t r = 0; r < rows; ++r) CHECK(std::memcmp(&dst[r * dp], &src[r * sp], rb) == 0);
            // contiguous rows take the one-long-row path
            std::vector<char> c(rows * rb);
            CHECK(tcsc_selftest_copy2d(c.data(), rb, src.data(), rb, rb, rows, t % 4, 0) == 0);
            CHECK(std::memcmp(c.data(), src.data(), rows * rb) == 0);
        });
    for (auto& x : th) x.join();
    tcsc_free(W);
    tcsc_free(W2);
}

int main() {
    setenv("TCSC_ON_ERROR", "continue", 1);
    check_from_dense(1, 1, 2);
    check_from_dense(0, 5, 2);
    check_from_dense(7, 0, 2);
    check_from_dense(257, 131, 2);
    check_from_dense(1000, 300, 10);
    check_sparse_format(48, 40);
    check_sparse_format(1, 1);
    pools_concurrently(8);

    // dense helpers (dense/dense.h)
    tcsc_set_seed(7);
    float* X = init_rand_dense(5, 9);
    float* Wd = init_rand_sparse(9, 4, 2);
    float* B = init_rand_dense(4, 1);
    float* Y = (float*)std::malloc(5 * 4 * sizeof(float));
    float* Y2 = (float*)std::malloc(5 * 4 * sizeof(float));
    gemm_basic(X, Wd, B, Y, 5, 4, 9);
    std::memcpy(Y2, Y, 5 * 4 * sizeof(float));
    CHECK(compare(Y, Y2, 5, 4));

    // the drop-in calls without a device: an error, no crash, Y untouched
    tcsc_t* W = tcsc_from_dense(Wd, 9, 4);
    for (int i = 0; i < 20; ++i) Y2[i] = 7.0f;
    tcsc_sgemm_basic(X, W, B, Y2, 5, 4, 9);
    tcsc_sgemm_prelu_basic(X, W, B, 0.2f, Y2, 5, 4, 9);
    for (int i = 0; i < 20; ++i) CHECK(Y2[i] == 7.0f);
    CHECK(std::strlen(tcsc_gpu_last_error()) > 0);
    tcsc_free(W);
    std::free(X);
    std::free(Wd);
    std::free(B);
    std::free(Y);
    std::free(Y2);
    std::printf("host_selftest: %s (%d failed checks)\n", g_fail ? "FAIL" : "OK", g_fail);
    return g_fail ? 1 : 0;
}
