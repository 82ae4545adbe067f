// bcsr_api.cpp -- the BCSR operator API (include/sparse/bcsr.h, reference
// sparse/bcsr.h:1-39 + sparse/bcsr.c) and its device API
// (include/bcsr_gpu.h), on top of the gfx950 kernel k_bcsr
// (bcsr_kernels.hip).
//
//  * bcsr_from_dense: host builder, same arrays as bcsr.c:19-139 (block
//    numbering, b_row_start written per non-empty block row, all values of a
//    stored block kept); the entries of b_row_start the reference leaves
//    uninitialised are set to k.
//  * plans: W re-indexed by block column in the reference's visiting order
//    (counting sort, stable), values uploaded as they are.
//  * bcsr_sgemm_*: W is passed by value and has no destructor in the
//    reference, so nothing is cached across calls: plan, X, B up; Y down.
//
// Errors go through the library's channel (tcsc_gpu_last_error(); stderr +
// abort in the host API unless TCSC_ON_ERROR=continue).  No GPU: every
// compute entry point fails; there is no CPU path.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

#include "../../include/bcsr_gpu.h"
#include "../../include/sparse/bcsr.h"
#include "../../include/tcsc_gpu.h"
#include "tcsc_internal.h"

struct bcsr_gpu_plan {
    int device = 0;
    int r = 1, c = 1, nbr = 0, nbc = 0, k = 0;
    long long visits = 0;  // block visits over all block columns
    bool ternary = false;  // every stored value is +-0 or +-1: every product is exact
    int* colptr = nullptr; // nbc + 1 offsets into ent
    int2* ent = nullptr;   // visits*r: per (block, block row i) {X row br*r+i, value offset (bi*r+i)*c}
    float* vals = nullptr; // k*r*c
    float* xt = nullptr;   // workspace: X^T
    size_t xt_bytes = 0;
    size_t bytes = 0;
    // what bcsr_gpu_prepare_x left in xt: (M, K) of the staged X, or -1 when
    // nothing is staged (never staged, the workspace was reallocated, or a
    // whole bcsr_gpu_sgemm overwrote it with its own X)
    int staged_M = -1, staged_K = -1;
};

namespace {

int fail(int rc, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    tcsc::set_error_msg(buf);
    return rc;
}

#define BCSR_HIP(call)                                                                                  \
    do {                                                                                                \
        hipError_t e_ = (call);                                                                         \
        if (e_ != hipSuccess) return fail(TCSC_E_HIP, "%s: %s (%d)", #call, hipGetErrorString(e_), (int)e_); \
    } while (0)

class DevGuard {
  public:
    explicit DevGuard(int dev) {
        if (hipGetDevice(&prev_) != hipSuccess) prev_ = -1;
        ok_ = hipSetDevice(dev) == hipSuccess;
    }
    ~DevGuard() {
        if (prev_ >= 0) (void)hipSetDevice(prev_);
    }
    bool ok() const { return ok_; }

  private:
    int prev_ = -1;
    bool ok_ = false;
};

void free_plan(bcsr_gpu_plan* p) {
    if (!p) return;
    DevGuard dg(p->device);
    if (p->colptr) (void)hipFree(p->colptr);
    if (p->ent) (void)hipFree(p->ent);
    if (p->vals) (void)hipFree(p->vals);
    if (p->xt) (void)hipFree(p->xt);
    delete p;
}

struct PlanDeleter {
    void operator()(bcsr_gpu_plan* p) const { free_plan(p); }
};

const char* variant_name(int v) {
    static const char* names[] = {"basic", "prelu_basic", "avx", "prelu_avx", "avx2"};
    return (v >= 0 && v <= 4) ? names[v] : "?";
}

// Shapes the reference's variants are defined for (bcsr.h comment).
int check_variant(int variant, int r, int c) {
    if (variant < BCSR_VARIANT_BASIC || variant > BCSR_VARIANT_AVX2)
        return fail(TCSC_E_ARG, "bcsr: bad variant %d", variant);
    if (variant >= BCSR_VARIANT_AVX && c != 8)
        return fail(TCSC_E_ARG,
                    "bcsr_sgemm_%s needs 8-column blocks (bcsr.c:250-256 move 8 floats per block row); W has c=%d",
                    variant_name(variant), c);
    if (variant == BCSR_VARIANT_AVX2 && r != 8)
        return fail(TCSC_E_ARG, "bcsr_sgemm_avx2 needs 8x8 blocks (bcsr.c:347-377 read 8 block rows); W has r=%d", r);
    return TCSC_OK;
}

int plan_create(const bcsr_t* W, int device, hipStream_t st, bcsr_gpu_plan** out) {
    if (!out) return fail(TCSC_E_ARG, "bcsr_gpu_plan_create: NULL out");
    *out = nullptr;
    if (!W || W->r < 1 || W->c < 1 || W->br < 0 || W->bc < 0 || W->k < 0 || !W->b_row_start ||
        (W->k > 0 && (!W->b_col_idx || !W->b_values)))
        return fail(TCSC_E_ARG, "bcsr_gpu_plan_create: malformed bcsr_t");
    const long long nvals = (long long)W->k * W->r * W->c;
    if (nvals > INT_MAX || (long long)W->br * W->r > INT_MAX || (long long)W->bc * W->c > INT_MAX)
        return fail(TCSC_E_ARG, "bcsr_gpu_plan_create: W too large for int offsets (k*r*c = %lld)", nvals);
    // visiting order of the reference (bcsr.c:157-160), counted per block column
    std::vector<int> colptr((size_t)W->bc + 1, 0);
    long long visits = 0;
    for (int b = 0; b < W->br; ++b) {
        const int lo = W->b_row_start[b], hi = W->b_row_start[b + 1];
        for (int bi = lo; bi < hi; ++bi) {
            if (bi < 0 || bi >= W->k)
                return fail(TCSC_E_ARG, "bcsr_gpu_plan_create: b_row_start[%d..%d] = [%d, %d) outside the %d blocks",
                            b, b + 1, lo, hi, W->k);
            const int bcol = W->b_col_idx[bi];
            if (bcol < 0 || bcol >= W->bc)
                return fail(TCSC_E_ARG, "bcsr_gpu_plan_create: b_col_idx[%d] = %d outside [0, %d)", bi, bcol, W->bc);
            colptr[bcol + 1] += W->r;
            ++visits;
        }
    }
    const long long rows_total = visits * W->r;  // stream entries: one per (block, block row)
    if (rows_total > INT_MAX) return fail(TCSC_E_ARG, "bcsr_gpu_plan_create: %lld block rows", rows_total);
    for (int j = 0; j < W->bc; ++j) colptr[j + 1] += colptr[j];
    std::vector<int2> ent((size_t)(rows_total > 0 ? rows_total : 1));
    {
        std::vector<int> cur(colptr.begin(), colptr.end() - 1);
        for (int b = 0; b < W->br; ++b)
            for (int bi = W->b_row_start[b]; bi < W->b_row_start[b + 1]; ++bi) {
                int& t = cur[W->b_col_idx[bi]];
                for (int i = 0; i < W->r; ++i) ent[t++] = make_int2(b * W->r + i, (bi * W->r + i) * W->c);
            }
    }
    bool ternary = true;
    for (long long i = 0; i < nvals && ternary; ++i) {
        const float v = W->b_values[i];
        ternary = (v == 0.0f || v == 1.0f || v == -1.0f);
    }
    DevGuard dg(device);
    if (!dg.ok()) return fail(TCSC_E_NODEV, "bcsr_gpu_plan_create: cannot select device %d", device);
    std::unique_ptr<bcsr_gpu_plan, PlanDeleter> p(new bcsr_gpu_plan);
    p->device = device;
    p->r = W->r;
    p->c = W->c;
    p->nbr = W->br;
    p->nbc = W->bc;
    p->k = W->k;
    p->visits = visits;
    p->ternary = ternary;
    const size_t cb = colptr.size() * sizeof(int), eb = ent.size() * sizeof(int2),
                 vb = (size_t)(nvals > 0 ? nvals : 1) * sizeof(float);
    BCSR_HIP(hipMalloc(&p->colptr, cb));
    BCSR_HIP(hipMalloc(&p->ent, eb));
    BCSR_HIP(hipMalloc(&p->vals, vb));
    BCSR_HIP(hipMemcpyAsync(p->colptr, colptr.data(), cb, hipMemcpyHostToDevice, st));
    BCSR_HIP(hipMemcpyAsync(p->ent, ent.data(), eb, hipMemcpyHostToDevice, st));
    if (nvals > 0) BCSR_HIP(hipMemcpyAsync(p->vals, W->b_values, (size_t)nvals * sizeof(float), hipMemcpyHostToDevice, st));
    BCSR_HIP(hipStreamSynchronize(st));
    p->bytes = cb + eb + vb;
    *out = p.release();
    return TCSC_OK;
}

size_t xt_need(int M, int K) { return (size_t)K * tcsc::ldxt_for(M) * sizeof(float); }

int reserve(bcsr_gpu_plan* p, int M, int K) {
    const size_t want = xt_need(M, K);
    if (want <= p->xt_bytes) return TCSC_OK;
    DevGuard dg(p->device);
    if (p->xt) {
        BCSR_HIP(hipDeviceSynchronize());  // a queued launch may still read it
        (void)hipFree(p->xt);
        p->xt = nullptr;
        p->xt_bytes = 0;
    }
    p->staged_M = p->staged_K = -1;
    BCSR_HIP(hipMalloc(&p->xt, want));
    p->xt_bytes = want;
    return TCSC_OK;
}

// stage 0: transpose + block kernel, 1: transpose only, 2: block kernel only
int run(const bcsr_gpu_plan* pc, const float* dX, const float* dB, float* dY, int M, int N, int K, int ldy,
        int variant, float a, hipStream_t st, int stage) {
    if (!pc) return fail(TCSC_E_ARG, "bcsr_gpu_sgemm: NULL plan");
    if (M < 0 || N < 0 || K < 0) return fail(TCSC_E_ARG, "bcsr_gpu_sgemm: negative size (M=%d N=%d K=%d)", M, N, K);
    if (K < pc->nbr * pc->r)
        return fail(TCSC_E_ARG, "bcsr_gpu_sgemm: K=%d < W.br*W.r=%d (X columns the blocks read)", K, pc->nbr * pc->r);
    int rc;
    if (stage != 1) {
        if ((rc = check_variant(variant, pc->r, pc->c)) != TCSC_OK) return rc;
        if (N < pc->nbc * pc->c)
            return fail(TCSC_E_ARG, "bcsr_gpu_sgemm: N=%d < W.bc*W.c=%d (Y columns the blocks write)", N,
                        pc->nbc * pc->c);
        if (ldy < N) return fail(TCSC_E_ARG, "bcsr_gpu_sgemm: ldy=%d < N=%d", ldy, N);
    }
    if (M == 0 || (stage != 1 && N == 0)) return TCSC_OK;
    bcsr_gpu_plan* p = const_cast<bcsr_gpu_plan*>(pc);
    // the gather reads X^T with the pitch of the M it was staged for
    if (stage == 2 && K > 0 && (p->staged_M != M || p->staged_K != K))
        return fail(TCSC_E_ARG, "bcsr_gpu_sgemm_prepared: M=%d K=%d but the staged X is %s (bcsr_gpu_prepare_x first)",
                    M, K, p->staged_M < 0 ? "absent" : "another shape");
    if (K > 0 && (rc = reserve(p, M, K)) != TCSC_OK) return rc;
    DevGuard dg(p->device);
    const int ldxt = tcsc::ldxt_for(M);
    if (stage != 2 && K > 0) {
        if (!dX) return fail(TCSC_E_ARG, "bcsr_gpu_sgemm: NULL X");
        p->staged_M = p->staged_K = -1;
        BCSR_HIP(tcsc::launch_transpose(dX, M, K, p->xt, ldxt, st));
        if (stage == 1) {
            p->staged_M = M;
            p->staged_K = K;
        }
    }
    if (stage == 1) return TCSC_OK;
    if (!dB || !dY) return fail(TCSC_E_ARG, "bcsr_gpu_sgemm: NULL B or Y");
    tcsc::BcsrArgs g;
    g.XT = p->xt;
    g.ldxt = ldxt;
    g.M = M;
    g.N = N;
    g.ldy = ldy;
    g.colptr = p->colptr;
    g.ent = p->ent;
    g.vals = p->vals;
    g.r = p->r;
    g.c = p->c;
    g.nbc = p->nbc;
    g.B = dB;
    g.Y = dY;
    g.a = a;
    // a fused multiply-add equals the rounded product + sum when every
    // product is exact (ternary values), so basic runs the FMA kernel then
    g.fma = variant >= BCSR_VARIANT_AVX || p->ternary;
    g.prelu = variant == BCSR_VARIANT_PRELU_BASIC || variant == BCSR_VARIANT_PRELU_AVX;
    BCSR_HIP(tcsc::launch_bcsr(g, st));
    return TCSC_OK;
}

// ---------------------------------------------------------------------------
// Host-pointer API
// ---------------------------------------------------------------------------
std::mutex g_bcsr_mu;

struct HostCall {
    hipStream_t st = nullptr;
    bcsr_gpu_plan* plan = nullptr;
    float *x = nullptr, *b = nullptr, *y = nullptr;
    ~HostCall() {
        if (st) (void)hipStreamSynchronize(st);
        if (x) (void)hipFree(x);
        if (b) (void)hipFree(b);
        if (y) (void)hipFree(y);
        free_plan(plan);
        if (st) (void)hipStreamDestroy(st);
    }
};

int host_call(int variant, const float* X, const bcsr_t& W, const float* B, float a, float* Y, int M, int N, int K) {
    if (M <= 0 || N <= 0) return TCSC_OK;  // the reference's loops do nothing
    if ((!X && K > 0) || !B || !Y) return fail(TCSC_E_ARG, "bcsr_sgemm_%s: NULL argument", variant_name(variant));
    int rc = check_variant(variant, W.r, W.c);
    if (rc != TCSC_OK) return rc;
    if (N < W.bc * W.c || K < W.br * W.r)
        return fail(TCSC_E_ARG, "bcsr_sgemm_%s: shape mismatch (W %d x %d blocks of %d x %d, M=%d N=%d K=%d)",
                    variant_name(variant), W.br, W.bc, W.r, W.c, M, N, K);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        return fail(TCSC_E_NODEV, "no HIP device visible: the BCSR kernels need a gfx950 GPU");
    }
    std::lock_guard<std::mutex> lk(g_bcsr_mu);
    int dev = 0;
    BCSR_HIP(hipGetDevice(&dev));
    HostCall hc;
    BCSR_HIP(hipStreamCreateWithFlags(&hc.st, hipStreamNonBlocking));
    if ((rc = plan_create(&W, dev, hc.st, &hc.plan)) != TCSC_OK) return rc;
    const size_t xb = (size_t)M * K * sizeof(float), bb = (size_t)N * sizeof(float), yb = (size_t)M * N * sizeof(float);
    BCSR_HIP(hipMalloc(&hc.x, xb ? xb : 4));
    BCSR_HIP(hipMalloc(&hc.b, bb));
    BCSR_HIP(hipMalloc(&hc.y, yb));
    if (xb) BCSR_HIP(hipMemcpyAsync(hc.x, X, xb, hipMemcpyHostToDevice, hc.st));
    BCSR_HIP(hipMemcpyAsync(hc.b, B, bb, hipMemcpyHostToDevice, hc.st));
    if ((rc = run(hc.plan, hc.x, hc.b, hc.y, M, N, K, N, variant, a, hc.st, 0)) != TCSC_OK) return rc;
    BCSR_HIP(hipMemcpyAsync(Y, hc.y, yb, hipMemcpyDeviceToHost, hc.st));
    BCSR_HIP(hipStreamSynchronize(hc.st));
    return TCSC_OK;
}

void host_sgemm(int variant, const float* X, const bcsr_t& W, const float* B, float a, float* Y, int M, int N, int K) {
    tcsc::report_status(host_call(variant, X, W, B, a, Y, M, N, K));
}

void* alloc32(size_t bytes) {
    void* p = nullptr;
    return posix_memalign(&p, 32, bytes ? bytes : 32) == 0 ? p : nullptr;
}

}  // namespace

extern "C" {

// ---------------------------------------------------------------------------
// bcsr_from_dense (bcsr.c:19-139)
// ---------------------------------------------------------------------------
bcsr_t* bcsr_from_dense(dense_t dense, int rows, int cols, int r, int c) {
    if (r < 1 || c < 1 || rows < 0 || cols < 0 || (!dense && (long long)rows * cols > 0)) return nullptr;
    const int nbr = rows / r, nbc = cols / c;  // trailing rows/columns are ignored (bcsr.c:23-24)
    // pass 1: a block is stored when one of its values compares equal to
    // +1 or -1 (bcsr.c:62); swept row by row (same set as the reference's
    // block-by-block walk), numbered block-row-major afterwards (bcsr.c:69)
    std::vector<unsigned char> hit((size_t)nbr * nbc, 0);
    for (int b = 0; b < nbr; ++b)
        for (int i = 0; i < r; ++i) {
            const float* row = dense + (size_t)(b * r + i) * cols;
            unsigned char* h = hit.data() + (size_t)b * nbc;
            for (int bc = 0; bc < nbc; ++bc) {
                if (h[bc]) continue;
                const float* v = row + (size_t)bc * c;
                for (int j = 0; j < c; ++j)
                    if (v[j] == 1.0f || v[j] == -1.0f) {
                        h[bc] = 1;
                        break;
                    }
            }
        }
    long long k = 0;
    for (unsigned char h : hit) k += h;
    if (k * r * c > INT_MAX) return nullptr;
    bcsr_t* m = static_cast<bcsr_t*>(alloc32(sizeof(bcsr_t)));
    if (!m) return nullptr;
    m->r = r;
    m->c = c;
    m->br = nbr;
    m->bc = nbc;
    m->k = (int)k;
    m->b_row_start = static_cast<int*>(alloc32(((size_t)nbr + 1) * sizeof(int)));
    m->b_col_idx = static_cast<int*>(alloc32((size_t)k * sizeof(int)));
    m->b_values = static_cast<float*>(alloc32((size_t)k * r * c * sizeof(float)));
    if (!m->b_row_start || !m->b_col_idx || !m->b_values) {
        bcsr_free(m);
        return nullptr;
    }
    // pass 2 (bcsr.c:101-137): b_row_start gets the first block of every
    // NON-EMPTY block row, then k; the rest (uninitialised there) is k too
    int w = 0, blk = 0;
    for (int b = 0; b < nbr; ++b) {
        bool first = true;
        for (int bc = 0; bc < nbc; ++bc) {
            if (!hit[(size_t)b * nbc + bc]) continue;
            if (first) {
                m->b_row_start[w++] = blk;
                first = false;
            }
            m->b_col_idx[blk] = bc;
            float* dst = m->b_values + (size_t)blk * r * c;
            for (int i = 0; i < r; ++i)
                std::memcpy(dst + (size_t)i * c, dense + (size_t)(b * r + i) * cols + (size_t)bc * c, (size_t)c * sizeof(float));
            ++blk;
        }
    }
    for (int i = w; i <= nbr; ++i) m->b_row_start[i] = blk;
    return m;
}

void bcsr_free(bcsr_t* W) {
    if (!W) return;
    std::free(W->b_row_start);
    std::free(W->b_col_idx);
    std::free(W->b_values);
    std::free(W);
}

void bcsr_sgemm_basic(const dense_t X, const bcsr_t W, const dense_t B, dense_t Y, int M, int N, int K) {
    host_sgemm(BCSR_VARIANT_BASIC, X, W, B, 0.0f, Y, M, N, K);
}

void bcsr_sgemm_prelu_basic(const dense_t X, const bcsr_t W, const dense_t B, float a, dense_t Y, int M, int N, int K) {
    host_sgemm(BCSR_VARIANT_PRELU_BASIC, X, W, B, a, Y, M, N, K);
}

void bcsr_sgemm_avx(const dense_t X, const bcsr_t W, const dense_t B, dense_t Y, int M, int N, int K) {
    host_sgemm(BCSR_VARIANT_AVX, X, W, B, 0.0f, Y, M, N, K);
}

void bcsr_sgemm_prelu_avx(const dense_t X, const bcsr_t W, const dense_t B, float a, dense_t Y, int M, int N, int K) {
    host_sgemm(BCSR_VARIANT_PRELU_AVX, X, W, B, a, Y, M, N, K);
}

void bcsr_sgemm_avx2(const dense_t X, const bcsr_t W, const dense_t B, dense_t Y, int M, int N, int K) {
    host_sgemm(BCSR_VARIANT_AVX2, X, W, B, 0.0f, Y, M, N, K);
}

// ---------------------------------------------------------------------------
// Device API (include/bcsr_gpu.h)
// ---------------------------------------------------------------------------
int bcsr_gpu_plan_create(const bcsr_t* W, int device, void* stream, bcsr_gpu_plan** out) {
    return plan_create(W, device, static_cast<hipStream_t>(stream), out);
}

int bcsr_gpu_plan_stats(const bcsr_gpu_plan* p, long long* block_visits, size_t* device_bytes) {
    if (!p) return fail(TCSC_E_ARG, "bcsr_gpu_plan_stats: NULL plan");
    if (block_visits) *block_visits = p->visits;
    if (device_bytes) *device_bytes = p->bytes + p->xt_bytes;
    return TCSC_OK;
}

int bcsr_gpu_plan_reserve(bcsr_gpu_plan* p, int max_M, int K) {
    if (!p || max_M < 0 || K < 0) return fail(TCSC_E_ARG, "bcsr_gpu_plan_reserve: bad arguments");
    return reserve(p, max_M, K);
}

void bcsr_gpu_plan_destroy(bcsr_gpu_plan* p) { free_plan(p); }

int bcsr_gpu_sgemm(const bcsr_gpu_plan* p, const float* dX, const float* dB, float* dY, int M, int N, int K, int ldy,
                   int variant, float a, void* stream) {
    return run(p, dX, dB, dY, M, N, K, ldy, variant, a, static_cast<hipStream_t>(stream), 0);
}

int bcsr_gpu_prepare_x(const bcsr_gpu_plan* p, const float* dX, int M, int K, void* stream) {
    return run(p, dX, nullptr, nullptr, M, 0, K, 0, BCSR_VARIANT_BASIC, 0.f, static_cast<hipStream_t>(stream), 1);
}

int bcsr_gpu_sgemm_prepared(const bcsr_gpu_plan* p, const float* dB, float* dY, int M, int N, int K, int ldy,
                            int variant, float a, void* stream) {
    return run(p, nullptr, dB, dY, M, N, K, ldy, variant, a, static_cast<hipStream_t>(stream), 2);
}

}  // extern "C"
