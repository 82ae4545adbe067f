// tcsc_internal.h -- shared between the kernels (tcsc_kernels.hip) and the
// C-ABI layer (tcsc_api.cpp).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace tcsc {

// K rows per LDS chunk (one 512-B LDS row per k: 128 rows x fp32).
constexpr int kChunkK = 128;
// Entries are padded by this many ints so unrolled scalar loads never run
// past the allocation.
constexpr int kEntPad = 16;

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

// Plan arrays (device).  lbp/lbn/cnt/scan_tmp are build-time scratch.
struct PlanOut {
    int chunk_k = kChunkK;
    int n_chunks = 0;
    int* ent = nullptr;   // nnz (+kEntPad) merged entries
    int* cptr = nullptr;  // n_chunks*ncols + 1 bucket starts (chunk-major)
    int* lbp = nullptr;
    int* lbn = nullptr;
    int* cnt = nullptr;
    void* scan_tmp = nullptr;
    size_t scan_tmp_bytes = 0;
};

struct GemmArgs {
    const float* X = nullptr;
    int M = 0, K = 0;
    const int* ent = nullptr;
    const int* cptr = nullptr;
    int ncols = 0;
    int chunk_k = kChunkK;
    const float* B = nullptr;
    float* Y = nullptr;
    int ldy = 0;
    float a = 0.f;
    bool bias_first = false;
    bool prelu = false;
};

hipError_t plan_build(const PlanDev& in, PlanOut& out, hipStream_t st);
hipError_t plan_scan_tmp_bytes(long long n, size_t* bytes);
hipError_t launch_gemm(const GemmArgs& g, hipStream_t st);
hipError_t dense_to_tcsc_counts(const float* D, int rows, int cols, int* cntp, int* cntn, hipStream_t st);
hipError_t dense_to_tcsc_fill(const float* D, int rows, int cols, const int* csp, const int* csn, int* rip,
                              int* rin, hipStream_t st);
hipError_t exclusive_scan_i32(const int* in, int* out, int n, void* tmp, size_t tmp_bytes, hipStream_t st);

}  // namespace tcsc
