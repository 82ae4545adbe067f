// tcsc_kernels.hip -- gfx950 (MI355X / CDNA4) kernels for the TCSC
// sparse-ternary GEMM  Y = act(X * W + b),  W in {-1,0,+1}.
//
// Replaces the CPU loops of /root/reference/sparse/tcsc.c:
//   tcsc_sgemm_basic                     tcsc.c:69-98
//   tcsc_sgemm_optimized                 tcsc.c:101-140
//   tcsc_sgemm_prelu_basic               tcsc.c:143-165
//   tcsc_sgemm_prelu_optimized_separate  tcsc.c:179-227
//   tcsc_sgemm_prelu_optimized_onthego   tcsc.c:231-275
// and tcsc_from_dense (tcsc.c:6-66) with a device builder.
//
// Kernel K1 (k_stream) -- DESIGN.md has the derivation and the measured
// primitive rates it rests on:
//  * lanes = rows.  A workgroup owns kTM = 256 rows of X (4 per lane) and
//    kWaves*kCW = 256 output columns; it walks K in chunks of kTK = 64 rows.
//    Each chunk of X is staged in LDS transposed (one 1-KiB row per k,
//    double-buffered), so one nonzero of W is ONE conflict-free ds_read_b128
//    that every lane issues at the same k, then two v_pk_fma_f32 with a +-1
//    scalar (an exact add/subtract).  No multiplies of data, no MFMA: W is
//    ternary and 98 % sparse at the headline size.
//  * W is re-laid out once per tcsc_t (the "plan"): for every (K chunk,
//    wave-column group) one flat stream of 8-byte entries {+-1.0f,
//    lds_row<<10 | 4*slot}, padded to a multiple of 8.  A wave reads its
//    stream with s_load_dwordx16 (8 entries per scalar load) and selects the
//    accumulator of the entry's column with s_set_gpr_idx_on (relative VGPR
//    addressing on the v_pk_fma DST/SRC2): no per-column loop, no branch per
//    nonzero, 2 SALU + 3 VALU + 1 LDS instruction per nonzero.
//  * Accumulators (4*kCW VGPRs) live in registers for the whole K range; the
//    epilogue adds the bias (first or last, matching the reference variant's
//    order) and applies PReLU before the only store of Y.  Small grids split
//    K over workgroups (k-slices) and reduce the fp32 partial slabs in a
//    fixed order (deterministic) in k_reduce.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "tcsc_internal.h"

namespace tcsc {

typedef float f32x32 __attribute__((ext_vector_type(32)));

// ---------------------------------------------------------------------------
// Plan building
// ---------------------------------------------------------------------------

__device__ __forceinline__ int lower_bound_i32(const int* __restrict__ a, int lo, int hi, int key) {
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (a[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// lbp/lbn[c*ncols + n] = absolute position of the first +1 (-1) entry of
// column n with row >= c*kTK  (c in [0, nch]; c == nch -> column end).
__global__ void k_chunk_bounds(const int* __restrict__ csp, const int* __restrict__ csn,
                               const int* __restrict__ rip, const int* __restrict__ rin,
                               int col_begin, int ncols, int nch, int* __restrict__ lbp, int* __restrict__ lbn) {
    const long long total = (long long)(nch + 1) * ncols;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int c = (int)(i / ncols), n = (int)(i % ncols);
        const int key = (c == nch) ? 0x7fffffff : c * kTK;
        const int gn = col_begin + n;
        lbp[i] = lower_bound_i32(rip, csp[gn], csp[gn + 1], key);
        lbn[i] = lower_bound_i32(rin, csn[gn], csn[gn + 1], key);
    }
}

// cnt[c*ncols + n] = nonzeros of column n inside chunk c.
__global__ void k_chunk_counts(const int* __restrict__ lbp, const int* __restrict__ lbn, int ncols, int nch,
                               int* __restrict__ cnt) {
    const long long total = (long long)nch * ncols;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x)
        cnt[i] = (lbp[i + ncols] - lbp[i]) + (lbn[i + ncols] - lbn[i]);
}

// gcnt[c*G + g] = entries of group g in chunk c, rounded up to kBatch.
__global__ void k_group_counts(const int* __restrict__ cptr, int ncols, int nch, int G, int* __restrict__ gcnt) {
    const long long total = (long long)nch * G;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int c = (int)(i / G), g = (int)(i % G);
        const int n0 = g * kCW, n1 = min(n0 + kCW, ncols);
        const int real = cptr[(long long)c * ncols + n1] - cptr[(long long)c * ncols + n0];
        gcnt[i] = (real + kBatch - 1) / kBatch * kBatch;
    }
}

__device__ __forceinline__ int lds_row_of(int c, int k_local) { return (c & 1) * kBufRows + k_local; }

// Scatter the +1 (SIGN=0) or -1 (SIGN=1) entries to their stream slot.
// Inside a (chunk, group) stream the columns follow each other and every
// column's entries are in ascending row order (the +1/-1 lists merged), so
// each output accumulates its nonzeros in ascending k.
template <int SIGN>
__global__ void k_scatter(const int* __restrict__ cs_own, const int* __restrict__ ri_own,
                          const int* __restrict__ cs_oth, const int* __restrict__ ri_oth,
                          const int* __restrict__ lb_own, const int* __restrict__ lb_oth,
                          const int* __restrict__ cptr, const int* __restrict__ sptr, int col_begin, int ncols,
                          int G, int2* __restrict__ ent) {
    const int base = cs_own[col_begin];
    const int total = cs_own[col_begin + ncols] - base;
    const int sgn = SIGN ? (int)0xbf800000u : 0x3f800000;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
        const int i = base + t;
        int lo = 0, hi = ncols;  // last n with cs_own[col_begin+n] <= i
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (cs_own[col_begin + mid] <= i) lo = mid; else hi = mid;
        }
        const int n = lo, gn = col_begin + n;
        const int k = ri_own[i];
        const int c = k / kTK;
        const long long b = (long long)c * ncols + n;
        const int g = n / kCW, j = n - g * kCW;
        const int rank_own = i - lb_own[b];
        const int rank_oth = lower_bound_i32(ri_oth, cs_oth[gn], cs_oth[gn + 1], k) - lb_oth[b];
        const int in_group = cptr[b] - cptr[(long long)c * ncols + g * kCW];
        const int pos = sptr[(long long)c * G + g] + in_group + rank_own + rank_oth;
        ent[pos] = make_int2(sgn, (lds_row_of(c, k - c * kTK) << 10) | (4 * j));
    }
}

// Padding entries: +1 x (the -0.0 row) -- an exact no-op on any accumulator.
__global__ void k_fill_pads(const int* __restrict__ cptr, const int* __restrict__ sptr, int ncols, int nch, int G,
                            int2* __restrict__ ent, long long n_entries) {
    const long long total = (long long)nch * G;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int c = (int)(i / G), g = (int)(i % G);
        const int n0 = g * kCW, n1 = min(n0 + kCW, ncols);
        const int real = cptr[(long long)c * ncols + n1] - cptr[(long long)c * ncols + n0];
        const int s0 = sptr[i], s1 = sptr[i + 1];
        const int2 pad = make_int2(0x3f800000, lds_row_of(c, kTK) << 10);
        for (int p = s0 + real; p < s1; ++p) ent[p] = pad;
    }
    // trailing guard block (never consumed; keeps the 64-entry block loads in bounds)
    if (blockIdx.x == 0 && threadIdx.x < kEntGuard) ent[n_entries + threadIdx.x] = make_int2(0x3f800000, kTK << 10);
}

// ---------------------------------------------------------------------------
// K1: the gather kernel
// ---------------------------------------------------------------------------

// Transposed staging of X[m0..m0+255][k0..k0+63] into an LDS buffer laid out
// [k][256 rows].  Each thread owns two 4x4 blocks (4 rows x 4 k): four
// coalesced float4 loads (rows), a register transpose, four ds_write_b128
// (k rows).  Lanes 0-7 of a wave own consecutive row quads so every 8-lane
// write group stores 128 contiguous bytes (conflict-free), and per load
// instruction the wave reads 8 rows x 128 B.
struct Stage {
    float4 v[2][4];
};

// Branch-free and select-free loads, so all eight issue back to back and are
// waited for once, at stage_store.  Values staged for rows >= M or k >= K are
// never used (no stream entry points at a k row past K, and rows past M are
// not stored), so only memory safety matters: VEC4 (K % 4 == 0, X 16-B
// aligned, (M+256)*K*4 < 2^31) uses raw buffer loads, whose range check
// returns 0 past the end of X; one 32-bit offset VGPR per row keeps address
// registers few, so the staged tile stays out of the registers the gather
// asm owns.  Otherwise clamped scalar loads.
template <bool VEC4>
__device__ __forceinline__ void stage_load(Stage& s, const float* __restrict__ X, int M, int K, int m0, int k0) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int mq = (lane & 7) + 8 * w;  // 0..63
    if (VEC4) {
        const __amdgpu_buffer_rsrc_t rsrc =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(X), (short)0, M * K * 4, 0x00020000);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int kk = k0 + 4 * ((lane >> 3) + 8 * h);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const unsigned off = (unsigned)((m0 + 4 * mq + r) * K + kk) * 4u;
                s.v[h][r] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0));
            }
        }
        return;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int kk = k0 + 4 * ((lane >> 3) + 8 * h);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = min(m0 + 4 * mq + r, M - 1);
            const float* src = X + (size_t)row * K;
            s.v[h][r] = make_float4(src[min(kk, K - 1)], src[min(kk + 1, K - 1)], src[min(kk + 2, K - 1)],
                                    src[min(kk + 3, K - 1)]);
        }
    }
}

__device__ __forceinline__ void stage_store(const Stage& s, char* __restrict__ buf) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int mq = (lane & 7) + 8 * w;
        const int kq = (lane >> 3) + 8 * h;
        char* p = buf + (4 * kq) * kRowBytes + mq * 16;
        *reinterpret_cast<float4*>(p + 0 * kRowBytes) = make_float4(s.v[h][0].x, s.v[h][1].x, s.v[h][2].x, s.v[h][3].x);
        *reinterpret_cast<float4*>(p + 1 * kRowBytes) = make_float4(s.v[h][0].y, s.v[h][1].y, s.v[h][2].y, s.v[h][3].y);
        *reinterpret_cast<float4*>(p + 2 * kRowBytes) = make_float4(s.v[h][0].z, s.v[h][1].z, s.v[h][2].z, s.v[h][3].z);
        *reinterpret_cast<float4*>(p + 3 * kRowBytes) = make_float4(s.v[h][0].w, s.v[h][1].w, s.v[h][2].w, s.v[h][3].w);
    }
}

#include "gather_asm.inc"

// Consume this wave's stream for one chunk: `nb` batches of 8 entries at
// `stream` (entries padded to a multiple of 8; the first 64-entry block is
// already in e_sgn/e_w1, lane i = entry i).  The schedule and register map
// are in tools/gen_gather_asm.py.  M0 is written by s_set_gpr_idx_*; it is a
// reserved register the compiler keeps nothing in for this kernel (no
// LDS-DMA, movrel or message instructions).
__device__ __forceinline__ void gather_stream(const int2* __restrict__ stream, unsigned nb, int e_sgn, int e_w1,
                                              unsigned lane_off, unsigned mask, f32x32& a0, f32x32& a1,
                                              f32x32& a2, f32x32& a3) {
    unsigned voff = (lane_off >> 4) * 8u;  // byte offset of this lane's entry in a block
    asm volatile(TCSC_GATHER_ASM
                 : [nb] "+s"(nb), "+{v[40:71]}"(a0), "+{v[72:103]}"(a1), "+{v[104:135]}"(a2),
                   "+{v[136:167]}"(a3), "+{v232}"(e_sgn), "+{v233}"(e_w1), "+{v236}"(voff)
                 : [ent] "s"(stream), [lane] "v"(lane_off), [mask] "v"(mask)
                 : "memory", "scc", "v168", "v169", "v170", "v171", "v172", "v173", "v174", "v175", "v176",
                   "v177", "v178", "v179", "v180", "v181", "v182", "v183", "v184", "v185", "v186", "v187", "v188",
                   "v189", "v190", "v191", "v192", "v193", "v194", "v195", "v196", "v197", "v198", "v199", "v200",
                   "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208", "v209", "v210", "v211", "v212",
                   "v213", "v214", "v215", "v216", "v217", "v218", "v219", "v220", "v221", "v222", "v223", "v224",
                   "v225", "v226", "v227", "v228", "v229", "v230", "v231", "v234", "v235", "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43",
                   "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", "s56", "s57",
                   "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67");
}

// i is a compile-time constant after unrolling
__device__ __forceinline__ float acc_get(const f32x32& a0, const f32x32& a1, const f32x32& a2, const f32x32& a3,
                                         int i) {
    return i < 32 ? a0[i] : (i < 64 ? a1[i - 32] : (i < 96 ? a2[i - 64] : a3[i - 96]));
}
__device__ __forceinline__ void acc_set(f32x32& a0, f32x32& a1, f32x32& a2, f32x32& a3, int i, float v) {
    if (i < 32) a0[i] = v;
    else if (i < 64) a1[i - 32] = v;
    else if (i < 96) a2[i - 64] = v;
    else a3[i - 96] = v;
}

// OUT: 0 = final Y (bias + activation), 1 = partial slab ws[slice][M][ncols]
template <bool BIAS_FIRST, bool PRELU, bool VEC4, int OUT>
__global__ void __launch_bounds__(kWaves * 64, 2)
k_stream(const float* __restrict__ X, int M, int K, const int2* __restrict__ ent, const int* __restrict__ sptr,
         int G, int ncols, int nch, int chunks_per_slice, const float* __restrict__ Bias, float* __restrict__ Y,
         int ldy, float a, float* __restrict__ ws) {
    __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = blockIdx.x * kWaves + wave;  // wave-column group
    const int m0 = blockIdx.y * kTM;
    const int c_begin = blockIdx.z * chunks_per_slice;
    const int c_end = min(nch, c_begin + chunks_per_slice);
    const bool active = g < G;

    f32x32 a0, a1, a2, a3;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        a0[i] = 0.f;
        a1[i] = 0.f;
        a2[i] = 0.f;
        a3[i] = 0.f;
    }
    if (BIAS_FIRST && OUT == 0 && active) {
        // one vector load of the wave's 32 bias values, then lane broadcasts
        // (keeps them out of the SGPRs the gather loop owns)
        const int cb = g * kCW + (lane & (kCW - 1));
        const float bv = cb < ncols ? Bias[cb] : 0.f;
#pragma unroll
        for (int j = 0; j < kCW; ++j) {
            const float b = __shfl(bv, j);
#pragma unroll
            for (int r = 0; r < 4; ++r) acc_set(a0, a1, a2, a3, 4 * j + r, b);
        }
    }

    // the -0.0 pad rows of both buffers (entries padding a stream point here)
    if (threadIdx.x < 64) {
        reinterpret_cast<float4*>(lds + kTK * kRowBytes)[threadIdx.x] = make_float4(-0.f, -0.f, -0.f, -0.f);
        reinterpret_cast<float4*>(lds + (kBufRows + kTK) * kRowBytes)[threadIdx.x] =
            make_float4(-0.f, -0.f, -0.f, -0.f);
    }
    Stage st;
    if (c_begin < c_end) {
        stage_load<VEC4>(st, X, M, K, m0, c_begin * kTK);
        stage_store(st, lds + (c_begin & 1) * kBufRows * kRowBytes);
    }
    __syncthreads();

    const unsigned lane_off = 16u * lane;
    const unsigned mask = 0x3ffu;
    // Software-pipelined chunk loop.  Stream bounds come 64 chunks at a time
    // (lane i = chunk cb+i) and are read with readlane; the first entry block
    // of chunk c+1 is loaded during chunk c, before the staging loads, so the
    // gather's input was issued a whole chunk earlier.  No branches around
    // the loads: staging the chunk after the last one and streams of idle
    // waves are harmless (clamped reads, nb = 0, an LDS buffer nobody reads).
    const int gi = active ? g : G - 1;
    int cb = c_begin;
    int vs0 = 0, vs1 = 0;
    int2 en = make_int2(0, 0);
    int s0n = 0, s1n = 0;
    if (c_begin < c_end) {
        const long long ci = (long long)min(cb + lane, nch - 1) * G + gi;
        vs0 = sptr[ci];
        vs1 = sptr[ci + 1];
        s0n = __builtin_amdgcn_readlane(vs0, 0);
        s1n = __builtin_amdgcn_readlane(vs1, 0);
        en = ent[s0n + lane];
    }
    for (int c = c_begin; c < c_end; ++c) {
        const int s0 = s0n, s1 = s1n;
        const int2 e = en;
        int idx = c + 1 - cb;
        if (idx == 64) {
            cb += 64;
            idx = 0;
            const long long ci = (long long)min(cb + lane, nch - 1) * G + gi;
            vs0 = sptr[ci];
            vs1 = sptr[ci + 1];
        }
        s0n = __builtin_amdgcn_readlane(vs0, idx);
        s1n = __builtin_amdgcn_readlane(vs1, idx);
        en = ent[s0n + lane];
        asm volatile("" ::: "memory");  // keep the entry load ahead of the staging loads
        stage_load<VEC4>(st, X, M, K, m0, (c + 1) * kTK);
        const unsigned nb = active ? (unsigned)(s1 - s0) / kBatch : 0u;
        gather_stream(ent + s0, nb, e.x, e.y, lane_off, mask, a0, a1, a2, a3);
        stage_store(st, lds + ((c + 1) & 1) * kBufRows * kRowBytes);
        __syncthreads();
    }

    if (!active) return;
#pragma unroll
    for (int j = 0; j < kCW; ++j) {
        const int col = g * kCW + j;
        if (col < ncols) {
            float b = 0.f;
            if (OUT == 0 && !BIAS_FIRST) b = Bias[col];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + 4 * lane + r;
                if (row < M) {
                    float v = acc_get(a0, a1, a2, a3, 4 * j + r);
                    if (OUT == 0) {
                        if (!BIAS_FIRST) v += b;
                        if (PRELU) v = (v < 0.0f) ? a * v : v;
                        Y[(size_t)row * ldy + col] = v;
                    } else {
                        ws[((size_t)blockIdx.z * M + row) * ncols + col] = v;
                    }
                }
            }
        }
    }
}

// Split-K combine in slice order (deterministic): y = act(b + s0 + s1 ...)
// or act(s0 + s1 + ... + b) depending on the variant's bias order.
template <bool BIAS_FIRST, bool PRELU>
__global__ void k_reduce(const float* __restrict__ ws, int slices, int M, int ncols, const float* __restrict__ Bias,
                         float* __restrict__ Y, int ldy, float a) {
    const long long total = (long long)M * ncols;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int row = (int)(i / ncols), col = (int)(i % ncols);
        float v = BIAS_FIRST ? Bias[col] : 0.f;
        for (int s = 0; s < slices; ++s) v += ws[(size_t)s * total + i];
        if (!BIAS_FIRST) v += Bias[col];
        if (PRELU) v = (v < 0.0f) ? a * v : v;
        Y[(size_t)row * ldy + col] = v;
    }
}

// ---------------------------------------------------------------------------
// Device tcsc_from_dense (bit-exact with tcsc.c:6-66): per-column counts,
// exclusive scans, then a fill that keeps rows ascending inside a column.
// ---------------------------------------------------------------------------
__global__ void k_dense_col_counts(const float* __restrict__ D, int rows, int cols, int* __restrict__ cntp,
                                   int* __restrict__ cntn) {
    for (int n = blockIdx.x * blockDim.x + threadIdx.x; n < cols; n += gridDim.x * blockDim.x) {
        int p = 0, q = 0;
        for (int i = 0; i < rows; ++i) {
            const float v = D[(size_t)i * cols + n];
            p += (v == 1.0f);
            q += (v == -1.0f);
        }
        cntp[n] = p;
        cntn[n] = q;
    }
}

__global__ void k_dense_fill(const float* __restrict__ D, int rows, int cols, const int* __restrict__ csp,
                             const int* __restrict__ csn, int* __restrict__ rip, int* __restrict__ rin) {
    for (int n = blockIdx.x * blockDim.x + threadIdx.x; n < cols; n += gridDim.x * blockDim.x) {
        int p = csp[n], q = csn[n];
        for (int i = 0; i < rows; ++i) {
            const float v = D[(size_t)i * cols + n];
            if (v == 1.0f) rip[p++] = i;
            else if (v == -1.0f) rin[q++] = i;
        }
    }
}

// ---------------------------------------------------------------------------
// Host-side launchers (called from tcsc_api.cpp)
// ---------------------------------------------------------------------------

static inline int grid_for(long long n, int block) {
    long long g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > 65535LL * 16) g = 65535LL * 16;
    return (int)g;
}

hipError_t plan_scan_tmp_bytes(long long n, size_t* bytes) {
    *bytes = 0;
    return hipcub::DeviceScan::ExclusiveSum(nullptr, *bytes, (int*)nullptr, (int*)nullptr, (int)n, (hipStream_t)0);
}

// Phase 1: chunk bounds, per-(chunk, column) counts and their scan (cptr),
// per-(chunk, group) padded stream lengths (gcnt, with a trailing 0).
hipError_t plan_counts(const PlanDev& in, PlanOut& out, hipStream_t st) {
    const int ncols = in.ncols, nch = out.n_chunks, G = out.n_groups;
    hipError_t e;
    const long long nb = (long long)(nch + 1) * ncols;
    hipLaunchKernelGGL(k_chunk_bounds, dim3(grid_for(nb, 256)), dim3(256), 0, st, in.csp, in.csn, in.rip, in.rin,
                       in.col_begin, ncols, nch, out.lbp, out.lbn);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const long long nc = (long long)nch * ncols;
    hipLaunchKernelGGL(k_chunk_counts, dim3(grid_for(nc, 256)), dim3(256), 0, st, out.lbp, out.lbn, ncols, nch,
                       out.cnt);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    size_t tb = out.scan_tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(out.scan_tmp, tb, out.cnt, out.cptr, (int)(nc + 1), st)) != hipSuccess)
        return e;
    const long long ng = (long long)nch * G;
    hipLaunchKernelGGL(k_group_counts, dim3(grid_for(ng, 256)), dim3(256), 0, st, out.cptr, ncols, nch, G, out.gcnt);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    tb = out.scan_tmp_bytes;
    return hipcub::DeviceScan::ExclusiveSum(out.scan_tmp, tb, out.gcnt, out.sptr, (int)(ng + 1), st);
}

// Phase 2 (ent allocated with n_entries + kBatch): scatter + padding.
hipError_t plan_fill(const PlanDev& in, PlanOut& out, hipStream_t st) {
    const int ncols = in.ncols, nch = out.n_chunks, G = out.n_groups;
    hipError_t e;
    if (in.n_pos > 0) {
        hipLaunchKernelGGL(k_scatter<0>, dim3(grid_for(in.n_pos, 256)), dim3(256), 0, st, in.csp, in.rip, in.csn,
                           in.rin, out.lbp, out.lbn, out.cptr, out.sptr, in.col_begin, ncols, G, out.ent);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (in.n_neg > 0) {
        hipLaunchKernelGGL(k_scatter<1>, dim3(grid_for(in.n_neg, 256)), dim3(256), 0, st, in.csn, in.rin, in.csp,
                           in.rip, out.lbn, out.lbp, out.cptr, out.sptr, in.col_begin, ncols, G, out.ent);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    const long long ng = (long long)nch * G;
    hipLaunchKernelGGL(k_fill_pads, dim3(grid_for(ng, 256)), dim3(256), 0, st, out.cptr, out.sptr, ncols, nch, G,
                       out.ent, out.n_entries);
    return hipGetLastError();
}

size_t workspace_bytes(int M, int ncols, int slices) {
    return slices > 1 ? (size_t)slices * M * ncols * sizeof(float) : 0;
}

// Cost model (cycles of one CU at ~2.1 GHz) for k-slicing: every workgroup
// runs on its own CU; gathers cost ~1 KiB / 220 B/clk per nonzero and
// wave, staging ~1 KiB / 79 B/clk per k row (MI355X_MICROARCH.md LDS rows,
// DESIGN.md measurements); the split-K slabs cost HBM time.
int choose_slices(int M, int ncols, int K, long long nnz, int G, size_t ws_bytes, int force) {
    const int nch = (K + kTK - 1) / kTK;
    if (nch <= 1) return 1;
    const int rt = (M + kTM - 1) / kTM;
    const int cb = (G + kWaves - 1) / kWaves;
    const long long base = (long long)rt * cb;
    auto cap = [&](int s) { return s <= nch && workspace_bytes(M, ncols, s) <= ws_bytes; };
    if (force > 0) return cap(force) ? force : 1;
    const double nz_per_chunk_block = (double)nnz / nch / cb;  // per workgroup and chunk (all its waves)
    const double chunk_cycles = nz_per_chunk_block * (1024.0 / 220.0) + kTK * (1024.0 / 79.0) + 600.0;
    double best = 1e300;
    int best_s = 1;
    for (int s = 1; s <= 16; ++s) {
        if (!cap(s)) break;
        const long long blocks = base * s;
        const long long rounds = (blocks + 255) / 256;
        const int cps = (nch + s - 1) / s;
        double t = (double)rounds * cps * chunk_cycles;
        if (s > 1) t += (double)(s + 1) * M * ncols * 4.0 / 5.0e12 * 2.1e9 + 4000.0;
        if (t < best * 0.97) {
            best = t;
            best_s = s;
        }
    }
    return best_s;
}

template <bool BF, bool PR>
static hipError_t launch_t(const GemmArgs& g, int slices, bool vec4, hipStream_t st) {
    const int nch = (g.K + kTK - 1) / kTK;
    int cps = nch > 0 ? (nch + slices - 1) / slices : 1;
    slices = nch > 0 ? (nch + cps - 1) / cps : 1;
    dim3 grid((g.n_groups + kWaves - 1) / kWaves, (g.M + kTM - 1) / kTM, slices);
    dim3 block(kWaves * 64);
    if (slices == 1) {
        if (vec4)
            hipLaunchKernelGGL((k_stream<BF, PR, true, 0>), grid, block, 0, st, g.X, g.M, g.K, g.ent, g.sptr,
                               g.n_groups, g.ncols, nch, cps, g.B, g.Y, g.ldy, g.a, g.ws);
        else
            hipLaunchKernelGGL((k_stream<BF, PR, false, 0>), grid, block, 0, st, g.X, g.M, g.K, g.ent, g.sptr,
                               g.n_groups, g.ncols, nch, cps, g.B, g.Y, g.ldy, g.a, g.ws);
        return hipGetLastError();
    }
    if (vec4)
        hipLaunchKernelGGL((k_stream<BF, PR, true, 1>), grid, block, 0, st, g.X, g.M, g.K, g.ent, g.sptr, g.n_groups,
                           g.ncols, nch, cps, g.B, g.Y, g.ldy, g.a, g.ws);
    else
        hipLaunchKernelGGL((k_stream<BF, PR, false, 1>), grid, block, 0, st, g.X, g.M, g.K, g.ent, g.sptr,
                           g.n_groups, g.ncols, nch, cps, g.B, g.Y, g.ldy, g.a, g.ws);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const long long total = (long long)g.M * g.ncols;
    hipLaunchKernelGGL((k_reduce<BF, PR>), dim3(grid_for(total, 256)), dim3(256), 0, st, g.ws, slices, g.M,
                       g.ncols, g.B, g.Y, g.ldy, g.a);
    return hipGetLastError();
}

hipError_t launch_gemm(const GemmArgs& g, hipStream_t st) {
    if (g.M <= 0 || g.ncols <= 0) return hipSuccess;
    const bool vec4 = (g.K % 4 == 0) && ((reinterpret_cast<uintptr_t>(g.X) & 15) == 0) &&
                      ((long long)(g.M + kTM) * g.K * 4 < (1LL << 31));
    const int s = choose_slices(g.M, g.ncols, g.K, g.nnz, g.n_groups, g.ws ? g.ws_bytes : 0, g.force_slices);
    if (g.bias_first) {
        return g.prelu ? launch_t<true, true>(g, s, vec4, st) : launch_t<true, false>(g, s, vec4, st);
    }
    return g.prelu ? launch_t<false, true>(g, s, vec4, st) : launch_t<false, false>(g, s, vec4, st);
}

hipError_t dense_to_tcsc_counts(const float* D, int rows, int cols, int* cntp, int* cntn, hipStream_t st) {
    hipLaunchKernelGGL(k_dense_col_counts, dim3(grid_for(cols, 256)), dim3(256), 0, st, D, rows, cols, cntp, cntn);
    return hipGetLastError();
}

hipError_t dense_to_tcsc_fill(const float* D, int rows, int cols, const int* csp, const int* csn, int* rip, int* rin,
                              hipStream_t st) {
    hipLaunchKernelGGL(k_dense_fill, dim3(grid_for(cols, 256)), dim3(256), 0, st, D, rows, cols, csp, csn, rip, rin);
    return hipGetLastError();
}

hipError_t exclusive_scan_i32(const int* in, int* out, int n, void* tmp, size_t tmp_bytes, hipStream_t st) {
    return hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, in, out, n, st);
}

}  // namespace tcsc
