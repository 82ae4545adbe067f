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
//    kWaves*kCW = 256 output columns; it walks K in chunks of kTK = 48 rows.
//    Each chunk of X^T is DMA'd into LDS (one 1-KiB row per k, a ring of
//    kNBuf = 3 buffers, two chunks in flight), so one nonzero of W is ONE
//    conflict-free ds_read_b128
//    that every lane issues at the same k, then two v_pk_fma_f32 with a +-1
//    scalar (an exact add/subtract).  No multiplies of data, no MFMA: W is
//    ternary and 98 % sparse at the headline size.
//  * W is re-laid out once per tcsc_t (the "plan"): for every (K chunk,
//    wave-column group) one flat stream of 8-byte entries {+-1.0f,
//    lds_row<<10 | 4*slot}, unpadded.  A wave reads its
//    stream with s_load_dwordx16 (8 entries per scalar load) and selects the
//    accumulator of the entry's column with s_set_gpr_idx_on (relative VGPR
//    addressing on the v_pk_fma DST/SRC2): no per-column loop, no branch per
//    nonzero, 2 SALU + 3 VALU + 1 LDS instruction per nonzero.  Each wave
//    also pulls its stream ~4 chunks ahead into L2 (one LDS-DMA dword load
//    per chunk into a scratch), so the next chunk's scalar load hits L2.
//  * Accumulators (4*kCW VGPRs) live in registers for the whole K range; the
//    epilogue adds the bias (first or last, matching the reference variant's
//    order) and applies PReLU before the only store of Y.  Small grids split
//    K over workgroups (k-slices) and reduce the fp32 partial slabs in a
//    fixed order (deterministic) in k_reduce.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "tcsc_internal.h"

namespace tcsc {

// The generated gather loop (tools/gen_gather_asm.py) and its geometry.
#ifdef TCSC_GATHER_INC
#include TCSC_GATHER_INC
#else
#include "gather_asm.inc"
#endif
#ifndef TCSC_ACC_W
#define TCSC_ACC_W 32
#endif
// accumulator registers in TCSC_ACC_VECS vectors of TCSC_ACC_W (the generated asm operands)
typedef float facc_t __attribute__((ext_vector_type(TCSC_ACC_W)));
static_assert(TCSC_GEN_CW == kCW && TCSC_GEN_BATCH == kBatch, "generated loop geometry");
static_assert(TCSC_GEN_CAP + kHdr <= kEntGuard, "stream prefetch stays inside the entry guard");
static_assert(TCSC_GEN_HDR == 2 * kHdr, "generated loop and plan agree on the chunk header");
static_assert(TCSC_GEN_BUDGET == (512 / kWavesPerSimd) / 8 * 8, "generated loop VGPR budget");
#ifndef TCSC_GEN_TAIL
#define TCSC_GEN_TAIL 0
#endif
// Stream padding.  The generated loop ends every stream with a tail that
// gathers only its last, partial batch, so streams are unpadded (kPad 1); a
// loop without the tail needs every (chunk, wave) stream padded to whole
// batches with no-op entries (+1 x the -0.0 row).
constexpr int kPad = TCSC_GEN_TAIL ? 1 : kBatch;

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

// first position in a[lo, hi) with a[pos] > key
__device__ __forceinline__ int upper_bound_i32(const int* __restrict__ a, int lo, int hi, int key) {
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (a[mid] <= key) lo = mid + 1; else hi = mid;
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

// gcnt[g*nch + c] = entries of group g in chunk c (rounded up to kPad) plus
// the chunk header: group-major, so one group's chunks follow each other.
__global__ void k_group_counts(const int* __restrict__ cptr, int ncols, int nch, int G, int* __restrict__ gcnt) {
    const long long total = (long long)nch * G;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int g = (int)(i / nch), c = (int)(i % nch);
        const int n0 = group_col0(g), n1 = min(n0 + group_cols(g), ncols);
        const int real = cptr[(long long)c * ncols + n1] - cptr[(long long)c * ncols + n0];
        gcnt[i] = kHdr + (real + kPad - 1) / kPad * kPad;
    }
}

__device__ __forceinline__ int lds_row_of(int c, int k_local) { return (c % kNBuf) * kBufRows + k_local; }

// Scatter the +1 (SIGN=0) or -1 (SIGN=1) entries to their stream slot.
// Inside a (chunk, group) stream the columns follow each other and every
// column's entries are in ascending row order (the +1/-1 lists merged), so
// each output accumulates its nonzeros in ascending k.  A row present in
// both lists of a column (a hand-built tcsc_t; tcsc_from_dense never makes
// one) puts its +1 entry first: a +1 entry counts the -1 entries with a
// smaller row, a -1 entry the +1 entries with a smaller or equal row, so
// every slot of the merged stream gets exactly one entry.
template <int SIGN>
__global__ void k_scatter(const int* __restrict__ cs_own, const int* __restrict__ ri_own,
                          const int* __restrict__ cs_oth, const int* __restrict__ ri_oth,
                          const int* __restrict__ lb_own, const int* __restrict__ lb_oth,
                          const int* __restrict__ cptr, const int* __restrict__ sptr, int col_begin, int ncols,
                          int ent_nch, int2* __restrict__ ent) {
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
        int g = (n / kWgCols) * kWaves, j = n - (n / kWgCols) * kWgCols;  // group of column n, its slot
        while (j >= wave_cols(g % kWaves)) j -= wave_cols(g++ % kWaves);
        const int rank_own = i - lb_own[b];
        const int rank_oth = (SIGN ? upper_bound_i32(ri_oth, cs_oth[gn], cs_oth[gn + 1], k)
                                   : lower_bound_i32(ri_oth, cs_oth[gn], cs_oth[gn + 1], k)) - lb_oth[b];
        const int in_group = cptr[b] - cptr[(long long)c * ncols + group_col0(g)];
        const int pos = sptr[(long long)g * (ent_nch) + c] + kHdr + in_group + rank_own + rank_oth;
        ent[pos] = make_int2(sgn, (lds_row_of(c, k - c * kTK) << 10) | (4 * j));
    }
}

// Chunk headers and padding.  Header of (group g, chunk c), kHdr entries
// at sptr[g*nch + c]: {nb, rem} = the chunk's entries as whole batches +
// the rest, {byte distance to the next chunk's header, 0}.  Padding
// entries (padded streams only): +1 x (the -0.0 row), an exact no-op.
// After the last stream: an empty chain for idle waves (a header of no
// entries that points at itself), then guard entries that keep the
// scalar-buffer loads past a stream's end inside the allocation.
__global__ void k_fill_headers(const int* __restrict__ cptr, const int* __restrict__ sptr, int ncols, int nch, int G,
                               int2* __restrict__ ent, long long n_entries) {
    const long long total = (long long)nch * G;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int g = (int)(i / nch), c = (int)(i % nch);
        const int n0 = group_col0(g), n1 = min(n0 + group_cols(g), ncols);
        const int real = cptr[(long long)c * ncols + n1] - cptr[(long long)c * ncols + n0];
        const int s0 = sptr[i], s1 = sptr[i + 1];
        const int n = s1 - s0 - kHdr;
        ent[s0] = make_int2(n / kBatch, n % kBatch);
        ent[s0 + 1] = make_int2((s1 - s0) * (int)sizeof(int2), 0);
        const int2 pad = make_int2(0x3f800000, lds_row_of(c, kTK) << 10);
        for (int p = s0 + kHdr + real; p < s1; ++p) ent[p] = pad;
    }
    if (blockIdx.x == 0)
        for (int i = threadIdx.x; i < kEntGuard; i += blockDim.x)
            ent[n_entries + i] = i < kHdr ? make_int2(0, 0) : make_int2(0x3f800000, kTK << 10);
}

// Plan-build precondition on device-resident TCSC arrays, one thread per
// column of [col_begin, col_begin + ncols): col_start non-decreasing inside
// [0, n_total], row indices in [0, rows) (flag bit 0 otherwise: the
// reference would read outside X) and ascending (flag bit 1 otherwise: the
// plan's merge by binary search needs them sorted).
__global__ void k_check_index(const int* __restrict__ cs, const int* __restrict__ ri, int col_begin, int ncols,
                              int rows, int n_total, int* __restrict__ flag) {
    for (int n = blockIdx.x * blockDim.x + threadIdx.x; n < ncols; n += gridDim.x * blockDim.x) {
        const int a = cs[col_begin + n], b = cs[col_begin + n + 1];
        int f = 0;
        if (a < 0 || b < a || b > n_total) {
            f = 1;
        } else {
            int prev = -1;
            for (int i = a; i < b; ++i) {
                const int k = ri[i];
                if (k < 0 || k >= rows) f |= 1;
                if (k < prev) f |= 2;
                prev = k;
            }
        }
        if (f) atomicOr(flag, f);
    }
}

// out[j] = cs[col_begin + j] - cs[col_begin], j in [0, ncols]
__global__ void k_rebase(const int* __restrict__ cs, int col_begin, int ncols, int* __restrict__ out) {
    const int base = cs[col_begin];
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j <= ncols; j += gridDim.x * blockDim.x)
        out[j] = cs[col_begin + j] - base;
}

// ---------------------------------------------------------------------------
// K1: the gather kernel
// ---------------------------------------------------------------------------

// X (M x K, row-major) -> XT (K x ldxt), ldxt = M rounded up to kTM; the
// rows m in [M, ldxt) are written as 0.  64x64 tiles through LDS (the +1
// column keeps the column reads conflict-free).  HBM-bound: 2*M*K*4 bytes
// per call.  VEC (K % 4 == 0, X 16-B aligned): 16-B loads along k and
// 16-B stores along m; otherwise scalar, guarded.
template <bool VEC>
__global__ void __launch_bounds__(256) k_transpose(const float* __restrict__ X, int M, int K, float* __restrict__ XT,
                                                   int ldxt) {
    if (VEC) {
        // 64 (m) x 128 (k) tile: 512-B row reads, all 8 float4 loads of a
        // thread in flight before the first LDS write.  Row stride 129 keeps
        // the column reads conflict-free (129 = 1 mod 64 banks).
        __shared__ float tv[64][129];
        const int k0 = blockIdx.x * 128, m0 = blockIdx.y * 64;
        const int q2 = threadIdx.x & 31, r2 = threadIdx.x >> 5;  // 32 float4 per 128-wide row
        float4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int m = m0 + r2 + 8 * i, k = k0 + 4 * q2;
            v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (m < M && k < K) {
                typedef float nt4 __attribute__((ext_vector_type(4)));
                const nt4 w = __builtin_nontemporal_load(reinterpret_cast<const nt4*>(X + (size_t)m * K + k));
                v[i] = make_float4(w.x, w.y, w.z, w.w);
            }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int r = r2 + 8 * i;
            tv[r][4 * q2 + 0] = v[i].x;
            tv[r][4 * q2 + 1] = v[i].y;
            tv[r][4 * q2 + 2] = v[i].z;
            tv[r][4 * q2 + 3] = v[i].w;
        }
        __syncthreads();
        const int q = threadIdx.x & 15, rr = threadIdx.x >> 4;  // 16 float4 per 64-wide XT row piece
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int kk = rr + 16 * i, k = k0 + kk;
            if (k < K)
                *reinterpret_cast<float4*>(XT + (size_t)k * ldxt + m0 + 4 * q) =
                    make_float4(tv[4 * q + 0][kk], tv[4 * q + 1][kk], tv[4 * q + 2][kk], tv[4 * q + 3][kk]);
        }
        return;
    }
    __shared__ float t[64][65];
    const int k0 = blockIdx.x * 64, m0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int r = ty + 4 * i, m = m0 + r, k = k0 + tx;
        t[r][tx] = (m < M && k < K) ? X[(size_t)m * K + k] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int kk = ty + 4 * i, k = k0 + kk;
        if (k < K) XT[(size_t)k * ldxt + m0 + tx] = t[tx][kk];
    }
}

typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(4))) const i32x16 const_i32x16;
// the scalar buffer's last, 4- or 8-SGPR piece (header + CAP entries is not
// a multiple of 16 dwords)
typedef int sbuf_tail_t __attribute__((ext_vector_type(TCSC_SBUF_TAIL ? TCSC_SBUF_TAIL : 4)));
typedef __attribute__((address_space(4))) const sbuf_tail_t const_sbuf_tail;

// Consume this wave's stream for one chunk.  The chunk's header {nb, rem,
// bytes to the next header, 0} and first TCSC_GEN_CAP entries are already in
// the pinned SGPR buffer (sb, sbt: the caller's scalar loads); `ptr` is the
// header's address, from which the loop reloads the buffer for streams
// longer than the capacity, and which it leaves at the NEXT chunk's header.
// The schedule and register map are in tools/gen_gather_asm.py.
__device__ __forceinline__ void gather_stream(i32x16 (&sb)[TCSC_SBUF_VECS], sbuf_tail_t& sbt,
                                              unsigned long long& ptr, unsigned lane, unsigned mask,
                                              facc_t (&acc)[TCSC_ACC_VECS]) {
    (void)sbt;
#if (defined(TCSC_GEN_PF) && TCSC_GEN_PF) || TCSC_GEN_TOUCH
    int junk = 0;  // destination of the scalar-cache touches (tools/gen_gather_asm.py --touch / --pf)
    unsigned m0sv;
    asm volatile(TCSC_GATHER_ASM
                 : TCSC_ACC_OPERANDS(acc), TCSC_SBUF_OPERANDS(sb, sbt), TCSC_PTR_OPERAND(ptr), TCSC_JUNK_OPERAND(junk),
                   [m0sv] "=&s"(m0sv)
                 : [lane] "v"(lane * 16u), [mask] "v"(mask)
                 : TCSC_GATHER_CLOBBERS);
#else
    unsigned m0sv;
    asm volatile(TCSC_GATHER_ASM
                 : TCSC_ACC_OPERANDS(acc), TCSC_SBUF_OPERANDS(sb, sbt), TCSC_PTR_OPERAND(ptr), [m0sv] "=&s"(m0sv)
                 : [lane] "v"(lane * 16u), [mask] "v"(mask)
                 : TCSC_GATHER_CLOBBERS);
#endif
}

// Scalar (SMEM) load of a chunk's header and its first TCSC_GEN_CAP entries.
__device__ __forceinline__ void load_stream(i32x16 (&sb)[TCSC_SBUF_VECS], sbuf_tail_t& sbt, const char* p) {
    const_i32x16* q = reinterpret_cast<const_i32x16*>(reinterpret_cast<uintptr_t>(p));
#pragma unroll
    for (int i = 0; i < TCSC_SBUF_VECS; ++i) sb[i] = q[i];
#if TCSC_SBUF_TAIL
    sbt = *reinterpret_cast<const_sbuf_tail*>(reinterpret_cast<uintptr_t>(p + 64 * TCSC_SBUF_VECS));
#endif
}

// i is a compile-time constant after unrolling
__device__ __forceinline__ float acc_get(const facc_t (&acc)[TCSC_ACC_VECS], int i) { return acc[i / TCSC_ACC_W][i % TCSC_ACC_W]; }
__device__ __forceinline__ void acc_set(facc_t (&acc)[TCSC_ACC_VECS], int i, float v) { acc[i / TCSC_ACC_W][i % TCSC_ACC_W] = v; }

// LDS-DMA of X^T chunks.  Row k of chunk c = XT[c*kTK + k][m0..m0+255] (1
// KiB); wave w moves rows w*D .. w*D+D-1 (D = kDmaPerWave), lane l the 16 B
// of rows m0+4l..4l+3.  Per-lane offsets are fixed for the whole kernel, so
// a chunk costs D x (s_add m0 + global_load_lds_dwordx4) and one 64-bit base
// advance.  X^T carries kNBuf-1 chunks of padding rows past the last chunk,
// so the look-ahead never needs a clamp (those rows are never gathered).
// M0 is written in the same statement that reads it (the compiler keeps
// nothing in M0 across statements), with the s_nop the M0 -> LDS-DMA hazard
// asks for; the gather asm saves and restores it anyway.
struct DmaState {
    const char* next;              // byte address of the next chunk's first row, column m0
    unsigned voff[kDmaPerWave];    // lane*16 + (w*D + i) * ldxt*4
    unsigned lds_wave;             // LDS address of this wave's first row in buffer 0
    size_t chunk_bytes;            // kTK * ldxt * 4
};

#ifndef TCSC_DMA_OFFSET
#define TCSC_DMA_OFFSET 1
#endif
// TCSC_DMA_OFFSET: one M0 write per group of up to 4 rows.  The instruction
// offset (13-bit signed, 0..3 KiB here) moves the LDS destination (M0 +
// offset + 16*lane) and the global source alike; voff[i] carries
// -(i % 4) KiB to cancel it on the global side: 3 instructions per row ->
// ~1.7 (A/B: -0.9 % k_stream at cfg4).  0 = one M0 write per row.
template <int N>
__device__ __forceinline__ void dma_rows(unsigned m0, const unsigned* v, const char* src) {
    unsigned sv;  // M0 is saved and restored around every statement that writes it
    if constexpr (N == 4)
        asm volatile("s_mov_b32 %[sv], m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %6\n\t"
                     "global_load_lds_dwordx4 %3, %6 offset:1024\n\tglobal_load_lds_dwordx4 %4, %6 offset:2048\n\t"
                     "global_load_lds_dwordx4 %5, %6 offset:3072\n\ts_mov_b32 m0, %[sv]"
                     : [sv] "=&s"(sv)
                     : "s"(m0), "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "s"(src)
                     : "memory");
    else if constexpr (N == 3)
        asm volatile("s_mov_b32 %[sv], m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %5\n\t"
                     "global_load_lds_dwordx4 %3, %5 offset:1024\n\tglobal_load_lds_dwordx4 %4, %5 offset:2048\n\t"
                     "s_mov_b32 m0, %[sv]"
                     : [sv] "=&s"(sv)
                     : "s"(m0), "v"(v[0]), "v"(v[1]), "v"(v[2]), "s"(src)
                     : "memory");
    else if constexpr (N == 2)
        asm volatile("s_mov_b32 %[sv], m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %4\n\t"
                     "global_load_lds_dwordx4 %3, %4 offset:1024\n\ts_mov_b32 m0, %[sv]"
                     : [sv] "=&s"(sv)
                     : "s"(m0), "v"(v[0]), "v"(v[1]), "s"(src)
                     : "memory");
    else
        asm volatile("s_mov_b32 %[sv], m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %3\n\t"
                     "s_mov_b32 m0, %[sv]"
                     : [sv] "=&s"(sv)
                     : "s"(m0), "v"(v[0]), "s"(src)
                     : "memory");
}

template <int I0>
__device__ __forceinline__ void dma_groups(const DmaState& d, unsigned m0base) {
    if constexpr (I0 < kDmaPerWave) {
        constexpr int n = kDmaPerWave - I0 < 4 ? kDmaPerWave - I0 : 4;
        dma_rows<n>(m0base + I0 * kRowBytes, d.voff + I0, d.next);
        dma_groups<I0 + 4>(d, m0base);
    }
}

__device__ __forceinline__ void dma_next_chunk(DmaState& d, int buf) {
#if !((defined(TCSC_ABLATION) && TCSC_ABLATION == 6) || defined(TCSC_NODMA))
    const unsigned m0base = d.lds_wave + (unsigned)(buf * (kBufRows * kRowBytes));
#if TCSC_DMA_OFFSET
    dma_groups<0>(d, m0base);
#else
#pragma unroll
    for (int i = 0; i < kDmaPerWave; ++i) {
        unsigned sv;
        asm volatile("s_mov_b32 %[sv], m0\n\ts_add_u32 m0, %1, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %3, %4\n\t"
                     "s_mov_b32 m0, %[sv]"
                     : [sv] "=&s"(sv)
                     : "s"(m0base), "n"(i * kRowBytes), "v"(d.voff[i]), "s"(d.next)
                     : "memory", "scc");
    }
#endif
#endif
    d.next += d.chunk_bytes;
}

// L2 prefetch of the entry stream (kPfS): one global_load_lds_dword per wave
// and chunk into the wave's 256-B scratch; the data is never read.
__device__ __forceinline__ void pf_touch(unsigned m0, unsigned voff, const char* base) {
    unsigned sv;
    asm volatile("s_mov_b32 %[sv], m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %2, %3\n\t"
                 "s_mov_b32 m0, %[sv]"
                 : [sv] "=&s"(sv)
                 : "s"(m0), "v"(voff), "s"(base)
                 : "memory");
}

// XCD-aware tile order.  Workgroups are dealt round-robin over the 8 XCDs
// (MI355X_MICROARCH.md "Workgroup dispatch"; speed only, never correctness),
// so launch order L puts L % 8 on one XCD.  Renumber so each XCD gets a
// contiguous range of the (column block fastest, row tile, slice) order: the
// ~32 workgroups an XCD runs at once then share one row tile of X^T, and its
// L2 serves the rows they all stream.  Bijective for any grid size.
struct Tile {
    int cb, rt, z;
};
__device__ __forceinline__ Tile xcd_tile() {
    const int ncb = gridDim.x, nrt = gridDim.y;
    const int T = ncb * nrt * gridDim.z;
    const int L = blockIdx.x + ncb * (blockIdx.y + nrt * blockIdx.z);
    const int q = T >> 3, r = T & 7, x = L & 7;
    const int Lg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (L >> 3);
    Tile t;
    t.cb = Lg % ncb;
    const int rest = Lg / ncb;
    t.rt = rest % nrt;
    t.z = rest / nrt;
    return t;
}

#ifdef TCSC_STAMPS
// Diagnostic build only (make lib/abl/libtcsc_amd_stamps.so): per wave, the
// chunk loop's cycles summed by segment -- gather, post-gather (stream load
// + DMA issue, waited for), top-of-chunk (vmcnt + barrier) -- and its total;
// read with tcsc_debug_stamps().  Stamps never feed an output.
constexpr int kStampWgs = 4096;
__device__ unsigned long long g_stamps[kStampWgs * kWaves * 4];
// per workgroup (wave 0), s_memrealtime (100 MHz, one clock for the whole
// chip): entry, chunk loop start, chunk loop end, epilogue end, kernel end
__device__ unsigned long long g_wgtime[kStampWgs * 8];
__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
__device__ __forceinline__ unsigned long long rtstamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#endif

// In-launch split-K combine (k_stream OUT 2; DESIGN.md §4 k_reduce).  The
// Z workgroups of a tile (its K slices) each own row band z of the tile.
// Each writes the other bands of its slab with sc1 (write-through) stores;
// at Z = 4 (a band is exactly one 64-row epilogue pass) its own band stays
// in the LDS, otherwise it is written too.  It drains the stores (vmcnt(0)
// in every wave, barrier) and adds 1 to the tile's arrival word (lane 0,
// agent scope), then polls the arrival word (sc1 loads, s_sleep) until all
// Z have arrived, marks its band taken (state word 1) and reduces it: its
// own partial from the LDS, the others' from their slabs with sc1 loads --
// the same adds in the same order as k_reduce4, so the same bits.  A
// workgroup whose poll gives up (after kCombineWaitTicks of wall time, ~50
// us: a slice that is not resident, or TCSC_COMBINE_GIVEUP) first writes its
// own band to its slab (sc1, drained, barrier) and then marks it abandoned
// (state 2).  The workgroup whose add came last knows the slabs are
// complete without polling; after its own band it waits for every other
// band's state word to leave 0 (each owner is running: it has arrived) and
// reduces the abandoned ones from the slabs, so no band is left undone and
// none is reduced twice.  The last workgroup to finish (the done word)
// zeroes the tile's words for the next launch.  The host takes this path
// only when the grid fits the chip at one workgroup per CU
// (MI355X_MICROARCH.md "Workgroup dispatch ... inter-workgroup visibility",
// the counter hand-off row: sc1 stores, vmcnt(0), barrier, one agent add or
// store, sc1 poll or the add's return value, barrier, sc1 loads).
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4c_t __attribute__((ext_vector_type(4)));
constexpr int kSc1 = 16;  // buffer cache-policy bits: sc1
// The hand-off leans on gfx942/gfx950's lowering of sc1 loads and stores
// (L1 bypassed, written through to the memory side) and of relaxed
// agent-scope atomics; other targets would need the release/acquire fences
// (DESIGN.md §4 k_reduce, the protocol and its conditions).
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__) && !defined(__gfx942__)
#error "combine_tile's sc1 hand-off is written for gfx942/gfx950 only"
#endif
// A slice waits for its tile's other slices at most this long (s_memrealtime
// ticks, 100 MHz: 50 us, against a few us of measured slab skew); then it
// leaves its band to the tile's last arrival.
constexpr unsigned long long kCombineWaitTicks = 5000;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slabs_rsrc(float* ws, int Z, int M, int ncols) {
    const long long bytes = (long long)Z * M * ncols * 4;
    return __builtin_amdgcn_make_buffer_rsrc(ws, 0, (int)(bytes < 0x7fffffffLL ? bytes : 0x7fffffffLL), 0x00020000);
}

// The tile's own band at Z = 4 (k_stream's epilogue keeps it there): row R
// of the band at byte kOwnBandOff + R * 1 KiB, column j at + 4 j.
constexpr int kOwnBandOff = kWaves * 64 * (kCW * 4 + 16);  // past the epilogue's 64-row staging
static_assert(kOwnBandOff + 64 * kRowBytes <= kLdsBytes - 16, "the own band fits beside the epilogue staging");

template <bool BIAS_FIRST, bool PRELU>
__device__ __forceinline__ void combine_tile(float* ws, int M, int ncols, const float* __restrict__ Bias,
                                             float* __restrict__ Y, int ldy, float a, unsigned* ccnt, const Tile t,
                                             char* lds, int giveup, bool own_lds) {
    const int Z = (int)gridDim.z;
    unsigned* w = ccnt + (size_t)(t.rt * (int)gridDim.x + t.cb) * kCombineWords;  // {arrivals, done, state[Z]}
    int* flag = reinterpret_cast<int*>(lds);  // the epilogue's staging is done (barrier below)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's slab stores have left
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned old = __hip_atomic_fetch_add(w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int st = old + 1 == (unsigned)Z ? 2 : 0;  // 2: the last arrival, 1: saw all arrive, 0: gave up
        if (st == 0 && !giveup) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            for (;;) {
                if (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)Z) {
                    st = 1;
                    break;
                }
                if (__builtin_amdgcn_s_memrealtime() - t0 > kCombineWaitTicks) break;
                __builtin_amdgcn_s_sleep(4);
            }
        }
        if (st != 0) __hip_atomic_store(w + 2 + t.z, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        flag[0] = st;
    }
    __syncthreads();
    const int st = __builtin_amdgcn_readfirstlane(flag[0]);
    const __amdgpu_buffer_rsrc_t rs = slabs_rsrc(ws, Z, M, ncols);
    const int m0 = t.rt * kTM, c0 = t.cb * kWgCols;
    const size_t slab = (size_t)M * ncols;
    constexpr int nq = kWgCols / 4;
    // own: slab q's band q is in this workgroup's LDS; poison: a band whose
    // owner never marked it (the bounded wait below ran out, i.e. a broken
    // launch) is written as quiet NaN, never finalized from an unpublished slab
    auto reduce_band = [&](int q, bool own, bool poison = false) {
        const int r0 = kTM * q / Z, r1 = kTM * (q + 1) / Z;
        for (int i = threadIdx.x; i < (r1 - r0) * nq; i += kWaves * 64) {
            const int row = m0 + r0 + i / nq, col = c0 + 4 * (i % nq);
            if (row >= M || col >= ncols) continue;
            const int off = (int)((size_t)row * ncols + col) * 4;
            f32x4c_t p[16];
#pragma unroll
            for (int s = 0; s < 16; ++s)
                if (s < Z) {
                    if (own && s == q)
                        p[s] = *reinterpret_cast<const f32x4c_t*>(lds + kOwnBandOff + (i / nq) * kRowBytes +
                                                                  16 * (i % nq));
                    else
                        p[s] = __builtin_bit_cast(
                            f32x4c_t, __builtin_amdgcn_raw_buffer_load_b128(rs, off, (int)(s * slab * 4), kSc1));
                }
            const float4 b = *reinterpret_cast<const float4*>(Bias + col);
            float4 v = BIAS_FIRST ? b : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int s = 0; s < 16; ++s)
                if (s < Z) {
                    v.x += p[s].x;
                    v.y += p[s].y;
                    v.z += p[s].z;
                    v.w += p[s].w;
                }
            if (!BIAS_FIRST) {
                v.x += b.x;
                v.y += b.y;
                v.z += b.z;
                v.w += b.w;
            }
            if (PRELU) {
                v.x = (v.x < 0.0f) ? a * v.x : v.x;
                v.y = (v.y < 0.0f) ? a * v.y : v.y;
                v.z = (v.z < 0.0f) ? a * v.z : v.z;
                v.w = (v.w < 0.0f) ? a * v.w : v.w;
            }
            if (poison) v = make_float4(__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""));
            typedef float nt4 __attribute__((ext_vector_type(4)));
            nt4 o = {v.x, v.y, v.z, v.w};
            __builtin_nontemporal_store(o, reinterpret_cast<nt4*>(Y + (size_t)row * ldy + col));
        }
    };
    if (st != 0) {
        reduce_band(t.z, own_lds);
    } else {
        if (own_lds) {
            // give the band up: its LDS partial into slab t.z (sc1), drained by every wave
            const int r0 = kTM * t.z / Z, r1 = kTM * (t.z + 1) / Z;
            for (int i = threadIdx.x; i < (r1 - r0) * nq; i += kWaves * 64) {
                const int row = m0 + r0 + i / nq, col = c0 + 4 * (i % nq);
                if (row >= M || col >= ncols) continue;
                const int off = (int)(((size_t)t.z * M + row) * ncols + col) * 4;
                const f32x4c_t v =
                    *reinterpret_cast<const f32x4c_t*>(lds + kOwnBandOff + (i / nq) * kRowBytes + 16 * (i % nq));
                // whole quads: the host combines in launch only when ncols % 4 == 0
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rs, off, 0, kSc1);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        if (threadIdx.x == 0) __hip_atomic_store(w + 2 + t.z, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (st == 2) {
        // every other owner has arrived, so it is running and will mark its band
        // taken or abandoned; the bound (100 ms) only keeps a broken launch from
        // hanging the device
        for (int q = 0; q < Z; ++q) {
            if (q == t.z) continue;
            __syncthreads();  // everyone has read the previous flag
            if (threadIdx.x == 0) {
                const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                unsigned v;
                while ((v = __hip_atomic_load(w + 2 + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u &&
                       __builtin_amdgcn_s_memrealtime() - t0 < 10000000ull)
                    __builtin_amdgcn_s_sleep(2);
                flag[1] = (int)v;
            }
            __syncthreads();
            const int fq = __builtin_amdgcn_readfirstlane(flag[1]);
            if (fq == 2) reduce_band(q, false);
            else if (fq == 0) reduce_band(q, false, true);  // timed out: NaN, not a stale slab
        }
    }
    __syncthreads();
    if (threadIdx.x == 0 && __hip_atomic_fetch_add(w + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 ==
                                (unsigned)Z) {
        for (int i = 0; i < 2 + Z; ++i) __hip_atomic_store(w + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// OUT: 0 = final Y (bias + activation), 1 = partial slab ws[slice][M][ncols]
// (k_reduce combines), 2 = the slab, then the in-launch combine (combine_tile)
// ORDER (the summation order, DESIGN.md "Numerics"):
//   0  one plan, each column's +1 and -1 entries merged by ascending k;
//   1  the reference's order for tcsc_sgemm_basic / _prelu_basic
//      (tcsc.c:84-93, 149-161): the +1 chain (ent, all chunks) then the -1
//      chain (ent2, all chunks) into the same accumulator;
//   2  the reference's order for the optimized family (tcsc.c:113-137,
//      184-216, 244-273): the +1 sums from 0 are added to the bias and
//      parked in Y, the -1 chain sums from 0 again (its entries carry -1,
//      so the sum is exactly -acc_neg), and the epilogue adds it to the
//      parked value.
// Orders 1 and 2 walk K twice (the X^T chunks are staged twice) and never
// split K.
template <bool BIAS_FIRST, bool PRELU, int OUT, int ORDER>
__global__ void __launch_bounds__(kWaves * 64, kWavesPerSimd)
k_stream(const float* __restrict__ XT, int ldxt, int M, int K, const int2* __restrict__ ent,
         const int* __restrict__ sptr, long long n_entries, const int2* __restrict__ ent2,
         const int* __restrict__ sptr2, long long n_entries2, int G, int ncols, int nch, int chunks_per_slice,
         const float* __restrict__ Bias, float* __restrict__ Y, int ldy, float a, float* __restrict__ ws, int pf_dist,
         int pf_lines, unsigned* __restrict__ ccnt, int combine_giveup) {
    static_assert(ORDER == 0 || OUT == 0, "the reference orders do not split K");
    static_assert(OUT >= 0 && OUT <= 3, "OUT: 0 Y, 1 slab, 2 slab + band combine, 3 pairwise combine (2 slices)");
    __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const Tile t = xcd_tile();
    const int g = t.cb * kWaves + wave;  // wave-column group
    const int m0 = t.rt * kTM;
    const int c_begin = t.z * chunks_per_slice;
    const int c_end = min(nch, c_begin + chunks_per_slice);
    const bool active = g < G;
#ifdef TCSC_STAMPS
    unsigned long long rt_[7] = {rtstamp(), 0, 0, 0, 0, 0, 0};  // + [5] loads drained, [6] epilogue barrier
#endif

    facc_t acc[TCSC_ACC_VECS];
#pragma unroll
    for (int v = 0; v < TCSC_ACC_VECS; ++v)
#pragma unroll
        for (int i = 0; i < TCSC_ACC_W; ++i) acc[v][i] = 0.f;
    if (BIAS_FIRST && OUT == 0 && active) {
        // one vector load of the wave's bias values, then lane broadcasts
        // (keeps them out of the SGPRs the gather loop owns)
        const int cb = group_col0(g) + lane;
        const float bv = (lane < wave_cols(wave) && cb < ncols) ? Bias[cb] : 0.f;
#pragma unroll
        for (int j = 0; j < kCW; ++j) {
            const float b = __shfl(bv, j);
#pragma unroll
            for (int r = 0; r < 4; ++r) acc_set(acc, 4 * j + r, b);
        }
    }

    // the -0.0 pad row of every ring buffer (entries padding a stream point here)
    auto pad_rows = [&]() {
        if (threadIdx.x < 64 * kNBuf) {
            const int b = threadIdx.x >> 6;
            reinterpret_cast<float4*>(lds + (b * kBufRows + kTK) * kRowBytes)[lane] =
                make_float4(-0.f, -0.f, -0.f, -0.f);
        }
    };
    pad_rows();

    // One walk over chunks [c_begin, c_end) of a plan's chains (stream
    // layout v4) into acc.
    auto run_chain = [&](const int2* __restrict__ e, const int* __restrict__ sp, long long ne) {
        if (c_begin >= c_end) return;
        // Chunk c lives in ring buffer c % kNBuf (the plan baked that into
        // every entry).  Ring of 3: DMA(c+2) is issued right after gather(c),
        // so two chunks are in flight while one is consumed; per wave the
        // VMEM order is
        //   ... DMA(c) | DMA(c+1) | ...
        // so at the top of chunk c, vmcnt(kDmaPerWave) means DMA(c) has
        // landed (entry streams are scalar loads, counted by lgkmcnt).  Ring
        // of 2: DMA(c+1) is issued right after the barrier of chunk c (its
        // buffer held chunk c-1), so it has gather(c) to land; the top of
        // chunk c+1 waits vmcnt(0).  Either way the barrier makes every
        // wave's rows of chunk c visible and says all waves are done with
        // chunk c-1's buffer.  All loads in the loop are asm or scalar, so the
        // compiler inserts no vmcnt waits of its own.
        DmaState dma;
        dma.chunk_bytes = (size_t)kTK * ldxt * 4;
        dma.next = reinterpret_cast<const char*>(XT + (size_t)c_begin * kTK * ldxt + m0);
#pragma unroll
        for (int i = 0; i < kDmaPerWave; ++i)
            dma.voff[i] = 16u * lane + (unsigned)((wave * kDmaPerWave + i) * ldxt * 4) -
                          (TCSC_DMA_OFFSET ? (unsigned)((i % 4) * kRowBytes) : 0u);
        dma.lds_wave = (unsigned)reinterpret_cast<uintptr_t>(lds) + (unsigned)(wave * kDmaPerWave * kRowBytes);
        const bool dma_wave = wave < kDmaWaves;  // uniform
        const int buf0 = c_begin % kNBuf;
        // stream prefetch (pf_stream_params): this wave's 256-B scratch and its lane offsets
        const unsigned pf_m0 = (unsigned)reinterpret_cast<uintptr_t>(lds) + kRingBytes + 256u * wave;
        // pf_lines is 1, 2, 4 or 8: lane groups of 64 / pf_lines lanes touch one line each
        const unsigned pf_s_off = (unsigned)pf_dist + 128u * (unsigned)(lane * pf_lines >> 6);
        // one stream prefetch right after every DMA issue (the prologue's
        // included), so the top-of-chunk vmcnt count is the same for every
        // chunk; `p` is the header of the next chunk to gather
        auto pf_issue = [&](unsigned long long p) {
            if (kPfS) pf_touch(pf_m0, pf_s_off, reinterpret_cast<const char*>(p));
        };
        if (dma_wave) dma_next_chunk(dma, buf0);  // DMA(c_begin)

        // This wave's chain of chunk streams (stream layout v4,
        // tcsc_internal.h): the header of (g, c_begin); an idle wave (g >= G,
        // last column block) walks the empty chain after the last stream.
        unsigned long long cur =
            reinterpret_cast<unsigned long long>(e + (active ? (long long)sp[(long long)g * nch + c_begin] : ne));
        i32x16 sb[TCSC_SBUF_VECS];
        sbuf_tail_t sbt;
        load_stream(sb, sbt, reinterpret_cast<const char*>(cur));
        pf_issue(cur);
        // DMA(c_begin+1 .. c_begin+kNBuf-2): a ring of n keeps n-1 chunks in flight
#pragma unroll
        for (int i = 1; i + 1 < kNBuf; ++i) {
            if (dma_wave) dma_next_chunk(dma, (buf0 + i) % kNBuf);
            pf_issue(cur);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                       // pad rows

        const unsigned mask = 0x3ffu;
        // ring buffer that DMA(c+2) (ring of 3) / DMA(c+1) (ring of 2) fills
        int dbuf = kNBuf >= 3 ? (buf0 + kNBuf - 1) % kNBuf : (buf0 ^ 1);
#ifdef TCSC_STAMPS
        unsigned long long st_g = 0, st_p = 0, st_w = 0, t2 = stamp();
        const unsigned long long t_begin = t2;
        rt_[1] = rtstamp();
#endif
        for (int c = c_begin; c < c_end; ++c) {
            // see the VMEM order above: ring of 3 keeps DMA(c+1) in flight
            // (+ the stream prefetches issued after DMA(c+1): two chunks' worth)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kNBuf >= 3 ? (kNBuf - 2) * kDmaPerWave + (kPfS ? 2 : 0) : 0)
                         : "memory");
            __builtin_amdgcn_s_barrier();
#ifdef TCSC_STAMPS
            const unsigned long long t0 = stamp();
            st_w += t0 - t2;
#endif
            if ((kNBuf == 2 || kDmaEarly) && dma_wave) dma_next_chunk(dma, dbuf);
            gather_stream(sb, sbt, cur, lane, mask, acc);  // leaves cur at the next chunk's header
#ifdef TCSC_STAMPS
            const unsigned long long t1 = stamp();
            st_g += t1 - t0;
#endif
            // next chunk's stream: lands behind the DMA issue and the barrier
            load_stream(sb, sbt, reinterpret_cast<const char*>(cur));
            // DMA(c+2) into the buffer chunk c-1 used
            if (kNBuf >= 3 && !kDmaEarly && dma_wave) dma_next_chunk(dma, dbuf);
            pf_issue(cur);
            dbuf = dbuf == kNBuf - 1 ? 0 : dbuf + 1;
#ifdef TCSC_STAMPS
            t2 = stamp();  // waits for the stream load too
            st_p += t2 - t1;
#endif
        }
#ifdef TCSC_STAMPS
        rt_[2] = rtstamp();
        if (lane == 0) {
            const int wg = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
            unsigned long long* o = g_stamps + ((size_t)(wg % kStampWgs) * kWaves + wave) * 4;
            o[0] = st_g;
            o[1] = st_p;
            o[2] = st_w;
            o[3] = t2 - t_begin;
        }
#endif
        // no LDS-DMA may still be writing when the workgroup's LDS is
        // released, and the last (unused) stream load must have landed
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#ifdef TCSC_STAMPS
        rt_[5] = rtstamp();
#endif
    };

    // Epilogue: lanes hold rows (4 per lane), so a direct store would put
    // 64 rows' 4-byte pieces in one instruction (partial-line writes that
    // cost ~16x the bytes in HBM writes).  Transpose through LDS instead:
    // per pass of 64 rows every wave parks its 64 x kCW block into the
    // pass's tile rows (1 KiB + 16 B apart), then each wave reads back whole
    // tile rows (wave, wave + 16, ...): lane l stores columns 4l..4l+3, so
    // one store instruction writes one full 1-KiB row.
    // HOW: 0 the final values (bias last unless BIAS_FIRST, PReLU); 1 (order 2,
    // after the +1 chain) acc + bias parked in Y as is; 2 (order 2, after the
    // -1 chain) the parked value + acc, then PReLU.  A thread re-reads in
    // HOW 2 exactly the elements it stored in HOW 1.
    // OUT 3 (split-K over exactly 2 slices, DESIGN.md §4 k_reduce "pairwise"):
    // the tile's first slice to finish its chunk loop (its add to the
    // arrival word returns 0) stores its partial slab (sc1) and then adds 1
    // to the tile's ready word; the second polls the ready word, re-zeroes
    // both words, and writes Y = act((0 + s0) + s1 + b) from its registers
    // and the partner's slab, in slice order -- k_reduce4's adds, the same
    // bits.  The first finisher never waits, so no residency is assumed.
    const bool own_lds = OUT == 2 && gridDim.z == 4;  // combine_tile: the own band stays in the LDS
    int pair_role = 0;  // OUT 3: 0 = the tile's first slice to finish, 1 = the second
    int pair_poison = 0;  // OUT 3: the partner's slab was never published (a bounded wait ran out): Y = NaN
    const bool pair_split = OUT == 3 && (combine_giveup & 2);  // OUT 3: split halves (resident grid)
    unsigned* const pw = OUT == 3 ? ccnt + (size_t)(t.rt * (int)gridDim.x + t.cb) * kCombineWords : nullptr;
    auto epilogue = [&](auto how_) {
        constexpr int HOW = decltype(how_)::value;
        __syncthreads();  // every wave is done with the tile ring
#ifdef TCSC_STAMPS
        rt_[6] = rtstamp();
#endif
        if constexpr (OUT == 3) {
            int* role = reinterpret_cast<int*>(lds + kLdsBytes - 16);
            if (threadIdx.x == 0) {
                int r = __hip_atomic_fetch_add(pw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u ? 0 : 1;
                if (r == 1 && !pair_split) {
                    // the partner has arrived, so it is running and will publish: the bound
                    // (100 ms) only keeps a broken launch from hanging the device, and
                    // running out of it poisons the tile (NaN) instead of reading a stale slab
                    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                    bool ready;
                    while (!(ready = __hip_atomic_load(pw + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) &&
                           __builtin_amdgcn_s_memrealtime() - t0 < 10000000ull)
                        __builtin_amdgcn_s_sleep(2);
                    if (!ready) r |= 2;
                    __hip_atomic_store(pw, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(pw + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                role[0] = r;
            }
            __syncthreads();
            const int rv = __builtin_amdgcn_readfirstlane(role[0]);
            pair_role = rv & 1;
            pair_poison = rv >> 1;
        }
        constexpr int kQ = kCW / 4;                 // 16-B quads of a wave's row
        constexpr int kEpiRows = 64;                // tile rows per pass
        constexpr int kStride = kRowBytes + 16;     // bytes per parked tile row
        static_assert(kEpiRows * kStride <= kOwnBandOff, "the epilogue staging stays below the own band");
        static_assert(kEpiRows % kWaves == 0 && kWgCols == 64 * 4, "each wave stores whole tile rows");
        constexpr int kLanesPerPass = kEpiRows / 4;
        const int pcol = group_col0(g) - t.cb * kWgCols;  // this wave's first column in a parked row
        const int col = t.cb * kWgCols + 4 * lane;        // the lane's 4 columns of a stored tile row
        const int col_end = ncols;
        const bool vec_ok = OUT == 0 ? ((ldy & 3) == 0 && ((reinterpret_cast<uintptr_t>(Y) & 15) == 0))
                                     : ((ncols & 3) == 0 && ((reinterpret_cast<uintptr_t>(ws) & 15) == 0));
        const __amdgpu_buffer_rsrc_t slab_rs = slabs_rsrc(ws, (int)gridDim.z, M, ncols);
        constexpr bool kAddBias = OUT == 0 && (HOW == 1 || (HOW == 0 && !BIAS_FIRST));
        constexpr bool kPrelu = PRELU && HOW != 1;
        constexpr bool kLoadBias = kAddBias || OUT == 3;
        float4 bq = make_float4(0.f, 0.f, 0.f, 0.f);
        if (kLoadBias) {
            bq.x = col + 0 < col_end ? Bias[col + 0] : 0.f;
            bq.y = col + 1 < col_end ? Bias[col + 1] : 0.f;
            bq.z = col + 2 < col_end ? Bias[col + 2] : 0.f;
            bq.w = col + 3 < col_end ? Bias[col + 3] : 0.f;
        }
        // one pass: park rows [64 h, 64 h + 64) of the tile, then store them (OUT 3:
        // fin = finalize Y from this slice's partial and the partner's slab,
        // else store the partial to this slice's slab); no trailing barrier
        auto pass = [&](const int h, const bool fin) {
            if (active && lane / kLanesPerPass == h) {
                const int lh = lane % kLanesPerPass;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int R = 4 * lh + r;
#pragma unroll
                    for (int q = 0; q < kQ; ++q) {
                        const float4 v =
                            make_float4(acc_get(acc, 4 * (4 * q + 0) + r), acc_get(acc, 4 * (4 * q + 1) + r),
                                        acc_get(acc, 4 * (4 * q + 2) + r), acc_get(acc, 4 * (4 * q + 3) + r));
                        *reinterpret_cast<float4*>(lds + R * kStride + pcol * 4 + q * 16) = v;
                    }
                }
            }
            __syncthreads();
            {
#pragma unroll
                for (int i = 0; i < kEpiRows / kWaves; ++i) {
                    const int R = wave + kWaves * i;  // whole 1-KiB tile rows: one full-line store per wave
                    const int row = m0 + kEpiRows * h + R;
                    float4 v = *reinterpret_cast<const float4*>(lds + R * kStride + lane * 16);
                    if (row < M && col < col_end) {
                        float* dst;
                        if (OUT == 0) {
                            dst = Y + (size_t)row * ldy + col;
                            if (HOW == 2) {  // the parked bias + (+1 sums), then + (-1 sums)
                                const bool full = vec_ok && col + 3 < col_end;
                                v.x = dst[0] + v.x;
                                v.y = (full || col + 1 < col_end) ? dst[1] + v.y : v.y;
                                v.z = (full || col + 2 < col_end) ? dst[2] + v.z : v.z;
                                v.w = (full || col + 3 < col_end) ? dst[3] + v.w : v.w;
                            }
                            if (kAddBias) {
                                v.x += bq.x;
                                v.y += bq.y;
                                v.z += bq.z;
                                v.w += bq.w;
                            }
                            if (kPrelu) {
                                v.x = (v.x < 0.0f) ? a * v.x : v.x;
                                v.y = (v.y < 0.0f) ? a * v.y : v.y;
                                v.z = (v.z < 0.0f) ? a * v.z : v.z;
                                v.w = (v.w < 0.0f) ? a * v.w : v.w;
                            }
                        } else {
                            dst = ws + ((size_t)t.z * M + row) * ncols + col;
                        }
                        if constexpr (OUT == 3) {
                            // vec_ok and whole quads (the launcher's conditions)
                            const int off = (int)(((size_t)t.z * M + row) * ncols + col) * 4;
                            if (!fin) {
                                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), slab_rs, off, 0,
                                                                       kSc1);
                            } else {
                                const int poff = (int)(((size_t)(1 - t.z) * M + row) * ncols + col) * 4;
                                const float4 pv = __builtin_bit_cast(
                                    float4, __builtin_amdgcn_raw_buffer_load_b128(slab_rs, poff, 0, kSc1));
                                const float4 lo = t.z == 0 ? v : pv, hi = t.z == 0 ? pv : v;
                                float4 o = BIAS_FIRST ? bq : make_float4(0.f, 0.f, 0.f, 0.f);
                                o.x += lo.x;
                                o.y += lo.y;
                                o.z += lo.z;
                                o.w += lo.w;
                                o.x += hi.x;
                                o.y += hi.y;
                                o.z += hi.z;
                                o.w += hi.w;
                                if (!BIAS_FIRST) {
                                    o.x += bq.x;
                                    o.y += bq.y;
                                    o.z += bq.z;
                                    o.w += bq.w;
                                }
                                if (PRELU) {
                                    o.x = (o.x < 0.0f) ? a * o.x : o.x;
                                    o.y = (o.y < 0.0f) ? a * o.y : o.y;
                                    o.z = (o.z < 0.0f) ? a * o.z : o.z;
                                    o.w = (o.w < 0.0f) ? a * o.w : o.w;
                                }
                                if (pair_poison) {
                                    const float qn = __builtin_nanf("");
                                    o = make_float4(qn, qn, qn, qn);
                                }
                                typedef float nt4 __attribute__((ext_vector_type(4)));
                                nt4 w = {o.x, o.y, o.z, o.w};
                                __builtin_nontemporal_store(w, reinterpret_cast<nt4*>(Y + (size_t)row * ldy + col));
                            }
                        } else if constexpr (OUT == 2) {
                            // write-through (sc1) slab stores: the tile's other
                            // workgroups read them with sc1 loads (combine_tile);
                            // at Z = 4 the own band (pass h == z) stays in the LDS
                            const int off = (int)(((size_t)t.z * M + row) * ncols + col) * 4;
                            if (own_lds && h == t.z) {
                                static_assert(kEpiRows == 64, "a pass is one band at Z = 4");
                                *reinterpret_cast<float4*>(lds + kOwnBandOff + R * kRowBytes +
                                                           (col - t.cb * kWgCols) * 4) = v;
                            } else {  // whole quads: the launcher combines in launch only when ncols % 4 == 0
                                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), slab_rs, off, 0,
                                                                       kSc1);
                            }
                        } else if (vec_ok && col + 3 < col_end) {
                            if (OUT == 0 && HOW != 1) {  // Y is never re-read here: keep it out of L2's way
                                typedef float nt4 __attribute__((ext_vector_type(4)));
                                nt4 w = {v.x, v.y, v.z, v.w};
                                __builtin_nontemporal_store(w, reinterpret_cast<nt4*>(dst));
                            } else {
                                *reinterpret_cast<float4*>(dst) = v;
                            }
                        } else {
                            dst[0] = v.x;
                            if (col + 1 < col_end) dst[1] = v.y;
                            if (col + 2 < col_end) dst[2] = v.z;
                            if (col + 3 < col_end) dst[3] = v.w;
                        }
                    }
                }
            }
        };
        if (!pair_split) {
#pragma unroll
            for (int h = 0; h < 256 / kEpiRows; ++h) {
                pass(h, OUT == 3 && pair_role == 1);
                if (h + 1 < 256 / kEpiRows) __syncthreads();  // region reused by the next pass
            }
            if (OUT == 3 && pair_role == 0) {  // publish the slab: every wave's sc1 stores drained, then one agent add
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (threadIdx.x == 0) __hip_atomic_fetch_add(pw + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else if constexpr (OUT == 3) {
            // Split pairwise (the grid is resident; DESIGN.md §4 k_reduce): the first
            // finisher F stores rows 0..127 of its partial, the second S rows 128..255;
            // each then finalizes the half the other stored, from its registers and
            // the partner's slab.  Words: pw[0] arrival, pw[1] F's half ready, pw[2]
            // who finalizes rows 128..255 (2: S stored its half, F finalizes; 1: F
            // gave up waiting, stored that half too, S finalizes), pw[3] done.
            int* dec = reinterpret_cast<int*>(lds + kLdsBytes - 16) + 1;
            const bool first = pair_role == 0;
            const int own = first ? 0 : 2;  // passes of the half this slice stores
            pass(own, false);
            __syncthreads();
            pass(own + 1, false);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's slab stores have left
            __syncthreads();
            if (threadIdx.x == 0) {
                int d;
                if (first) {
                    __hip_atomic_fetch_add(pw + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    unsigned v = 0;
                    if (!(combine_giveup & 1)) {  // the partner may not be resident: a bounded wait
                        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                        while ((v = __hip_atomic_load(pw + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u &&
                               __builtin_amdgcn_s_memrealtime() - t0 < kCombineWaitTicks)
                            __builtin_amdgcn_s_sleep(2);
                    }
                    d = v == 2u ? 1 : 0;  // 1: finalize rows 128..255; 0: gave up
                } else {
                    unsigned expect = 0u;
                    const bool mine = __hip_atomic_compare_exchange_strong(
                        pw + 2, &expect, 2u, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    d = mine ? 0 : 1;  // 1: F gave up and stored rows 128..255 as well
                    // F has arrived, so it is running and publishes its half without
                    // waiting; the bound (100 ms) only keeps a broken launch from hanging,
                    // and running out of it poisons what S finalizes (NaN)
                    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                    bool ready;
                    while (!(ready = __hip_atomic_load(pw + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) &&
                           __builtin_amdgcn_s_memrealtime() - t0 < 10000000ull)
                        __builtin_amdgcn_s_sleep(2);
                    if (!ready) d |= 2;
                }
                dec[0] = d;
            }
            __syncthreads();
            const int dv = __builtin_amdgcn_readfirstlane(dec[0]);
            const int d = dv & 1;
            if (!first) pair_poison = dv >> 1;
            if (first) {
                if (d == 0) {  // give the second half up: store it, then try to hand it over
                    pass(2, false);
                    __syncthreads();
                    pass(3, false);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __syncthreads();
                    if (threadIdx.x == 0) {
                        unsigned expect = 0u;
                        dec[0] = __hip_atomic_compare_exchange_strong(pw + 2, &expect, 1u, __ATOMIC_RELAXED,
                                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     ? 0
                                     : 1;  // 1: S stored its half in the meantime, so finalize it here
                    }
                    __syncthreads();
                }
                if (__builtin_amdgcn_readfirstlane(dec[0]) == 1) {
                    pass(2, true);
                    __syncthreads();
                    pass(3, true);
                }
            } else {
                pass(0, true);
                __syncthreads();
                pass(1, true);
                if (d == 1) {
                    __syncthreads();
                    pass(2, true);
                    __syncthreads();
                    pass(3, true);
                }
            }
            __syncthreads();
            if (threadIdx.x == 0 &&
                __hip_atomic_fetch_add(pw + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1u) {
                for (int i = 0; i < 4; ++i) __hip_atomic_store(pw + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    };

    run_chain(ent, sptr, n_entries);
    if constexpr (ORDER == 0) {
        epilogue(std::integral_constant<int, 0>{});
#ifdef TCSC_STAMPS
        rt_[3] = rtstamp();
#endif
        if constexpr (OUT == 2) combine_tile<BIAS_FIRST, PRELU>(ws, M, ncols, Bias, Y, ldy, a, ccnt, t, lds, combine_giveup,
                                                         own_lds);
#ifdef TCSC_STAMPS
        rt_[4] = rtstamp();
        if (threadIdx.x == 0) {
            const int wg = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
            if (wg < kStampWgs)
                for (int i = 0; i < 7; ++i) g_wgtime[wg * 8 + i] = rt_[i];
        }
#endif
    } else if constexpr (ORDER == 1) {
        __syncthreads();  // every wave is done with the ring before the -1 chain refills it
        run_chain(ent2, sptr2, n_entries2);
        epilogue(std::integral_constant<int, 0>{});
    } else {
        epilogue(std::integral_constant<int, 1>{});
#pragma unroll
        for (int v = 0; v < TCSC_ACC_VECS; ++v)
#pragma unroll
            for (int i = 0; i < TCSC_ACC_W; ++i) acc[v][i] = 0.f;
        __syncthreads();  // the epilogue's LDS staging is done before the ring is refilled
        pad_rows();
        run_chain(ent2, sptr2, n_entries2);
        epilogue(std::integral_constant<int, 2>{});
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

// The same with 4 columns per thread (16-B slab loads, all slices' loads in
// flight before the adds); same order per element, so the same bits.  Needs
// ncols % 4 == 0, ldy % 4 == 0 and 16-B aligned ws, Y.
typedef float f32x4_t __attribute__((ext_vector_type(4)));
#ifndef TCSC_REDUCE_NT
#define TCSC_REDUCE_NT 1  // slab loads nontemporal (A/B: tools/ab.mk lib/abl/libtcsc_amd_rnt0.so)
#endif
template <bool BIAS_FIRST, bool PRELU>
__global__ void k_reduce4(const f32x4_t* __restrict__ ws, int slices, int M, int ncols,
                          const float* __restrict__ Bias, float* __restrict__ Y, int ldy, float a) {
    const int nq = ncols / 4;
    const long long total = (long long)M * nq;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int row = (int)(i / nq), col = 4 * (int)(i % nq);
        f32x4_t p[16];
#pragma unroll
        for (int s = 0; s < 16; ++s)
            if (s < slices) p[s] = TCSC_REDUCE_NT ? __builtin_nontemporal_load(ws + (size_t)s * total + i)
                                                  : ws[(size_t)s * total + i];
        const float4 b = *reinterpret_cast<const float4*>(Bias + col);
        float4 v = BIAS_FIRST ? b : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int s = 0; s < 16; ++s)
            if (s < slices) {
                v.x += p[s].x;
                v.y += p[s].y;
                v.z += p[s].z;
                v.w += p[s].w;
            }
        if (!BIAS_FIRST) {
            v.x += b.x;
            v.y += b.y;
            v.z += b.z;
            v.w += b.w;
        }
        if (PRELU) {
            v.x = (v.x < 0.0f) ? a * v.x : v.x;
            v.y = (v.y < 0.0f) ? a * v.y : v.y;
            v.z = (v.z < 0.0f) ? a * v.z : v.z;
            v.w = (v.w < 0.0f) ? a * v.w : v.w;
        }
        typedef float nt4 __attribute__((ext_vector_type(4)));
        nt4 w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, reinterpret_cast<nt4*>(Y + (size_t)row * ldy + col));
    }
}

// Dense-baseline epilogue (gemm_basic order, dense/dense.c:64-77: the bias
// after the sum): Y = act(Y + B), one float4 of a row per thread where the
// row pitch allows, HBM-bound (2*M*N*4 bytes).
template <bool PRELU>
__global__ void k_bias_act(float* __restrict__ Y, int M, int N, int ldy, const float* __restrict__ B, float a) {
    const int nq = (N + 3) / 4;
    const long long total = (long long)M * nq;
    const bool vec = (ldy & 3) == 0 && (N & 3) == 0 && ((reinterpret_cast<uintptr_t>(Y) & 15) == 0);
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
        const int m = (int)(i / nq), n = 4 * (int)(i % nq);
        float* y = Y + (size_t)m * ldy + n;
        if (vec) {
            float4 v = *reinterpret_cast<float4*>(y);
            v.x += B[n + 0];
            v.y += B[n + 1];
            v.z += B[n + 2];
            v.w += B[n + 3];
            if (PRELU) {
                v.x = (v.x < 0.0f) ? a * v.x : v.x;
                v.y = (v.y < 0.0f) ? a * v.y : v.y;
                v.z = (v.z < 0.0f) ? a * v.z : v.z;
                v.w = (v.w < 0.0f) ? a * v.w : v.w;
            }
            *reinterpret_cast<float4*>(y) = v;
        } else {
            for (int j = 0; j < 4 && n + j < N; ++j) {
                float v = y[j] + B[n + j];
                if (PRELU) v = (v < 0.0f) ? a * v : v;
                y[j] = v;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Device tcsc_from_dense (bit-exact with tcsc.c:6-66): the K x N matrix is cut
// into tiles of `tr` rows; one thread per (row tile, column) -- a wave reads
// 64 consecutive columns of a row, 256 B coalesced, 8 rows in flight --
// counts its +1.0f / -1.0f entries (k_dense_tile_counts), a per-column pass
// turns the tile counts into tile offsets and column totals
// (k_dense_tile_scan), the totals are scanned into col_start, and the same
// threads walk their tile again writing row indices from their offsets
// (k_dense_tile_fill): within a column the tiles follow each other in row
// order and each walks its rows ascending, so every column's rows ascend as
// in the reference's fill (tcsc.c:48-60).  Only == 1.0f / == -1.0f count
// (tcsc.c:14-17,54-58).  HBM-bound: the matrix is read once per pass.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_dense_tile_counts(const float* __restrict__ D, int rows, int cols, int tr,
                                                           int* __restrict__ cp, int* __restrict__ cn) {
    const int col = blockIdx.x * 256 + threadIdx.x;
    if (col >= cols) return;
    const int tile = blockIdx.y;
    const int r0 = tile * tr, r1 = min(rows, r0 + tr);
    const float* d = D + (size_t)r0 * cols + col;
    int p = 0, q = 0, r = r0;
    for (; r + 8 <= r1; r += 8) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = __builtin_nontemporal_load(d + (size_t)(r - r0 + i) * cols);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            p += v[i] == 1.0f;
            q += v[i] == -1.0f;
        }
    }
    for (; r < r1; ++r) {
        const float v = d[(size_t)(r - r0) * cols];
        p += v == 1.0f;
        q += v == -1.0f;
    }
    cp[(size_t)tile * cols + col] = p;
    cn[(size_t)tile * cols + col] = q;
}

// In place: tile counts -> exclusive offsets inside the column; totals into
// totp/totn[col] (their [cols] entry is 0, so an exclusive scan of cols+1
// entries ends in the grand total).
__global__ void k_dense_tile_scan(int* __restrict__ cp, int* __restrict__ cn, int ntiles, int cols,
                                  int* __restrict__ totp, int* __restrict__ totn) {
    const int col = blockIdx.x * blockDim.x + threadIdx.x;
    if (col > cols) return;
    if (col == cols) {
        totp[cols] = 0;
        totn[cols] = 0;
        return;
    }
    int sp = 0, sn = 0;
    for (int t = 0; t < ntiles; ++t) {
        const size_t i = (size_t)t * cols + col;
        const int a = cp[i], b = cn[i];
        cp[i] = sp;
        cn[i] = sn;
        sp += a;
        sn += b;
    }
    totp[col] = sp;
    totn[col] = sn;
}

// Writes at most the tile's counted entries (offsets of the next tile, or the
// column's end): the arrays the caller sized from the counts are never
// overrun, whatever the matrix holds by now.
__global__ void __launch_bounds__(256) k_dense_tile_fill(const float* __restrict__ D, int rows, int cols, int tr,
                                                         int ntiles, const int* __restrict__ csp,
                                                         const int* __restrict__ csn, const int* __restrict__ op,
                                                         const int* __restrict__ on, int* __restrict__ rip,
                                                         int* __restrict__ rin) {
    const int col = blockIdx.x * 256 + threadIdx.x;
    if (col >= cols) return;
    const int tile = blockIdx.y;
    const size_t i = (size_t)tile * cols + col;
    int p = csp[col] + op[i], q = csn[col] + on[i];
    const int pend = tile + 1 < ntiles ? csp[col] + op[i + cols] : csp[col + 1];
    const int qend = tile + 1 < ntiles ? csn[col] + on[i + cols] : csn[col + 1];
    if (p == pend && q == qend) return;
    const int r0 = tile * tr, r1 = min(rows, r0 + tr);
    const float* d = D + (size_t)r0 * cols + col;
    int r = r0;
    for (; r + 8 <= r1; r += 8) {
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = __builtin_nontemporal_load(d + (size_t)(r - r0 + k) * cols);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (v[k] == 1.0f) {
                if (p < pend) rip[p] = r + k;
                ++p;
            } else if (v[k] == -1.0f) {
                if (q < qend) rin[q] = r + k;
                ++q;
            }
        }
    }
    for (; r < r1; ++r) {
        const float v = d[(size_t)(r - r0) * cols];
        if (v == 1.0f) {
            if (p < pend) rip[p] = r;
            ++p;
        } else if (v == -1.0f) {
            if (q < qend) rin[q] = r;
            ++q;
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
                           in.rin, out.lbp, out.lbn, out.cptr, out.sptr, in.col_begin, ncols, nch, out.ent);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (in.n_neg > 0) {
        hipLaunchKernelGGL(k_scatter<1>, dim3(grid_for(in.n_neg, 256)), dim3(256), 0, st, in.csn, in.rin, in.csp,
                           in.rip, out.lbn, out.lbp, out.cptr, out.sptr, in.col_begin, ncols, nch, out.ent);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    const long long ng = (long long)nch * G;
    hipLaunchKernelGGL(k_fill_headers, dim3(grid_for(ng, 256)), dim3(256), 0, st, out.cptr, out.sptr, ncols, nch, G,
                       out.ent, out.n_entries);
    return hipGetLastError();
}

size_t workspace_bytes(int M, int ncols, int slices) {
    return slices > 1 ? (size_t)slices * M * ncols * sizeof(float) : 0;
}

static inline int ldxt_of(int M) { return (M + kTM - 1) / kTM * kTM; }

// X^T of one call: (chunks + kNBuf-1 look-ahead chunks) * kTK rows of ldxt
// floats (rows >= K are never gathered), 256-B aligned size.
size_t xt_bytes(int M, int K) {
    const size_t rows = ((size_t)(K + kTK - 1) / kTK + kNBuf - 1) * kTK;
    const size_t b = rows * ldxt_of(M) * sizeof(float);
    return (b + 255) / 256 * 256;
}

// Cost model (cycles of one CU at ~2.1 GHz) for k-slicing: every workgroup
// runs on its own CU; gathers cost ~1 KiB / 220 B/clk per nonzero and
// wave, the LDS-DMA ~1 KiB / 100 B/clk per k row (DESIGN.md
// measurements); the split-K slabs cost HBM time.
int choose_slices(int M, int ncols, int K, long long nnz, int G, size_t ws_bytes, int force) {
    const int nch = (K + kTK - 1) / kTK;
    if (nch <= 1) return 1;
    const int rt = (M + kTM - 1) / kTM;
    const int cb = (G + kWaves - 1) / kWaves;
    const long long base = (long long)rt * cb;
    auto cap = [&](int s) { return s <= nch && workspace_bytes(M, ncols, s) <= ws_bytes; };
    if (force > 0) return cap(force) ? force : 1;
    const double nz_per_chunk_block = (double)nnz / nch / cb;  // per workgroup and chunk (all its waves)
    const double chunk_cycles = nz_per_chunk_block * (1024.0 / 220.0) + kTK * (1024.0 / 100.0) + 400.0;
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

// Stream prefetch parameters: about four chunks ahead and 1.5 chunks wide
// (tools/ab.sh sweep, DESIGN.md §4: cfg 4 streams average ~140 B per chunk
// and take 512 B x 2 lines, cfg 2/3's ~320 B take 4 lines).
static int env_int(const char* name, int dflt) {
    const char* v = std::getenv(name);
    return v ? std::atoi(v) : dflt;
}

void pf_stream_params(long long n_entries, int n_groups, int n_chunks, int* dist, int* lines) {
    const int env_dist = env_int("TCSC_PF_DIST", -1), env_lines = env_int("TCSC_PF_LINES", 0);  // read per launch
    const double per_chunk = n_groups > 0 && n_chunks > 0 ? 8.0 * (double)n_entries / ((double)n_groups * n_chunks) : 0.0;
    int l = env_lines > 0 ? env_lines : (int)std::ceil(1.5 * per_chunk / 128.0);
    l = l <= 1 ? 1 : l <= 2 ? 2 : l <= 4 ? 4 : 8;
    int d = env_dist >= 0 ? env_dist : (int)std::lround(4.0 * per_chunk / 128.0) * 128;
    d = std::min(std::max(d, 0), kPfWindow - 128 * l) & ~3;
    *dist = d;
    *lines = l;
}

// Split-K slabs combined inside the k_stream launch or by k_reduce4 after it.
//  * 2 slices: pairwise (k_stream OUT 3): the tile's first slice to finish
//    stores its slab, the second combines -- no reduce launch, half the slab
//    bytes, and no wait on a workgroup that has not started, so any grid (3);
//    where the grid is resident each slice stores one half and finalizes the
//    other (4, the split halves; TCSC_PAIR_SPLIT=0 keeps 3).
//  * 3 or more: row bands (combine_tile, OUT 2) where the whole grid is
//    resident (one workgroup per CU), from 64 workgroups on (measured: cfg
//    2/3 at 4 slices 79 -> 74 us; cfg 1's 6 workgroups 23 -> 27 us: the
//    hand-off's atomics in series cost more than a launch).
// TCSC_COMBINE unset: that policy; 1: in-launch wherever it can run; 0: never;
// 2: row bands wherever the grid is resident, 2 slices included (A/B).
int combine_mode(int slices, long long wgs, long long tiles, long long slab_floats, int num_cus, bool have_words,
                 bool vec) {
    if (slices < 2 || slices > 16 || !vec || !have_words || tiles > kCombineTiles ||
        slab_floats * slices * 4 >= 0x7fffffffLL)
        return 0;
    const int c = env_int("TCSC_COMBINE", -1);
    if (c == 0) return 0;
    if (slices == 2 && (c != 2 || num_cus <= 0 || wgs > num_cus))  // pairwise: split halves on a resident grid
        return (num_cus > 0 && wgs <= num_cus && env_int("TCSC_PAIR_SPLIT", 1) != 0) ? 4 : 3;
    if (num_cus <= 0 || wgs > num_cus) return 0;
    return (c > 0 || wgs >= 64) ? 2 : 0;
}

int normalized_slices(int K, int slices) {
    const int nch = (K + kTK - 1) / kTK;
    if (nch <= 0) return 1;
    const int cps = (nch + slices - 1) / slices;
    return (nch + cps - 1) / cps;
}

template <bool BF, bool PR>
static hipError_t launch_t(const GemmArgs& g, int slices, hipStream_t st) {
    const int nch = (g.K + kTK - 1) / kTK;
    if (g.order != 0) slices = 1;  // the reference orders walk K in order
    int cps = nch > 0 ? (nch + slices - 1) / slices : 1;
    slices = nch > 0 ? (nch + cps - 1) / cps : 1;
    const int ldxt = ldxt_of(g.M);
    dim3 grid((g.n_groups + kWaves - 1) / kWaves, (g.M + kTM - 1) / kTM, slices);
    dim3 block(kWaves * 64);
    int pfd = 0, pfl = 1;
    pf_stream_params(g.n_entries, g.n_groups, nch, &pfd, &pfl);
    if (g.order == 1) {
        hipLaunchKernelGGL((k_stream<BF, PR, 0, 1>), grid, block, 0, st, g.XT, ldxt, g.M, g.K, g.ent, g.sptr,
                           g.n_entries, g.ent2, g.sptr2, g.n_entries2, g.n_groups, g.ncols, nch, cps, g.B, g.Y, g.ldy,
                           g.a, g.ws, pfd, pfl, nullptr, 0);
        return hipGetLastError();
    }
    if (g.order == 2) {
        hipLaunchKernelGGL((k_stream<false, PR, 0, 2>), grid, block, 0, st, g.XT, ldxt, g.M, g.K, g.ent, g.sptr,
                           g.n_entries, g.ent2, g.sptr2, g.n_entries2, g.n_groups, g.ncols, nch, cps, g.B, g.Y, g.ldy,
                           g.a, g.ws, pfd, pfl, nullptr, 0);
        return hipGetLastError();
    }
    if (slices == 1) {
        hipLaunchKernelGGL((k_stream<BF, PR, 0, 0>), grid, block, 0, st, g.XT, ldxt, g.M, g.K, g.ent, g.sptr,
                           g.n_entries, g.ent, g.sptr, g.n_entries, g.n_groups, g.ncols, nch, cps, g.B, g.Y, g.ldy,
                           g.a, g.ws, pfd, pfl, nullptr, 0);
        return hipGetLastError();
    }
    const long long total = (long long)g.M * g.ncols;
    const bool vec = slices <= 16 && g.ncols % 4 == 0 && g.ldy % 4 == 0 &&
                     ((reinterpret_cast<uintptr_t>(g.Y) | reinterpret_cast<uintptr_t>(g.ws) |
                       reinterpret_cast<uintptr_t>(g.B)) & 15) == 0;
    const int cm = combine_mode(slices, (long long)grid.x * grid.y * grid.z, (long long)grid.x * grid.y, total,
                                g.num_cus, g.ccnt != nullptr, vec);
    if (cm == 3 || cm == 4) {  // pairwise: no residency needed (3); the split halves on a resident grid (4)
        const int split = cm == 4 ? 2 : 0;
        hipLaunchKernelGGL((k_stream<BF, PR, 3, 0>), grid, block, 0, st, g.XT, ldxt, g.M, g.K, g.ent, g.sptr,
                           g.n_entries, g.ent, g.sptr, g.n_entries, g.n_groups, g.ncols, nch, cps, g.B, g.Y, g.ldy, g.a,
                           g.ws, pfd, pfl, g.ccnt, split | (g.combine_giveup & 1));
        return hipGetLastError();
    }
    if (cm == 2) {  // row bands: every workgroup of the grid resident at once (one per CU)
        hipLaunchKernelGGL((k_stream<BF, PR, 2, 0>), grid, block, 0, st, g.XT, ldxt, g.M, g.K, g.ent, g.sptr,
                           g.n_entries, g.ent, g.sptr, g.n_entries, g.n_groups, g.ncols, nch, cps, g.B, g.Y, g.ldy, g.a,
                           g.ws, pfd, pfl, g.ccnt, g.combine_giveup);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((k_stream<BF, PR, 1, 0>), grid, block, 0, st, g.XT, ldxt, g.M, g.K, g.ent, g.sptr, g.n_entries,
                       g.ent, g.sptr, g.n_entries, g.n_groups, g.ncols, nch, cps, g.B, g.Y, g.ldy, g.a, g.ws, pfd,
                       pfl, nullptr, 0);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (vec)
        hipLaunchKernelGGL((k_reduce4<BF, PR>), dim3(grid_for(total / 4, 256)), dim3(256), 0, st,
                           reinterpret_cast<const f32x4_t*>(g.ws), slices, g.M, g.ncols, g.B, g.Y, g.ldy, g.a);
    else
        hipLaunchKernelGGL((k_reduce<BF, PR>), dim3(grid_for(total, 256)), dim3(256), 0, st, g.ws, slices, g.M,
                           g.ncols, g.B, g.Y, g.ldy, g.a);
    return hipGetLastError();
}

// g.XT must hold xt_bytes(M, K) (the API layer carves it out of the plan's
// workspace, ahead of the split-K slabs in g.ws).
hipError_t launch_gemm(const GemmArgs& g, hipStream_t st) {
    if (g.M <= 0 || g.ncols <= 0) return hipSuccess;
    if (g.K > 0 && g.stage != 2) {
        if (!g.XT) return hipErrorInvalidValue;
        const int ldxt = ldxt_of(g.M);
        const bool vec = (g.K % 4 == 0) && ((reinterpret_cast<uintptr_t>(g.X) & 15) == 0);
        if (vec)
            hipLaunchKernelGGL(k_transpose<true>, dim3((g.K + 127) / 128, ldxt / 64), dim3(256), 0, st, g.X, g.M, g.K,
                               g.XT, ldxt);
        else
            hipLaunchKernelGGL(k_transpose<false>, dim3((g.K + 63) / 64, ldxt / 64), dim3(256), 0, st, g.X, g.M,
                               g.K, g.XT, ldxt);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (g.stage == 1) return hipSuccess;
    const int s = choose_slices(g.M, g.ncols, g.K, g.nnz, g.n_groups, g.ws ? g.ws_bytes : 0, g.force_slices);
    if (g.bias_first) return g.prelu ? launch_t<true, true>(g, s, st) : launch_t<true, false>(g, s, st);
    return g.prelu ? launch_t<false, true>(g, s, st) : launch_t<false, false>(g, s, st);
}

int dense_tile_rows(int rows) {
    // 256-row tiles; taller ones when the grid's y extent (65535) needs them
    int tr = 256;
    while ((rows + tr - 1) / tr > 65535) tr *= 2;
    return tr;
}

hipError_t dense_to_tcsc_counts(const float* D, int rows, int cols, int* cp, int* cn, int* totp, int* totn,
                                hipStream_t st) {
    const int tr = dense_tile_rows(rows), nt = (rows + tr - 1) / tr;
    if (rows > 0 && cols > 0) {
        hipLaunchKernelGGL(k_dense_tile_counts, dim3((cols + 255) / 256, nt), dim3(256), 0, st, D, rows, cols, tr, cp,
                           cn);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_dense_tile_scan, dim3(cols / 256 + 1), dim3(256), 0, st, cp, cn, rows > 0 ? nt : 0, cols,
                       totp, totn);
    return hipGetLastError();
}

hipError_t dense_to_tcsc_fill(const float* D, int rows, int cols, const int* csp, const int* csn, const int* op,
                              const int* on, int* rip, int* rin, hipStream_t st) {
    const int tr = dense_tile_rows(rows), nt = (rows + tr - 1) / tr;
    if (rows <= 0 || cols <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_dense_tile_fill, dim3((cols + 255) / 256, nt), dim3(256), 0, st, D, rows, cols, tr, nt, csp,
                       csn, op, on, rip, rin);
    return hipGetLastError();
}

hipError_t launch_bias_act(float* Y, int M, int N, int ldy, const float* B, bool prelu, float a, hipStream_t st) {
    const long long total = (long long)M * ((N + 3) / 4);
    if (total == 0) return hipSuccess;
    if (prelu)
        hipLaunchKernelGGL(k_bias_act<true>, dim3(grid_for(total, 256)), dim3(256), 0, st, Y, M, N, ldy, B, a);
    else
        hipLaunchKernelGGL(k_bias_act<false>, dim3(grid_for(total, 256)), dim3(256), 0, st, Y, M, N, ldy, B, a);
    return hipGetLastError();
}

hipError_t check_index_device(const int* cs, const int* ri, int col_begin, int ncols, int rows, int n_total,
                              int* d_flag, hipStream_t st) {
    if (ncols <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_check_index, dim3(grid_for(ncols, 256)), dim3(256), 0, st, cs, ri, col_begin, ncols, rows,
                       n_total, d_flag);
    return hipGetLastError();
}

hipError_t rebase_offsets(const int* cs, int col_begin, int ncols, int* out, hipStream_t st) {
    hipLaunchKernelGGL(k_rebase, dim3(grid_for((long long)ncols + 1, 256)), dim3(256), 0, st, cs, col_begin, ncols, out);
    return hipGetLastError();
}

hipError_t sort_columns_tmp_bytes(int n, int ncols, size_t* bytes) {
    *bytes = 0;
    return hipcub::DeviceSegmentedRadixSort::SortKeys(nullptr, *bytes, (const int*)nullptr, (int*)nullptr, n, ncols,
                                                      (const int*)nullptr, (const int*)nullptr, 0, 32, (hipStream_t)0);
}

// Sort every column's row indices (segments off[j] .. off[j+1] of in, all
// rows >= 0) into out.
hipError_t sort_columns(const int* in, int* out, int n, int ncols, const int* off, void* tmp, size_t tmp_bytes,
                        hipStream_t st) {
    if (n <= 0 || ncols <= 0) return hipSuccess;
    return hipcub::DeviceSegmentedRadixSort::SortKeys(tmp, tmp_bytes, in, out, n, ncols, off, off + 1, 0, 32, st);
}

hipError_t exclusive_scan_i32(const int* in, int* out, int n, void* tmp, size_t tmp_bytes, hipStream_t st) {
    return hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, in, out, n, st);
}

int ldxt_for(int M) { return ldxt_of(M); }

}  // namespace tcsc

// include/tcsc_gpu.h: which diagnostic macros this kernel object was built with
extern "C" __attribute__((visibility("default"))) int tcsc_gpu_build_flags(void) {
    int f = 0;
#ifdef TCSC_ABLATION
    f |= 1;
#endif
#ifdef TCSC_NODMA
    f |= 2;
#endif
#ifdef TCSC_STAMPS
    f |= 4;
#endif
#ifdef TCSC_TRACE
    f |= 8;
#endif
    return f;
}

namespace tcsc {

#ifdef TCSC_STAMPS
extern "C" __attribute__((visibility("default"))) int tcsc_debug_stamps(void* dst, size_t bytes) {
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stamps), bytes < sizeof(g_stamps) ? bytes : sizeof(g_stamps));
}
extern "C" __attribute__((visibility("default"))) int tcsc_debug_wgtimes(void* dst, size_t bytes) {
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_wgtime), bytes < sizeof(g_wgtime) ? bytes : sizeof(g_wgtime));
}
#endif

hipError_t launch_transpose(const float* X, int M, int K, float* XT, int ldxt, hipStream_t st) {
    if (M <= 0 || K <= 0) return hipSuccess;
    const bool vec = (K % 4 == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
    if (vec)
        hipLaunchKernelGGL(k_transpose<true>, dim3((K + 127) / 128, ldxt / 64), dim3(256), 0, st, X, M, K, XT, ldxt);
    else
        hipLaunchKernelGGL(k_transpose<false>, dim3((K + 63) / 64, ldxt / 64), dim3(256), 0, st, X, M, K, XT, ldxt);
    return hipGetLastError();
}

}  // namespace tcsc
