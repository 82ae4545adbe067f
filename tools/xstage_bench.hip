// xstage_bench.hip -- the chunk loop of k_stream without its gather: can
// the Xᵀ staging read row-major X directly, with no k_transpose launch?
//
//   mode 0 (the kernel today): each chunk is 48 rows of X^T (1 KiB each),
//          4 DMA waves x 12 global_load_lds_dwordx4 (16 B per lane).
//   mode 1 (transposing DMA): each chunk is read from row-major X with
//          global_load_lds_dword: lane l loads X[m0 + 64j + l][k] (one row
//          per lane), so LDS gets the same [k][256 m] 1-KiB rows.  192
//          instructions per chunk, spread over all 16 waves (3 k x 4 row
//          groups each), one M0 write per k.
//   mode 2: as 1, issued by the 4 oldest waves only (12 k x 4 each).
//   mode 3 (round 3's direct staging, commit 19e8dbb): every wave loads 3
//          16-B pieces of row-major X per chunk into VGPRs (lane pair = 32 B
//          of a row, 32 rows per instruction) two chunks ahead, and writes
//          the previous set transposed into a ring of 2 (4 ds_write_b32 per
//          piece, paired as ds_write2st64).
//
// Workgroups are mapped XCD-aware as in k_stream (--xcd 1, the default):
// launch order L goes to XCD L % 8, and each XCD takes a contiguous range of
// (row tile, column block, slice) items, so the workgroups of a row tile
// share one L2.
//
// Geometry as k_stream: one workgroup of 16 waves per CU, 256 rows, ring of
// 3 x (48 + 1) rows, two chunks in flight, counted vmcnt + s_barrier per
// chunk.  grid = (ncb, nrt, z); each workgroup walks nch/z chunks.
// --check dumps workgroup (0,0,0)'s buffer after chunk 0 and compares it
// with X transposed.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

constexpr int kTK = 48, kTM = 256, kNBuf = 3, kBufRows = kTK + 1, kRow = kTM * 4;
constexpr int kLds = kNBuf * kBufRows * kRow;

template <int MODE>
__global__ void __launch_bounds__(1024, 4) stage(const float* X, const float* __restrict__ XT, int M, int K, int ldxt,
                                                  int nch, int cps, float* __restrict__ dump, int xcd) {
    __shared__ __attribute__((aligned(16))) char lds[kLds];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int cb = blockIdx.x, rt = blockIdx.y, z = blockIdx.z;
    if (xcd) {  // item i = (rt * ncb + cb) * nz + z, dealt in contiguous ranges per XCD
        const int n = gridDim.x * gridDim.y * gridDim.z;
        const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        const int per = n / 8;
        const int i = (n % 8 == 0) ? (L % 8) * per + L / 8 : L;
        z = i % gridDim.z;
        cb = (i / gridDim.z) % gridDim.x;
        rt = i / (gridDim.z * gridDim.x);
    }
    (void)cb;
    const int m0 = rt * kTM;
    const int c0 = z * cps, c1 = min(nch, c0 + cps);
    const unsigned ldsb = (unsigned)reinterpret_cast<uintptr_t>(lds);
    // mode 0
    unsigned voffA[12];
    for (int i = 0; i < 12; ++i) voffA[i] = 16u * lane + (unsigned)((wave * 12 + i) * ldxt * 4) - (unsigned)((i % 4) * kRow);
    // mode 1/2: per-lane row offsets, one per 64-row group, minus the group's LDS step (inst offset j*256)
    unsigned voffB[4];
    for (int j = 0; j < 4; ++j) {
        const int m = min(m0 + 64 * j + lane, M - 1);
        voffB[j] = (unsigned)((size_t)(m - m0) * K * 4) - 256u * j;
    }
    // mode 3: lane's row and first k inside the chunk (piece 0), LDS offset in buffer 0
    typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
    const int r3 = 32 * (wave & 7) + (lane >> 1), k3 = 8 * (wave >> 3) + 4 * (lane & 1);
    const int rows3 = min(kTM, M - m0);
    const __amdgpu_buffer_rsrc_t rs3 = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(X + (size_t)m0 * K), (short)0,
                                                                         (int)((unsigned)rows3 * (unsigned)K * 4u),
                                                                         0x00020000);
    const unsigned voff3 = (unsigned)(r3 * K + k3) * 4u;
    const unsigned lds3 = (unsigned)(k3 * kRow + 4 * r3);
    auto load3 = [&](u32x4_t (&v)[3], int c) {
        const unsigned base = voff3 + (unsigned)(c * kTK * 4);
#pragma unroll
        for (int q = 0; q < 3; ++q) v[q] = __builtin_amdgcn_raw_buffer_load_b128(rs3, base + 64u * q, 0, 0);
    };
    auto write3 = [&](const u32x4_t (&v)[3], int buf) {
        char* p = lds + lds3 + buf * (kBufRows * kRow);
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int j = 0; j < 4; ++j) *reinterpret_cast<unsigned*>(p + (16 * q + j) * kRow) = v[q][j];
    };
    if constexpr (MODE == 3) {
        float acc = 0.f;
        if (c0 < c1) {
            u32x4_t va[3], vb[3];
            load3(va, c0);
            load3(vb, c0 + 1);
            write3(va, c0 & 1);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            auto chunk = [&](int c, u32x4_t(&now)[3], u32x4_t(&nxt)[3]) {
                __builtin_amdgcn_s_barrier();
                load3(now, c + 2);
                asm volatile("" ::: "memory");
                acc += reinterpret_cast<const float*>(lds + (c & 1) * kBufRows * kRow)[threadIdx.x];
                if (dump && c == c0 && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && !xcd)
                    for (int i = threadIdx.x; i < kTK * kTM; i += 1024)
                        dump[i] = reinterpret_cast<const float*>(lds + (c & 1) * kBufRows * kRow)[i];
                if (c + 1 < c1) write3(nxt, (c + 1) & 1);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            };
            int c = c0;
            for (; c + 1 < c1; c += 2) {
                chunk(c, va, vb);
                chunk(c + 1, vb, va);
            }
            if (c < c1) chunk(c, va, vb);
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        }
        if (acc == 12345.f && dump) dump[0] = acc;
        return;
    }
    auto issue = [&](int c) {
        const int buf = c % kNBuf;
        const unsigned bb = ldsb + buf * kBufRows * kRow;
        if (MODE == 0) {
            if (wave < 4) {
                const char* src = reinterpret_cast<const char*>(XT + (size_t)c * kTK * ldxt + m0);
                for (int g = 0; g < 3; ++g) {
                    const unsigned m0v = bb + (wave * 12 + 4 * g) * kRow;
                    unsigned sv;
                    asm volatile(
                        "s_mov_b32 %[sv], m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %6\n\t"
                        "global_load_lds_dwordx4 %3, %6 offset:1024\n\tglobal_load_lds_dwordx4 %4, %6 offset:2048\n\t"
                        "global_load_lds_dwordx4 %5, %6 offset:3072\n\ts_mov_b32 m0, %[sv]"
                        : [sv] "=&s"(sv)
                        : "s"(m0v), "v"(voffA[4 * g]), "v"(voffA[4 * g + 1]), "v"(voffA[4 * g + 2]),
                          "v"(voffA[4 * g + 3]), "s"(src)
                        : "memory");
                }
            }
        } else {
            constexpr int kPer = MODE == 1 ? 3 : 12;  // k rows per issuing wave
            if (MODE == 1 || wave < 4) {
                const int kw = wave * kPer;
                const char* src = reinterpret_cast<const char*>(X + (size_t)m0 * K + (size_t)c * kTK + kw);
#pragma unroll
                for (int kk = 0; kk < kPer; ++kk) {
                    // M0 + inst offset (4kk + 256j) = bb + (kw+kk)*1 KiB + 256 j
                    const unsigned m0v = bb + (kw + kk) * kRow - 4 * kk;
                    unsigned sv;
                    asm volatile(
                        "s_mov_b32 %[sv], m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                        "global_load_lds_dword %2, %6 offset:%7\n\t"
                        "global_load_lds_dword %3, %6 offset:%8\n\t"
                        "global_load_lds_dword %4, %6 offset:%9\n\t"
                        "global_load_lds_dword %5, %6 offset:%10\n\ts_mov_b32 m0, %[sv]"
                        : [sv] "=&s"(sv)
                        : "s"(m0v), "v"(voffB[0]), "v"(voffB[1]), "v"(voffB[2]), "v"(voffB[3]), "s"(src),
                          "n"(4 * kk), "n"(4 * kk + 256), "n"(4 * kk + 512), "n"(4 * kk + 768)
                        : "memory");
                }
            }
        }
    };
    if (c0 < c1) issue(c0);
    if (c0 + 1 < c1) issue(c0 + 1);
    float acc = 0.f;
    for (int c = c0; c < c1; ++c) {
        // chunk c landed: everything but the next chunk's loads
        if (c + 1 < c1) {
            if (MODE == 0)
                asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
            else if (MODE == 1)
                asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
            else
                asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        if (c + 2 < c1) issue(c + 2);
        // a token read so the buffer is "used"
        acc += reinterpret_cast<const float*>(lds + (c % kNBuf) * kBufRows * kRow)[threadIdx.x];
        if (dump && c == c0 && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && !xcd) {
            for (int i = threadIdx.x; i < kTK * kTM; i += 1024)
                dump[i] = reinterpret_cast<const float*>(lds + (c % kNBuf) * kBufRows * kRow)[i];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (acc == 12345.f && dump) dump[0] = acc;
}

int main(int argc, char** argv) {
    int M = 4096, K = 16384, ncb = 8, z = 2, reps = 20, xcd = 1;
    bool check = false;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--M")) M = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--K")) K = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--ncb")) ncb = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--z")) z = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--reps")) reps = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--check")) check = true;
        else if (!strcmp(argv[i], "--xcd")) xcd = atoi(argv[++i]);
    }
    const int nrt = (M + kTM - 1) / kTM, nch = (K + kTK - 1) / kTK, cps = (nch + z - 1) / z;
    const int ldxt = nrt * kTM;
    const size_t xn = (size_t)M * K, xtn = (size_t)(nch + 2) * kTK * ldxt;
    float *X, *XT, *dump;
    hipMalloc(&X, xn * 4 + 4096);
    hipMalloc(&XT, xtn * 4);
    hipMalloc(&dump, (size_t)kTK * kTM * 4);
    std::vector<float> h(xn);
    for (size_t i = 0; i < xn; ++i) h[i] = (float)(i % 1000003);
    hipMemcpy(X, h.data(), xn * 4, hipMemcpyHostToDevice);
    {
        std::vector<float> t(xtn, 0.f);
        for (int k = 0; k < K; ++k)
            for (int m = 0; m < M; ++m) t[(size_t)k * ldxt + m] = h[(size_t)m * K + k];
        hipMemcpy(XT, t.data(), xtn * 4, hipMemcpyHostToDevice);
    }
    dim3 grid(ncb, nrt, z);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("M=%d K=%d grid %dx%dx%d = %d WGs, %d chunks per WG, XCD-aware order %d\n", M, K, ncb, nrt, z,
           ncb * nrt * z, cps, xcd);
    for (int mode = 0; mode < 4; ++mode) {
        auto launch = [&](float* d) {
            if (mode == 0) hipLaunchKernelGGL(stage<0>, grid, dim3(1024), 0, 0, X, XT, M, K, ldxt, nch, cps, d, xcd);
            if (mode == 1) hipLaunchKernelGGL(stage<1>, grid, dim3(1024), 0, 0, X, XT, M, K, ldxt, nch, cps, d, xcd);
            if (mode == 2) hipLaunchKernelGGL(stage<2>, grid, dim3(1024), 0, 0, X, XT, M, K, ldxt, nch, cps, d, xcd);
            if (mode == 3) hipLaunchKernelGGL(stage<3>, grid, dim3(1024), 0, 0, X, XT, M, K, ldxt, nch, cps, d, xcd);
        };
        if (check && !xcd) {
            hipMemset(dump, 0, (size_t)kTK * kTM * 4);
            launch(dump);
            hipDeviceSynchronize();
            std::vector<float> d((size_t)kTK * kTM);
            hipMemcpy(d.data(), dump, d.size() * 4, hipMemcpyDeviceToHost);
            int bad = 0;
            for (int k = 0; k < kTK; ++k)
                for (int m = 0; m < kTM && m < M; ++m)
                    if (d[(size_t)k * kTM + m] != h[(size_t)m * K + k]) ++bad;
            printf("mode %d check: %d wrong of %d\n", mode, bad, kTK * kTM);
        }
        for (int w = 0; w < 3; ++w) launch(nullptr);
        hipEventRecord(e0);
        for (int r = 0; r < reps; ++r) launch(nullptr);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double per = ms / reps;
        const double waves_rounds = (double)ncb * nrt * z / 256.0;
        printf("mode %d: %.4f ms per launch, %.3f us per chunk per round (rounds %.2f)\n", mode, per,
               per * 1e3 / (cps * (waves_rounds < 1 ? 1 : waves_rounds)), waves_rounds);
    }
    return 0;
}
