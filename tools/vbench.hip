// vbench.hip -- issue cost of the gather loop's instruction forms on gfx950.
// Every CU runs WPS waves per SIMD (blocks of 4 waves, one per SIMD); each
// wave loops ITERS times over a body of the instruction form under test with
// independent accumulators, timing itself with s_memtime (shader clock).
// Prints cycles per body per wave and per instruction per SIMD.
//   Build: hipcc --offload-arch=gfx950 -O3 -o vbench vbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// 16 instructions per body unless noted
#define PKFMA_S(a, b) "v_pk_fma_f32 v[" #a ":" #b "], v[40:41], s[20:21], v[" #a ":" #b "] op_sel_hi:[1,0,1]\n"
#define PKFMA_V(a, b) "v_pk_fma_f32 v[" #a ":" #b "], v[40:41], v[42:43], v[" #a ":" #b "]\n"
#define PKADD(a, b) "v_pk_add_f32 v[" #a ":" #b "], v[40:41], v[" #a ":" #b "]\n"
#define ADD2(a, b) "v_add_f32 v" #a ", v40, v" #a "\n v_add_f32 v" #b ", v41, v" #b "\n"

// One asm block per mode: setup, s_memtime, the loop (s_cbranch on an SGPR
// counter) and the closing s_memtime, so no compiler value lives in the
// registers the body uses.  Body registers: v0..v31 accumulators, v32..v43
// operands/temps, s20..s21 sign pair, s22..s29 index words, s30..s45 temps.
#define SETUP \
    "v_mov_b32 v40, 1.0\n v_mov_b32 v41, 1.0\n v_mov_b32 v42, 1.0\n v_mov_b32 v43, 1.0\n" \
    "s_mov_b32 s20, 1.0\n s_mov_b32 s21, 1.0\n" \
    "s_mov_b32 s22, 0\n s_mov_b32 s23, 4\n s_mov_b32 s24, 8\n s_mov_b32 s25, 12\n" \
    "s_mov_b32 s26, 16\n s_mov_b32 s27, 20\n s_mov_b32 s28, 24\n s_mov_b32 s29, 28\n" \
    "v_mov_b32 v0, 0\n v_mov_b32 v1, 0\n v_mov_b32 v2, 0\n v_mov_b32 v3, 0\n" \
    "v_mov_b32 v4, 0\n v_mov_b32 v5, 0\n v_mov_b32 v6, 0\n v_mov_b32 v7, 0\n" \
    "v_mov_b32 v8, 0\n v_mov_b32 v9, 0\n v_mov_b32 v10, 0\n v_mov_b32 v11, 0\n" \
    "v_mov_b32 v12, 0\n v_mov_b32 v13, 0\n v_mov_b32 v14, 0\n v_mov_b32 v15, 0\n" \
    "v_mov_b32 v16, 0\n v_mov_b32 v17, 0\n v_mov_b32 v18, 0\n v_mov_b32 v19, 0\n" \
    "v_mov_b32 v20, 0\n v_mov_b32 v21, 0\n v_mov_b32 v22, 0\n v_mov_b32 v23, 0\n" \
    "v_mov_b32 v24, 0\n v_mov_b32 v25, 0\n v_mov_b32 v26, 0\n v_mov_b32 v27, 0\n" \
    "v_mov_b32 v28, 0\n v_mov_b32 v29, 0\n v_mov_b32 v30, 0\n v_mov_b32 v31, 0\n"
#define CLOBBERS                                                                                                    \
    "memory", "scc", "m0", "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13",   \
        "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28",     \
        "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43",     \
        "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", "s29", "s30", "s31", "s32", "s33", "s34",     \
        "s35", "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45"
#define LOOP(BODY)                                                                                          \
    asm volatile(SETUP                                                                                        \
                 "s_waitcnt lgkmcnt(0)\n s_memtime %[t0]\n s_waitcnt lgkmcnt(0)\n s_mov_b32 s46, %[n]\n"   \
                 ".Lloop%=:\n" BODY BODY BODY BODY "s_sub_u32 s46, s46, 1\n s_cmp_lg_u32 s46, 0\n s_cbranch_scc1 .Lloop%=\n" \
                 "s_memtime %[t1]\n s_waitcnt lgkmcnt(0)\n v_add_f32 %[r], v0, v31\n"                         \
                 : [t0] "=&s"(t0), [t1] "=&s"(t1), [r] "=&v"(r)                                               \
                 : [n] "s"(iters)                                                                             \
                 : CLOBBERS, "s46")

template <int MODE>
__global__ void __launch_bounds__(256) k_body(int iters, long long* cyc, float* out) {
    long long t0 = 0, t1 = 0;
    float r = 0.f;
    if (MODE == 0) LOOP(PKFMA_S(0, 1) PKFMA_S(2, 3) PKFMA_S(4, 5) PKFMA_S(6, 7) PKFMA_S(8, 9) PKFMA_S(10, 11) PKFMA_S(12, 13) PKFMA_S(14, 15) PKFMA_S(16, 17) PKFMA_S(18, 19) PKFMA_S(20, 21) PKFMA_S(22, 23) PKFMA_S(24, 25) PKFMA_S(26, 27) PKFMA_S(28, 29) PKFMA_S(30, 31));
    if (MODE == 1) LOOP(PKFMA_V(0, 1) PKFMA_V(2, 3) PKFMA_V(4, 5) PKFMA_V(6, 7) PKFMA_V(8, 9) PKFMA_V(10, 11) PKFMA_V(12, 13) PKFMA_V(14, 15) PKFMA_V(16, 17) PKFMA_V(18, 19) PKFMA_V(20, 21) PKFMA_V(22, 23) PKFMA_V(24, 25) PKFMA_V(26, 27) PKFMA_V(28, 29) PKFMA_V(30, 31));
    if (MODE == 2) LOOP(PKADD(0, 1) PKADD(2, 3) PKADD(4, 5) PKADD(6, 7) PKADD(8, 9) PKADD(10, 11) PKADD(12, 13) PKADD(14, 15) PKADD(16, 17) PKADD(18, 19) PKADD(20, 21) PKADD(22, 23) PKADD(24, 25) PKADD(26, 27) PKADD(28, 29) PKADD(30, 31));
    if (MODE == 3) LOOP(ADD2(0, 1) ADD2(2, 3) ADD2(4, 5) ADD2(6, 7) ADD2(8, 9) ADD2(10, 11) ADD2(12, 13) ADD2(14, 15) ADD2(16, 17) ADD2(18, 19) ADD2(20, 21) ADD2(22, 23) ADD2(24, 25) ADD2(26, 27) ADD2(28, 29) ADD2(30, 31));
    if (MODE == 4) LOOP("s_set_gpr_idx_on s22, gpr_idx(SRC2,DST)\n" PKFMA_S(0, 1) PKFMA_S(2, 3) "s_set_gpr_idx_idx s23\n" PKFMA_S(0, 1) PKFMA_S(2, 3) "s_set_gpr_idx_idx s24\n" PKFMA_S(0, 1) PKFMA_S(2, 3) "s_set_gpr_idx_idx s25\n" PKFMA_S(0, 1) PKFMA_S(2, 3) "s_set_gpr_idx_idx s26\n" PKFMA_S(0, 1) PKFMA_S(2, 3) "s_set_gpr_idx_idx s27\n" PKFMA_S(0, 1) PKFMA_S(2, 3) "s_set_gpr_idx_idx s28\n" PKFMA_S(0, 1) PKFMA_S(2, 3) "s_set_gpr_idx_idx s29\n" PKFMA_S(0, 1) PKFMA_S(2, 3) "s_set_gpr_idx_off\n");
    if (MODE == 5) LOOP("v_readlane_b32 s30, v40, 0\n v_readlane_b32 s31, v40, 1\n v_readlane_b32 s32, v40, 2\n v_readlane_b32 s33, v40, 3\n v_readlane_b32 s34, v40, 4\n v_readlane_b32 s35, v40, 5\n v_readlane_b32 s36, v40, 6\n v_readlane_b32 s37, v40, 7\n v_readlane_b32 s38, v41, 0\n v_readlane_b32 s39, v41, 1\n v_readlane_b32 s40, v41, 2\n v_readlane_b32 s41, v41, 3\n v_readlane_b32 s42, v41, 4\n v_readlane_b32 s43, v41, 5\n v_readlane_b32 s44, v41, 6\n v_readlane_b32 s45, v41, 7\n v_bfi_b32 v32, v42, v43, s30\n v_bfi_b32 v33, v42, v43, s31\n v_bfi_b32 v34, v42, v43, s32\n v_bfi_b32 v35, v42, v43, s33\n v_bfi_b32 v36, v42, v43, s34\n v_bfi_b32 v37, v42, v43, s35\n v_bfi_b32 v38, v42, v43, s36\n v_bfi_b32 v39, v42, v43, s37\n");
    if (MODE == 6) LOOP("v_bfi_b32 v32, v42, v43, s22\n v_bfi_b32 v33, v42, v43, s23\n v_bfi_b32 v34, v42, v43, s24\n v_bfi_b32 v35, v42, v43, s25\n v_bfi_b32 v36, v42, v43, s26\n v_bfi_b32 v37, v42, v43, s27\n v_bfi_b32 v38, v42, v43, s28\n v_bfi_b32 v39, v42, v43, s29\n");
    if (MODE == 7) LOOP("v_readlane_b32 s30, v40, 0\n v_readlane_b32 s31, v40, 1\n v_readlane_b32 s32, v40, 2\n v_readlane_b32 s33, v40, 3\n v_readlane_b32 s34, v40, 4\n v_readlane_b32 s35, v40, 5\n v_readlane_b32 s36, v40, 6\n v_readlane_b32 s37, v40, 7\n v_readlane_b32 s38, v41, 0\n v_readlane_b32 s39, v41, 1\n v_readlane_b32 s40, v41, 2\n v_readlane_b32 s41, v41, 3\n v_readlane_b32 s42, v41, 4\n v_readlane_b32 s43, v41, 5\n v_readlane_b32 s44, v41, 6\n v_readlane_b32 s45, v41, 7\n");
    if (MODE == 8) LOOP("s_set_gpr_idx_on s22, gpr_idx(SRC1,DST)\n" PKADD(0, 1) PKADD(2, 3) "s_set_gpr_idx_idx s23\n" PKADD(0, 1) PKADD(2, 3) "s_set_gpr_idx_idx s24\n" PKADD(0, 1) PKADD(2, 3) "s_set_gpr_idx_idx s25\n" PKADD(0, 1) PKADD(2, 3) "s_set_gpr_idx_idx s26\n" PKADD(0, 1) PKADD(2, 3) "s_set_gpr_idx_idx s27\n" PKADD(0, 1) PKADD(2, 3) "s_set_gpr_idx_idx s28\n" PKADD(0, 1) PKADD(2, 3) "s_set_gpr_idx_idx s29\n" PKADD(0, 1) PKADD(2, 3) "s_set_gpr_idx_off\n");
    if (MODE == 9) LOOP("v_add_u32 v32, s22, v42\n v_add_u32 v33, s23, v42\n v_add_u32 v34, s24, v42\n v_add_u32 v35, s25, v42\n v_add_u32 v36, s26, v42\n v_add_u32 v37, s27, v42\n v_add_u32 v38, s28, v42\n v_add_u32 v39, s29, v42\n v_add_u32 v32, s22, v42\n v_add_u32 v33, s23, v42\n v_add_u32 v34, s24, v42\n v_add_u32 v35, s25, v42\n v_add_u32 v36, s26, v42\n v_add_u32 v37, s27, v42\n v_add_u32 v38, s28, v42\n v_add_u32 v39, s29, v42\n ");
    if (MODE == 10) LOOP("v_add_u32_e64 v32, s22, v42\n v_add_u32_e64 v33, s23, v42\n v_add_u32_e64 v34, s24, v42\n v_add_u32_e64 v35, s25, v42\n v_add_u32_e64 v36, s26, v42\n v_add_u32_e64 v37, s27, v42\n v_add_u32_e64 v38, s28, v42\n v_add_u32_e64 v39, s29, v42\n v_add_u32_e64 v32, s22, v42\n v_add_u32_e64 v33, s23, v42\n v_add_u32_e64 v34, s24, v42\n v_add_u32_e64 v35, s25, v42\n v_add_u32_e64 v36, s26, v42\n v_add_u32_e64 v37, s27, v42\n v_add_u32_e64 v38, s28, v42\n v_add_u32_e64 v39, s29, v42\n ");
    if (MODE == 11) LOOP("s_set_gpr_idx_on s22, gpr_idx(DST)\n s_set_gpr_idx_off\n s_set_gpr_idx_on s23, gpr_idx(DST)\n s_set_gpr_idx_off\n s_set_gpr_idx_on s24, gpr_idx(DST)\n s_set_gpr_idx_off\n s_set_gpr_idx_on s25, gpr_idx(DST)\n s_set_gpr_idx_off\n s_set_gpr_idx_on s26, gpr_idx(DST)\n s_set_gpr_idx_off\n s_set_gpr_idx_on s27, gpr_idx(DST)\n s_set_gpr_idx_off\n s_set_gpr_idx_on s28, gpr_idx(DST)\n s_set_gpr_idx_off\n s_set_gpr_idx_on s29, gpr_idx(DST)\n s_set_gpr_idx_off\n ");
    if (MODE == 12) LOOP("v_mov_b32 v32, s22\n v_mov_b32 v33, s23\n v_mov_b32 v34, s24\n v_mov_b32 v35, s25\n v_mov_b32 v36, s26\n v_mov_b32 v37, s27\n v_mov_b32 v38, s28\n v_mov_b32 v39, s29\n v_mov_b32 v32, s22\n v_mov_b32 v33, s23\n v_mov_b32 v34, s24\n v_mov_b32 v35, s25\n v_mov_b32 v36, s26\n v_mov_b32 v37, s27\n v_mov_b32 v38, s28\n v_mov_b32 v39, s29\n ");
    if (MODE == 13) LOOP("s_add_u32 s30, s22, 1\n s_add_u32 s31, s23, 1\n s_add_u32 s32, s24, 1\n s_add_u32 s33, s25, 1\n s_add_u32 s34, s26, 1\n s_add_u32 s35, s27, 1\n s_add_u32 s36, s28, 1\n s_add_u32 s37, s29, 1\n s_add_u32 s30, s22, 1\n s_add_u32 s31, s23, 1\n s_add_u32 s32, s24, 1\n s_add_u32 s33, s25, 1\n s_add_u32 s34, s26, 1\n s_add_u32 s35, s27, 1\n s_add_u32 s36, s28, 1\n s_add_u32 s37, s29, 1\n ");
    if (MODE == 14) LOOP("v_add_u32 v32, s22, v42\n v_pk_add_f32 v[0:1], v[40:41], v[0:1]\n v_add_u32 v33, s23, v42\n v_pk_add_f32 v[2:3], v[40:41], v[2:3]\n v_add_u32 v34, s24, v42\n v_pk_add_f32 v[4:5], v[40:41], v[4:5]\n v_add_u32 v35, s25, v42\n v_pk_add_f32 v[6:7], v[40:41], v[6:7]\n v_add_u32 v36, s26, v42\n v_pk_add_f32 v[8:9], v[40:41], v[8:9]\n v_add_u32 v37, s27, v42\n v_pk_add_f32 v[10:11], v[40:41], v[10:11]\n v_add_u32 v38, s28, v42\n v_pk_add_f32 v[12:13], v[40:41], v[12:13]\n v_add_u32 v39, s29, v42\n v_pk_add_f32 v[14:15], v[40:41], v[14:15]\n v_add_u32 v32, s22, v42\n v_pk_add_f32 v[16:17], v[40:41], v[16:17]\n v_add_u32 v33, s23, v42\n v_pk_add_f32 v[18:19], v[40:41], v[18:19]\n v_add_u32 v34, s24, v42\n v_pk_add_f32 v[20:21], v[40:41], v[20:21]\n v_add_u32 v35, s25, v42\n v_pk_add_f32 v[22:23], v[40:41], v[22:23]\n v_add_u32 v36, s26, v42\n v_pk_add_f32 v[24:25], v[40:41], v[24:25]\n v_add_u32 v37, s27, v42\n v_pk_add_f32 v[26:27], v[40:41], v[26:27]\n v_add_u32 v38, s28, v42\n v_pk_add_f32 v[28:29], v[40:41], v[28:29]\n v_add_u32 v39, s29, v42\n v_pk_add_f32 v[30:31], v[40:41], v[30:31]\n ");
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

static const char* kName[] = {"16 pk_fma (sgpr src1)", "16 pk_fma (vgpr src1)", "16 pk_add", "32 v_add_f32",
                              "FMA phase: 8x(idx + 2 pk_fma)", "16 readlane + 8 bfi", "8 bfi", "16 readlane",
                              "FMA phase with pk_add", "16 v_add_u32 (VOP2)", "16 v_add_u32_e64 (VOP3)",
                              "8 x (gpr_idx_on + off)", "16 v_mov_b32 (VOP1)", "16 s_add_u32",
                              "16 x (v_add_u32 + v_pk_add)"};
static const int kInstr[] = {16, 16, 16, 32, 16, 24, 8, 16, 16, 16, 16, 16, 16, 16, 32};

template <int MODE>
void run(int cus, int wps, long long* cyc, float* out) {
    const int iters = 4096;
    const int blocks = cus * wps;
    hipLaunchKernelGGL((k_body<MODE>), dim3(blocks), dim3(256), 0, 0, iters, cyc, out);
    CHECK(hipDeviceSynchronize());
    hipLaunchKernelGGL((k_body<MODE>), dim3(blocks), dim3(256), 0, 0, iters, cyc, out);
    CHECK(hipDeviceSynchronize());
    long long* h = (long long*)malloc(sizeof(long long) * blocks * 4);
    CHECK(hipMemcpy(h, cyc, sizeof(long long) * blocks * 4, hipMemcpyDeviceToHost));
    double s = 0;
    for (int i = 0; i < blocks * 4; ++i) s += (double)h[i];
    s /= blocks * 4;
    const double per_body = s / iters / 4;  // LOOP repeats the body 4x
    // per SIMD: wps waves share it
    printf("%-34s wps=%d: %7.1f cyc/body/wave  %5.2f cyc/instr/SIMD\n", kName[MODE], wps, per_body,
           per_body / kInstr[MODE] / wps);
    free(h);
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    long long* cyc;
    float* out;
    CHECK(hipMalloc(&cyc, sizeof(long long) * cus * 64 * 4));
    CHECK(hipMalloc(&out, sizeof(float) * cus * 64 * 256));
    for (int wps : {1, 2, 4}) {
        run<0>(cus, wps, cyc, out);
        run<1>(cus, wps, cyc, out);
        run<2>(cus, wps, cyc, out);
        run<3>(cus, wps, cyc, out);
        run<4>(cus, wps, cyc, out);
        run<8>(cus, wps, cyc, out);
        run<5>(cus, wps, cyc, out);
        run<6>(cus, wps, cyc, out);
        run<7>(cus, wps, cyc, out);
        run<9>(cus, wps, cyc, out);
        run<10>(cus, wps, cyc, out);
        run<11>(cus, wps, cyc, out);
        run<12>(cus, wps, cyc, out);
        run<13>(cus, wps, cyc, out);
        run<14>(cus, wps, cyc, out);
    }
    return 0;
}
