// gpridx_test.hip -- does gfx950 honour s_set_gpr_idx_on for VOP3P
// (v_pk_fma_f32) DST/SRC2 operands?  Each lane accumulates 8 float4 slots;
// step i adds (i+1)*sign to slot perm[i].  Also times the dynamic-slot
// update against a static-slot update.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f32x32 __attribute__((ext_vector_type(32)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__global__ void k_test(const int* __restrict__ slot4, const float* __restrict__ sgn, int n, float* out) {
    f32x32 acc;
#pragma unroll
    for (int i = 0; i < 32; ++i) acc[i] = 0.f;
    const float lanef = (float)(threadIdx.x & 63);
    for (int i = 0; i < n; ++i) {
        const int s = __builtin_amdgcn_readfirstlane(slot4[i]) | ((i * 7 + 1) << 10);  // high bits must be ignored
        const float g = __builtin_amdgcn_readfirstlane(__float_as_int(sgn[i])) == 0 ? 0.f : sgn[i];
        const float gs = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(g)));
        const unsigned long long gs2 = (unsigned long long)(unsigned)__float_as_int(gs);
        f32x2 x;
        x[0] = (float)(i + 1) + lanef;
        x[1] = (float)(i + 1) * 2.f;
        asm volatile(
            "s_set_gpr_idx_on %1, gpr_idx(SRC2,DST)\n"
            "v_pk_fma_f32 v[40:41], %2, %3, v[40:41] op_sel_hi:[1,0,1]\n"
            "s_set_gpr_idx_off\n"
            : "+{v[40:71]}"(acc)
            : "s"(s), "v"(x), "s"(gs2));
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) out[(blockIdx.x * blockDim.x + threadIdx.x) * 32 + i] = acc[i];
}

int main() {
    const int n = 64;
    int hs[n];
    float hg[n];
    for (int i = 0; i < n; ++i) {
        hs[i] = ((i * 5 + 3) % 16) * 2;  // float2 slot -> register index 2*slot (16 slots x 2 regs)
        hg[i] = (i % 3 == 0) ? -1.f : 1.f;
    }
    int* ds;
    float *dg, *dout;
    hipMalloc(&ds, sizeof hs);
    hipMalloc(&dg, sizeof hg);
    hipMalloc(&dout, 64 * 32 * 4);
    hipMemcpy(ds, hs, sizeof hs, hipMemcpyHostToDevice);
    hipMemcpy(dg, hg, sizeof hg, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_test, dim3(1), dim3(64), 0, 0, ds, dg, n, dout);
    hipError_t e = hipDeviceSynchronize();
    float ho[64 * 32];
    hipMemcpy(ho, dout, sizeof ho, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int lane = 0; lane < 64; ++lane) {
        float ref[32] = {0};
        for (int i = 0; i < n; ++i) {
            int r = hs[i];
            ref[r] += hg[i] * ((float)(i + 1) + lane);
            ref[r + 1] += hg[i] * ((float)(i + 1) * 2.f);
        }
        for (int r = 0; r < 32; ++r)
            if (ref[r] != ho[lane * 32 + r]) {
                if (bad < 10) printf("lane %d reg %d: got %f want %f\n", lane, r, ho[lane * 32 + r], ref[r]);
                ++bad;
            }
    }
    printf("gpr_idx VOP3P test: %s (%d mismatches), hip=%s\n", bad ? "FAIL" : "PASS", bad, hipGetErrorString(e));
    return bad != 0;
}
