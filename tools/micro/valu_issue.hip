// Microbenchmark: VALU issue cost per wave64 instruction class on gfx950, the
// per-class costs of bench.py's weighted VALU-issue floor (roofline.valu_issue).
//
// Each wave runs kIters x kChains independent instructions of one class (kChains
// independent register chains, so latency hides behind issue), timed with
// s_memtime (shader clock).  waves_per_simd 1 / 2 / 4: one wave alone on its
// SIMD, or several sharing it (cycles per instruction PER SIMD = elapsed *
// SIMDs / instructions).  Build + run:
//   hipcc --offload-arch=gfx950 -O3 tools/micro/valu_issue.hip -o /tmp/valu_issue && /tmp/valu_issue
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kChains = 16;
constexpr int kIters = 256;

enum Op { ADD_F64, FMA_F64, MUL_F64, RCP_F64, SQRT_F64, ADD_F32, FMA_F32, PK_FMA_F32, EXP_F32, RCP_F32, ADD_U32,
          CNDMASK, CVT_F64_I32, READLANE, LDEXP_F64, FRACT_F64, NOP_OPS };
const char* kName[] = {"v_add_f64", "v_fma_f64", "v_mul_f64", "v_rcp_f64", "v_sqrt_f64", "v_add_f32", "v_fma_f32",
                       "v_pk_fma_f32", "v_exp_f32", "v_rcp_f32", "v_add_u32", "v_cndmask_b32", "v_cvt_f64_i32",
                       "v_readlane_b32", "v_ldexp_f64", "v_fract_f64"};

template <int OP>
__global__ void k_issue(const double* in, double* out, unsigned long long* cyc) {
    const int t = threadIdx.x;
    double d[kChains];
    float f[kChains];
    unsigned u[kChains];
    for (int i = 0; i < kChains; ++i) {
        d[i] = in[(t + i) & 63];
        f[i] = (float)d[i];
        u[i] = (unsigned)(t * 7 + i);
    }
    const double dc = in[1];
    const float fc = (float)in[2];
    __syncthreads();
    const unsigned long long c0 = clock64();
#pragma unroll 1
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int i = 0; i < kChains; ++i) {
            if constexpr (OP == ADD_F64) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i]) : "v"(dc));
            if constexpr (OP == FMA_F64) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[i]) : "v"(dc));
            if constexpr (OP == MUL_F64) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[i]) : "v"(dc));
            if constexpr (OP == RCP_F64) asm volatile("v_rcp_f64 %0, %0" : "+v"(d[i]));
            if constexpr (OP == SQRT_F64) asm volatile("v_sqrt_f64 %0, %0" : "+v"(d[i]));
            if constexpr (OP == ADD_F32) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[i]) : "v"(fc));
            if constexpr (OP == FMA_F32) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[i]) : "v"(fc));
            if constexpr (OP == PK_FMA_F32) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(d[i]) : "v"(dc));
            if constexpr (OP == EXP_F32) asm volatile("v_exp_f32 %0, %0" : "+v"(f[i]));
            if constexpr (OP == RCP_F32) asm volatile("v_rcp_f32 %0, %0" : "+v"(f[i]));
            if constexpr (OP == ADD_U32) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[i]) : "v"(t));
            if constexpr (OP == CNDMASK) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[i]) : "v"(t));
            if constexpr (OP == CVT_F64_I32) asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(d[i]) : "v"(u[i]));
            if constexpr (OP == READLANE) asm volatile("v_readlane_b32 %0, %1, 5" : "=s"(u[i]) : "v"(f[i]));
            if constexpr (OP == LDEXP_F64) asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(d[i]) : "v"(t));
            if constexpr (OP == FRACT_F64) asm volatile("v_fract_f64 %0, %0" : "+v"(d[i]));
        }
    }
    const unsigned long long c1 = clock64();
    double s = 0.0;
    for (int i = 0; i < kChains; ++i) s += d[i] + (double)f[i] + (double)u[i];
    out[blockIdx.x * blockDim.x + t] = s;
    if ((t & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + t / 64] = c1 - c0;
}

template <int OP>
void run(const double* in, double* out, unsigned long long* cyc, int wps) {
    // one workgroup per CU (256 CUs), 4 * wps waves: wps waves on each SIMD
    const int threads = 256 * wps, blocks = 256;
    hipLaunchKernelGGL(k_issue<OP>, dim3(blocks), dim3(threads), 0, 0, in, out, cyc);
    hipDeviceSynchronize();
    const int nw = blocks * threads / 64;
    unsigned long long h[4096];
    hipMemcpy(h, cyc, nw * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    double mx = 0, sum = 0;
    for (int i = 0; i < nw; ++i) { sum += (double)h[i]; mx = h[i] > mx ? (double)h[i] : mx; }
    const double per_wave = (sum / nw) / (double)(kIters * kChains);
    printf("%-16s waves/SIMD %d: %6.2f cycles per instruction per wave, %6.2f per SIMD\n", kName[OP], wps, per_wave,
           per_wave / wps);
}

template <int OP>
void run_all(const double* in, double* out, unsigned long long* cyc) {
    for (int wps : {1, 2, 4}) run<OP>(in, out, cyc, wps);
    if constexpr (OP + 1 < NOP_OPS) run_all<OP + 1>(in, out, cyc);
}

int main() {
    double *in, *out;
    unsigned long long* cyc;
    hipMalloc(&in, 64 * 8);
    hipMalloc(&out, 256 * 1024 * 8);
    hipMalloc(&cyc, 4096 * 8);
    double h[64];
    for (int i = 0; i < 64; ++i) h[i] = 1.0 + 1e-3 * i;
    hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    run<ADD_F64>(in, out, cyc, 1);                       // warm-up (clock ramp)
    run_all<0>(in, out, cyc);
    return 0;
}
