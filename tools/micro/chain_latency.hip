// Microbenchmark: dependent fp64 add chain latency on gfx950, alone and next
// to 15 busy waves of the same workgroup (the k_score_split chain-wave setting).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(1024) void k_chain(const double* in, double* out, long long* cyc, int busy, int prio) {
    __shared__ double lds[4096];
    const int t = threadIdx.x;
    for (int i = t; i < 4096; i += blockDim.x) lds[i] = in[i & 255];
    __syncthreads();
    if (t >= 960) {                        // chain wave
        if (prio) __builtin_amdgcn_s_setprio(3);
        double acc = 0.0;
        const double x0 = in[t & 7], x1 = in[(t + 1) & 7];
        const long long c0 = clock64();
        for (int i = 0; i < 4096; i += 2) { acc += x0; acc += x1; }
        const long long c1 = clock64();
        double acc2 = 0.0;
        const long long c2 = clock64();
#pragma unroll 1
        for (int i = 0; i < 4096; i += 8) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = lds[(i + u) & 4095];
#pragma unroll
            for (int u = 0; u < 8; ++u) acc2 += v[u];
        }
        const long long c3 = clock64();
        if (t == 960) { cyc[0] = c1 - c0; cyc[1] = c3 - c2; }
        out[t] = acc + acc2;
    } else if (busy == 1) {                // 15 compute waves: independent fp64 FMAs
        double a = in[t & 255], b = in[(t + 3) & 255], c = 0.5, d = 0.25, e = 0.125, f = 0.0625;
        for (int i = 0; i < 20000; ++i) {
            a = __builtin_fma(a, b, 1e-9); c = __builtin_fma(c, b, 1e-9);
            d = __builtin_fma(d, b, 1e-9); e = __builtin_fma(e, b, 1e-9); f = __builtin_fma(f, b, 1e-9);
        }
        out[t] = a + c + d + e + f;
    } else if (busy == 2) {                // 15 compute waves: LDS traffic
        double s = 0.0;
        for (int i = 0; i < 4000; ++i) { s += lds[(t * 8 + i * 64) & 4095]; lds[(t + i * 17) & 4095] = s; }
        out[t] = s;
    }
}

int main() {
    double *in, *out;
    long long* cyc;
    hipMalloc(&in, 4096 * 8); hipMalloc(&out, 1024 * 8); hipMalloc(&cyc, 16);
    double h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = 1.0 + 1e-3 * (i % 13);
    hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    for (int busy = 0; busy < 3; ++busy)
        for (int prio = 0; prio < 2; ++prio) {
            hipLaunchKernelGGL(k_chain, dim3(1), dim3(1024), 0, 0, in, out, cyc, busy, prio);
            long long c[2];
            hipMemcpy(c, cyc, 16, hipMemcpyDeviceToHost);
            printf("busy=%d prio=%d  reg-chain %.2f cyc/add   lds-chain(8-ahead) %.2f cyc/add\n", busy, prio,
                   c[0] / 4096.0, c[1] / 4096.0);
        }
    return 0;
}
