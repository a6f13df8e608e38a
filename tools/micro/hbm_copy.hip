// Microbenchmark: streaming-copy variants on gfx950, to pick the shape of the
// engine's measured-HBM-peak probe (k_hbm_copy, gcr_measure_hbm).
// Reports read + write bytes / kernel time, best of 10 per variant.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/hbm_copy.hip -o /tmp/hbm_copy
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double v2d __attribute__((ext_vector_type(2)));

// A: grid-stride, U loads in flight per lane (the round-2 probe)
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_gs(const v2d* __restrict__ s, v2d* __restrict__ d, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        v2d v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(s + i + u * stride) : s[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NT) __builtin_nontemporal_store(v[u], d + i + u * stride);
            else d[i + u * stride] = v[u];
        }
    }
    for (; i < n; i += stride) d[i] = s[i];
}

// B: one tile per workgroup (no grid stride), U loads per lane, T threads
template <int T, int U, bool NT>
__global__ __launch_bounds__(T) void k_tile(const v2d* __restrict__ s, v2d* __restrict__ d, size_t n) {
    const size_t base = (size_t)blockIdx.x * T * U + threadIdx.x;
    v2d v[U];
    if (base + (size_t)(U - 1) * T < n) {
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(s + base + u * T) : s[base + u * T];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NT) __builtin_nontemporal_store(v[u], d + base + u * T);
            else d[base + u * T] = v[u];
        }
    } else {
        for (int u = 0; u < U; ++u)
            if (base + (size_t)u * T < n) d[base + u * T] = s[base + u * T];
    }
}

// C: read-only reduction (one value per workgroup), the read half alone
template <int U>
__global__ __launch_bounds__(256) void k_read(const v2d* __restrict__ s, double* __restrict__ d, size_t n) {
    const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    double acc = 0.0;
    if (base + (size_t)(U - 1) * 256 < n) {
        v2d v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(s + base + u * 256);
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y;
    }
    if (acc == 12345.678) d[blockIdx.x] = acc;     // never true: keeps the loads
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <class L>
static double timeit(L launch, double bytes) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    double best = 0.0;
    for (int it = -2; it < 10; ++it) {
        CK(hipEventRecord(a));
        launch();
        CK(hipGetLastError());
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, a, b));
        if (it >= 0 && ms > 0.f) best = best > bytes / (ms * 1e6) ? best : bytes / (ms * 1e6);
    }
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return best;
}

int main(int argc, char** argv) {
    const size_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 2048ull) << 20;
    const size_t n = bytes / sizeof(v2d);
    v2d *s, *d;
    CK(hipMalloc(&s, bytes));
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(s, 0x3f, bytes));
    CK(hipMemset(d, 0, bytes));
    CK(hipDeviceSynchronize());
    const double rw = 2.0 * (double)bytes;
#define GS(U, NT, G) printf("grid-stride U=%d nt=%d grid=%d: %.0f GB/s\n", U, NT, G, \
        timeit([&] { hipLaunchKernelGGL((k_gs<U, NT>), dim3(G), dim3(256), 0, 0, s, d, n); }, rw))
#define TL(T, U, NT) printf("tile T=%d U=%d nt=%d: %.0f GB/s\n", T, U, NT, \
        timeit([&] { hipLaunchKernelGGL((k_tile<T, U, NT>), dim3((n + (size_t)T * U - 1) / ((size_t)T * U)), dim3(T), 0, 0, s, d, n); }, rw))
    GS(8, false, 2048);
    GS(8, true, 2048);
    GS(4, false, 8192);
    GS(4, true, 8192);
    GS(2, true, 16384);
    TL(256, 1, false);
    TL(256, 2, false);
    TL(256, 4, false);
    TL(256, 4, true);
    TL(256, 8, false);
    TL(256, 8, true);
    TL(512, 4, false);
    TL(512, 4, true);
    TL(1024, 2, false);
    TL(1024, 4, true);
    double* r;
    CK(hipMalloc(&r, 1 << 20));
    printf("read-only U=8 nt: %.0f GB/s\n",
           timeit([&] { hipLaunchKernelGGL((k_read<8>), dim3(n / (256 * 8)), dim3(256), 0, 0, s, r, n); }, (double)bytes));
    printf("read-only U=4 nt: %.0f GB/s\n",
           timeit([&] { hipLaunchKernelGGL((k_read<4>), dim3(n / (256 * 4)), dim3(256), 0, 0, s, r, n); }, (double)bytes));
    CK(hipFree(r));
    CK(hipFree(s));
    CK(hipFree(d));
    return 0;
}
