// Host wake-up latency after a short kernel (LO-round sized, ~25 us of work):
//   (a) hipStreamSynchronize (HIP's default wait: active spin, then blocking),
//   (b) hipEventSynchronize on a blocking-sync-free event,
//   (c) a host spin on a flag the kernel writes into coherent pinned memory
//       (after __threadfence_system), then hipStreamSynchronize (already done).
// Prints median wall time per launch for each, for a few kernel lengths.
// Build: hipcc --offload-arch=gfx950 -O2 tools/micro/sync_latency.hip -o /tmp/sync_latency
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_spin(long long cycles, volatile unsigned* flag, unsigned epoch, double* sink) {
    const long long t0 = clock64();
    double a = threadIdx.x;
    while (clock64() - t0 < cycles) a = a * 1.0000001 + 1e-9;
    if (a == -1.0) sink[0] = a;
    __syncthreads();
    if (threadIdx.x == 0 && flag) {
        __threadfence_system();
        *flag = epoch;
    }
}

int main(int argc, char** argv) {
    // argv[1] == "spin": hipSetDeviceFlags(hipDeviceScheduleSpin) before any
    // other HIP call (HIP's host wait policy); ROC_ACTIVE_WAIT_TIMEOUT in the
    // environment sets the runtime's active-wait window instead
    if (argc > 1 && argv[1][0] == 's') CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
    if (argc > 1 && argv[1][0] == 'y') CK(hipSetDeviceFlags(hipDeviceScheduleYield));
    if (argc > 1 && argv[1][0] == 'b') CK(hipSetDeviceFlags(hipDeviceScheduleBlockingSync));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned* flag = nullptr;
    CK(hipHostMalloc((void**)&flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
    unsigned* dflag = nullptr;
    CK(hipHostGetDevicePointer((void**)&dflag, flag, 0));
    double* sink;
    CK(hipMalloc(&sink, 64));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    // clock64 runs at the shader clock; calibrate cycles per us
    auto wall = [] { return std::chrono::steady_clock::now(); };
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, 1000LL, nullptr, 0u, sink);
    CK(hipStreamSynchronize(s));
    const int R = 200;
    unsigned epoch = 1;
    for (long long cyc : {0LL, 10000LL, 40000LL, 100000LL}) {
        std::vector<double> a, b, c;
        for (int r = 0; r < R; ++r) {
            auto t0 = wall();
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, cyc, nullptr, 0u, sink);
            CK(hipStreamSynchronize(s));
            a.push_back(us(t0, wall()));
            t0 = wall();
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, cyc, nullptr, 0u, sink);
            CK(hipEventRecord(ev, s));
            CK(hipEventSynchronize(ev));
            b.push_back(us(t0, wall()));
            ++epoch;
            t0 = wall();
            hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, cyc, dflag, epoch, sink);
            while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != epoch) {}
            c.push_back(us(t0, wall()));
            CK(hipStreamSynchronize(s));
        }
        auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
        printf("cycles %7lld: streamSync %7.2f us  eventSync %7.2f us  flag spin %7.2f us\n", cyc, med(a), med(b), med(c));
    }
    return 0;
}
