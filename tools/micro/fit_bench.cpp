// Host LO-trial fit timing (host_fit.cpp fit_nonminimal): the 2-SIFT hybrid
// fit of 14 scale + 14 orientation points (an M2 LO trial, 7 m per class) on
// synthetic features, per call on one thread.  Build:
//   g++ -O3 -std=c++17 -ffp-contract=off -I graph-cut-ransac_amd/csrc -I include \
//       tools/micro/fit_bench.cpp graph-cut-ransac_amd/csrc/host_fit.cpp -o /tmp/fit_bench
#include "host_fit.h"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

using namespace gcr;

int main() {
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    HostClass cls[2];
    const size_t n = 5000;
    for (int c = 0; c < 2; ++c) {
        cls[c].n = n;
        for (size_t i = 0; i < n; ++i) {
            cls[c].x.push_back(1000 * U(rng));
            cls[c].y.push_back(800 * U(rng));
            const double th = 6.283185307179586 * U(rng);
            cls[c].a.push_back(1.0 + U(rng));
            cls[c].c0.push_back(c == 0 ? 1.0 + U(rng) : std::cos(th));
            cls[c].c1.push_back(std::sin(th));
        }
    }
    const int calls = 2000;
    std::vector<std::vector<uint32_t>> idx(2 * calls);
    for (auto& v : idx) {
        for (int k = 0; k < 14; ++k) v.push_back((uint32_t)(U(rng) * n));
    }
    int ok = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < calls; ++k) {
        RectModel m{};
        std::vector<uint32_t> two[2] = {idx[2 * k], idx[2 * k + 1]};
        ok += fit_nonminimal(2, cls, two, m, nullptr, 0) ? 1 : 0;
    }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / calls;
    std::printf("fit_nonminimal (2-SIFT, 14 + 14 points): %.2f us per call, %d / %d fitted\n", us, ok, calls);
    return 0;
}
