// Host LO-trial fit breakdown (host_fit.cpp fit_nonminimal, 2-SIFT, 14 + 14
// points): whole fit, and its parts -- the 105-row system + QR, the rectified
// angles (glibc atan2), the weighted mode -- per call on one thread, min of 7
// repetitions.  Build (see tools/README.md):
//   g++ -O3 -std=c++17 -ffp-contract=off -I graph-cut-ransac_amd/csrc -I include \
//       tools/micro/fit_parts.cpp graph-cut-ransac_amd/csrc/host_fit.cpp -o tools/micro/fit_parts.bin
#include "host_fit.h"
#include "qr3.h"
#include "rect.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

using namespace gcr;
using Clock = std::chrono::steady_clock;

int main() {
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    HostClass cls[2];
    const size_t n = 5000;
    for (int c = 0; c < 2; ++c) {
        cls[c].n = n;
        for (size_t i = 0; i < n; ++i) {
            cls[c].x.push_back(1368 * U(rng));
            cls[c].y.push_back(1824 * U(rng));
            const double th = 6.283185307179586 * U(rng);
            cls[c].a.push_back(c == 0 ? 2.0 + U(rng) : th);
            cls[c].c0.push_back(c == 0 ? std::cbrt(cls[c].a.back()) : std::cos(th));
            cls[c].c1.push_back(c == 0 ? 0.0 : std::sin(th));
        }
    }
    const int R = 4000;
    std::vector<std::vector<uint32_t>> idx(2 * R);
    for (auto& v : idx)
        for (int k = 0; k < 14; ++k) v.push_back((uint32_t)(U(rng) * n));
    double best[4] = {1e30, 1e30, 1e30, 1e30}, acc = 0;
    for (int rep = 0; rep < 7; ++rep) {
        RectModel m{};
        auto t0 = Clock::now();
        for (int r = 0; r < R; ++r) {
            fit_nonminimal(2, cls, &idx[2 * r], m, nullptr, 0);
            acc += m.phi;
        }
        auto t1 = Clock::now();
        // QR of a 105-row system alone
        std::vector<double> A0(105 * 4);
        for (auto& v : A0) v = U(rng);
        for (int r = 0; r < R; ++r) {
            double A[4 * 105];
            std::copy(A0.begin(), A0.end(), A);
            HostQRStore st{{A, A + 105, A + 210, A + 315}};
            double x[3];
            qr3_solve(st, 105, x);
            acc += x[0];
        }
        auto t2 = Clock::now();
        for (int r = 0; r < R; ++r)
            for (int i = 0; i < 14; ++i) {
                const uint32_t j = idx[2 * r + 1][i];
                acc += rectified_angle<GlibcMath>(cls[1].x[j], cls[1].y[j], cls[1].c0[j], cls[1].c1[j], 1e-4, 2e-4);
            }
        auto t3 = Clock::now();
        std::vector<double> ang(14), w(14, 1.0 / 14);
        for (int r = 0; r < R; ++r) {
            for (int i = 0; i < 14; ++i) ang[i] = 3.1 * U(rng);
            acc += weighted_mode(ang, w, 0.5 * (3.141592653589793 / 180.0));
        }
        auto t4 = Clock::now();
        auto us = [&](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count() / R; };
        best[0] = std::min(best[0], us(t0, t1));
        best[1] = std::min(best[1], us(t1, t2));
        best[2] = std::min(best[2], us(t2, t3));
        best[3] = std::min(best[3], us(t3, t4) - 0.0);
    }
    printf("fit_nonminimal 2-SIFT 14+14: %.3f us; qr3 105 rows %.3f us; 14 glibc rectified angles %.3f us; "
           "weighted mode (+14 rng) %.3f us  (%g)\n", best[0], best[1], best[2], best[3], acc);
    return 0;
}
