// The engine's labeling path (graphcut.h gc_schedule + graphcut_labeling_jobs:
// cost-balanced cell jobs writing cell-ordered labels, then the assembly
// ranges; jobs in any order or concurrently)
// against the serial driver (terminal test for every point, then every cell
// in key order), on random 4-D grids with clustered points (cells of 2 to
// ~100 points), ties at the truncated threshold, and several pool sizes; jobs
// run in schedule order, reversed, shuffled, and on 4 threads.
#include "../../graph-cut-ransac_amd/csrc/graphcut.h"

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <random>
#include <thread>

// optional argument: the number of random grids (default 60; the sanitizer
// builds in tests/test_sanitizers.py run fewer)
int main(int argc, char** argv) {
    const int grids = argc > 1 ? atoi(argv[1]) : 60;
    std::mt19937_64 rng(777);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long bad = 0, runs = 0;
    for (int it = 0; it < grids; ++it) {
        const size_t n = 200 + rng() % 6000;
        const int clusters = 1 + (int)(rng() % 40);
        std::vector<double> cols[4];
        for (auto& c : cols) c.resize(n);
        std::vector<double> cx(clusters * 4);
        for (auto& v : cx) v = U(rng) * 1000.0;
        for (size_t i = 0; i < n; ++i) {
            const bool cl = U(rng) < 0.6;
            const int k = (int)(rng() % clusters);
            for (int d = 0; d < 4; ++d) cols[d][i] = cl ? cx[k * 4 + d] + U(rng) * 40.0 : U(rng) * 1000.0;
        }
        const double* cp[4] = {cols[0].data(), cols[1].data(), cols[2].data(), cols[3].data()};
        const double cs[4] = {125.0, 125.0, 125.0, 125.0};
        gcr::NeighbourEdges e;
        gcr::grid_edges(cp, 4, n, cs, 8, e, false);
        const double sqt = 0.5 + U(rng) * 4.0;
        std::vector<double> r2(n);
        for (size_t i = 0; i < n; ++i) {
            const int c = (int)(rng() % 6);
            r2[i] = c == 0 ? sqt : c == 1 ? 0.0 : c == 2 ? sqt * 2.0 : U(rng) * 2.0 * sqt;
        }
        const double lam = (it % 3 == 0) ? 0.975 : (it % 3 == 1 ? 1.0 : U(rng));
        std::vector<double> q;
        std::vector<uint8_t> ref;
        gcr::graphcut_labeling(r2.data(), n, sqt, lam, e, q, ref);
        for (size_t parts : {1, 3, 8, 16, 64}) {
            gcr::gc_schedule(e, parts);
            for (int order = 0; order < 4; ++order) {
                std::vector<uint8_t> cseg(e.nodes.size() + 1, 9);
                std::vector<uint8_t> seg(n, 9);
                auto for_jobs = [&](size_t nj, const auto& fn) {
                    std::vector<size_t> ord(nj);
                    for (size_t j = 0; j < nj; ++j) ord[j] = j;
                    if (order == 1) std::reverse(ord.begin(), ord.end());
                    if (order == 2) std::shuffle(ord.begin(), ord.end(), rng);
                    if (order < 3) {
                        gcr::CellScratch s;
                        for (size_t j : ord) fn(j, s);
                        return;
                    }
                    std::atomic<size_t> next{0};
                    std::vector<std::thread> th;
                    for (int t = 0; t < 4; ++t)
                        th.emplace_back([&] {
                            gcr::CellScratch s;
                            for (size_t j; (j = next.fetch_add(1)) < nj;) fn(j, s);
                        });
                    for (auto& t : th) t.join();
                };
                gcr::graphcut_labeling_jobs(r2.data(), sqt, lam, e, cseg.data(), seg.data(), for_jobs);
                ++runs;
                if (std::memcmp(seg.data(), ref.data(), n) != 0) {
                    if (++bad <= 5) std::printf("mismatch it %d parts %zu order %d\n", it, parts, order);
                }
            }
        }
    }
    std::printf("runs %ld mismatches %ld\n", runs, bad);
    return bad ? 1 : 0;
}
