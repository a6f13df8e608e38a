// Host graph-cut labeling timing (graphcut.h): the per-round cost of one
// labeling on a dumped problem (points, squared residuals), with the grid
// built once as the engine does -- the serial driver, and the engine's
// cost-balanced jobs (gc_schedule) drawn dynamically by T persistent spinning
// threads (the host pool's pattern).  Input: gc_bench <file> [threads] with
// n, dims, cell_number (u64), cell sizes (4 f64), sqt, lambda (f64),
// points (n x dims f64, row-major), r2 (n f64).
#include "../../graph-cut-ransac_amd/csrc/graphcut.h"

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    const int T = argc > 2 ? std::atoi(argv[2]) : 8;
    uint64_t hdr[3];
    double cs[4], sl[2];
    if (std::fread(hdr, 8, 3, f) != 3 || std::fread(cs, 8, 4, f) != 4 || std::fread(sl, 8, 2, f) != 2) return 2;
    const size_t n = hdr[0], dims = hdr[1];
    std::vector<double> pts(n * dims), r2(n);
    if (std::fread(pts.data(), 8, n * dims, f) != n * dims || std::fread(r2.data(), 8, n, f) != n) return 2;
    std::fclose(f);
    std::vector<std::vector<double>> cols(dims, std::vector<double>(n));
    for (size_t i = 0; i < n; ++i)
        for (size_t d = 0; d < dims; ++d) cols[d][i] = pts[i * dims + d];
    std::vector<const double*> cp(dims);
    for (size_t d = 0; d < dims; ++d) cp[d] = cols[d].data();
    gcr::NeighbourEdges e;
    gcr::grid_edges(cp.data(), (int)dims, n, cs, hdr[2], e, false);
    gcr::gc_schedule(e, (size_t)T);
    size_t k2 = 0, kmax = 0;
    for (size_t c = 0; c + 1 < e.off.size(); ++c) {
        const size_t k = e.off[c + 1] - e.off[c];
        k2 += k * (k - 1) / 2;
        kmax = k > kmax ? k : kmax;
    }
    std::vector<double> q;
    std::vector<uint8_t> seg;
    const int reps = 200;
    gcr::graphcut_labeling(r2.data(), n, sl[0], sl[1], e, q, seg);
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; ++r) gcr::graphcut_labeling(r2.data(), n, sl[0], sl[1], e, q, seg);
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
    size_t ns = 0;
    for (auto v : seg) ns += v;
    std::printf("n %zu cells(>=2) %zu pairs %zu kmax %zu sink %zu: %.1f us per labeling (serial)\n", n, e.cells(), k2,
                kmax, ns, us);

    // the jobs on T spinning threads
    std::vector<uint8_t> q2(e.nodes.size() + 1);
    std::vector<uint8_t> seg2(n);
    std::atomic<size_t> next{0}, done{0};
    std::atomic<int> gen{0};
    std::atomic<bool> stop{false};
    const std::function<void(size_t, gcr::CellScratch&)>* job = nullptr;
    size_t njobs = 0;
    auto work = [&](gcr::CellScratch& s) {
        for (size_t j; (j = next.fetch_add(1)) < njobs;) (*job)(j, s);
    };
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t)
        th.emplace_back([&] {
            gcr::CellScratch s;
            int seen = 0;
            while (!stop.load()) {
                if (gen.load(std::memory_order_acquire) == seen) continue;
                seen = gen.load();
                work(s);
                done.fetch_add(1);
            }
        });
    gcr::CellScratch s0;
    auto for_jobs = [&](size_t nj, const auto& fn) {
        std::function<void(size_t, gcr::CellScratch&)> w = fn;
        job = &w;
        njobs = nj;
        next.store(0);
        done.store(0);
        gen.fetch_add(1, std::memory_order_release);
        work(s0);
        while (done.load() != (size_t)(T - 1)) {
        }
    };
    gcr::graphcut_labeling_jobs(r2.data(), sl[0], sl[1], e, q2.data(), seg2.data(), for_jobs);
    t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; ++r) gcr::graphcut_labeling_jobs(r2.data(), sl[0], sl[1], e, q2.data(), seg2.data(), for_jobs);
    const double us2 = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
    stop.store(true);
    gen.fetch_add(1);
    for (auto& t : th) t.join();
    std::printf("%zu jobs on %d threads: %.1f us per labeling, seg %s\n", e.jobs.size(), T, us2,
                std::memcmp(seg.data(), seg2.data(), n) == 0 ? "identical" : "DIFFERS");
    return std::memcmp(seg.data(), seg2.data(), n) == 0 ? 0 : 1;
}
