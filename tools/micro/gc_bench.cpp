// Host graph-cut labeling timing (graphcut.h, serial driver): the per-round
// cost of labeling() on a dumped problem (points, squared residuals), with the
// grid built once as the engine does.  Input: gc_bench <file> with
// n, dims, cell_number (u64), cell sizes (4 f64), sqt, lambda (f64),
// points (n x dims f64, row-major), r2 (n f64).
#include "../../graph-cut-ransac_amd/csrc/graphcut.h"

#include <chrono>
#include <cstdio>
#include <vector>

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 2;
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
    std::printf("n %zu cells(>=2) %zu pairs %zu kmax %zu sink %zu: %.1f us per labeling\n", n, e.cells(), k2, kmax, ns, us);
    return 0;
}
