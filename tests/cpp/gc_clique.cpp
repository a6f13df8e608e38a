// graphcut_clique (a cell with at most one source node, decided without BK)
// against the BK max-flow it skips (graphcut_cell_bk), over random cells of
// 3 .. 40 points and deliberate ties: residuals exactly at the truncated
// threshold, zero residuals, equal residuals, q in {0, 1/2, 1}, lambda in
// {1/2, 0.975, 1, tiny, huge} and random, NaN residuals.
#include "../../graph-cut-ransac_amd/csrc/graphcut.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

// optional argument: the number of random cells (default 2 M; the
// sanitizer builds in tests/test_sanitizers.py run fewer)
int main(int argc, char** argv) {
    const long cells = argc > 1 ? atol(argv[1]) : 2000000;
    std::mt19937_64 rng(20261018);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    const double lams[] = {0.5, 0.975, 1.0, 1e-300, 1e300, 0.0, -1.0};
    gcr::CellScratch cs;
    long checked = 0, bad = 0, skipped = 0, one_source = 0;
    for (long it = 0; it < cells; ++it) {
        const uint32_t k = 3 + (uint32_t)(rng() % (it & 1 ? 6 : 38));
        const double sqt = (it & 7) == 0 ? 1.0 : 0.1 + 4.0 * U(rng);
        std::vector<double> r2(k), q(k);
        for (uint32_t a = 0; a < k; ++a) {
            const int c = (int)(rng() % 10);
            r2[a] = c == 0 ? sqt : c == 1 ? 0.0 : c == 2 ? sqt * 0.5 : c == 3 ? 2.0 * sqt
                  : c == 4 && a > 0 ? r2[a - 1] : c == 5 && (it % 97) == 0 ? NAN : U(rng) * 2.0 * sqt;
        }
        double lam = lams[rng() % 7];
        if (lam < 0) lam = U(rng);
        for (uint32_t a = 0; a < k; ++a) q[a] = gcr::gc_q(r2[a], sqt);
        std::vector<uint32_t> nodes(k);
        for (uint32_t a = 0; a < k; ++a) nodes[a] = a;
        std::vector<uint8_t> s1(k, 9), s2(k, 9);
        if (!gcr::graphcut_clique(q.data(), r2.data(), sqt, lam, nodes.data(), k, cs, s1.data())) {
            ++skipped;
            continue;
        }
        gcr::graphcut_cell_bk(q.data(), r2.data(), sqt, lam, nodes.data(), k, cs, s2.data());
        ++checked;
        int pos = 0;
        for (uint32_t a = 0; a < k; ++a) pos += r2[a] > sqt;
        one_source += pos > 0;
        if (s1 != s2) {
            if (++bad <= 10) {
                std::printf("mismatch k %u sqt %.17g lam %.17g:", k, sqt, lam);
                for (uint32_t a = 0; a < k; ++a) std::printf(" %.17g/%d%d", r2[a], s1[a], s2[a]);
                std::printf("\n");
            }
        }
    }
    std::printf("checked %ld (with outliers %ld) skipped %ld mismatches %ld\n", checked, one_source, skipped, bad);
    return bad || checked < 10000 ? 1 : 0;
}
