// graphcut_pair (the two-point cell in closed form) against the BK max-flow
// it replaces (graphcut_cell_bk), over random cells and deliberate ties:
// residuals exactly at the truncated threshold (tr == 0), equal points,
// q in {0, 1/2, 1}, lambda in {0, 1/2, 0.975, 1} and random.
#include "../../graph-cut-ransac_amd/csrc/graphcut.h"

#include <cmath>
#include <cstdio>
#include <random>

int main() {
    std::mt19937_64 rng(12345);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    const double lams[] = {0.0, 0.5, 0.975, 1.0, -1.0};
    gcr::CellScratch cs;
    long checked = 0, bad = 0, skipped = 0;
    for (long it = 0; it < 2000000; ++it) {
        const double sqt = (it & 7) == 0 ? 1.0 : 0.1 + 4.0 * U(rng);
        double r2[2];
        for (int a = 0; a < 2; ++a) {
            const int c = (int)(rng() % 8);
            r2[a] = c == 0 ? sqt : c == 1 ? 0.0 : c == 2 ? sqt * 0.5 : c == 3 ? 2.0 * sqt
                  : c == 4 && a == 1 ? r2[0] : U(rng) * 2.0 * sqt;
        }
        double lam = lams[rng() % 5];
        if (lam < 0) lam = U(rng);
        double q[2];
        for (int a = 0; a < 2; ++a) q[a] = std::clamp(r2[a] / sqt, 0.0, 1.0);
        const uint32_t nodes[2] = {0, 1};
        uint8_t s1[2] = {9, 9}, s2[2] = {9, 9};
        if (!gcr::graphcut_pair(q, r2, sqt, lam, nodes, s1)) {
            ++skipped;
            continue;
        }
        gcr::graphcut_cell_bk(q, r2, sqt, lam, nodes, 2, cs, s2);
        ++checked;
        if (s1[0] != s2[0] || s1[1] != s2[1]) {
            if (++bad <= 10)
                std::printf("mismatch r2 %.17g %.17g sqt %.17g lam %.17g: pair %d%d bk %d%d\n", r2[0], r2[1], sqt, lam,
                            s1[0], s1[1], s2[0], s2[1]);
        }
    }
    std::printf("checked %ld skipped %ld mismatches %ld\n", checked, skipped, bad);
    return bad ? 1 : 0;
}
