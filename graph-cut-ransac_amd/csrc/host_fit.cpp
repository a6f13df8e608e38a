// host_fit.cpp -- non-minimal fits for LO and the final refit (host C++).
//
// Reference: estimators/rectifying_homography_estimator.h:164-227 (wrapper),
// solver_rectifying_homography_three_sift.hpp:195-254 (+original :233-234),
// solver_rectifying_homography_two_sift.hpp:239-259 (pair rows), :354-394
// (findWeightedMode), :423-579 (non-minimal), :715-848 (normalizePoints, whose
// transform is reset to identity), and Eigen's ColPivHouseholderQR for the
// least-squares solve.  Weights are always empty on the Python path, i.e. 1.0.
// Models are the reference's: the rectified angles of the mode (and the
// minimal 2-SIFT phi) use glibc's atan2 (GlibcMath), as the reference does.
#include "host_fit.h"
#include "qr3.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <memory_resource>
#include <unordered_map>

namespace gcr {

void colpiv_qr_solve3(std::vector<double>& A, size_t m, std::vector<double>& b, double x[3]) {
    HostQRStore st{{A.data(), A.data() + m, A.data() + 2 * m, b.data()}};
    qr3_solve(st, m, x);
}

double weighted_mode(const std::vector<double>& angles, const std::vector<double>& weights, double bin_width) {
    // findWeightedMode (two_sift.hpp:354-394): per-bin weight and weighted
    // angle sums in input order, the mode = the first maximum in
    // std::unordered_map<int, double> iteration order.  That order depends
    // only on the sequence in which NEW keys were inserted (lookups of
    // existing keys do not touch the table), so the sums are accumulated in
    // flat arrays and only each bin's first occurrence goes into the map.
    // small calls (the LO trials' 7 m angles) run out of a stack arena: the
    // same containers and hash table (so the same iteration order), no heap
    alignas(16) unsigned char arena[12288];
    std::pmr::monotonic_buffer_resource mr(arena, sizeof(arena));
    const size_t n = angles.size();
    std::pmr::vector<int> bins(n, &mr);
    int lo = 0, hi = -1;
    for (size_t i = 0; i < n; i++) {
        bins[i] = static_cast<int>(std::round(angles[i] / bin_width));
        if (i == 0 || bins[i] < lo) lo = bins[i];
        if (i == 0 || bins[i] > hi) hi = bins[i];
    }
    const bool dense = n > 0 && (int64_t)hi - (int64_t)lo < (int64_t)(4 * n + 1024);
    if (!dense) {                                        // sparse / pathological bins: the maps themselves
        std::unordered_map<int, double> wmap, vmap;
        for (size_t i = 0; i < n; i++) {
            wmap[bins[i]] += weights[i];
            vmap[bins[i]] += angles[i] * weights[i];
        }
        int mode_bin = 0;
        double max_w = -1;
        for (const auto& kv : wmap)
            if (kv.second > max_w) { max_w = kv.second; mode_bin = kv.first; }
        return vmap[mode_bin] / wmap[mode_bin];
    }
    const size_t span = (size_t)((int64_t)hi - (int64_t)lo + 1);
    std::pmr::vector<double> w(span, 0.0, &mr), v(span, 0.0, &mr);
    std::pmr::vector<char> seen(span, 0, &mr);
    std::pmr::unordered_map<int, double> order(&mr);     // the reference's wmap keys, in its insertion order
    for (size_t i = 0; i < n; i++) {
        const size_t k = (size_t)(bins[i] - lo);
        if (!seen[k]) {
            seen[k] = 1;
            order.emplace(bins[i], 0.0);
        }
        w[k] += weights[i];
        v[k] += angles[i] * weights[i];
    }
    int mode_bin = 0;
    double max_w = -1;
    for (const auto& kv : order) {
        const double wk = w[(size_t)(kv.first - lo)];
        if (wk > max_w) { max_w = wk; mode_bin = kv.first; }
    }
    if (max_w < 0) {                                     // no weight > -1 (NaN weights): vmap[0] / wmap[0]
        if (0 < lo || 0 > hi || !seen[(size_t)(0 - lo)]) return 0.0 / 0.0;
    }
    return v[(size_t)(mode_bin - lo)] / w[(size_t)(mode_bin - lo)];
}

void homography_of(const RectModel& md, double H[9]) {
    const double s = md.s, x0 = md.x0, y0 = md.y0;
    const double N[9] = {s, 0, -s * x0, 0, s, -s * y0, 0, 0, 1};
    const double Hn[9] = {1, 0, 0, 0, 1, 0, md.h7, md.h8, 1};
    auto cof = [&](int i, int j) {
        const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
        return N[i1 * 3 + j1] * N[i2 * 3 + j2] - N[i1 * 3 + j2] * N[i2 * 3 + j1];
    };
    const double det = (cof(0, 0) * N[0] + cof(1, 0) * N[3]) + cof(2, 0) * N[6];
    const double invdet = 1.0 / det;
    double Ni[9], T[9], R[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) Ni[r * 3 + c] = cof(c, r) * invdet;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            T[i * 3 + j] = (Ni[i * 3] * Hn[j] + Ni[i * 3 + 1] * Hn[3 + j]) + Ni[i * 3 + 2] * Hn[6 + j];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            R[i * 3 + j] = (T[i * 3] * N[j] + T[i * 3 + 1] * N[3 + j]) + T[i * 3 + 2] * N[6 + j];
    const double d = R[8];
    for (int i = 0; i < 9; ++i) H[i] = R[i] / d;
}

namespace {

// normalizePoints' failure test (three_sift.hpp:350-433 / two_sift.hpp:715-848);
// the transform itself is reset to identity by the reference.
bool normalize_ok(int K, const HostClass* cls, const std::vector<uint32_t>* idx) {
    size_t tot = 0;
    for (int c = 0; c < K; ++c) tot += idx[c].size();
    if (tot < 1) return false;
    // Shortcut (same answer): the mean distance to ANY centre is at least
    // diameter / (2 n), and the computed mean is within (3 n u) of the real
    // one, so two points more than 4 n 1e-9 apart in x or y make it > 1e-9.
    // The first point against the next few settles every ordinary call; NaN
    // and degenerate sets take the full computation below.
    {
        const double thr = 4.0 * (double)tot * 1e-9;
        const HostClass* c0 = nullptr;
        uint32_t j0 = 0;
        int seen = 0;
        for (int c = 0; c < K && seen < 64; ++c)
            for (uint32_t j : idx[c]) {
                if (++seen > 64) break;
                if (!c0) {
                    c0 = &cls[c];
                    j0 = j;
                    continue;
                }
                if (std::fabs(cls[c].x[j] - c0->x[j0]) > thr || std::fabs(cls[c].y[j] - c0->y[j0]) > thr) return true;
            }
    }
    double x0 = 0.0, y0 = 0.0;
    for (int c = 0; c < K; ++c)
        for (uint32_t j : idx[c]) { x0 += cls[c].x[j]; y0 += cls[c].y[j]; }
    const double inv_n = 1.0 / static_cast<double>(tot);
    x0 *= inv_n;
    y0 *= inv_n;
    double avg = 0.0;
    for (int c = 0; c < K; ++c)
        for (uint32_t j : idx[c]) {
            const double dx = cls[c].x[j] - x0, dy = cls[c].y[j] - y0;
            avg += std::sqrt(dx * dx + dy * dy);
        }
    avg *= inv_n;
    return !(avg < 1e-9);
}

bool finish_model(const double sol[3], RectModel& out) {
    if (std::isnan(sol[0]) || std::isnan(sol[1]) || std::isnan(sol[2])) return false;
    out = default_model();
    out.h7 = sol[0];
    out.h8 = sol[1];
    out.alpha = sol[2];
    return !(out.alpha < kEps9);
}

bool fit_scale3(bool original, const HostClass& c, const std::vector<uint32_t>& idx, RectModel& out) {
    const size_t n = idx.size();
    if (n < 3) return false;
    if (n == 3) {
        double x[3], y[3], p[3];
        for (int i = 0; i < 3; ++i) { x[i] = c.x[idx[i]]; y[i] = c.y[idx[i]]; p[i] = c.c0[idx[i]]; }
        return original ? solve_scale3<true>(x, y, p, out) : solve_scale3<false>(x, y, p, out);
    }
    std::vector<double> A(n * 3), b(n);
    for (size_t i = 0; i < n; ++i) {
        const uint32_t j = idx[i];
        const double w = 1.0;
        A[i] = w * c.x[j];
        A[n + i] = w * c.y[j];
        if (original) { A[2 * n + i] = -w * c.c0[j]; b[i] = -w; }
        else { A[2 * n + i] = w * c.c0[j]; b[i] = w; }
    }
    double sol[3];
    colpiv_qr_solve3(A, n, b, sol);
    return finish_model(sol, out);
}

// Rows of the hybrid system (assembly two_sift.hpp:474-509): scale rows
// (setScaleConstraint :228-236: w x, w y, w s^(1/3) | w), then one row per orientation
// pair i < j in index order.  Column-major A (rows x 3) and b.
void sift_rows_host(const HostClass& sc, const HostClass& oc, const std::vector<uint32_t>& si,
                    const std::vector<uint32_t>& oi, size_t rows, double* A, double* b) {
    const size_t ns = si.size(), no = oi.size();
    size_t r = 0;
    for (size_t i = 0; i < ns; ++i, ++r) {
        const uint32_t j = si[i];
        const double w = 1.0;
        A[r] = w * sc.x[j];
        A[rows + r] = w * sc.y[j];
        A[2 * rows + r] = w * sc.c0[j];
        b[r] = w;
    }
    for (size_t i = 0; i + 1 < no; ++i) {
        const uint32_t p = oi[i];
        for (size_t j = i + 1; j < no; ++j, ++r) {
            const uint32_t q = oi[j];
            double row[4];
            sift_pair_row(oc.x[p], oc.y[p], oc.c0[p], oc.c1[p], oc.x[q], oc.y[q], oc.c0[q], oc.c1[q], row);
            A[r] = row[0];
            A[rows + r] = row[1];
            A[2 * rows + r] = row[2];
            b[r] = row[3];
        }
    }
}

}  // namespace

bool gram_refit_on() {
    const char* e = getenv("GCR_REFIT");              // read per fit (tests switch it)
    return !(e && e[0] == 'q');
}

void gram_sift_host(const HostClass& sc, const HostClass& oc, const std::vector<uint32_t>& si,
                    const std::vector<uint32_t>& oi, size_t rows, DD g[kGramN]) {
    const size_t ns = si.size(), no = oi.size();
    std::vector<DD> lane((size_t)kGramLanes * kGramN), tiles;
    for (size_t base = 0; base < rows; base += kGramTile) {
        for (auto& v : lane) v = DD{0.0, 0.0};
        for (int l = 0; l < kGramLanes; ++l) {
            DD* acc = &lane[(size_t)l * kGramN];
            for (size_t u = 0; u < kGramTile / kGramLanes; ++u) {
                const size_t r = base + (size_t)l + (size_t)kGramLanes * u;
                if (r >= rows) break;
                double row[4];
                if (r < ns) {
                    const uint32_t j = si[r];
                    const double w = 1.0;
                    row[0] = w * sc.x[j];
                    row[1] = w * sc.y[j];
                    row[2] = w * sc.c0[j];
                    row[3] = w;
                } else {
                    uint64_t i, j;
                    pair_of(r - ns, no, i, j);
                    const uint32_t a = oi[i], c = oi[j];
                    sift_pair_row(oc.x[a], oc.y[a], oc.c0[a], oc.c1[a], oc.x[c], oc.y[c], oc.c0[c], oc.c1[c], row);
                }
                gram_add_row(acc, row);
            }
        }
        gram_lane_tree(lane.data());
        tiles.insert(tiles.end(), lane.begin(), lane.begin() + kGramN);
    }
    gram_combine_tiles(tiles.data(), tiles.size() / kGramN, g);
}

void gram_solve3(const DD g[kGramN], size_t rows, double x[3]) {
    // S: the Gram matrix of [A | b], updated to its Schur complements
    DD S[4][4];
    for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) S[a][b] = g[gram_index(a, b)];
    int ord[3] = {0, 1, 2};                  // pivot order: stored column of step k
    const double eps = std::numeric_limits<double>::epsilon();
    double maxn = 0.0;
    for (int k = 0; k < 3; ++k) {
        const double nk = dd_sqrt(S[k][k]).hi;
        if (k == 0 || maxn < nk) maxn = nk;
    }
    const double thr_helper = ((maxn * eps) * (maxn * eps)) / (double)rows;
    int nonzero = 3;
    DD R[3][4];                              // R[k][c]: row k of R at stored column c (c = 3: Q^T b)
    for (int k = 0; k < 3; ++k) {
        // the largest remaining squared column norm, first on ties
        int big = k;
        for (int j = k + 1; j < 3; ++j)
            if (dd_lt(S[ord[big]][ord[big]], S[ord[j]][ord[j]])) big = j;
        const double big_sq = S[ord[big]][ord[big]].hi;
        if (nonzero == 3 && big_sq < thr_helper * (double)(rows - (size_t)k)) nonzero = k;
        std::swap(ord[k], ord[big]);
        const int p = ord[k];
        const DD rkk = dd_sqrt(S[p][p]);
        R[k][p] = rkk;
        int rest[3], nr = 0;                 // the remaining stored columns and b
        for (int j = k + 1; j < 3; ++j) rest[nr++] = ord[j];
        rest[nr++] = 3;
        for (int q = 0; q < nr; ++q) R[k][rest[q]] = rkk.hi > 0.0 ? dd_div(S[p][rest[q]], rkk) : DD{0.0, 0.0};
        // Schur complement of the remaining columns and b
        for (int a = 0; a < nr; ++a)
            for (int b = a; b < nr; ++b) {
                const int ca = rest[a], cb = rest[b];
                S[ca][cb] = dd_sub(S[ca][cb], dd_mul(R[k][ca], R[k][cb]));
                S[cb][ca] = S[ca][cb];
            }
    }
    DD c[3] = {R[0][3], R[1][3], R[2][3]};
    for (int jj = nonzero - 1; jj >= 0; --jj) {
        c[jj] = dd_div(c[jj], R[jj][ord[jj]]);
        for (int i = 0; i < jj; ++i) c[i] = dd_sub(c[i], dd_mul(c[jj], R[i][ord[jj]]));
    }
    for (int k = 0; k < 3; ++k) x[ord[k]] = k < nonzero ? c[k].hi : 0.0;
}

namespace {

bool fit_sift22(const HostClass* cls, const std::vector<uint32_t>* idx, RectModel& out, SiftSystemSolver* big,
                size_t big_rows) {
    const HostClass& sc = cls[0];
    const HostClass& oc = cls[1];
    const std::vector<uint32_t>& si = idx[0];
    const std::vector<uint32_t>& oi = idx[1];
    const size_t ns = si.size(), no = oi.size();
    const size_t npairs = no == 0 ? 0 : (no * (no - 1)) / 2;
    if (ns < 2 || npairs < 1) return false;
    if (ns == 2 && npairs == 1) {
        const double sx[2] = {sc.x[si[0]], sc.x[si[1]]}, sy[2] = {sc.y[si[0]], sc.y[si[1]]};
        const double sp[2] = {sc.c0[si[0]], sc.c0[si[1]]};
        const double ox[2] = {oc.x[oi[0]], oc.x[oi[1]]}, oy[2] = {oc.y[oi[0]], oc.y[oi[1]]};
        const double ocs[2] = {oc.c0[oi[0]], oc.c0[oi[1]]}, osn[2] = {oc.c1[oi[0]], oc.c1[oi[1]]};
        return solve_sift22<GlibcMath>(sx, sy, sp, ox, oy, ocs, osn, out);
    }
    const size_t rows = ns + npairs;
    double sol[3];
    if (rows >= kGramRows && gram_refit_on()) {
        DD g[kGramN];
        if (!(big && big->gram(si, oi, rows, g))) gram_sift_host(sc, oc, si, oi, rows, g);
        gram_solve3(g, rows, sol);
    } else if (big && rows >= big_rows) {
        big->solve(si, oi, rows, sol);
    } else if (rows <= 256) {
        // LO trials (<= 14 + C(14, 2) rows): the system on the stack
        double A[4 * 256];
        sift_rows_host(sc, oc, si, oi, rows, A, A + 3 * rows);
        HostQRStore st{{A, A + rows, A + 2 * rows, A + 3 * rows}};
        qr3_solve(st, rows, sol);
    } else {
        std::vector<double> A(rows * 3), b(rows);
        sift_rows_host(sc, oc, si, oi, rows, A.data(), b.data());
        colpiv_qr_solve3(A, rows, b, sol);
    }
    if (!finish_model(sol, out)) return false;
    // the calling thread's scratch, bound to references: the angle lambda
    // below runs on the host pool's threads too, and a thread_local named
    // inside it would be each worker's own instance
    thread_local std::vector<double> tl_ang, tl_wts;
    std::vector<double>& ang = tl_ang;
    std::vector<double>& wts = tl_wts;
    ang.resize(no);
    wts.resize(no);
    double wsum = 0;
    // the rectified angles are independent (a big refit spreads them over
    // the solver's threads); the weights and the mode stay in order
    auto angles = [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i) {
            const uint32_t j = oi[i];
            ang[i] = rectified_angle<GlibcMath>(oc.x[j], oc.y[j], oc.c0[j], oc.c1[j], out.h7, out.h8);
        }
    };
    if (big && rows >= big_rows) big->for_ranges(no, angles);
    else angles(0, no);
    for (size_t i = 0; i < no; ++i) {
        wts[i] = 1.0;
        wsum += 1.0;
    }
    if (wsum < kEps9) return false;
    for (size_t i = 0; i < no; ++i) {
        if (ang[i] > kPi) ang[i] -= kPi;
        wts[i] /= wsum;
    }
    out.phi = weighted_mode(ang, wts, 0.5 * (kPi / 180.0));
    return true;
}

}  // namespace

bool fit_nonminimal(int solver, const HostClass* cls, const std::vector<uint32_t>* idx, RectModel& out,
                    SiftSystemSolver* big, size_t big_rows) {
    const int K = (solver == 2) ? 2 : 1;
    const size_t m[2] = {solver == 2 ? 2u : 3u, 2u};
    for (int c = 0; c < K; ++c)
        if (idx[c].size() < m[c]) return false;
    if (!normalize_ok(K, cls, idx)) return false;
    bool ok;
    if (solver == 2) ok = fit_sift22(cls, idx, out, big, big_rows);
    else ok = fit_scale3(solver == 1, cls[0], idx[0], out);
    if (ok) { out.x0 = 0.0; out.y0 = 0.0; out.s = 1.0; }
    return ok;
}

bool fit_h4_nonminimal(const HostClass& c, const std::vector<uint32_t>& idx, GeoModel& out) {
    const size_t n = idx.size();
    if (n < 4) return false;
    if (n == 4) {
        double x1[4], y1[4], x2[4], y2[4];
        for (int i = 0; i < 4; ++i) {
            x1[i] = c.x[idx[i]]; y1[i] = c.y[idx[i]]; x2[i] = c.a[idx[i]]; y2[i] = c.c0[idx[i]];
        }
        return solve_h4(x1, y1, x2, y2, out);
    }
    // Hartley normalisation of both point sets (blocked-order sums)
    const double inv_n = 1.0 / static_cast<double>(n);
    const double mx1 = blocked_sum(0, n, [&](size_t i) { return c.x[idx[i]]; }) * inv_n;
    const double my1 = blocked_sum(0, n, [&](size_t i) { return c.y[idx[i]]; }) * inv_n;
    const double mx2 = blocked_sum(0, n, [&](size_t i) { return c.a[idx[i]]; }) * inv_n;
    const double my2 = blocked_sum(0, n, [&](size_t i) { return c.c0[idx[i]]; }) * inv_n;
    const double d1 = blocked_sum(0, n, [&](size_t i) {
        const double dx = c.x[idx[i]] - mx1, dy = c.y[idx[i]] - my1;
        return std::sqrt(dx * dx + dy * dy);
    }) * inv_n;
    const double d2 = blocked_sum(0, n, [&](size_t i) {
        const double dx = c.a[idx[i]] - mx2, dy = c.c0[idx[i]] - my2;
        return std::sqrt(dx * dx + dy * dy);
    }) * inv_n;
    if (!(d1 > 1e-12) || !(d2 > 1e-12)) return false;
    const double s1 = std::sqrt(2.0) / d1, s2 = std::sqrt(2.0) / d2;
    // 2n x 8 system (column-major) and right-hand side
    const size_t m = 2 * n;
    std::vector<double> A(9 * m);
    double* col[9];
    for (int k = 0; k < 9; ++k) col[k] = A.data() + k * m;
    for (size_t i = 0; i < n; ++i) {
        const double u1 = (c.x[idx[i]] - mx1) * s1, v1 = (c.y[idx[i]] - my1) * s1;
        const double u2 = (c.a[idx[i]] - mx2) * s2, v2 = (c.c0[idx[i]] - my2) * s2;
        const size_t r0 = 2 * i, r1 = 2 * i + 1;
        col[0][r0] = u1; col[1][r0] = v1; col[2][r0] = 1.0; col[3][r0] = 0.0; col[4][r0] = 0.0; col[5][r0] = 0.0;
        col[6][r0] = -u2 * u1; col[7][r0] = -u2 * v1; col[8][r0] = u2;
        col[0][r1] = 0.0; col[1][r1] = 0.0; col[2][r1] = 0.0; col[3][r1] = u1; col[4][r1] = v1; col[5][r1] = 1.0;
        col[6][r1] = -v2 * u1; col[7][r1] = -v2 * v1; col[8][r1] = v2;
    }
    HostQRStoreN<8> st;
    for (int k = 0; k < 9; ++k) st.col[k] = col[k];
    double hn[8];
    qr_solve<8>(st, m, hn);
    const double Hn[9] = {hn[0], hn[1], hn[2], hn[3], hn[4], hn[5], hn[6], hn[7], 1.0};
    // H = T2^-1 * Hn * T1, T1 = [s1 0 -s1 mx1; 0 s1 -s1 my1; 0 0 1],
    // T2^-1 = [1/s2 0 mx2; 0 1/s2 my2; 0 0 1]
    const double T1[9] = {s1, 0.0, -s1 * mx1, 0.0, s1, -s1 * my1, 0.0, 0.0, 1.0};
    const double T2i[9] = {1.0 / s2, 0.0, mx2, 0.0, 1.0 / s2, my2, 0.0, 0.0, 1.0};
    double M[9], H[9];
    for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 3; ++q)
            M[r * 3 + q] = (Hn[r * 3] * T1[q] + Hn[r * 3 + 1] * T1[3 + q]) + Hn[r * 3 + 2] * T1[6 + q];
    for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 3; ++q)
            H[r * 3 + q] = (T2i[r * 3] * M[q] + T2i[r * 3 + 1] * M[3 + q]) + T2i[r * 3 + 2] * M[6 + q];
    if (!(std::fabs(H[8]) > 1e-300)) return false;
    for (int k = 0; k < 9; ++k) {
        out.h[k] = H[k] / H[8];
        if (std::isnan(out.h[k])) return false;
    }
    return true;
}

// Cyclic Jacobi, rotations in (p, q) row order until the off-diagonal sum
// is exactly zero.  Stored as padded rows so that the two rotated rows are
// updated four entries per instruction: for k outside {p, q} the row update
// cs * a[p][k] - sn * a[q][k] is bit for bit the column update of a[k][p]
// (the matrix stays exactly symmetric), so the columns are mirrored from the
// rows, and the 2 x 2 block is computed in the column-then-row order of the
// plain loop.  The eigenvectors are kept transposed (rows contiguous).
// Identical to the scalar loop bit for bit (the oracle's), 1.36x faster
// (MEASUREMENTS.md).
template <int N>
void jacobi_eigen(double (&a)[N][N], double (&v)[N][N], double (&d)[N]) {
    constexpr int L = (N + 3) & ~3;
    typedef double v4d __attribute__((vector_size(32)));
    alignas(32) double A[N][L] = {}, VT[N][L] = {};
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j) {
            A[i][j] = a[i][j];
            VT[i][j] = i == j ? 1.0 : 0.0;
        }
    auto rotate = [](double* rp, double* rq, double cs, double sn) {
        const v4d cv = {cs, cs, cs, cs}, sv = {sn, sn, sn, sn};
        for (int k = 0; k < L; k += 4) {
            v4d x, y;
            __builtin_memcpy(&x, rp + k, sizeof x);
            __builtin_memcpy(&y, rq + k, sizeof y);
            const v4d nx = cv * x - sv * y, ny = sv * x + cv * y;
            __builtin_memcpy(rp + k, &nx, sizeof nx);
            __builtin_memcpy(rq + k, &ny, sizeof ny);
        }
    };
    for (int sweep = 0; sweep < 64; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < N; ++p)
            for (int q = p + 1; q < N; ++q) off += A[p][q] * A[p][q];
        if (!(off > 0.0)) break;
        for (int p = 0; p < N; ++p)
            for (int q = p + 1; q < N; ++q) {
                const double apq = A[p][q];
                if (apq == 0.0) continue;
                const double app = A[p][p], aqq = A[q][q], aqp = A[q][p];
                const double theta = (aqq - app) / (2.0 * apq);
                double t = 1.0 / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
                if (theta < 0.0) t = -t;
                const double cs = 1.0 / std::sqrt(t * t + 1.0), sn = t * cs;
                // the block: columns p, q first (k = p, q), then rows p, q
                const double cpp = cs * app - sn * apq, cpq = sn * app + cs * apq;
                const double cqp = cs * aqp - sn * aqq, cqq = sn * aqp + cs * aqq;
                const double npp = cs * cpp - sn * cqp, nqq = sn * cpq + cs * cqq;
                rotate(A[p], A[q], cs, sn);
                for (int k = 0; k < N; ++k) {
                    A[k][p] = A[p][k];
                    A[k][q] = A[q][k];
                }
                A[p][p] = npp;
                A[q][q] = nqq;
                A[p][q] = 0.0;
                A[q][p] = 0.0;
                rotate(VT[p], VT[q], cs, sn);
            }
    }
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j) {
            a[i][j] = A[i][j];
            v[i][j] = VT[j][i];
        }
    for (int k = 0; k < N; ++k) d[k] = A[k][k];
}

template void jacobi_eigen<3>(double (&)[3][3], double (&)[3][3], double (&)[3]);
template void jacobi_eigen<9>(double (&)[9][9], double (&)[9][9], double (&)[9]);

namespace {
// column of v with the smallest eigenvalue (first on ties)
template <int N>
int argmin_eig(const double (&d)[N]) {
    int k = 0;
    for (int i = 1; i < N; ++i)
        if (d[i] < d[k]) k = i;
    return k;
}
}  // namespace

bool fit_f8_nonminimal(const HostClass& c, const std::vector<uint32_t>& idx, GeoModel& out) {
    const size_t n = idx.size();
    if (n < 7) return false;
    if (n == 7) {
        double x1[7], y1[7], x2[7], y2[7];
        for (int i = 0; i < 7; ++i) {
            x1[i] = c.x[idx[i]]; y1[i] = c.y[idx[i]]; x2[i] = c.a[idx[i]]; y2[i] = c.c0[idx[i]];
        }
        GeoModel ms[kFModels];
        if (solve_f7(x1, y1, x2, y2, ms) == 0) return false;
        out = ms[0];
        return true;
    }
    const double inv_n = 1.0 / static_cast<double>(n);
    const double mx1 = blocked_sum(0, n, [&](size_t i) { return c.x[idx[i]]; }) * inv_n;
    const double my1 = blocked_sum(0, n, [&](size_t i) { return c.y[idx[i]]; }) * inv_n;
    const double mx2 = blocked_sum(0, n, [&](size_t i) { return c.a[idx[i]]; }) * inv_n;
    const double my2 = blocked_sum(0, n, [&](size_t i) { return c.c0[idx[i]]; }) * inv_n;
    const double d1 = blocked_sum(0, n, [&](size_t i) {
        const double dx = c.x[idx[i]] - mx1, dy = c.y[idx[i]] - my1;
        return std::sqrt(dx * dx + dy * dy);
    }) * inv_n;
    const double d2 = blocked_sum(0, n, [&](size_t i) {
        const double dx = c.a[idx[i]] - mx2, dy = c.c0[idx[i]] - my2;
        return std::sqrt(dx * dx + dy * dy);
    }) * inv_n;
    if (!(d1 > 1e-12) || !(d2 > 1e-12)) return false;
    const double s1 = std::sqrt(2.0) / d1, s2 = std::sqrt(2.0) / d2;
    // A^T A, upper triangle, accumulated in blocked order.  Each block's rows
    // r = (u2 u1, u2 v1, u2, v2 u1, v2 v1, v2, u1, v1, 1) go to a scratch
    // block first; two passes over it then add r[p] * r[0..7] four entries
    // per instruction (rows 0..3 of the triangle, then rows 4..7; column 8 is
    // r[p] * 1 = r[p], entry (8, 8) the row count).  Every entry is still its
    // own row-ordered sum of r[p] * r[q] (the lower 4 x 4 halves computed on
    // the way are dropped), so the result is the scalar loop's bit for bit,
    // 1.5x faster with the box's compiler (MEASUREMENTS.md).
    typedef double v4d __attribute__((vector_size(32)));
    alignas(64) static thread_local double rows[kSumBlock][8];
    auto ld4 = [](const double* p) {
        v4d v;
        __builtin_memcpy(&v, p, sizeof v);
        return v;
    };
    double ata[9][9] = {};
    size_t i = 0;
    while (i < n) {
        const size_t m = std::min(n, (i / kSumBlock + 1) * kSumBlock) - i;
        for (size_t t = 0; t < m; ++t, ++i) {
            const double u1 = (c.x[idx[i]] - mx1) * s1, v1 = (c.y[idx[i]] - my1) * s1;
            const double u2 = (c.a[idx[i]] - mx2) * s2, v2 = (c.c0[idx[i]] - my2) * s2;
            double* r = rows[t];
            r[0] = u2 * u1; r[1] = u2 * v1; r[2] = u2; r[3] = v2 * u1;
            r[4] = v2 * v1; r[5] = v2; r[6] = u1; r[7] = v1;
        }
        v4d lo[8] = {}, c8lo = {};
        for (size_t t = 0; t < m; ++t) {
            const v4d R0 = ld4(rows[t]), R1 = ld4(rows[t] + 4);
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const v4d b = {rows[t][p], rows[t][p], rows[t][p], rows[t][p]};
                lo[2 * p] += b * R0;
                lo[2 * p + 1] += b * R1;
            }
            c8lo += R0;
        }
        v4d hi[4] = {}, c8hi = {};
        double c88 = 0.0;
        for (size_t t = 0; t < m; ++t) {
            const v4d R1 = ld4(rows[t] + 4);
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const v4d b = {rows[t][4 + p], rows[t][4 + p], rows[t][4 + p], rows[t][4 + p]};
                hi[p] += b * R1;
            }
            c8hi += R1;
            c88 += 1.0;
        }
        for (int p = 0; p < 4; ++p) {
            for (int q = p; q < 8; ++q) ata[p][q] += q < 4 ? lo[2 * p][q] : lo[2 * p + 1][q - 4];
            for (int q = 4 + p; q < 8; ++q) ata[4 + p][q] += hi[p][q - 4];
            ata[p][8] += c8lo[p];
            ata[4 + p][8] += c8hi[p];
        }
        ata[8][8] += c88;
    }
    for (int p = 0; p < 9; ++p)
        for (int q = 0; q < p; ++q) ata[p][q] = ata[q][p];
    double V[9][9], D[9];
    jacobi_eigen<9>(ata, V, D);
    const int k9 = argmin_eig<9>(D);
    double fn[9];
    for (int k = 0; k < 9; ++k) fn[k] = V[k][k9];
    // rank 2: Fn (I - v v^T), v the right singular vector of the smallest
    // singular value (smallest eigenvector of Fn^T Fn)
    double ftf[3][3];
    for (int p = 0; p < 3; ++p)
        for (int q = 0; q < 3; ++q) ftf[p][q] = (fn[p] * fn[q] + fn[3 + p] * fn[3 + q]) + fn[6 + p] * fn[6 + q];
    double V3[3][3], D3[3];
    jacobi_eigen<3>(ftf, V3, D3);
    const int k3 = argmin_eig<3>(D3);
    const double v[3] = {V3[0][k3], V3[1][k3], V3[2][k3]};
    double f2[9];
    for (int r = 0; r < 3; ++r) {
        const double fv = (fn[3 * r] * v[0] + fn[3 * r + 1] * v[1]) + fn[3 * r + 2] * v[2];
        for (int q = 0; q < 3; ++q) f2[3 * r + q] = fn[3 * r + q] - fv * v[q];
    }
    return denormalize_f(f2, s1, mx1, my1, s2, mx2, my2, out.h);
}

}  // namespace gcr
