// host_fit.cpp -- non-minimal fits for LO and the final refit (host C++).
//
// Reference: estimators/rectifying_homography_estimator.h:164-227 (wrapper),
// solver_rectifying_homography_three_sift.hpp:195-254 (+original :233-234),
// solver_rectifying_homography_two_sift.hpp:239-259 (pair rows), :354-394
// (findWeightedMode), :423-579 (non-minimal), :715-848 (normalizePoints, whose
// transform is reset to identity), and Eigen's ColPivHouseholderQR for the
// least-squares solve.  Weights are always empty on the Python path, i.e. 1.0.
#include "host_fit.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <unordered_map>

namespace gcr {

namespace {

inline double sq(double v) { return v * v; }

// Householder reflector applied from the left to one column (rows k..m-1),
// essential part stored in column k of A below the diagonal.
inline void apply_reflector(const double* ess_col, size_t k, size_t m, double tau, double* col) {
    if (m - k == 1) {
        col[k] *= (1.0 - tau);
        return;
    }
    if (tau == 0.0) return;
    double t = 0;
    for (size_t i = k + 1; i < m; ++i) t += ess_col[i] * col[i];
    t += col[k];
    col[k] -= tau * t;
    for (size_t i = k + 1; i < m; ++i) col[i] -= (tau * ess_col[i]) * t;
}

}  // namespace

void colpiv_qr_solve3(std::vector<double>& A, size_t m, std::vector<double>& b, double x[3]) {
    constexpr size_t cols = 3;
    const size_t size = std::min(m, cols);
    double* col[3] = {A.data(), A.data() + m, A.data() + 2 * m};
    double tau_k[3] = {0, 0, 0};
    size_t transp[3] = {0, 1, 2};
    double nu[3], nd[3];
    for (size_t k = 0; k < cols; ++k) {
        double s = 0;
        for (size_t i = 0; i < m; ++i) s += col[k][i] * col[k][i];
        nd[k] = std::sqrt(s);
        nu[k] = nd[k];
    }
    const double eps = std::numeric_limits<double>::epsilon();
    double maxn = nu[0];
    for (size_t k = 1; k < cols; ++k)
        if (maxn < nu[k]) maxn = nu[k];
    const double thr_helper = sq(maxn * eps) / (double)m;
    const double downdate_thr = std::sqrt(eps);
    size_t nonzero = size;
    for (size_t k = 0; k < size; ++k) {
        size_t big = k;
        double bign = nu[k];
        for (size_t j = k + 1; j < cols; ++j)
            if (bign < nu[j]) { bign = nu[j]; big = j; }
        if (nonzero == size && sq(bign) < thr_helper * (double)(m - k)) nonzero = k;
        transp[k] = big;
        if (k != big) {
            std::swap(col[k], col[big]);   // swap column storage
            std::swap(nu[k], nu[big]);
            std::swap(nd[k], nd[big]);
        }
        double* ck = col[k];
        double tail = 0;
        for (size_t i = k + 1; i < m; ++i) tail += ck[i] * ck[i];
        const double c0 = ck[k];
        double tau, beta;
        if (tail <= std::numeric_limits<double>::min()) {
            tau = 0.0;
            beta = c0;
            for (size_t i = k + 1; i < m; ++i) ck[i] = 0.0;
        } else {
            beta = std::sqrt(c0 * c0 + tail);
            if (c0 >= 0.0) beta = -beta;
            const double den = c0 - beta;
            for (size_t i = k + 1; i < m; ++i) ck[i] = ck[i] / den;
            tau = (beta - c0) / beta;
        }
        tau_k[k] = tau;
        ck[k] = beta;
        for (size_t j = k + 1; j < cols; ++j) apply_reflector(ck, k, m, tau, col[j]);
        for (size_t j = k + 1; j < cols; ++j) {
            if (nu[j] != 0.0) {
                double temp = std::fabs(col[j][k]) / nu[j];
                temp = (1.0 + temp) * (1.0 - temp);
                temp = temp < 0.0 ? 0.0 : temp;
                const double temp2 = temp * sq(nu[j] / nd[j]);
                if (temp2 <= downdate_thr) {
                    double s = 0;
                    for (size_t i = k + 1; i < m; ++i) s += col[j][i] * col[j][i];
                    nd[j] = std::sqrt(s);
                    nu[j] = nd[j];
                } else {
                    nu[j] *= std::sqrt(temp);
                }
            }
        }
    }
    size_t perm[3] = {0, 1, 2};
    for (size_t k = 0; k < size; ++k) std::swap(perm[k], perm[transp[k]]);
    if (nonzero == 0) {
        x[0] = x[1] = x[2] = 0.0;
        return;
    }
    for (size_t k = 0; k < nonzero; ++k) apply_reflector(col[k], k, m, tau_k[k], b.data());
    double c[3] = {b[0], m > 1 ? b[1] : 0.0, m > 2 ? b[2] : 0.0};
    for (size_t jj = nonzero; jj-- > 0;) {
        c[jj] = c[jj] / col[jj][jj];
        for (size_t i = 0; i < jj; ++i) c[i] -= c[jj] * col[jj][i];
    }
    for (size_t i = 0; i < nonzero; ++i) x[perm[i]] = c[i];
    for (size_t i = nonzero; i < cols; ++i) x[perm[i]] = 0.0;
}

double weighted_mode(const std::vector<double>& angles, const std::vector<double>& weights, double bin_width) {
    std::unordered_map<int, double> wmap;
    std::unordered_map<int, double> vmap;
    for (size_t i = 0; i < angles.size(); i++) {
        const int bin = static_cast<int>(std::round(angles[i] / bin_width));
        wmap[bin] += weights[i];
        vmap[bin] += angles[i] * weights[i];
    }
    int mode_bin = 0;
    double max_w = -1;
    for (const auto& kv : wmap)
        if (kv.second > max_w) { max_w = kv.second; mode_bin = kv.first; }
    return vmap[mode_bin] / wmap[mode_bin];
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

bool fit_sift22(const HostClass* cls, const std::vector<uint32_t>* idx, RectModel& out) {
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
        return solve_sift22(sx, sy, sp, ox, oy, ocs, osn, out);
    }
    const size_t rows = ns + npairs;
    std::vector<double> A(rows * 3), b(rows);
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
        double l1[3];
        line_from(oc.x[oi[i]], oc.y[oi[i]], oc.c0[oi[i]], oc.c1[oi[i]], l1);
        for (size_t j = i + 1; j < no; ++j, ++r) {
            const double w = 1.0 * 1.0;
            double l2[3], vp[3];
            line_from(oc.x[oi[j]], oc.y[oi[j]], oc.c0[oi[j]], oc.c1[oi[j]], l2);
            cross3(l1, l2, vp);
            const double a0 = std::fabs(vp[0]), a1 = std::fabs(vp[1]), a2 = std::fabs(vp[2]);
            double mx = (a0 < a1) ? a1 : a0;
            mx = (mx < a2) ? a2 : mx;
            if (mx > 1.0)
                for (int q = 0; q < 3; ++q) vp[q] = vp[q] / mx;
            A[r] = w * vp[0];
            A[rows + r] = w * vp[1];
            A[2 * rows + r] = 0.0;
            b[r] = w * vp[2];
        }
    }
    double sol[3];
    colpiv_qr_solve3(A, rows, b, sol);
    if (!finish_model(sol, out)) return false;
    std::vector<double> ang(no), wts(no);
    double wsum = 0;
    for (size_t i = 0; i < no; ++i) {
        const uint32_t j = oi[i];
        ang[i] = rectified_angle(oc.x[j], oc.y[j], oc.c0[j], oc.c1[j], out.h7, out.h8);
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

bool fit_nonminimal(int solver, const HostClass* cls, const std::vector<uint32_t>* idx, RectModel& out) {
    const int K = (solver == 2) ? 2 : 1;
    const size_t m[2] = {solver == 2 ? 2u : 3u, 2u};
    for (int c = 0; c < K; ++c)
        if (idx[c].size() < m[c]) return false;
    if (!normalize_ok(K, cls, idx)) return false;
    bool ok;
    if (solver == 2) ok = fit_sift22(cls, idx, out);
    else ok = fit_scale3(solver == 1, cls[0], idx[0], out);
    if (ok) { out.x0 = 0.0; out.y0 = 0.0; out.s = 1.0; }
    return ok;
}

}  // namespace gcr
