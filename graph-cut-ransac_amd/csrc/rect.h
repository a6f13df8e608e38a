// rect.h -- rectifying-homography model, residuals and minimal solvers, written
// once for the gfx950 kernels and the host engine (GCR_HD).
//
// Each function restates one reference routine with the SAME IEEE operation
// order (compiled with -ffp-contract=off), so a residual, a sample-validity
// decision or a minimal solution computed on the GPU is bit-identical to the
// host's.  Per-feature transcendental constants (pow(s, +-1/3), cos(theta),
// sin(theta)) are evaluated once on the host with glibc exactly as the
// reference does and uploaded; hypothesis-dependent ones use detmath.h.
//
// Reference map (src/pygcransac/include/...):
//   RectModel                 model.h:42-246
//   scale_sq_residual         estimators/solver_rectifying_homography_three_sift.hpp:293-317,
//                             ..._three_sift_original.hpp:316, ..._two_sift.hpp:621-645
//   orient_sq_residual        ..._two_sift.hpp:647-665, model.h:156-165, math_utils.hpp:78-102
//   scale_sq_value,           the same residuals in the product's value form
//   orient_sq_value           (what the kernels evaluate, see "values")
//   are_collinear             math_utils.hpp:138-155
//   gauss3                    math_utils.hpp:164-221
//   convex hull / inside      math_utils.hpp:223-321
//   solve_scale3              ..._three_sift.hpp:145-193 (+ original :172-173)
//   valid_sample_sift22       ..._two_sift.hpp:141-215
//   solve_sift22              ..._two_sift.hpp:261-344
//   valid_model_sift22        ..._two_sift.hpp:45-61
#pragma once

#include "gcr_hd.h"
#include "detmath.h"

namespace gcr {

constexpr double kPi = dm::cf(0x400921fb54442d18ull);      // M_PI
constexpr double kPi2 = dm::cf(0x3ff921fb54442d18ull);     // M_PI_2
constexpr double kTwoPi = 2.0 * dm::cf(0x400921fb54442d18ull);
constexpr double kEps9 = 1e-9;                              // solvers' kEpsilon

// The three hypothesis-dependent libm calls of the residuals and of the
// 2-SIFT minimal solver, as a policy: TwinMath (detmath.h, host and device,
// what every kernel evaluates) or, on the host only, GlibcMath -- the
// reference's own std::log / std::pow(t, -3.0) / std::atan2, with which the
// engine takes every decision and model (exact.h).  Same operations around
// them either way.
struct TwinMath {
    static GCR_HD double log(double x) { return dm::dm_log(x); }
    static GCR_HD double pm3(double t) { return dm::dm_pow_m3(t); }
    static GCR_HD double atan2(double y, double x) { return dm::dm_atan2(y, x); }
};
struct GlibcMath {                       // host only (the engine's recheck, host fits)
    static double log(double x) { return ::log(x); }
    static double pm3(double t) { return ::pow(t, -3.0); }
    static double atan2(double y, double x) { return ::atan2(y, x); }
};

// model.h: NormalizingTransform{x0,y0,s} + RectifyingHomography{h7,h8} +
// ScaleBased{alpha} + OrientationBased{phi}.  56 bytes, POD on both sides.
struct RectModel {
    double x0, y0, s, h7, h8, alpha, phi;
};

GCR_HD RectModel default_model() { return RectModel{0.0, 0.0, 1.0, 0.0, 0.0, 1.0, 0.0}; }

GCR_HD bool identity_norm(const RectModel& m) { return m.x0 == 0.0 && m.y0 == 0.0 && m.s == 1.0; }

// ---------------------------------------------------------------- scale ----
// Per-hypothesis constant: cube(alpha) = alpha*alpha*alpha (math_utils.hpp:52).
GCR_HD double alpha_cube(const RectModel& m) { return m.alpha * m.alpha * m.alpha; }

// r^2 of one scale feature (x, y, s); DBL_MAX*DBL_MAX (= +inf) for rectified
// scales below 1e-9 as in the reference.  kOriginal selects log(rs/alpha^3).
template <bool kOriginal, bool kIdentity, class M = TwinMath>
GCR_HD double scale_sq_residual(double x, double y, double sc, const RectModel& m, double ac) {
    double px = x, py = y, ps = sc;
    if (!kIdentity) {
        px = m.s * (x - m.x0 * 1.0);
        py = m.s * (y - m.y0 * 1.0);
        ps = sc * m.s;
    }
    const double t = (-m.h7 * px - m.h8 * py) + 1.0;
    const double rs = ps * M::pm3(t);
    if (rs < kEps9) return DBL_MAX * DBL_MAX;
    const double arg = kOriginal ? rs / ac : ac * rs;
    const double r = __builtin_fabs(M::log(arg));
    return r * r;
}

// ---------------------------------------------------------- orientation ----
struct OrientConst {
    double cphi;    // clipAngle(phi)
    double cphi2;   // clipAngle(clipAngle(phi + M_PI_2))
};

GCR_HD OrientConst orient_const(const RectModel& m) {
    OrientConst c;
    c.cphi = dm::clip_angle(m.phi);
    c.cphi2 = dm::clip_angle(dm::clip_angle(m.phi + kPi2));
    return c;
}

// minAngleDiff with both arguments already clipped (math_utils.hpp:90-95).
GCR_HD double min_angle_diff_c(double ca, double cb) {
    const double d = __builtin_fabs(ca - cb);
    return __builtin_fmin(d, kTwoPi - d);
}

// RectifyingHomography::rectifiedAngle (model.h:156-165) with the feature's
// cos/sin supplied; (px, py) are already normalised coordinates.
template <class M = TwinMath>
GCR_HD double rectified_angle(double px, double py, double ct, double st, double h7, double h8) {
    const double numer = (-px * st + py * ct) * h7 + st;
    const double denom = (px * st - py * ct) * h8 + ct;
    return dm::clip_angle_small(M::atan2(numer, denom));   // |atan2| <= pi
}

template <bool kIdentity, class M = TwinMath>
GCR_HD double orient_sq_residual(double x, double y, double ct, double st, const RectModel& m,
                                 const OrientConst& oc) {
    double px = x, py = y;
    if (!kIdentity) {
        px = m.s * (x - m.x0 * 1.0);
        py = m.s * (y - m.y0 * 1.0);
    }
    // rectifiedAngle's clipAngle(atan2) and linesAnglesDiff's clipAngle(th),
    // clipAngle(th - pi), with the ranges known: atan2 lies in [-pi, pi] (or is
    // NaN), so th = clipAngle(atan2) is one conditional + 2 pi and lies in
    // [0, 2 pi]; clipAngle(th) is th except 0 for th == 2 pi (a tiny negative
    // atan2 rounds up to it); th - pi lies in [-pi, pi].  The same values as
    // clip_angle_small on each (NaN stays NaN), with fewer operations.
    const double numer = (-px * st + py * ct) * m.h7 + st;
    const double denom = (px * st - py * ct) * m.h8 + ct;
    const double a = M::atan2(numer, denom);
    const double th = a < 0.0 ? a + kTwoPi : a;
    const double c0 = th == kTwoPi ? 0.0 : th;
    const double dpi = th - kPi;
    const double c1 = dpi < 0.0 ? dpi + kTwoPi : dpi;
    const double l1 = __builtin_fmin(min_angle_diff_c(oc.cphi, c0), min_angle_diff_c(oc.cphi, c1));
    const double l2 = __builtin_fmin(min_angle_diff_c(oc.cphi2, c0), min_angle_diff_c(oc.cphi2, c1));
    const double r = __builtin_fmin(l1, l2);
    return r * r;
}

// ------------------------------------------------------------- values ----
// The product's residual VALUES: what the kernels evaluate, fold into the
// MSAC sums and test against the thresholds (the oracle's TWIN mode restates
// them).  Equal in real arithmetic to the reference's residuals above and
// within exact.h's bound of the glibc ones, with fewer operations:
//   scale:   r = |log((ac ps) / t^3)|, |log(ps / (ac t^3))| for the original
//            solver: one division and the table log (dm_log, no division),
//            the reference's cut rs < 1e-9 becomes arg < ac 1e-9 (1e-9 / ac),
//            a per-model constant;
//   orient:  the distance of the rectified direction's angle to the model's
//            line family {phi + k pi/2} (the reference's min over phi,
//            phi + pi/2 and both line directions, two_sift.hpp:647-665) is
//            the angle of the direction rotated by -phi to its nearest axis,
//            atan(min(|u|, |v|) / max(|u|, |v|)) of (u, v) = R(-phi) (denom,
//            numer): one division, no quadrant or clipping logic, with the
//            model's twin cos / sin (dm_sincos).  Directions whose magnitude
//            leaves [2^-900, 2^1000] (subnormal or overflowing rotations,
//            inf / NaN) and models with |phi| > 16 take the reference formula
//            with the twin atan2 (orient_sq_residual).
struct ValueConst {
    double ac;             // alpha^3
    double cut;            // scale: arg below it <-> the reference's rs < 1e-9
    double c, s;           // orientation: twin cos / sin of phi (NaN: reference formula)
    double cphi, cphi2;    // orientation: orient_const (the reference formula's)
};

GCR_HD ValueConst value_const(const RectModel& m, bool original, bool orient) {
    ValueConst v;
    v.ac = alpha_cube(m);
    v.cut = original ? kEps9 / v.ac : v.ac * kEps9;
    v.c = 1.0;
    v.s = 0.0;
    v.cphi = v.cphi2 = 0.0;
    if (orient) {
        const OrientConst oc = orient_const(m);
        v.cphi = oc.cphi;
        v.cphi2 = oc.cphi2;
        if (__builtin_fabs(m.phi) <= 16.0) {
            dm::dm_sincos(m.phi, v.s, v.c);
        } else {
            v.c = v.s = __builtin_nan("");
        }
    }
    return v;
}

template <bool kOriginal, bool kIdentity>
GCR_HD double scale_sq_value(double x, double y, double sc, const RectModel& m, double ac, double cut,
                             const double* __restrict__ logtab = dm::kLogTab) {
    double px = x, py = y, ps = sc;
    if (!kIdentity) {
        px = m.s * (x - m.x0 * 1.0);
        py = m.s * (y - m.y0 * 1.0);
        ps = sc * m.s;
    }
    const double t = (-m.h7 * px - m.h8 * py) + 1.0;
    const double u = (t * t) * t;
    const double arg = kOriginal ? ps / (ac * u) : (ac * ps) / u;
    if (!(arg >= cut)) return DBL_MAX * DBL_MAX;          // the cut, negative, NaN: outlier
    const double r = __builtin_fabs(dm::dm_log(arg, logtab));
    return r * r;
}

// the reference formula with the twin atan2, out of line (rare)
GCR_COLD GCR_HD double orient_sq_slow(double px, double py, double ct, double st, double h7, double h8, double cphi,
                                      double cphi2) {
    RectModel m = default_model();
    m.h7 = h7;
    m.h8 = h8;
    return orient_sq_residual<true, TwinMath>(px, py, ct, st, m, OrientConst{cphi, cphi2});
}

template <bool kIdentity>
GCR_HD double orient_sq_value(double x, double y, double ct, double st, const RectModel& m, double c, double s,
                              double cphi, double cphi2) {
    double px = x, py = y;
    if (!kIdentity) {
        px = m.s * (x - m.x0 * 1.0);
        py = m.s * (y - m.y0 * 1.0);
    }
    const double numer = (-px * st + py * ct) * m.h7 + st;
    const double denom = (px * st - py * ct) * m.h8 + ct;
    const double an = __builtin_fabs(numer), ad = __builtin_fabs(denom);
    if (an < 0x1p1000 && ad < 0x1p1000 && __builtin_fmax(an, ad) >= 0x1p-900 && c == c) {
        const double u = __builtin_fabs(denom * c + numer * s);
        const double w = __builtin_fabs(numer * c - denom * s);
        const double r = dm::atan_ratio(__builtin_fmin(u, w), __builtin_fmax(u, w));
        return r * r;
    }
    return orient_sq_slow(px, py, ct, st, m.h7, m.h8, cphi, cphi2);
}

// ---------------------------------------------------------- geometry -------
// utils::areCollinear: SIGNED distance of p3 to line(p1, p2) < tol.
GCR_HD bool are_collinear(double x1, double y1, double x2, double y2, double x3, double y3, double tol) {
    double l0 = y1 * 1.0 - 1.0 * y2;
    double l1 = 1.0 * x2 - x1 * 1.0;
    double l2 = x1 * y2 - y1 * x2;
    const double nrm = sqrt(l0 * l0 + l1 * l1);
    l0 = l0 / nrm;
    l1 = l1 / nrm;
    l2 = l2 / nrm;
    const double dist = (l0 * x3 + l1 * y3) + l2 * 1.0;
    return dist < tol;
}

// Pivoting in-place Gauss elimination on [A | b], 3x3 (gaussElimination<3>).
GCR_HD void gauss3(double a[3][4], double out[3]) {
    for (int i = 0; i < 3; ++i)
        for (int k = i + 1; k < 3; ++k)
            if (__builtin_fabs(a[i][i]) < __builtin_fabs(a[k][i]))
                for (int j = 0; j <= 3; ++j) {
                    const double tmp = a[i][j];
                    a[i][j] = a[k][j];
                    a[k][j] = tmp;
                }
    for (int i = 0; i < 2; ++i)
        for (int k = i + 1; k < 3; ++k) {
            const double temp = a[k][i] / a[i][i];
            for (int j = 0; j <= 3; ++j) a[k][j] = a[k][j] - temp * a[i][j];
        }
    for (int i = 0; i < 3; ++i) {
        const int r = 2 - i;
        out[r] = a[r][3];
        for (int c = r + 1; c < 3; ++c) out[r] = out[r] - a[r][c] * out[c];
        out[r] = out[r] / a[r][r];
    }
}

GCR_HD double cross2(double ox, double oy, double px, double py, double qx, double qy) {
    return (px - ox) * (qy - oy) - (py - oy) * (qx - ox);
}

// computeConvexHull (monotone chain) of n <= 4 points followed by
// pointInConvexPolygon (edges and vertices count as inside).
GCR_HD bool point_in_hull4(const double* px_in, const double* py_in, double qx, double qy) {
    constexpr int n = 4;
    double px[n], py[n];
    for (int i = 0; i < n; ++i) { px[i] = px_in[i]; py[i] = py_in[i]; }
    // lexicographic sort (insertion sort; equal keys are identical points)
    for (int i = 1; i < n; ++i) {
        const double kx = px[i], ky = py[i];
        int j = i - 1;
        while (j >= 0 && (kx < px[j] || (kx == px[j] && ky < py[j]))) {
            px[j + 1] = px[j]; py[j + 1] = py[j];
            --j;
        }
        px[j + 1] = kx; py[j + 1] = ky;
    }
    double hx[2 * n], hy[2 * n];
    int k = 0;
    for (int i = 0; i < n; ++i) {
        while (k >= 2 && cross2(hx[k - 2], hy[k - 2], hx[k - 1], hy[k - 1], px[i], py[i]) <= 0) k--;
        hx[k] = px[i]; hy[k] = py[i]; k++;
    }
    const int t = k + 1;
    for (int i = n - 1; i > 0; --i) {
        while (k >= t && cross2(hx[k - 2], hy[k - 2], hx[k - 1], hy[k - 1], px[i - 1], py[i - 1]) <= 0) k--;
        hx[k] = px[i - 1]; hy[k] = py[i - 1]; k++;
    }
    int nv = k - 1;
    if (nv == 2) {
        const bool cx = __builtin_fabs(hx[0] - hx[1]) < 1e-9;
        const bool cy = __builtin_fabs(hy[0] - hy[1]) < 1e-9;
        if (cx && cy) nv = 1;
    }
    if (nv < 3) return false;
    bool pos = false, neg = false;
    for (int i = 0; i < nv; ++i) {
        const int j = (i + 1) % nv;
        const double cp = cross2(hx[i], hy[i], hx[j], hy[j], qx, qy);
        if (cp > 0) pos = true;
        else if (cp < 0) neg = true;
        if (pos && neg) return false;
    }
    return true;
}

// lineFromPointAndAngle with cos/sin supplied: (s, -c, y*c - x*s).
GCR_HD void line_from(double x, double y, double c, double s, double l[3]) {
    l[0] = s;
    l[1] = -c;
    l[2] = y * c - x * s;
}

GCR_HD void cross3(const double a[3], const double b[3], double o[3]) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

// One orientation-pair row of the hybrid non-minimal system
// (setOrientationConstraint, two_sift.hpp:238-258): vp = l_i x l_j scaled by
// 1 / max|vp| when that exceeds 1 (cwiseAbs().maxCoeff(), left fold), weight
// w_i * w_j = 1 on the Python path; row (w vp0, w vp1, 0 | w vp2).
// ... from the two lines (line_from of features i and j)
GCR_HD void sift_pair_row_lines(const double l1[3], const double l2[3], double row[4]) {
    double vp[3];
    cross3(l1, l2, vp);
    const double a0 = __builtin_fabs(vp[0]), a1 = __builtin_fabs(vp[1]), a2 = __builtin_fabs(vp[2]);
    double mx = (a0 < a1) ? a1 : a0;
    mx = (mx < a2) ? a2 : mx;
    if (mx > 1.0)
        for (int q = 0; q < 3; ++q) vp[q] = vp[q] / mx;
    const double w = 1.0 * 1.0;
    row[0] = w * vp[0];
    row[1] = w * vp[1];
    row[2] = 0.0;
    row[3] = w * vp[2];
}
GCR_HD void sift_pair_row(double xi, double yi, double ci, double si, double xj, double yj, double cj, double sj,
                          double row[4]) {
    double l1[3], l2[3];
    line_from(xi, yi, ci, si, l1);
    line_from(xj, yj, cj, sj, l2);
    sift_pair_row_lines(l1, l2, row);
}

// ------------------------------------------------------- minimal solvers ---
// 3-SIFT minimal fit.  p[i] = pow(s_i, kScalePower) precomputed with glibc
// (+1/3 for the new solver, -1/3 for the original one).
template <bool kOriginal>
GCR_HD bool solve_scale3(const double x[3], const double y[3], const double p[3], RectModel& out) {
    double a[3][4];
    for (int i = 0; i < 3; ++i) {
        a[i][0] = x[i];
        a[i][1] = y[i];
        a[i][2] = kOriginal ? -p[i] : p[i];
        a[i][3] = kOriginal ? -1.0 : 1.0;
    }
    double sol[3];
    gauss3(a, sol);
    if (is_nan(sol[0]) || is_nan(sol[1]) || is_nan(sol[2])) return false;
    out = default_model();
    out.h7 = sol[0];
    out.h8 = sol[1];
    out.alpha = sol[2];
    return !(out.alpha < kEps9);
}

// 2-SIFT sample validity: vanishing point of the two orientation lines must be
// non-degenerate, not (signed-)collinear with the two scale points and outside
// the hull of the four sample points.
GCR_HD bool valid_sample_sift22(const double sx[2], const double sy[2], const double ox[2], const double oy[2],
                                const double oc[2], const double os[2]) {
    double l1[3], l2[3], vp[3];
    line_from(ox[0], oy[0], oc[0], os[0], l1);
    line_from(ox[1], oy[1], oc[1], os[1], l2);
    cross3(l1, l2, vp);
    if (__builtin_fabs(vp[0]) < 1e-6 && __builtin_fabs(vp[1]) < 1e-6 && __builtin_fabs(vp[2]) < 1e-6) return false;
    if (__builtin_fabs(vp[2]) < 1e-6) return true;
    const double vz = vp[2];
    const double vx = vp[0] / vz, vy = vp[1] / vz;
    if (are_collinear(sx[0], sy[0], sx[1], sy[1], vx, vy, 1.0)) return false;
    const double hxs[4] = {sx[0], sx[1], ox[0], ox[1]};
    const double hys[4] = {sy[0], sy[1], oy[0], oy[1]};
    return !point_in_hull4(hxs, hys, vx, vy);
}

template <class M = TwinMath>
GCR_HD bool solve_sift22(const double sx[2], const double sy[2], const double sp[2], const double ox[2],
                         const double oy[2], const double oc[2], const double os[2], RectModel& out) {
    double a[3][4];
    for (int i = 0; i < 2; ++i) {
        a[i][0] = sx[i];
        a[i][1] = sy[i];
        a[i][2] = sp[i];
        a[i][3] = 1.0;
    }
    double l1[3], l2[3], vp[3];
    line_from(ox[0], oy[0], oc[0], os[0], l1);
    line_from(ox[1], oy[1], oc[1], os[1], l2);
    cross3(l1, l2, vp);
    a[2][0] = vp[0];
    a[2][1] = vp[1];
    a[2][2] = 0.0;
    a[2][3] = vp[2];
    double sol[3];
    gauss3(a, sol);
    if (is_nan(sol[0]) || is_nan(sol[1]) || is_nan(sol[2])) return false;
    out = default_model();
    out.h7 = sol[0];
    out.h8 = sol[1];
    out.alpha = sol[2];
    if (out.alpha < kEps9) return false;
    const double vz = (-out.h7 * vp[0] - out.h8 * vp[1]) + vp[2];   // rectifyPoint(vp)
    if (__builtin_fabs(vz) > kEps9) return false;
    out.phi = dm::clip_angle_small(M::atan2(vp[1], vp[0]));
    return true;
}

GCR_HD bool valid_model_sift22(const RectModel& m) {
    return !(__builtin_fmax(__builtin_fabs(m.h7), __builtin_fabs(m.h8)) >= 1e-3);
}

}  // namespace gcr
