// fund.h -- fundamental-matrix estimator of the hot path (SURVEY.md §8(f)
// row 3, BASELINE configs[3]), host and device (GCR_HD).
//
// Like the homography (geo.h) this estimator is absent from the fork (SURVEY
// finding 0.1) and upstream GC-RANSAC is not in the container: parity is
// UNPINNED against any reference and rests on the oracle restatement
// (oracle/gcr_oracle.cpp FSolver) plus synthetic two-view ground truth.  The
// structure follows upstream's published 7-point estimator:
//   * minimal solver: 7 correspondences, Hartley-normalised, the 2-D null space
//     of the 7 x 9 epipolar system by Gaussian elimination with partial
//     pivoting, det(F1 + l F2) = 0 as a cubic, up to three real roots -- so a
//     sample may yield 1..3 models, every one of which is scored;
//   * model validity: the oriented epipolar constraint on the 7 sample points
//     (models violating it are dropped by the solver);
//   * residual: squared Sampson distance;
//   * non-minimal fit (LO, final refit; host only): normalised 8-point --
//     smallest eigenvector of A^T A, then rank-2 projection.
// Everything a device kernel evaluates uses +, -, *, / and sqrt only (all
// correctly rounded on gfx950 and x86-64 with -ffp-contract=off): the cubic is
// solved by bracketing between the critical points and safeguarded Newton,
// not by Cardano (which would need cbrt / acos / cos twins).
#pragma once

#include <type_traits>

#include "gcr_hd.h"
#include "geo.h"

namespace gcr {

constexpr int kFModels = 3;          // real roots of the cubic, models per sample

GCR_HD double det3(const double* m) {
    return (m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6])) +
           m[2] * (m[3] * m[7] - m[4] * m[6]);
}

// ((l + a) l + b) l + c and its derivative (3 l + 2 a) l + b
GCR_HD double cubic_monic(double a, double b, double c, double l) { return ((l + a) * l + b) * l + c; }
GCR_HD double cubic_monic_d(double a, double b, double l) { return (3.0 * l + 2.0 * a) * l + b; }

// Root of the monic cubic in a bracket [lo, hi] with p(lo) p(hi) < 0:
// safeguarded Newton (Newton steps while they stay inside the shrinking
// bracket and halve it fast enough, bisection otherwise; "rtsafe"), ~5-8
// iterations instead of ~60 for plain bisection.  Basic ops only.
GCR_HD double cubic_root_in(double a, double b, double c, double lo, double hi, double flo) {
    double xl = lo, xh = hi;                       // p(xl) < 0 < p(xh)
    if (!(flo < 0.0)) { xl = hi; xh = lo; }
    double rts = 0.5 * (lo + hi);
    double dxold = __builtin_fabs(hi - lo), dx = dxold;
    double f = cubic_monic(a, b, c, rts), df = cubic_monic_d(a, b, rts);
    for (int it = 0; it < 100; ++it) {
        if (f == 0.0) break;
        if ((((rts - xh) * df - f) * ((rts - xl) * df - f) > 0.0) ||
            (__builtin_fabs(2.0 * f) > __builtin_fabs(dxold * df))) {
            dxold = dx;
            dx = 0.5 * (xh - xl);
            rts = xl + dx;
            if (xl == rts) break;
        } else {
            dxold = dx;
            dx = f / df;
            const double prev = rts;
            rts = rts - dx;
            if (prev == rts) break;
        }
        if (__builtin_fabs(dx) < 1e-14 * (1.0 + __builtin_fabs(rts))) break;
        f = cubic_monic(a, b, c, rts);
        df = cubic_monic_d(a, b, rts);
        if (f < 0.0) xl = rts;
        else xh = rts;
    }
    return rts;
}

// cubic_root_in as a branch-free state machine, so the three brackets of a
// cubic run their iterations side by side (three independent dependency
// chains per lane instead of one after another).  Every chain performs
// exactly cubic_root_in's operations in its order; a step of a finished chain
// is a no-op, so the roots are bit-identical to three sequential calls.
struct RtSafe {
    double xl, xh, rts, dxold, dx, f, df;
    bool on;
};

GCR_HD RtSafe rtsafe_init(double a, double b, double c, double lo, double hi, double flo, bool on) {
    RtSafe s;
    const bool neg = flo < 0.0;
    s.xl = neg ? lo : hi;
    s.xh = neg ? hi : lo;
    s.rts = 0.5 * (lo + hi);
    s.dxold = __builtin_fabs(hi - lo);
    s.dx = s.dxold;
    s.f = cubic_monic(a, b, c, s.rts);
    s.df = cubic_monic_d(a, b, s.rts);
    s.on = on;
    return s;
}

GCR_HD void rtsafe_step(RtSafe& s, double a, double b, double c) {
    const bool run = s.on && !(s.f == 0.0);
    const bool bis = (((s.rts - s.xh) * s.df - s.f) * ((s.rts - s.xl) * s.df - s.f) > 0.0) ||
                     (__builtin_fabs(2.0 * s.f) > __builtin_fabs(s.dxold * s.df));
    const double bdx = 0.5 * (s.xh - s.xl);
    const double brts = s.xl + bdx;
    const double ndx = s.f / s.df;
    const double nrts = s.rts - ndx;
    const double dx = bis ? bdx : ndx;
    const double rts = bis ? brts : nrts;
    const bool same = bis ? (s.xl == rts) : (s.rts == rts);
    const bool cont = run && !same && !(__builtin_fabs(dx) < 1e-14 * (1.0 + __builtin_fabs(rts)));
    const double f = cubic_monic(a, b, c, rts);
    const double df = cubic_monic_d(a, b, rts);
    s.dxold = run ? s.dx : s.dxold;
    s.dx = run ? dx : s.dx;
    s.rts = run ? rts : s.rts;
    s.f = cont ? f : s.f;
    s.df = cont ? df : s.df;
    const bool lo_side = f < 0.0;
    s.xl = (cont && lo_side) ? rts : s.xl;
    s.xh = (cont && !lo_side) ? rts : s.xh;
    s.on = cont;
}

// Real roots of c3 l^3 + c2 l^2 + c1 l + c0 in ascending order (basic ops +
// sqrt only): brackets between the derivative's critical points and the
// Cauchy bound, one safeguarded-Newton root per sign change.  Returns the
// count.  Scalars only (no arrays): on the device a dynamically indexed
// bracket or root array went to LDS / scratch.
GCR_HD int real_roots_cubic(double c3, double c2, double c1, double c0, double& r0, double& r1, double& r2) {
    r0 = r1 = r2 = 0.0;
    const double big = __builtin_fmax(__builtin_fabs(c2), __builtin_fmax(__builtin_fabs(c1), __builtin_fabs(c0)));
    if (!(__builtin_fabs(c3) > 1e-12 * big)) {
        // degenerate leading coefficient: quadratic / linear
        if (c2 != 0.0) {
            const double disc = c1 * c1 - 4.0 * c2 * c0;
            if (disc < 0.0) return 0;
            const double sq = sqrt(disc);
            double u = (-c1 - sq) / (2.0 * c2), v = (-c1 + sq) / (2.0 * c2);
            if (v < u) { const double t = u; u = v; v = t; }
            r0 = u;
            if (v == u) return 1;
            r1 = v;
            return 2;
        }
        if (c1 != 0.0) {
            r0 = -c0 / c1;
            return 1;
        }
        return 0;
    }
    const double a = c2 / c3, b = c1 / c3, c = c0 / c3;
    const double R = 1.0 + __builtin_fmax(__builtin_fabs(a), __builtin_fmax(__builtin_fabs(b), __builtin_fabs(c)));
    const double dd = a * a - 3.0 * b;          // discriminant of the derivative / 4
    // brackets [-R, e1], [e1, e2], [e2, R] between the critical points (only
    // [-R, R] when the cubic is monotone)
    const bool crit = dd > 0.0;
    double e1 = R, e2 = R;
    if (crit) {
        const double sq = sqrt(dd);
        e1 = (-a - sq) / 3.0;
        e2 = (-a + sq) / 3.0;
    }
    int n = 0;
    double o0 = 0.0, o1 = 0.0, o2 = 0.0;
    // value selects, not an if-chain of stores (which the device compiler
    // turned into a pointer table in LDS and stores through it)
    auto push = [&](double v) {
        o0 = n == 0 ? v : o0;
        o1 = n == 1 ? v : o1;
        o2 = n >= 2 ? v : o2;
        ++n;
    };
    // the three brackets [-R, e1], [e1, e2], [e2, R] (the last two only with
    // critical points): their safeguarded-Newton roots side by side, then the
    // sequential bookkeeping (an exact zero at a bracket end is pushed once)
    const double f0 = cubic_monic(a, b, c, -R), f1 = cubic_monic(a, b, c, e1);
    const double f2 = cubic_monic(a, b, c, e2), f3 = cubic_monic(a, b, c, R);
    auto newton = [](double flo, double fhi) { return !(flo == 0.0) && ((flo < 0.0) != (fhi < 0.0)) && !(fhi == 0.0); };
    RtSafe s0 = rtsafe_init(a, b, c, -R, e1, f0, newton(f0, f1));
    RtSafe s1 = rtsafe_init(a, b, c, e1, e2, f1, crit && newton(f1, f2));
    RtSafe s2 = rtsafe_init(a, b, c, e2, R, f2, crit && newton(f2, f3));
    for (int it = 0; it < 100 && (s0.on || s1.on || s2.on); ++it) {
        rtsafe_step(s0, a, b, c);
        rtsafe_step(s1, a, b, c);
        rtsafe_step(s2, a, b, c);
    }
    double prev = 0.0;
    auto bracket = [&](double lo, double flo, double fhi, double root) {
        if (flo == 0.0) {
            if (n == 0 || prev != lo) { push(lo); prev = lo; }
            return;
        }
        if (!((flo < 0.0) != (fhi < 0.0)) || fhi == 0.0) return;
        prev = root;
        push(prev);
    };
    bracket(-R, f0, f1, s0.rts);
    if (crit) {
        bracket(e1, f1, f2, s1.rts);
        bracket(e2, f2, f3, s2.rts);
    }
    r0 = o0;
    r1 = o1;
    r2 = o2;
    return n;
}

GCR_HD int real_roots_cubic(double c3, double c2, double c1, double c0, double r[3]) {
    return real_roots_cubic(c3, c2, c1, c0, r[0], r[1], r[2]);
}

// Hartley normalisation of n points: centroid, mean distance, s = sqrt(2) / d;
// normalised u = s * (x - cx).  Sequential sums in index order.
template <int N>
GCR_HD bool hartley7(const double* x, const double* y, double& cx, double& cy, double& s) {
    double sx = 0.0, sy = 0.0;
    for (int i = 0; i < N; ++i) { sx += x[i]; sy += y[i]; }
    cx = sx / (double)N;
    cy = sy / (double)N;
    double sd = 0.0;
    for (int i = 0; i < N; ++i) {
        const double dx = x[i] - cx, dy = y[i] - cy;
        sd += sqrt(dx * dx + dy * dy);
    }
    const double d = sd / (double)N;
    if (!(d > 0.0)) return false;
    s = 1.4142135623730951 / d;
    return true;
}

// F = T2^T Fn T1 with Ti = [[si, 0, -si cxi], [0, si, -si cyi], [0, 0, 1]],
// then scaled to unit Frobenius norm.
GCR_HD bool denormalize_f(const double* fn, double s1, double cx1, double cy1, double s2, double cx2, double cy2,
                          double* f) {
    const double tx1 = -s1 * cx1, ty1 = -s1 * cy1, tx2 = -s2 * cx2, ty2 = -s2 * cy2;
    double m[9];
    for (int i = 0; i < 3; ++i) {
        m[3 * i] = fn[3 * i] * s1;
        m[3 * i + 1] = fn[3 * i + 1] * s1;
        m[3 * i + 2] = (fn[3 * i] * tx1 + fn[3 * i + 1] * ty1) + fn[3 * i + 2];
    }
    for (int j = 0; j < 3; ++j) {
        f[j] = s2 * m[j];
        f[3 + j] = s2 * m[3 + j];
        f[6 + j] = (tx2 * m[j] + ty2 * m[3 + j]) + m[6 + j];
    }
    double nn = 0.0;
    for (int k = 0; k < 9; ++k) nn += f[k] * f[k];
    const double nrm = sqrt(nn);
    // branch-free: a failed norm divides by 1.0, which leaves f exactly as is
    const bool ok = (nrm > 0.0) & (nrm < 1e300);
    const double d = ok ? nrm : 1.0;
    for (int k = 0; k < 9; ++k) f[k] = f[k] / d;
    return ok;
}

// Oriented epipolar constraint (Chum, Werner, Matas 2004): with e2 the
// epipole of image 2 (F^T e2 = 0), (e2 x x2_i) . (F x1_i) has one sign for
// every correspondence of the sample.
template <int N>
GCR_HD bool oriented_ok(const double* f, const double* x1, const double* y1, const double* x2, const double* y2) {
    // e2 orthogonal to every column of F: the largest cross product of two columns
    const double c[3][3] = {{f[0], f[3], f[6]}, {f[1], f[4], f[7]}, {f[2], f[5], f[8]}};
    const int pa[3] = {0, 0, 1}, pb[3] = {1, 2, 2};
    double e[3] = {0.0, 0.0, 0.0}, best = -1.0;
    for (int q = 0; q < 3; ++q) {
        const double* u = c[pa[q]];
        const double* v = c[pb[q]];
        const double w0 = u[1] * v[2] - u[2] * v[1];
        const double w1 = u[2] * v[0] - u[0] * v[2];
        const double w2 = u[0] * v[1] - u[1] * v[0];
        const double nn = (w0 * w0 + w1 * w1) + w2 * w2;
        if (nn > best) { best = nn; e[0] = w0; e[1] = w1; e[2] = w2; }
    }
    const bool epi = best > 0.0;   // tested last: the sign loop stays branch-free
    int pos = 0, neg = 0;
    for (int i = 0; i < N; ++i) {
        const double fx0 = (f[0] * x1[i] + f[1] * y1[i]) + f[2];
        const double fx1 = (f[3] * x1[i] + f[4] * y1[i]) + f[5];
        const double fx2 = (f[6] * x1[i] + f[7] * y1[i]) + f[8];
        // e2 x (x2, y2, 1)
        const double l0 = e[1] - e[2] * y2[i];
        const double l1 = e[2] * x2[i] - e[0];
        const double l2 = e[0] * y2[i] - e[1] * x2[i];
        const double sgn = (l0 * fx0 + l1 * fx1) + l2 * fx2;
        pos += sgn > 0.0;
        neg += sgn < 0.0;
    }
    return epi & ((pos == N) | (neg == N));
}

// The 7-point solver's intermediate state: normalisation, the null-space
// basis and the real roots of the cubic, with the oriented-valid roots in a
// bit mask.  Kept in registers; a model is rebuilt from it on demand
// (f7_model), so the generator never holds three 9-double models per lane.
struct F7Basis {
    double F1[9], F2[9];
    double s1, cx1, cy1, s2, cx2, cy2;
    double root0, root1, root2;
    unsigned valid;              // bit q: root q gives an oriented-valid model
};

GCR_HD double f7_root(const F7Basis& b, int q) { return q == 0 ? b.root0 : (q == 1 ? b.root1 : b.root2); }

// model of root q (false if it does not denormalise)
GCR_HD bool f7_model(const F7Basis& b, double l, double fm[9]) {
    double fn[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) fn[k] = b.F1[k] + l * b.F2[k];
    return denormalize_f(fn, b.s1, b.cx1, b.cy1, b.s2, b.cx2, b.cy2, fm);
}

// 7-point solver: fills the basis; returns the number of oriented-valid
// models (0 = the sample yields no model).  Models are in ascending root order.
GCR_HD int solve_f7_basis(const double x1[7], const double y1[7], const double x2[7], const double y2[7],
                          F7Basis& out) {
    out.valid = 0;
    double cx1, cy1, s1, cx2, cy2, s2;
    if (!hartley7<7>(x1, y1, cx1, cy1, s1) || !hartley7<7>(x2, y2, cx2, cy2, s2)) return 0;
    out.s1 = s1; out.cx1 = cx1; out.cy1 = cy1; out.s2 = s2; out.cx2 = cx2; out.cy2 = cy2;
    double a[7][9];
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        const double u1 = s1 * (x1[i] - cx1), v1 = s1 * (y1[i] - cy1);
        const double u2 = s2 * (x2[i] - cx2), v2 = s2 * (y2[i] - cy2);
        a[i][0] = u2 * u1; a[i][1] = u2 * v1; a[i][2] = u2;
        a[i][3] = v2 * u1; a[i][4] = v2 * v1; a[i][5] = v2;
        a[i][6] = u1;      a[i][7] = v1;      a[i][8] = 1.0;
    }
    // forward elimination, partial pivoting on columns 0..6 (fully unrolled:
    // the row swap is a compare-select per row, so the matrix stays in
    // registers instead of going to scratch through a dynamic row index)
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        int p = k;
        double pm = __builtin_fabs(a[k][k]);
#pragma unroll
        for (int i = k + 1; i < 7; ++i)
            if (__builtin_fabs(a[i][k]) > pm) { pm = __builtin_fabs(a[i][k]); p = i; }
        if (!(pm > 1e-10)) return 0;                 // rank < 7: degenerate sample
#pragma unroll
        for (int i = k + 1; i < 7; ++i) {
            const bool sw = i == p;
#pragma unroll
            for (int j = k; j < 9; ++j) {
                const double u = a[k][j], v = a[i][j];
                a[k][j] = sw ? v : u;
                a[i][j] = sw ? u : v;
            }
        }
#pragma unroll
        for (int i = k + 1; i < 7; ++i) {
            const double fct = a[i][k] / a[k][k];
#pragma unroll
            for (int j = k + 1; j < 9; ++j) a[i][j] = a[i][j] - fct * a[k][j];
            a[i][k] = 0.0;
        }
    }
    // null-space basis: (f7, f8) = (1, 0) and (0, 1)
    auto back_substitute = [&](double (&fv)[9], double f7, double f8) {
        fv[7] = f7;
        fv[8] = f8;
#pragma unroll
        for (int r = 6; r >= 0; --r) {
            double acc = a[r][7] * fv[7];
            acc = acc + a[r][8] * fv[8];
#pragma unroll
            for (int cc = r + 1; cc < 7; ++cc) acc = acc + a[r][cc] * fv[cc];
            fv[r] = -acc / a[r][r];
        }
    };
    back_substitute(out.F1, 1.0, 0.0);
    back_substitute(out.F2, 0.0, 1.0);
    // det(F1 + l F2) = c3 l^3 + c2 l^2 + c1 l + c0 from four evaluations
    double P[9], M[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) { P[k] = out.F1[k] + out.F2[k]; M[k] = out.F1[k] - out.F2[k]; }
    const double c0 = det3(out.F1), c3 = det3(out.F2), d1 = det3(P), dm1 = det3(M);
    const double c2 = (d1 + dm1) * 0.5 - c0;
    const double c1 = (d1 - dm1) * 0.5 - c3;
    double q0, q1, q2;
    const int nr = real_roots_cubic(c3, c2, c1, c0, q0, q1, q2);
    out.root0 = q0;
    out.root1 = q1;
    out.root2 = q2;
    // all three roots tested without branches (absent roots give inert
    // models), so their denormalisations and orientation tests overlap
    int n = 0;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        double fm[9];
        const bool den = f7_model(out, f7_root(out, q), fm);
        const bool ori = oriented_ok<7>(fm, x1, y1, x2, y2);
        const bool v = (q < nr) & den & ori;
        out.valid |= v ? 1u << q : 0u;
        n += v;
    }
    return n;
}

// 7-point solver, models materialised: up to kFModels oriented-valid models in
// ascending root order (host paths and tests)
GCR_HD int solve_f7(const double x1[7], const double y1[7], const double x2[7], const double y2[7],
                    GeoModel out[kFModels]) {
    F7Basis b;
    const int n = solve_f7_basis(x1, y1, x2, y2, b);
    int k = 0;
    for (int q = 0; q < 3 && k < n; ++q)
        if (b.valid & (1u << q)) f7_model(b, f7_root(b, q), out[k++].h);
    return n;
}

// squared Sampson distance of (x1, y1) <-> (x2, y2) under F
GCR_HD double f_sq_sampson(double x1, double y1, double x2, double y2, const double* h) {
    const double fx0 = (h[0] * x1 + h[1] * y1) + h[2];
    const double fx1 = (h[3] * x1 + h[4] * y1) + h[5];
    const double fx2 = (h[6] * x1 + h[7] * y1) + h[8];
    const double ft0 = (h[0] * x2 + h[3] * y2) + h[6];
    const double ft1 = (h[1] * x2 + h[4] * y2) + h[7];
    const double num = (x2 * fx0 + y2 * fx1) + fx2;
    const double den = ((fx0 * fx0 + fx1 * fx1) + ft0 * ft0) + ft1 * ft1;
    return (num * num) / den;
}

// residual of the correspondence estimators: 3 = homography, 4 = fundamental
template <int KIND>
GCR_HD double geo_sq_residual(double x1, double y1, double x2, double y2, const double* h) {
    if constexpr (KIND == 4) return f_sq_sampson(x1, y1, x2, y2, h);
    else return h_sq_residual(x1, y1, x2, y2, h);
}

}  // namespace gcr
