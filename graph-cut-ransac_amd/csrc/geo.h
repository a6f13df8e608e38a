// geo.h -- homography estimator of the hot path,
// host and device (GCR_HD).
//
// This fork has no homography / fundamental estimators (SURVEY finding 0.1) and
// upstream GC-RANSAC is not in the container, so these follow upstream's
// published structure as closely as it can be restated -- parity is UNPINNED
// against any reference and rests on the oracle restatement
// (oracle/gcr_oracle.cpp) plus synthetic ground truth:
//   * minimal solver: 4 correspondences, DLT with h33 = 1 -> an 8 x 9
//     augmented system solved by the reference's own gaussElimination<N>
//     (math_utils.hpp:164-221: one bubble pivot pass, elimination, back
//     substitution) with N = 8;
//   * sample validity: the four triangles of the sample keep their
//     orientation between the images (non-degenerate, no reflection);
//   * residual: squared forward transfer error in the second image;
//   * non-minimal fit (LO, final refit): Hartley-normalised DLT with h33 = 1 as
//     an 8-column least-squares problem, solved by the column-pivoted
//     Householder QR of qr3.h (blocked summation order).
// Correspondence layout in the engine: class 0 SoA x = x1, y = y1, a = x2,
// c0 = y2.
#pragma once

#include "gcr_hd.h"

namespace gcr {

// row-major 3x3 homography, h[8] = 1 after the minimal / non-minimal fits
struct GeoModel {
    double h[9];
};

GCR_HD GeoModel default_geo() { return GeoModel{{1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0}}; }

// gaussElimination<N> (math_utils.hpp:164-221) for the augmented N x (N+1) matrix
template <int N>
GCR_HD void gauss_n(double (&a)[N][N + 1], double (&out)[N]) {
    for (int i = 0; i < N; ++i)
        for (int k = i + 1; k < N; ++k)
            if (__builtin_fabs(a[i][i]) < __builtin_fabs(a[k][i]))
                for (int j = 0; j <= N; ++j) {
                    const double tmp = a[i][j];
                    a[i][j] = a[k][j];
                    a[k][j] = tmp;
                }
    for (int i = 0; i < N - 1; ++i)
        for (int k = i + 1; k < N; ++k) {
            const double temp = a[k][i] / a[i][i];
            for (int j = 0; j <= N; ++j) a[k][j] = a[k][j] - temp * a[i][j];
        }
    for (int i = 0; i < N; ++i) {
        const int r = N - 1 - i;
        out[r] = a[r][N];
        for (int c = r + 1; c < N; ++c) out[r] = out[r] - a[r][c] * out[c];
        out[r] = out[r] / a[r][r];
    }
}

// signed doubled area of the triangle (a, b, c)
GCR_HD double tri2(double ax, double ay, double bx, double by, double cx, double cy) {
    return (bx - ax) * (cy - ay) - (by - ay) * (cx - ax);
}

// A homography preserves the orientation of every triangle of a sample that
// lies on one side of the line at infinity: all four triples must have the
// same, non-zero orientation sign in both images.
GCR_HD bool valid_sample_h4(const double x1[4], const double y1[4], const double x2[4], const double y2[4]) {
    const int tri[4][3] = {{0, 1, 2}, {1, 2, 3}, {2, 3, 0}, {3, 0, 1}};
    for (int t = 0; t < 4; ++t) {
        const int a = tri[t][0], b = tri[t][1], c = tri[t][2];
        const double s1 = tri2(x1[a], y1[a], x1[b], y1[b], x1[c], y1[c]);
        const double s2 = tri2(x2[a], y2[a], x2[b], y2[b], x2[c], y2[c]);
        if (!(s1 * s2 > 0.0)) return false;
    }
    return true;
}

// 4-point DLT, h33 = 1: rows (x1, y1, 1, 0, 0, 0, -x2 x1, -x2 y1 | x2) and
// (0, 0, 0, x1, y1, 1, -y2 x1, -y2 y1 | y2).
GCR_HD bool solve_h4(const double x1[4], const double y1[4], const double x2[4], const double y2[4], GeoModel& out) {
    double a[8][9];
    for (int i = 0; i < 4; ++i) {
        double* r0 = a[2 * i];
        double* r1 = a[2 * i + 1];
        r0[0] = x1[i]; r0[1] = y1[i]; r0[2] = 1.0; r0[3] = 0.0; r0[4] = 0.0; r0[5] = 0.0;
        r0[6] = -x2[i] * x1[i]; r0[7] = -x2[i] * y1[i]; r0[8] = x2[i];
        r1[0] = 0.0; r1[1] = 0.0; r1[2] = 0.0; r1[3] = x1[i]; r1[4] = y1[i]; r1[5] = 1.0;
        r1[6] = -y2[i] * x1[i]; r1[7] = -y2[i] * y1[i]; r1[8] = y2[i];
    }
    double h[8];
    gauss_n<8>(a, h);
    for (int k = 0; k < 8; ++k) {
        if (is_nan(h[k]) || !(__builtin_fabs(h[k]) < 1e300)) return false;
        out.h[k] = h[k];
    }
    out.h[8] = 1.0;
    return true;
}

// squared forward transfer error of correspondence (x1, y1) -> (x2, y2)
GCR_HD double h_sq_residual(double x1, double y1, double x2, double y2, const double* h) {
    const double w = (h[6] * x1 + h[7] * y1) + h[8];
    const double u = ((h[0] * x1 + h[1] * y1) + h[2]) / w;
    const double v = ((h[3] * x1 + h[4] * y1) + h[5]) / w;
    const double du = u - x2, dv = v - y2;
    return du * du + dv * dv;
}

}  // namespace gcr
