// The orientation residual's angle clipping (rect.h orient_sq_residual) uses
// the known ranges of its arguments instead of three general clipAngle calls.
// This checks, on the host build of the same header, that the squared
// residual is bit-identical to the general form (rectified_angle +
// clip_angle_small twice, as before) on random, near-axis, tiny-negative-atan2
// and special-operand inputs.  Built and run by tests/test_orient_clip.py.
#include <stdio.h>
#include <string.h>

#include <random>

#include "rect.h"

using namespace gcr;

static double general_form(double x, double y, double ct, double st, const RectModel& m, const OrientConst& oc) {
    const double th = rectified_angle(x, y, ct, st, m.h7, m.h8);
    const double c0 = dm::clip_angle_small(th);
    const double c1 = dm::clip_angle_small(th - kPi);
    const double l1 = __builtin_fmin(min_angle_diff_c(oc.cphi, c0), min_angle_diff_c(oc.cphi, c1));
    const double l2 = __builtin_fmin(min_angle_diff_c(oc.cphi2, c0), min_angle_diff_c(oc.cphi2, c1));
    const double r = __builtin_fmin(l1, l2);
    return r * r;
}

static uint64_t bits(double v) {
    uint64_t u;
    memcpy(&u, &v, 8);
    return u;
}

int main() {
    std::mt19937_64 rng(20251121);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long n = 0, bad = 0;
    auto check = [&](double x, double y, double t, const RectModel& m) {
        const OrientConst oc = orient_const(m);
        const double ct = cos(t), st = sin(t);
        const double a = general_form(x, y, ct, st, m, oc), b = orient_sq_residual<true>(x, y, ct, st, m, oc);
        ++n;
        const bool same = bits(a) == bits(b) || (a != a && b != b);
        if (!same) {
            if (bad < 10) printf("mismatch x=%.17g y=%.17g t=%.17g h7=%.17g h8=%.17g phi=%.17g: %.17g vs %.17g\n", x, y,
                                 t, m.h7, m.h8, m.phi, a, b);
            ++bad;
        }
    };
    for (int i = 0; i < 2000000; ++i) {
        RectModel m = default_model();
        m.h7 = (U(rng) - 0.5) * 4e-3;
        m.h8 = (U(rng) - 0.5) * 4e-3;
        m.phi = U(rng) * 2 * kPi;
        check(U(rng) * 2000, U(rng) * 2000, U(rng) * 2 * kPi, m);
    }
    // angles whose rectified direction sits on the axes (atan2 = 0, -0, +-pi,
    // tiny negative: th rounds up to 2 pi), and special operands
    const double ts[] = {0.0, -0.0, kPi, -kPi, 1e-300, -1e-300, -1e-17, -1e-16, 2 * kPi, kPi / 2, -kPi / 2,
                         NAN, INFINITY};
    const double ps[] = {0.0, kPi / 2, kPi, 1.5 * kPi, 2 * kPi - 1e-16, 1e-17};
    for (double t : ts)
        for (double phi : ps)
            for (double h : {0.0, 1e-4, -1e-4, 1e300, (double)NAN}) {
                RectModel m = default_model();
                m.h7 = h;
                m.h8 = -h;
                m.phi = phi;
                check(0.0, 0.0, t, m);
                check(10.0, -3.0, t, m);
                check(1e308, 1e-308, t, m);
            }
    printf("%ld inputs, %ld mismatches\n", n, bad);
    return bad != 0;
}
