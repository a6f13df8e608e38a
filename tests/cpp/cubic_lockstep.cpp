// Lockstep root finder (fund.h real_roots_cubic: three RtSafe chains side by
// side) against the sequential form it replaces (one cubic_root_in call per
// bracket, pushed in order), bitwise, on random and adversarial cubics.
// Built and run by tests/test_cubic_lockstep.py with g++ -ffp-contract=off.
#include <stdio.h>
#include <string.h>

#include <random>

#include "fund.h"

using namespace gcr;

static int roots_sequential(double c3, double c2, double c1, double c0, double r[3]) {
    r[0] = r[1] = r[2] = 0.0;
    const double big = __builtin_fmax(__builtin_fabs(c2), __builtin_fmax(__builtin_fabs(c1), __builtin_fabs(c0)));
    if (!(__builtin_fabs(c3) > 1e-12 * big)) return -1;   // quadratic branch: unchanged code, not compared
    const double a = c2 / c3, b = c1 / c3, c = c0 / c3;
    const double R = 1.0 + __builtin_fmax(__builtin_fabs(a), __builtin_fmax(__builtin_fabs(b), __builtin_fabs(c)));
    const double dd = a * a - 3.0 * b;
    const bool crit = dd > 0.0;
    double e1 = R, e2 = R;
    if (crit) {
        const double sq = sqrt(dd);
        e1 = (-a - sq) / 3.0;
        e2 = (-a + sq) / 3.0;
    }
    int n = 0;
    double prev = 0.0;
    auto bracket = [&](double lo, double hi) {
        const double flo = cubic_monic(a, b, c, lo);
        const double fhi = cubic_monic(a, b, c, hi);
        if (flo == 0.0) {
            if (n == 0 || prev != lo) { r[n < 3 ? n : 2] = lo; ++n; prev = lo; }
            return;
        }
        if (!((flo < 0.0) != (fhi < 0.0)) || fhi == 0.0) return;
        prev = cubic_root_in(a, b, c, lo, hi, flo);
        r[n < 3 ? n : 2] = prev;
        ++n;
    };
    bracket(-R, e1);
    if (crit) {
        bracket(e1, e2);
        bracket(e2, R);
    }
    return n;
}

static bool same(double x, double y) { return memcmp(&x, &y, sizeof x) == 0; }

int main() {
    std::mt19937_64 rng(12345);
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    std::uniform_int_distribution<int> ex(-12, 12);
    long checked = 0, bad = 0, three = 0;
    auto check = [&](double c3, double c2, double c1, double c0) {
        double s[3], l[3];
        const int ns = roots_sequential(c3, c2, c1, c0, s);
        if (ns < 0) return;
        const int nl = real_roots_cubic(c3, c2, c1, c0, l[0], l[1], l[2]);
        ++checked;
        three += ns == 3;
        if (ns != nl || !same(s[0], l[0]) || !same(s[1], l[1]) || !same(s[2], l[2])) {
            if (bad++ < 5)
                printf("MISMATCH %.17g %.17g %.17g %.17g: %d [%.17g %.17g %.17g] vs %d [%.17g %.17g %.17g]\n", c3, c2,
                       c1, c0, ns, s[0], s[1], s[2], nl, l[0], l[1], l[2]);
        }
    };
    for (int i = 0; i < 400000; ++i) {
        // random coefficients over many magnitudes
        check(ldexp(u(rng), ex(rng)), ldexp(u(rng), ex(rng)), ldexp(u(rng), ex(rng)), ldexp(u(rng), ex(rng)));
        // cubics from chosen real roots (three, double, triple, integer roots
        // that put exact zeros at bracket ends)
        const double p = u(rng) * 10, q = (i & 1) ? p : u(rng) * 10, r = (i & 2) ? q : u(rng) * 10;
        check(1.0, -(p + q + r), p * q + q * r + r * p, -p * q * r);
        const double ip = (double)(int)(u(rng) * 5), iq = (double)(int)(u(rng) * 5), ir = (double)(int)(u(rng) * 5);
        check(1.0, -(ip + iq + ir), ip * iq + iq * ir + ir * ip, -ip * iq * ir);
        check(2.0, -2.0 * (ip + iq + ir), 2.0 * (ip * iq + iq * ir + ir * ip), -2.0 * ip * iq * ir);
    }
    // special operands
    const double sp[] = {0.0, -0.0, 1.0, -1.0, 1e-300, 1e300, __builtin_inf(), -__builtin_inf(), __builtin_nan("")};
    for (double a : sp)
        for (double b : sp)
            for (double c : sp) check(1.0, a, b, c);
    printf("checked %ld cubics (%ld with three roots), %ld mismatches\n", checked, three, bad);
    return bad != 0;
}
