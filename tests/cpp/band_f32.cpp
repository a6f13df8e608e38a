// The packed-fp32 rectification pre-band of k_score_fm (csrc/kernels.hip
// RPairBand / rpb_setup / rpb_scale / rpb_orient) restated per lane in host
// fp32 (fmaf is correctly rounded, -ffp-contract=off keeps every other
// operation a separate rounding, as on the device), against the fp64 bands it
// stands in for (scale_band / orient_band, restated from the same file).
// The claim checked: a pair the fp32 pre-band rejects is rejected by the
// fp64 band too (so the exact pass still sees every pair the fp64 band kept,
// and the results cannot change).  Cases: random models and features,
// features placed by bisection ON the fp64 band's edges (scale s = lo t^3 or
// hi t^3 to the last ulp; orientation angle where min(u, v) = tan_tau max),
// t near 0, scales near the range limits, huge / NaN coordinates, subnormal
// model terms.  Prints "violations 0" and the rejection rates.
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

namespace {

constexpr double kU = 0x1p-24;

float fpb_up(double v) { return (v < 1e30) ? (float)(v * (1.0 + 1e-6)) + 1e-30f : INFINITY; }

struct Hyp {
    double h7, h8, lo, hi, cf, sf;
};

// ---- fp64 bands (kernels.hip scale_band, orient_band) ----
bool scale_band64(double x, double y, double s, const Hyp& q) {
    const double t = (-q.h7 * x - q.h8 * y) + 1.0;
    const double t3 = (t * t) * t;
    const bool odd = !(t > 0.0 && s > 0.0);
    return odd | !(s < q.lo * t3 || s > q.hi * t3);
}
bool orient_band64(double x, double y, double ct, double st, const Hyp& q, double tan_tau) {
    const double numer = (-x * st + y * ct) * q.h7 + st;
    const double denom = (x * st - y * ct) * q.h8 + ct;
    const double u = std::fabs(denom * q.cf + numer * q.sf);
    const double v = std::fabs(numer * q.cf - denom * q.sf);
    const double mx = std::fmax(u, v);
    return !(std::fmin(u, v) > tan_tau * mx) | !(mx >= 0x1p-900);
}

// ---- fp32 pre-band (kernels.hip rpb_setup / rpb_scale / rpb_orient), one hypothesis ----
struct RB {
    float nh7, nh8, tb, lo, hi, h7, h8, cf, sf, tq, eq;
};
RB setup(const Hyp& q, double X0, double Y0, double X1, double Y1, double tan_tau) {
    RB b;
    const double a7 = std::fabs(q.h7), a8 = std::fabs(q.h8);
    const double tb = 6.0 * kU * ((a7 * X0 + a8 * Y0) + 1.0) + (X0 + Y0) * 0x1p-140;
    b.nh7 = (float)(-q.h7);
    b.nh8 = (float)(-q.h8);
    b.tb = fpb_up(tb);
    const bool lo_ok = q.lo >= 0x1p-20 && q.lo <= 0x1p20;
    const bool hi_ok = q.hi >= 0x1p-20 && q.hi <= 0x1p20;
    b.lo = lo_ok ? (float)(q.lo * (1.0 - 0x1p-19)) : 0.0f;
    b.hi = hi_ok ? (float)(q.hi * (1.0 + 0x1p-19)) : INFINITY;
    const double G = X1 + Y1;
    const double e = 32.0 * kU * (G * std::fmax(a7, a8) + 1.0) + G * 0x1p-140 + 0x1p-90;
    const double tq = tan_tau * (1.0 + 0x1p-18);
    b.h7 = (float)q.h7;
    b.h8 = (float)q.h8;
    b.cf = (float)q.cf;
    b.sf = (float)q.sf;
    b.tq = fpb_up(tq);
    b.eq = fpb_up(e * (1.0 + tq) * 1.01);
    return b;
}
bool scale_reject32(const RB& b, double x, double y, double s) {
    const float xf = (float)x, yf = (float)y;
    const float sf = (s >= 0x1p-100 && s <= 0x1p100) ? (float)s : NAN;
    const float t = fmaf(b.nh7, xf, fmaf(b.nh8, yf, 1.0f));
    const float tl = t - b.tb, th = t + b.tb;
    const float a = ((tl * tl) * tl) * b.lo;
    const float c = ((th * th) * th) * b.hi;
    return tl > 0.0f && (sf < a || sf > c);
}
bool orient_reject32(const RB& b, double x, double y, double ct, double st) {
    const float xf = (float)x, yf = (float)y, ctf = (float)ct, stf = (float)st;
    const float g = fmaf(xf, stf, -(yf * ctf));
    const float N = fmaf(-g, b.h7, stf), D = fmaf(g, b.h8, ctf);
    const float U = std::fabs(fmaf(D, b.cf, N * b.sf));
    const float V = std::fabs(fmaf(N, b.cf, -(D * b.sf)));
    const float P1 = fmaf(-b.tq, V, U), P2 = fmaf(-b.tq, U, V);
    return P1 > b.eq && P2 > b.eq;
}

}  // namespace

int main(int argc, char** argv) {
    const long iters = argc > 1 ? atol(argv[1]) : 400;
    std::mt19937_64 rng(20261018);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long r64s = 0, r32s = 0, r64o = 0, r32o = 0;
    long viol = 0, n64s = 0, n32s = 0, n64o = 0, n32o = 0, pairs_s = 0, pairs_o = 0, edge_s = 0, edge_o = 0;
    for (long it = 0; it < iters; ++it) {
        // a class of features (scale: x, y, s; orientation: x, y, theta)
        const int n = 256;
        const double span = (it % 7 == 0) ? 1e6 : (it % 7 == 1 ? 1.0 : 4000.0);
        std::vector<double> x(n), y(n), s(n), th(n);
        for (int i = 0; i < n; ++i) {
            x[i] = (U(rng) - 0.3) * span;
            y[i] = (U(rng) - 0.3) * span;
            s[i] = std::exp((U(rng) - 0.5) * 6.0);
            th[i] = U(rng) * 6.283185307179586;
        }
        if (it % 11 == 0) s[3] = 0x1p-101, s[4] = 0x1p-99, s[5] = 0x1p100, s[6] = -1.0, s[7] = NAN, s[8] = 0.0;
        if (it % 13 == 0) x[9] = 1e200;
        if (it % 17 == 0) y[10] = NAN;
        double X = 0, Y = 0;
        bool bad = false;
        for (int i = 0; i < n; ++i) {
            if (!std::isfinite(x[i]) || !std::isfinite(y[i])) bad = true;
            else X = std::fmax(X, std::fabs(x[i])), Y = std::fmax(Y, std::fabs(y[i]));
        }
        if (bad) X = Y = HUGE_VAL;
        // models: h7, h8 so that t = 1 - h7 x - h8 y spans positive values
        // and crosses 0 for some features; alpha^3 around 1 (and extremes)
        for (int m = 0; m < 24; ++m) {
            Hyp q;
            const double hs = (m % 5 == 0) ? 1.0 / span : 0.2 / span;
            q.h7 = (U(rng) - 0.5) * hs;
            q.h8 = (U(rng) - 0.5) * hs;
            if (m == 7) q.h7 = 1e-42, q.h8 = -3e-41;                 // subnormal in fp32
            const double tau = 0.01 + U(rng) * 0.6;
            double ac = std::exp((U(rng) - 0.5) * 4.0);
            if (m == 11) ac = 1e-8;
            if (m == 12) ac = 1e8;
            const double band0 = std::exp(tau) * (1.0 + 1e-9);
            q.lo = (1.0 / ac) * (1.0 / band0) * (1.0 - 1e-9);
            q.hi = (1.0 / ac) * band0 * (1.0 + 1e-9);
            const double phi = (U(rng) - 0.5) * 2.0;
            q.cf = std::cos(phi);
            q.sf = std::sin(phi);
            if (m == 13) q.cf = NAN;
            const double tan_tau = (tau < 0.7) ? std::tan(tau) * (1.0 + 1e-6) + 1e-12 : HUGE_VAL;
            const RB b = setup(q, X, Y, X, Y, tan_tau);
            for (int i = 0; i < n; ++i) {
                // scale: the feature as drawn, and placed on both band edges
                double ss[5] = {s[i], s[i], s[i], s[i], s[i]};
                const double t = (-q.h7 * x[i] - q.h8 * y[i]) + 1.0;
                if (t > 0.0 && std::isfinite(t)) {
                    const double t3 = (t * t) * t;
                    const double e0 = q.lo * t3, e1 = q.hi * t3;
                    ss[1] = std::nextafter(e0, 0.0);                   // just rejected by fp64
                    ss[2] = e0;
                    ss[3] = std::nextafter(e1, HUGE_VAL);              // just rejected by fp64
                    ss[4] = e1 * (1.0 + 0x1p-22);
                    edge_s += 4;
                }
                for (int e = 0; e < 5; ++e) {
                    const double sv = ss[e];
                    const bool keep64 = scale_band64(x[i], y[i], sv, q);
                    const bool rej32 = scale_reject32(b, x[i], y[i], sv);
                    if (e == 0) r64s += !keep64, r32s += rej32;
                    ++pairs_s;
                    n64s += !keep64;
                    n32s += rej32;
                    if (rej32 && keep64) {
                        if (++viol <= 10)
                            printf("scale violation: x %.17g y %.17g s %.17g h7 %.17g h8 %.17g lo %.17g hi %.17g\n",
                                   x[i], y[i], sv, q.h7, q.h8, q.lo, q.hi);
                    }
                }
                // orientation: the feature's angle, and angles on the band's
                // edges found by bisection of f(theta) = min - tan_tau max
                double tv[3] = {th[i], th[i], th[i]};
                if (std::isfinite(tan_tau) && std::isfinite(q.cf)) {
                    auto f = [&](double a) {
                        const double ct = std::cos(a), st = std::sin(a);
                        const double numer = (-x[i] * st + y[i] * ct) * q.h7 + st;
                        const double denom = (x[i] * st - y[i] * ct) * q.h8 + ct;
                        const double u = std::fabs(denom * q.cf + numer * q.sf);
                        const double v = std::fabs(numer * q.cf - denom * q.sf);
                        return std::fmin(u, v) - tan_tau * std::fmax(u, v);
                    };
                    for (int e = 1; e < 3; ++e) {
                        double lo = th[i], hi = th[i] + (e == 1 ? 0.05 : -0.05);
                        double flo = f(lo), fhi = f(hi);
                        if (!(std::isfinite(flo) && std::isfinite(fhi)) || (flo > 0) == (fhi > 0)) continue;
                        for (int k = 0; k < 80; ++k) {
                            const double mid = 0.5 * (lo + hi);
                            if ((f(mid) > 0) == (flo > 0)) lo = mid;
                            else hi = mid;
                        }
                        tv[e] = f(lo) > 0 ? lo : hi;                  // the rejected side, at the edge
                        ++edge_o;
                    }
                }
                for (int e = 0; e < 3; ++e) {
                    const double a = tv[e];
                    const double ct = std::cos(a), st = std::sin(a);
                    const bool keep64 = orient_band64(x[i], y[i], ct, st, q, tan_tau);
                    const bool rej32 = orient_reject32(b, x[i], y[i], ct, st);
                    if (e == 0) r64o += !keep64, r32o += rej32;
                    ++pairs_o;
                    n64o += !keep64;
                    n32o += rej32;
                    if (rej32 && keep64) {
                        if (++viol <= 10)
                            printf("orientation violation: x %.17g y %.17g theta %.17g h7 %.17g h8 %.17g\n", x[i],
                                   y[i], a, q.h7, q.h8);
                    }
                }
            }
        }
    }
    printf("scale pairs %ld (edge %ld): fp64 rejects %ld, fp32 rejects %ld\n", pairs_s, edge_s, n64s, n32s);
    printf("orientation pairs %ld (edge %ld): fp64 rejects %ld, fp32 rejects %ld\n", pairs_o, edge_o, n64o, n32o);
    printf("drawn pairs only: scale fp64 rejects %ld, fp32 %ld; orientation fp64 %ld, fp32 %ld\n", r64s, r32s, r64o,
           r32o);
    printf("violations %ld\n", viol);
    return viol == 0 ? 0 : 1;
}
