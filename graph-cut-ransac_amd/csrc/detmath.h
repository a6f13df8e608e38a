// detmath.h -- deterministic fp64 transcendental kernels for the MSAC hot loop.
//
// The reference evaluates std::log, std::pow(t, -3.0) and std::atan2 from glibc
// inside every residual (solver_rectifying_homography_three_sift.hpp:293-317,
// ..._two_sift.hpp:621-665, model.h:156-165, 194-204).  gfx950 has no fp64
// transcendental instructions and ocml's expansions are not glibc's, so the GPU
// engine evaluates these three functions with the code below, compiled
// identically for the host (engine, LO/refit) and for gfx950 (kernels).  All
// other arithmetic is IEEE +,-,*,/,sqrt, which both sides round identically.
//
//   dm_log      fdlibm e_log.c reduction and minimax polynomial (< 1 ulp),
//               the two fdlibm tail formulas selected without branches.
//   dm_pow_m3   t^-3 via a double-double t^3 and one Newton correction of the
//               IEEE reciprocal (nearly correctly rounded).
//   dm_atan2    fdlibm e_atan2.c / s_atan.c; the five-way argument reduction
//               of s_atan.c is rewritten as one (a*x+b)/(c*x+d) with selected
//               coefficients, which is the same IEEE operation sequence as each
//               fdlibm branch but runs without lane divergence.
//
// The accuracy against glibc/mpmath is pinned by tests/test_detmath.py; the
// oracle's "twin" mode uses these same three functions so GPU-vs-oracle
// comparisons are bitwise, and its "glibc" mode is cross-checked against twin.
#pragma once

#include "gcr_hd.h"

namespace gcr {
namespace dm {

constexpr double cf(uint64_t u) { return __builtin_bit_cast(double, u); }

// ------------------------------------------------------------------ log ----
GCR_HD double dm_log(double x) {
    constexpr double ln2_hi = cf(0x3fe62e42fee00000ull);
    constexpr double ln2_lo = cf(0x3dea39ef35793c76ull);
    constexpr double two54 = cf(0x4350000000000000ull);
    constexpr double Lg1 = cf(0x3fe5555555555593ull);
    constexpr double Lg2 = cf(0x3fd999999997fa04ull);
    constexpr double Lg3 = cf(0x3fd2492494229359ull);
    constexpr double Lg4 = cf(0x3fcc71c51d8e78afull);
    constexpr double Lg5 = cf(0x3fc7466496cb03deull);
    constexpr double Lg6 = cf(0x3fc39a09d078c69full);
    constexpr double Lg7 = cf(0x3fc2f112df3e5244ull);

    uint64_t u = as_u64(x);
    int32_t hx = (int32_t)(u >> 32);
    uint32_t lx = (uint32_t)u;
    int32_t k = 0;
    if (hx < 0x00100000) {                       // x < 2^-1022 (incl. <= 0)
        if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -HUGE_VAL;   // log(+-0)
        if (hx < 0) return __builtin_nan("");       // log(<0) = NaN
        k -= 54;
        x *= two54;                              // subnormal: scale up
        u = as_u64(x);
        hx = (int32_t)(u >> 32);
    }
    if (hx >= 0x7ff00000) return x + x;          // +inf or NaN
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    const int32_t i = (hx + 0x95f64) & 0x100000;
    // normalise x (or x/2) into [sqrt(2)/2, sqrt(2))
    x = as_f64(((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (uint64_t)(uint32_t)as_u64(x));
    k += (i >> 20);
    const double f = x - 1.0;
    const double dk = (double)k;
    const double s = f / (2.0 + f);
    const double z = s * s;
    const double w = z * z;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    const double R = t2 + t1;
    const int32_t sel = (hx - 0x6147a) | (0x6b851 - hx);
    const double hfsq = 0.5 * f * f;
    const double ra = dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    const double rb = dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
    return sel > 0 ? ra : rb;
}

// --------------------------------------------------------------- t^-3 -----
GCR_HD double pm3_core(double t) {
    const double h = t * t;
    const double l = fma_rn(t, t, -h);           // t^2 = h + l exactly
    const double H = h * t;
    const double L = fma_rn(h, t, -H) + l * t;   // t^3 ~= H + L
    const double y = 1.0 / H;
    double e = fma_rn(-y, H, 1.0);               // 1 - y*H (exact)
    e = fma_rn(-y, L, e);                        // 1 - y*(H + L)
    return fma_rn(y, e, y);
}

GCR_HD double dm_pow_m3(double t) {
    const double a = __builtin_fabs(t);
    if (a >= 0x1p-300 && a <= 0x1p300) return pm3_core(t);
    if (a != a) return t + t;                             // NaN
    if (a == 0.0) return 1.0 / (t * t * t);               // +-0 -> +-inf
    if (a == HUGE_VAL) return (t > 0.0) ? 0.0 : -0.0;     // +-inf -> +-0
    // extreme finite |t|: t = m 2^e, m in [0.5, 1)
    int e = 0;
    const double m = frexp(t, &e);
    return ldexp(pm3_core(m), -3 * e);
}

// -------------------------------------------------------------- atan2 -----
// atan(x) for x >= 0 (finite or +inf), fdlibm s_atan.c.
GCR_HD double dm_atan_nonneg(double x) {
    constexpr double aT0 = cf(0x3fd555555555550dull);
    constexpr double aT1 = cf(0xbfc999999998ebc4ull);
    constexpr double aT2 = cf(0x3fc24924920083ffull);
    constexpr double aT3 = cf(0xbfbc71c6fe231671ull);
    constexpr double aT4 = cf(0x3fb745cdc54c206eull);
    constexpr double aT5 = cf(0xbfb3b0f2af749a6dull);
    constexpr double aT6 = cf(0x3fb10d66a0d03d51ull);
    constexpr double aT7 = cf(0xbfadde2d52defd9aull);
    constexpr double aT8 = cf(0x3fa97b4b24760debull);
    constexpr double aT9 = cf(0xbfa2b4442c6a6c2full);
    constexpr double aT10 = cf(0x3f90ad3ae322da11ull);
    constexpr double hi0 = cf(0x3fddac670561bb4full), lo0 = cf(0x3c7a2b7f222f65e2ull);
    constexpr double hi1 = cf(0x3fe921fb54442d18ull), lo1 = cf(0x3c81a62633145c07ull);
    constexpr double hi2 = cf(0x3fef730bd281f69bull), lo2 = cf(0x3c7007887af0cbbdull);
    constexpr double hi3 = cf(0x3ff921fb54442d18ull), lo3 = cf(0x3c91a62633145c07ull);

    if (x >= 0x1p66) return hi3 + lo3;           // also +inf
    // reduction: xr = (ca*x + cb) / (cc*x + cd), result = hi - ((xr*S - lo) - xr)
    double ca = 1.0, cb = 0.0, cc = 0.0, cd = 1.0, hi = 0.0, lo = 0.0;
    if (x >= 0.4375) {
        if (x < 0.6875)      { ca = 2.0; cb = -1.0;  cc = 1.0; cd = 2.0; hi = hi0; lo = lo0; }
        else if (x < 1.1875) { ca = 1.0; cb = -1.0;  cc = 1.0; cd = 1.0; hi = hi1; lo = lo1; }
        else if (x < 2.4375) { ca = 1.0; cb = -1.5;  cc = 1.5; cd = 1.0; hi = hi2; lo = lo2; }
        else                 { ca = 0.0; cb = -1.0;  cc = 1.0; cd = 0.0; hi = hi3; lo = lo3; }
    }
    const double xr = (ca * x + cb) / (cc * x + cd);
    const double z = xr * xr;
    const double w = z * z;
    const double s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const double s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    return hi - ((xr * (s1 + s2) - lo) - xr);
}

GCR_HD double dm_atan2(double y, double x) {
    constexpr double pi_o_4 = cf(0x3fe921fb54442d18ull);
    constexpr double pi_o_2 = cf(0x3ff921fb54442d18ull);
    constexpr double pi = cf(0x400921fb54442d18ull);
    constexpr double pi_lo = cf(0x3ca1a62633145c07ull);

    const uint64_t ux = as_u64(x), uy = as_u64(y);
    const int32_t hx = (int32_t)(ux >> 32), hy = (int32_t)(uy >> 32);
    const int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    const uint32_t lx = (uint32_t)ux, ly = (uint32_t)uy;
    if (x != x || y != y) return x + y;          // NaN
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);   // 2*sign(x) + sign(y)

    if ((iy | (int32_t)ly) == 0) {               // y = +-0
        if (m < 2) return y;
        return (m == 2) ? pi : -pi;
    }
    if ((ix | (int32_t)lx) == 0) return (hy < 0) ? -pi_o_2 : pi_o_2;   // x = +-0
    if (ix == 0x7ff00000) {                      // x = +-inf
        if (iy == 0x7ff00000) {
            switch (m) {
                case 0: return pi_o_4;
                case 1: return -pi_o_4;
                case 2: return 3.0 * pi_o_4;
                default: return -3.0 * pi_o_4;
            }
        }
        switch (m) {
            case 0: return 0.0;
            case 1: return -0.0;
            case 2: return pi;
            default: return -pi;
        }
    }
    if (iy == 0x7ff00000) return (hy < 0) ? -pi_o_2 : pi_o_2;          // y = +-inf

    const int32_t k = (iy - ix) >> 20;
    double z;
    if (k > 60) z = pi_o_2 + 0.5 * pi_lo;        // |y/x| > 2^60
    else if (hx < 0 && k < -60) z = 0.0;         // |y|/x < -2^60
    else z = dm_atan_nonneg(__builtin_fabs(y / x));
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// -------------------------------------------------------- angle clipping ---
// std::fmod(a, c) for the reference's clipAngle (math_utils.hpp:78-88).  For
// |a| < 2c the remainder is a or a -+ c, both exact (Sterbenz); every call site
// on the hot path stays in that range.  Larger arguments (and inf/NaN) use the
// platform fmod, which is exact by definition on both sides.
GCR_HD double fmod_2pi(double a) {
    constexpr double c = 2.0 * cf(0x400921fb54442d18ull);   // 2.0 * M_PI
    const double aa = __builtin_fabs(a);
    if (aa < c) return a;
    if (aa < 2.0 * c) return (a > 0.0) ? a - c : a + c;
    return fmod(a, c);
}

GCR_HD double clip_angle(double a) {
    constexpr double c = 2.0 * cf(0x400921fb54442d18ull);
    double r = fmod_2pi(a);
    if (r < 0.0) r += c;
    return r;
}

}  // namespace dm
}  // namespace gcr
