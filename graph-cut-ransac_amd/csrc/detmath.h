// detmath.h -- deterministic fp64 transcendental kernels for the MSAC hot loop.
//
// The reference evaluates std::log, std::pow(t, -3.0) and std::atan2 from glibc
// inside every residual (solver_rectifying_homography_three_sift.hpp:293-317,
// ..._two_sift.hpp:621-665, model.h:156-165, 194-204).  gfx950 has no fp64
// transcendental instructions and ocml's expansions are not glibc's, so the GPU
// engine evaluates its residual VALUES with the code below, compiled
// identically for the host (engine, LO/refit) and for gfx950 (kernels).  All
// other arithmetic is IEEE +,-,*,/,sqrt, which both sides round identically.
// Decisions are the reference's own (glibc), see exact.h.
//
//   dm_log      table-driven (128 subintervals of [0.686, 1.371), logtab.h):
//               log x = k ln2 + log c + log1p(z / c - 1), the quotient as one
//               FMA against the tabulated 1 / c (no division), log1p by its
//               degree-7 Taylor polynomial (|r| <= 2^-8); the subinterval
//               around 1 has c = 1 (log 1 = 0, relative accuracy near 1);
//               < 1.8 ulp (measured max 1.72 ulp on 6M points against long
//               double, glibc 0.52).
//   dm_log_fd   fdlibm e_log.c reduction and minimax polynomial (< 1 ulp),
//               FMA Horner form (round 3's twin; the oracle's PURE_TWIN mode).
//   dm_pow_m3   t^-3 as 1 / ((t t) t) (< 2 ulp).
//   dm_atan2    fdlibm s_atan.c polynomial behind a branch-free two-step
//               reduction (octant swap, then pi/4 shift) with a single IEEE
//               division; special operands out of line (fdlibm e_atan2.c).
//   dm_sincos   sin and cos of a model angle: Cody-Waite reduction by pi/2
//               (fdlibm's 33-bit split) and fdlibm's k_sin / k_cos
//               polynomials (< 1.5 ulp for |x| <= 16).
//
// The accuracy against glibc is pinned by tests/test_exact.py and
// tests/test_oracle_modes.py; the oracle's TWIN mode uses these same functions
// so GPU-vs-oracle comparisons are bitwise.
#pragma once

#include "gcr_hd.h"
#include "logtab.h"

namespace gcr {
namespace dm {

constexpr double cf(uint64_t u) { return __builtin_bit_cast(double, u); }

// ------------------------------------------------------------------ log ----
#if defined(__HIP_DEVICE_COMPILE__)
#define GCR_COLD __attribute__((noinline))
#else
#define GCR_COLD
#endif

constexpr double kLn2Hi = cf(0x3fe62e42fee00000ull);
constexpr double kLn2Lo = cf(0x3dea39ef35793c76ull);

// fdlibm reduction + minimax polynomial for a normal, finite, positive x
// (k already includes any subnormal pre-scaling).
GCR_HD double log_core(uint64_t u, int32_t k) {
    constexpr double Lg1 = cf(0x3fe5555555555593ull);
    constexpr double Lg2 = cf(0x3fd999999997fa04ull);
    constexpr double Lg3 = cf(0x3fd2492494229359ull);
    constexpr double Lg4 = cf(0x3fcc71c51d8e78afull);
    constexpr double Lg5 = cf(0x3fc7466496cb03deull);
    constexpr double Lg6 = cf(0x3fc39a09d078c69full);
    constexpr double Lg7 = cf(0x3fc2f112df3e5244ull);
    int32_t hx = (int32_t)(u >> 32);
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    const int32_t i = (hx + 0x95f64) & 0x100000;
    // normalise x (or x/2) into [sqrt(2)/2, sqrt(2))
    const double x = as_f64(((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (uint64_t)(uint32_t)u);
    k += (i >> 20);
    const double f = x - 1.0;
    const double dk = (double)k;
    const double s = f / (2.0 + f);
    const double z = s * s;
    const double w = z * z;
    const double t1 = w * fma_rn(w, fma_rn(w, Lg6, Lg4), Lg2);
    const double t2 = z * fma_rn(w, fma_rn(w, fma_rn(w, Lg7, Lg5), Lg3), Lg1);
    const double R = t2 + t1;
    const int32_t sel = (hx - 0x6147a) | (0x6b851 - hx);
    const double hfsq = 0.5 * f * f;
    const double ra = dk * kLn2Hi - ((hfsq - (s * (hfsq + R) + dk * kLn2Lo)) - f);
    const double rb = dk * kLn2Hi - ((s * (f - R) - dk * kLn2Lo) - f);
    return sel > 0 ? ra : rb;
}

GCR_COLD GCR_HD double log_special(double x) {
    const uint64_t u = as_u64(x);
    const int32_t hx = (int32_t)(u >> 32);
    const uint32_t lx = (uint32_t)u;
    if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -HUGE_VAL;   // log(+-0)
    if (hx < 0) return __builtin_nan("");                           // log(<0), log(-inf)
    if (hx >= 0x7ff00000) return x + x;                               // +inf, NaN
    return log_core(as_u64(x * cf(0x4350000000000000ull)), -54);    // subnormal: x * 2^54
}

// log(x): fdlibm e_log.c algorithm (< 1 ulp), polynomial in FMA Horner form.
GCR_HD double dm_log_fd(double x) {
    if (!(x >= 0x1p-1022 && x < HUGE_VAL)) return log_special(x);
    return log_core(as_u64(x), 0);
}

// The table of dm_log: (1 / c_i, -log(1 / c_i)) pairs, the same doubles on
// both sides (tools/gen_logtab.py).
#if defined(__HIP_DEVICE_COMPILE__)
static __constant__ double kLogTab[256] = {GCR_LOGTAB_ENTRIES};
#else
static const double kLogTab[256] = {GCR_LOGTAB_ENTRIES};
#endif

// k ln2 with ln2's high part ending in 11 zero bits: exact for |k| <= 1075
constexpr double kLn2HiT = cf(0x3fe62e42fefa3800ull);
constexpr double kLn2LoT = cf(0x3d2ef35793c76730ull);

// table log of a normal, finite, positive x, x = 2^k z, z in [OFF, 2 OFF),
// OFF = 0x1.5fp-1 (1.0 in the middle of subinterval 80)
GCR_HD double log_tab_core(uint64_t ix, int32_t kadj, const double* __restrict__ tab = kLogTab) {
    constexpr uint64_t kOff = 0x3fe5f00000000000ull;
    const uint64_t tmp = ix - kOff;
    const uint32_t i = (uint32_t)(tmp >> 45) & 127u;
    const int32_t k = ((int32_t)(uint32_t)(tmp >> 32) >> 20) + kadj;   // the exponent of x / OFF (32-bit ops)
    const double z = as_f64(ix - (tmp & 0xfff0000000000000ull));
    const double invc = tab[2 * i], logc = tab[2 * i + 1];
    const double r = fma_rn(z, invc, -1.0);                 // z / c - 1, one rounding
    const double kd = (double)k;
    const double w = fma_rn(kd, kLn2HiT, logc);              // k ln2hi exact
    const double hi = w + r;
    const double lo = fma_rn(kd, kLn2LoT, (w - hi) + r);
    // log1p(r) - r = -r^2/2 + r^3/3 - r^4/4 + r^5/5 - r^6/6 + r^7/7 (+ O(r^8) < 1e-20)
    constexpr double A1 = cf(0x3fd5555555555555ull), A2 = -0.25, A3 = cf(0x3fc999999999999aull),
                     A4 = cf(0xbfc5555555555555ull), A5 = cf(0x3fc2492492492492ull);
    const double r2 = r * r;
    const double p = fma_rn(r2, fma_rn(r2, A5, fma_rn(r, A4, A3)), fma_rn(r, A2, A1));
    return fma_rn(r * r2, p, fma_rn(r2, -0.5, lo)) + hi;
}

GCR_COLD GCR_HD double log_tab_special(double x) {
    const uint64_t u = as_u64(x);
    const int32_t hx = (int32_t)(u >> 32);
    const uint32_t lx = (uint32_t)u;
    if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -HUGE_VAL;   // log(+-0)
    if (hx < 0) return __builtin_nan("");                           // log(<0), log(-inf)
    if (hx >= 0x7ff00000) return x + x;                               // +inf, NaN
    return log_tab_core(as_u64(x * cf(0x4350000000000000ull)), -54); // subnormal: x * 2^54
}

// log(x), table-driven, no division (the residuals' log)
GCR_HD double dm_log(double x) {
    if (!(x >= 0x1p-1022 && x < HUGE_VAL)) return log_tab_special(x);
    return log_tab_core(as_u64(x), 0);
}
// the same log reading the table from a copy (k_score_fm keeps one in LDS:
// a dependent lookup in L2 sat on the exact pass's critical path)
GCR_HD double dm_log(double x, const double* __restrict__ tab) {
    if (!(x >= 0x1p-1022 && x < HUGE_VAL)) return log_tab_special(x);
    return log_tab_core(as_u64(x), 0, tab);
}
// the table's size in doubles (for such copies)
constexpr int kLogTabSize = 256;

// --------------------------------------------------------------- t^-3 -----
// t^-3 = 1 / ((t*t)*t): two roundings in the cube and one in the IEEE
// division (< 2 ulp), valid while t^3 is normal (round 3's scale residual;
// the oracle's PURE_TWIN mode).
GCR_HD double pm3_core(double t) { return 1.0 / ((t * t) * t); }

GCR_COLD GCR_HD double pm3_special(double t) {
    const double a = __builtin_fabs(t);
    if (a != a) return t + t;                             // NaN
    if (a == 0.0) return 1.0 / (t * t * t);               // +-0 -> +-inf
    if (a == HUGE_VAL) return (t > 0.0) ? 0.0 : -0.0;     // +-inf -> +-0
    // extreme finite |t|: t = m 2^e, m in [0.5, 1)
    int e = 0;
    const double m = frexp(t, &e);
    return ldexp(pm3_core(m), -3 * e);
}

GCR_HD double dm_pow_m3(double t) {
    const double a = __builtin_fabs(t);
    if (a >= 0x1p-300 && a <= 0x1p300) return pm3_core(t);
    return pm3_special(t);
}

// -------------------------------------------------------------- atan2 -----
// fdlibm s_atan.c odd minimax polynomial, valid for |x| <= 7/16.
GCR_HD double atan_poly(double x, double hi, double lo) {
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
    const double z = x * x;
    const double w = z * z;
    const double s1 = z * fma_rn(w, fma_rn(w, fma_rn(w, fma_rn(w, fma_rn(w, aT10, aT8), aT6), aT4), aT2), aT0);
    const double s2 = w * fma_rn(w, fma_rn(w, fma_rn(w, fma_rn(w, aT9, aT7), aT5), aT3), aT1);
    return hi - ((x * (s1 + s2) - lo) - x);
}

constexpr double kPiO2 = cf(0x3ff921fb54442d18ull);
constexpr double kPiO4 = cf(0x3fe921fb54442d18ull);
constexpr double kPiF = cf(0x400921fb54442d18ull);
constexpr double kPiLo = cf(0x3ca1a62633145c07ull);     // pi - kPiF
constexpr double kPiO4Lo = cf(0x3c81a62633145c07ull);   // pi/4 - kPiO4
constexpr double kPiO2Lo = cf(0x3c91a62633145c07ull);   // pi/2 - kPiO2
constexpr double kTanPiO8 = cf(0x3fda827999fcef32ull);   // tan(pi/8)

// atan(n / d) for 0 <= n <= d, d > 0: the same reduction as dm_atan2's first
// octant (one division), without quadrant restoration
GCR_HD double atan_ratio(double n, double d) {
    const bool red = n > kTanPiO8 * d;
    const double xr = (red ? n - d : n) / (red ? n + d : d);
    return atan_poly(xr, red ? kPiO4 : 0.0, red ? kPiO4Lo : 0.0);
}

// IEEE special operands (NaN, zeros, infinities) as fdlibm e_atan2.c.
GCR_COLD GCR_HD double atan2_special(double y, double x) {
    if (x != x || y != y) return x + y;
    const int32_t hx = (int32_t)(as_u64(x) >> 32), hy = (int32_t)(as_u64(y) >> 32);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (y == 0.0) {
        if (m < 2) return y;
        return (m == 2) ? kPiF : -kPiF;
    }
    if (x == 0.0) return (hy < 0) ? -kPiO2 : kPiO2;
    if (__builtin_fabs(x) == HUGE_VAL) {
        if (__builtin_fabs(y) == HUGE_VAL) {
            switch (m) {
                case 0: return kPiO4;
                case 1: return -kPiO4;
                case 2: return 3.0 * kPiO4;
                default: return -3.0 * kPiO4;
            }
        }
        switch (m) {
            case 0: return 0.0;
            case 1: return -0.0;
            case 2: return kPiF;
            default: return -kPiF;
        }
    }
    return (hy < 0) ? -kPiO2 : kPiO2;                     // y = +-inf, x finite
}

// atan2(y, x) for finite non-zero operands with a two-step, branch-free
// reduction: t = min(|y|,|x|) / max(|y|,|x|) in (0, 1]; for t > tan(pi/8) the
// argument (n - d) / (n + d) is used around pi/4 (one IEEE division either
// way); |reduced| <= tan(pi/8) < 7/16 feeds fdlibm's polynomial.  Octant and
// quadrant are restored with fdlibm's hi/lo constants.  Max error ~1.1 ulp.
GCR_HD double dm_atan2(double y, double x) {
    const double ay = __builtin_fabs(y), ax = __builtin_fabs(x);
    if (!(ay > 0.0 && ay < HUGE_VAL && ax > 0.0 && ax < HUGE_VAL)) return atan2_special(y, x);
    const bool swap = ay > ax;
    const double n = swap ? ax : ay;
    const double d = swap ? ay : ax;
    const bool red = n > kTanPiO8 * d;
    const double xr = (red ? n - d : n) / (red ? n + d : d);
    double a = atan_poly(xr, red ? kPiO4 : 0.0, red ? kPiO4Lo : 0.0);   // atan(n / d)
    if (swap) a = (kPiO2 - a) + kPiO2Lo;
    if (x > 0.0) return (y > 0.0) ? a : -a;
    return (y > 0.0) ? kPiF - (a - kPiLo) : (a - kPiLo) - kPiF;
}

// ------------------------------------------------------------ sin / cos ---
// fdlibm k_sin.c / k_cos.c polynomials on |r| <= pi/4 (tail y = 0)
GCR_HD double ksin(double x) {
    constexpr double S1 = cf(0xbfc5555555555549ull), S2 = cf(0x3f8111111110f8a6ull), S3 = cf(0xbf2a01a019c161d5ull),
                     S4 = cf(0x3ec71de357b1fe7dull), S5 = cf(0xbe5ae5e68a2b9cebull), S6 = cf(0x3de5d93a5acfd57cull);
    const double z = x * x;
    const double v = z * x;
    const double r = fma_rn(z, fma_rn(z, fma_rn(z, fma_rn(z, S6, S5), S4), S3), S2);
    return fma_rn(v, fma_rn(z, r, S1), x);
}
GCR_HD double kcos(double x) {
    constexpr double C1 = cf(0x3fa555555555554cull), C2 = cf(0xbf56c16c16c15177ull), C3 = cf(0x3efa01a019cb1590ull),
                     C4 = cf(0xbe927e4f809c52adull), C5 = cf(0x3e21ee9ebdb4b1c4ull), C6 = cf(0xbda8fae9be8838d4ull);
    const double z = x * x;
    const double r = z * fma_rn(z, fma_rn(z, fma_rn(z, fma_rn(z, fma_rn(z, C6, C5), C4), C3), C2), C1);
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + z * r);
}

// sin and cos of x, |x| <= 16: x = n pi/2 + r with fdlibm's
// 33 + 53-bit split of pi/2 (n pio2_1 exact for |n| < 2^20, the subtraction
// exact by Sterbenz), quadrant n mod 4; < 1.5 ulp.  Larger |x| loses accuracy (callers
// keep to the range); NaN / inf give NaN.
GCR_HD void dm_sincos(double x, double& s, double& c) {
    constexpr double kInvPiO2 = cf(0x3fe45f306dc9c883ull);
    constexpr double kPio2_1 = cf(0x3ff921fb54400000ull);
    constexpr double kPio2_1t = cf(0x3dd0b4611a626331ull);
    const double n = __builtin_rint(x * kInvPiO2);
    const double r = (x - n * kPio2_1) - n * kPio2_1t;
    const double sr = ksin(r), cr = kcos(r);
    const int q = (int)((n == n && __builtin_fabs(n) < 0x1p30) ? n : 0.0) & 3;   // NaN / huge: any quadrant
    const double ss = (q & 1) ? cr : sr, cc = (q & 1) ? sr : cr;
    s = (q & 2) ? -ss : ss;
    c = ((q + 1) & 2) ? -cc : cc;
}

// -------------------------------------------------------- angle clipping ---
// std::fmod(a, c) for the reference's clipAngle (math_utils.hpp:78-88).  For
// |a| < 2c the remainder is a or a -+ c, both exact (Sterbenz); every call site
// on the hot path stays in that range.  Larger arguments (and inf/NaN) use the
// platform fmod, which is exact by definition on both sides.
GCR_COLD GCR_HD double fmod_2pi_slow(double a) { return fmod(a, 2.0 * cf(0x400921fb54442d18ull)); }

GCR_HD double fmod_2pi(double a) {
    constexpr double c = 2.0 * cf(0x400921fb54442d18ull);   // 2.0 * M_PI
    const double aa = __builtin_fabs(a);
    if (!(aa < 2.0 * c)) return fmod_2pi_slow(a);          // |a| >= 4 pi, inf, NaN
    // the remainder keeps the dividend's sign (fmod(-c, c) = -0.0)
    return (aa < c) ? a : ((a < 0.0) ? -(aa - c) : a - c);
}

GCR_HD double clip_angle(double a) {
    constexpr double c = 2.0 * cf(0x400921fb54442d18ull);
    double r = fmod_2pi(a);
    if (r < 0.0) r += c;
    return r;
}

// clip_angle for arguments known to satisfy |a| < 4 pi or to be NaN (atan2
// results and their shifts by pi): the same value as clip_angle, without the
// out-of-line fmod path, branch-free
GCR_HD double clip_angle_small(double a) {
    constexpr double c = 2.0 * cf(0x400921fb54442d18ull);
    const double aa = __builtin_fabs(a);
    const double r = (aa < c) ? a : ((a < 0.0) ? -(aa - c) : a - c);   // NaN stays NaN, unnegated
    return r < 0.0 ? r + c : r;
}

}  // namespace dm
}  // namespace gcr
