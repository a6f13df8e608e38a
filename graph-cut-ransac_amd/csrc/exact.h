// exact.h -- inlier decisions in the reference's arithmetic (glibc).
//
// The reference evaluates std::log, std::pow(t, -3.0) and std::atan2 from glibc
// inside every residual (solver_rectifying_homography_three_sift.hpp:293-317,
// ..._two_sift.hpp:621-665, model.h:156-204) and in the 2-SIFT minimal solver's
// phi (..._two_sift.hpp:341), and decides with them: MSAC `r^2 <= 2.25 thr^2`
// (MSAC_scoring_function.hpp:53-107), the LO relabel `r^2 <= (1.5 thr)^2`
// (GCRANSAC.h:921-942), the 1-class labeling's `fl(r^2 / T) < 1`
// (GCRANSAC.h:789-870) and the final masks.  The kernels evaluate the detmath
// twins (detmath.h), whose results can differ from glibc's in the last bits.
//
// The kernels evaluate the residual VALUES of rect.h ("values": the same
// residuals in a division-light form over the detmath twins), whose deviation
// from the reference's glibc residuals is bounded.  For the residual r (r^2
// the squared residual) of one (feature, model) pair,
//   scale:        |r_value - r_glibc| <= 1.0e-15 + 5.2e-16 r
//     (the value's argument (ac ps) / ((t t) t) carries 4 roundings, the
//     reference's ac (ps pow(t, -3)) glibc pow's 0.52 ulp and 2 roundings:
//     the two arguments agree within 7 ulp = 1.0e-15 relative, i.e. their
//     logs within 1.0e-15 absolute; dm_log <= 1.8 ulp and glibc log <= 0.52
//     ulp of r: 2.3 ulp(r) <= 5.2e-16 r), valid while ps ac, t^3 and the
//     argument are normal numbers and the argument is not at the cut
//     (scale_unsafe);
//   orientation:  |r_value - r_glibc| <= 5e-15
//     (value: the rotation by the model's twin cos / sin (< 1.5 ulp each) moves
//     the direction by < 6e-16 rad, the division and dm's atan polynomial add
//     < 3.1e-16; a minimal model's twin phi against its glibc one 1.3e-15;
//     reference: glibc atan2 <= 1 ulp of |a| <= pi and the clipping's roundings
//     of ulp(2 pi) / 2, <= 2.2e-15; the rare reference-formula fallback of the
//     value keeps round 3's bound 3.6e-15).
// tests/test_exact.py measures the deviations on random pairs far inside
// these bounds.
//
// The kernels therefore flag every pair whose twin r^2 lies within the band
// [lo, hi] = [((sqrt(T) - D)(1 - 1e-12))^2, ((sqrt(T) + D)(1 + 1e-12))^2]
// around a decision threshold T, with D = kDevScale / kDevOrient (the bounds
// above with a 4-8x margin; the 1e-12 relative margin covers the relative
// term, sqrt's and the squares' roundings).  Outside the band the twin and the
// glibc residual fall on the same side of T (and of fl(r^2 / T) < 1, which
// only differs from r^2 < T within 2^-53 T).  Inside it the host recomputes
// the pair with glibc (engine.cpp, RunnerT::exact_*).  The conservative
// prefilters of the batch scorers keep every flagged pair: their slack is
// >= 1e-9 absolute in log scale and tan(1.5 thr) 1e-6 + 1e-12 in angle.
//
// Values: the MSAC running sums add the value r^2 of the pairs the glibc
// decision makes inliers (a definition, restated by the oracle's TWIN mode);
// a pair whose decision the recheck flips makes the host re-fold that model's
// sums in that definition.  A flip moves the finished score by
// |1 - r^2 / T| <= (hi - lo) / T (r^2 is inside the band), i.e. by ~1e-13 at
// the bench thresholds: score comparisons between different hypotheses are
// unaffected unless their scores tie to that level.
#pragma once

#include "gcr_hd.h"

namespace gcr {

constexpr double kDevScale = 4e-15;      // bound on |r_value - r_glibc|, scale class (absolute part)
constexpr double kDevScaleRel = 1e-12;   // ... its relative part (and the band's rounding margin)
constexpr double kDevOrient = 4e-14;     // orientation class (radians)

// Per class c: a pair is flagged iff |r2 - mid[c]| <= half[c].
struct FlagBand {
    double mid[2];
    double half[2];
};

GCR_HD bool in_flag_band(double r2, double mid, double half) { return __builtin_fabs(r2 - mid) <= half; }

// The inlier rule of a squared residual (k_mask, the LO lists, the host's
// glibc recheck): rule 0 r^2 <= T (MSAC_scoring_function.hpp:64-66, the LO
// relabel GCRANSAC.h:921-942); rule 2 the 1-class labeling of an empty
// neighbourhood graph (GCRANSAC.h:789-811, gcransac_python.cpp:63-68): SINK iff
// the terminal capacity of add_term1(clamp(r^2 / T) energies) is < 0.
GCR_HD bool mask_rule(double r2, int rule, double T, double lambda) {
    if (rule == 2) {
        const double oml = 1.0 - lambda;
        double q = r2 / T;
        q = (q < 0.0) ? 0.0 : ((1.0 < q) ? 1.0 : q);      // std::clamp
        const double energy = 1.0 - q;
        const double tr = (r2 <= T) ? (0.0 - oml * energy) : (oml * (1.0 - energy) - 0.0);
        return tr < 0.0;
    }
    return r2 <= T;
}

// host-side helpers (launchers and engine)
// the band around threshold T (squared) of class c (0 scale, 1 orientation)
inline void flag_band_1(double T, int c, double& mid, double& half) {
    const double D = c == 0 ? kDevScale : kDevOrient;
    const double rT = sqrt(T);
    double rlo = (rT - D) * (1.0 - kDevScaleRel), rhi = (rT + D) * (1.0 + kDevScaleRel);
    if (!(rlo > 0.0)) rlo = 0.0;
    const double lo = rlo * rlo, hi = rhi * rhi;
    mid = 0.5 * (lo + hi);
    half = 0.5 * (hi - lo) * (1.0 + 1e-9) + 1e-300;
    if (!(T >= 0.0)) {                   // NaN threshold: nothing is an inlier on either side
        mid = 0.0;
        half = -1.0;
    }
}
inline FlagBand flag_band(const double T[2]) {
    FlagBand b;
    for (int c = 0; c < 2; ++c) flag_band_1(T[c], c, b.mid[c], b.half[c]);
    return b;
}

// Score comparisons in the reference's arithmetic.
// With the decisions glibc's, a hypothesis's MSAC score in the value
// definition (what the kernels fold) and in glibc's (what the reference
// compares, GCRANSAC.h:440, :662, :1036, :1054) differ only through the
// inliers' r^2 values and the two sums' roundings.  For counts n_c,
//   |Δv_c|   <= n_c d_c + 2 n_c^2 u T_c            (d_c: |r^2_value - r^2_glibc|
//   |Δtot|   <= sum_c n_c d_c + 2 n^2 u max T_c      of one inlier, r <= sqrt(T_c) + D_c;
//                                                   each sequential sum of n terms
//                                                   of size <= T_c rounds by <= (n-1) u n T_c)
//   |Δscore| <= |Δtot| + sum_c (1 + 1/T_c) |Δv_c| + 16 u (|tot| + |v| + |v'| + |score|)
// (the finish's few operations round on both sides), doubled for margin.
// Two scores further apart than the sum of their bounds compare the same in
// both arithmetics; closer ones are compared in glibc on the host.
struct ScoreBound {
    double a[2];     // per inlier of class c
    double b[2];     // per (inlier of class c)^2
    double g;        // per (inlier of both classes)^2
    bool finite;
};
inline ScoreBound score_bound(const double T[2], int K) {
    const double u = 0x1p-53;
    ScoreBound sb{{0.0, 0.0}, {0.0, 0.0}, 0.0, true};
    double tmax = 0.0;
    for (int c = 0; c < K; ++c) {
        const double Tc = T[c];
        if (!(Tc > 0.0) || !(Tc < HUGE_VAL)) {
            sb.finite = false;
            continue;
        }
        const double R0 = sqrt(Tc) * (1.0 + 1e-9) + 1e-12;
        const double D = c == 0 ? 4.0 * (1.0e-15 + 5.2e-16 * R0) : kDevOrient;
        const double d = D * (2.0 * (R0 + D) + D);
        const double inv = 1.0 + 1.0 / Tc;
        sb.a[c] = 2.0 * (d * inv + d + 16.0 * u * (2.0 * Tc + 2.0));
        sb.b[c] = 2.0 * (2.0 * u * Tc * inv);
        if (Tc > tmax) tmax = Tc;
    }
    sb.g = 2.0 * 2.0 * u * tmax;
    return sb;
}
// the bound of one hypothesis (+inf when a threshold is not positive finite
// and the class has inliers)
GCR_HD double score_dev(const ScoreBound& sb, double n0, double n1, double score) {
    if (!sb.finite && (n0 > 0.0 || n1 > 0.0)) return __builtin_huge_val();
    const double n = n0 + n1;
    return ((n0 * (sb.a[0] + n0 * sb.b[0]) + n1 * (sb.a[1] + n1 * sb.b[1])) + n * n * sb.g) +
           32.0 * 0x1p-53 * __builtin_fabs(score);
}

// A rectification model whose scale residuals the bound above does not cover:
// sqrt(T) >= 60 (arguments of log near the ends of the normal range),
// alpha^3 outside [2^-200, 2^200], a problem with a positive finite scale
// outside [2^-200, 2^200] (`scales_ok` false) -- with both in range, log's
// argument within [e^-60, e^60] keeps ac ps, t^3, t^-3 and rs normal, so the
// error analysis holds; other features give inf / NaN on both sides -- or the
// rectified-scale cut rs < 1e-9 (the value's arg < ac 1e-9, scale_sq_value)
// inside the inlier band (|log(alpha^3 1e-9)| close to sqrt(T): the value's
// and glibc's sides of the cut can differ).  The engine decides every pair of such a model on
// the host.  `solver`: 0, 1 (original: arg = rs / alpha^3) or 2.
inline bool scale_unsafe(int solver, double alpha, double T0, bool scales_ok) {
    const double rT = sqrt(T0);
    if (!(rT < 60.0) || !scales_ok) return true;
    const double ac = (alpha * alpha) * alpha;
    if (!(ac >= 0x1p-200 && ac <= 0x1p200)) return true;
    const double at_cut = fabs(log(solver == 1 ? 1e-9 / ac : ac * 1e-9));
    return !(at_cut > rT + 1e-3);
}
// the problem-level half of it: every positive finite scale feature in
// [2^-200, 2^200]
inline bool scales_in_range(const double* s, size_t n) {
    for (size_t i = 0; i < n; ++i)
        if (s[i] > 0.0 && s[i] < HUGE_VAL && !(s[i] >= 0x1p-200 && s[i] <= 0x1p200)) return false;
    return true;
}

}  // namespace gcr
