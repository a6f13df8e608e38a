// kernels.hip -- gfx950 kernels of the hypothesize-and-verify hot path.
//
//   k_generate   G lanes per outer-iteration slot evaluate its up-to-101
//                attempts (Philox sample -> sample validity -> 3x4 Gauss
//                minimal solve, fp64 registers) G at a time and keep the lowest
//                success (GCRANSAC.h:296-339, solvers' minimal fits)
//   k_score      one lane per hypothesis, features streamed in index order
//                through the scalar unit (uniform addresses), exact sequential
//                MSAC accumulation (MSAC_scoring_function.hpp:53-130): the
//                running sums are bit-identical to the reference's loop order
//   k_mask       one lane per feature, inlier mask of one model (LO relabel,
//                graph-cut labeling, final inlier sets)
//
// Compiled with -ffp-contract=off: every fp64 expression rounds exactly like
// the host restatement.
#include "kernels.h"
#include "philox.h"
#include "qr3.h"

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace gcr {

namespace {

typedef __attribute__((address_space(1))) void gvoid;   // global
typedef __attribute__((address_space(3))) void lvoid;   // LDS

constexpr int kGenBlock = 256;
constexpr int kScoreBlock = 256;
constexpr int kMaskBlock = 256;

// ------------------------------------------------------------- generate ----
// One attempt of one outer-iteration slot: Philox sample -> sample validity ->
// minimal solve.  Attempts of a slot are independent draws (the counter RNG is
// keyed by (slot, attempt)), so they may be evaluated in any order/parallel.
template <int KIND>
GCR_DEVICE bool attempt(const DevProblem& p, uint64_t seed, uint64_t slot, uint32_t a,
                        typename ModelOf<KIND>::type& m) {
    if constexpr (KIND == 3) {
        // homography: 4 correspondences, orientation check, 4-point DLT (geo.h)
        const DevClass& c = p.cls[0];
        uint32_t idx[4];
        WordStream ws(seed, slot, a, kStreamMain, 0);
        if (!sample_distinct<4>(ws, c.n, 4, idx)) return false;
        double x1[4], y1[4], x2[4], y2[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            x1[j] = c.x[idx[j]];
            y1[j] = c.y[idx[j]];
            x2[j] = c.a[idx[j]];
            y2[j] = c.c0[idx[j]];
        }
        if (!valid_sample_h4(x1, y1, x2, y2)) return false;
        return solve_h4(x1, y1, x2, y2, m);
    } else if constexpr (KIND != 2) {
        const DevClass& c = p.cls[0];
        uint32_t idx[3];
        WordStream ws(seed, slot, a, kStreamMain, 0);
        if (!sample_distinct<3>(ws, c.n, 3, idx)) return false;
        double x[3], y[3], pw[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            x[j] = c.x[idx[j]];
            y[j] = c.y[idx[j]];
            pw[j] = c.c0[idx[j]];
        }
        // areAllPointsCollinear on the single consecutive triplet
        if (are_collinear(x[0], y[0], x[1], y[1], x[2], y[2], 1.0)) return false;
        return (KIND == 1) ? solve_scale3<true>(x, y, pw, m) : solve_scale3<false>(x, y, pw, m);
    } else {
        const DevClass& sc = p.cls[0];
        const DevClass& oc = p.cls[1];
        uint32_t si[2], oi[2];
        WordStream ws0(seed, slot, a, kStreamMain, 0);
        if (!sample_distinct<2>(ws0, sc.n, 2, si)) return false;
        WordStream ws1(seed, slot, a, kStreamMain, 1);
        if (!sample_distinct<2>(ws1, oc.n, 2, oi)) return false;
        double sx[2], sy[2], sp[2], ox[2], oy[2], oco[2], osi[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            sx[j] = sc.x[si[j]];
            sy[j] = sc.y[si[j]];
            sp[j] = sc.c0[si[j]];
            ox[j] = oc.x[oi[j]];
            oy[j] = oc.y[oi[j]];
            oco[j] = oc.c0[oi[j]];
            osi[j] = oc.c1[oi[j]];
        }
        if (!valid_sample_sift22(sx, sy, ox, oy, oco, osi)) return false;
        return solve_sift22(sx, sy, sp, ox, oy, oco, osi, m);
    }
}

// G lanes per slot (G | 64, groups aligned inside a wave).  Round r evaluates
// attempts r*G .. r*G+G-1 in parallel; the slot's result is the lowest
// successful attempt, exactly the first success of the reference's sequential
// retry loop (GCRANSAC.h:296-339).  inc = attempt + 1, or 102 if all 101 fail.
template <int KIND, int G>
__global__ __launch_bounds__(kGenBlock) void k_generate(DevProblem p, uint64_t seed, uint64_t slot0,
                                                        uint32_t nslots, uint8_t* __restrict__ inc,
                                                        typename ModelOf<KIND>::type* __restrict__ models) {
    static_assert(G >= 1 && G <= 64 && (64 % G) == 0, "group size");
    const uint32_t tid = blockIdx.x * kGenBlock + threadIdx.x;
    const uint32_t s = tid / G;
    const uint32_t g = tid % G;
    if (s >= nslots) return;                 // whole groups exit together
    const uint64_t slot = slot0 + s;
    const int lane = threadIdx.x & 63;
    const int gbase = lane & ~(G - 1);
    for (uint32_t r = 0; r * G < 101; ++r) {
        const uint32_t a = r * G + g;
        typename ModelOf<KIND>::type m = ModelOf<KIND>::def();
        const bool ok = a < 101 && attempt<KIND>(p, seed, slot, a, m);
        const uint64_t mask = __ballot(ok);
        const uint64_t grp = G == 64 ? mask : (mask >> gbase) & ((1ull << G) - 1ull);
        if (grp) {
            if (g == (uint32_t)__builtin_ctzll(grp)) {
                models[s] = m;
                inc[s] = (uint8_t)(a + 1);
            }
            return;
        }
    }
    if (g == 0) {
        models[s] = ModelOf<KIND>::def();
        inc[s] = 102;
    }
}

// Fundamental matrix: one attempt = Philox sample of 7 correspondences ->
// 7-point solver (fund.h) into a register-resident basis; 0..3 models.  No
// sample-validity test beyond the solver's own rank and orientation checks.
GCR_DEVICE int attempt_f(const DevProblem& p, uint64_t seed, uint64_t slot, uint32_t a, F7Basis& b) {
    const DevClass& c = p.cls[0];
    uint32_t idx[7];
    WordStream ws(seed, slot, a, kStreamMain, 0);
    if (!sample_distinct<7>(ws, c.n, 7, idx)) return 0;
    double x1[7], y1[7], x2[7], y2[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) {
        x1[j] = c.x[idx[j]];
        y1[j] = c.y[idx[j]];
        x2[j] = c.a[idx[j]];
        y2[j] = c.c0[idx[j]];
    }
    return solve_f7_basis(x1, y1, x2, y2, b);
}

// k_generate for the fundamental matrix: a sample yields up to kFModels
// models, stored as hypotheses 3s + k.  inc[3s] = attempt + 1 (102: all 101
// attempts failed); inc[3s + k], k >= 1, = 0 if the k-th model exists (scored,
// no extra iterations) and 255 if not (skipped).  The winning lane rebuilds
// its models from the basis and writes them straight to global memory.
template <int G>
__global__ __launch_bounds__(kGenBlock) void k_generate_f(DevProblem p, uint64_t seed, uint64_t slot0,
                                                          uint32_t nslots, uint8_t* __restrict__ inc,
                                                          GeoModel* __restrict__ models) {
    static_assert(G >= 1 && G <= 64 && (64 % G) == 0, "group size");
    const uint32_t tid = blockIdx.x * kGenBlock + threadIdx.x;
    const uint32_t s = tid / G;
    const uint32_t g = tid % G;
    if (s >= nslots) return;
    const uint64_t slot = slot0 + s;
    const int lane = threadIdx.x & 63;
    const int gbase = lane & ~(G - 1);
    for (uint32_t r = 0; r * G < 101; ++r) {
        const uint32_t a = r * G + g;
        F7Basis b;
        const int cnt = a < 101 ? attempt_f(p, seed, slot, a, b) : 0;
        const uint64_t mask = __ballot(cnt > 0);
        const uint64_t grp = G == 64 ? mask : (mask >> gbase) & ((1ull << G) - 1ull);
        if (grp) {
            if (g == (uint32_t)__builtin_ctzll(grp)) {
                GeoModel* out = models + (size_t)kFModels * s;
                uint8_t* oi = inc + (size_t)kFModels * s;
                int k = 0;
#pragma unroll
                for (int q = 0; q < 3; ++q)
                    if (b.valid & (1u << q)) {
                        double fm[9];
                        f7_model(b, f7_root(b, q), fm);
                        for (int j = 0; j < 9; ++j) out[k].h[j] = fm[j];
                        ++k;
                    }
                for (int q = k; q < kFModels; ++q) out[q] = default_geo();
                oi[0] = (uint8_t)(a + 1);
                oi[1] = cnt > 1 ? 0 : 255;
                oi[2] = cnt > 2 ? 0 : 255;
            }
            return;
        }
    }
    if (g == 0) {
#pragma unroll
        for (int q = 0; q < kFModels; ++q) {
            models[(size_t)kFModels * s + q] = default_geo();
            inc[(size_t)kFModels * s + q] = q == 0 ? 102 : 255;
        }
    }
}

// k_generate_f with widening groups.  A wave starts with S = 64 / G slots of
// G lanes each.  After every round the lanes of finished slots go to the
// unfinished ones: with k slots left, each gets 64 / pow2ceil(k) lanes.  All
// unfinished slots of a wave advance by the same width each round, so one
// wave-uniform counter holds every such slot's lowest untried attempt; each
// round tries a contiguous range from it and keeps the range's lowest
// success, so a slot's result is the sequential retry loop's first success,
// as with fixed groups.  The rare slot that needs many attempts (7.7 on
// average at 80 % outliers, p99 35) then gets the lanes its finished
// neighbours no longer use, instead of holding the launch for many rounds of
// G lanes.
template <int KIND, int G>
__global__ __launch_bounds__(kGenBlock) void k_generate_fw(DevProblem p, uint64_t seed, uint64_t slot0,
                                                           uint32_t nslots, uint8_t* __restrict__ inc,
                                                           typename ModelOf<KIND>::type* __restrict__ models) {
    constexpr int S = 64 / G;
    static_assert(S >= 1 && S * G == 64, "slots per wave");
    const int lane = threadIdx.x & 63;
    const uint32_t s0 = (blockIdx.x * kGenBlock + (threadIdx.x & ~63u)) / G;   // the wave's first slot
    const uint32_t live = s0 < nslots ? nslots - s0 : 0;
    uint64_t pend = live >= (uint32_t)S ? (S == 64 ? ~0ull : (1ull << S) - 1ull) : (1ull << live) - 1ull;
    uint32_t nx = 0;                    // wave-uniform: lowest untried attempt of every unfinished slot
    while (pend) {
        const int k = __builtin_popcountll(pend);
        const int lw = 6 - (k == 1 ? 0 : 32 - __builtin_clz((uint32_t)(k - 1)));   // log2 of lanes per slot
        const int j = lane >> lw;
        const uint32_t a = nx + (uint32_t)(lane & ((1 << lw) - 1));
        int si = -1;                    // this lane's slot: the j-th unfinished one
        {
            uint64_t m = pend;
            for (int c = 0; m; ++c) {
                const int i = __builtin_ctzll(m);
                m &= m - 1;
                si = c == j ? i : si;
            }
        }
        // KIND 4: the 7-point basis (0..3 models); otherwise one model
        std::conditional_t<KIND == 4, F7Basis, typename ModelOf<KIND>::type> b;
        int cnt = 0;
        if constexpr (KIND == 4) {
            cnt = (si >= 0 && a < 101) ? attempt_f(p, seed, slot0 + s0 + (uint32_t)si, a, b) : 0;
        } else {
            b = ModelOf<KIND>::def();
            cnt = (si >= 0 && a < 101 && attempt<KIND>(p, seed, slot0 + s0 + (uint32_t)si, a, b)) ? 1 : 0;
        }
        const uint64_t mask = __ballot(cnt > 0);
        nx += 1u << lw;
        const bool out_of_attempts = nx >= 101;
        uint64_t np = out_of_attempts ? 0ull : pend;
        bool win = false;
        {
            uint64_t m = pend;
            for (int c = 0; m; ++c) {
                const int i = __builtin_ctzll(m);
                m &= m - 1;
                const uint64_t grp = lw == 6 ? mask : (mask >> (c << lw)) & ((1ull << (1 << lw)) - 1ull);
                if (grp) {
                    np &= ~(1ull << i);
                    win |= lane == (c << lw) + __builtin_ctzll(grp);
                }
            }
        }
        // slots with no success and no attempts left report failure (lane 0
        // of their group)
        const bool fail = out_of_attempts && si >= 0 && !((mask >> (j << lw)) & ((lw == 6) ? ~0ull : ((1ull << (1 << lw)) - 1ull))) &&
                          (lane & ((1 << lw) - 1)) == 0;
        pend = np;
        const uint32_t s = s0 + (uint32_t)si;   // the winner's / failure writer's own slot
        if (win) {
          if constexpr (KIND == 4) {
            GeoModel* out = models + (size_t)kFModels * s;
            uint8_t* oi = inc + (size_t)kFModels * s;
            int m = 0;
#pragma unroll
            for (int q = 0; q < 3; ++q)
                if (b.valid & (1u << q)) {
                    double fm[9];
                    f7_model(b, f7_root(b, q), fm);
                    for (int t = 0; t < 9; ++t) out[m].h[t] = fm[t];
                    ++m;
                }
            for (int q = m; q < kFModels; ++q) out[q] = default_geo();
            oi[0] = (uint8_t)(a + 1);
            oi[1] = cnt > 1 ? 0 : 255;
            oi[2] = cnt > 2 ? 0 : 255;
          } else {
            models[s] = b;
            inc[s] = (uint8_t)(a + 1);
          }
        } else if (fail) {
            constexpr int kM = KIND == 4 ? kFModels : 1;
#pragma unroll
            for (int q = 0; q < kM; ++q) {
                models[(size_t)kM * s + q] = ModelOf<KIND>::def();
                inc[(size_t)kM * s + q] = q == 0 ? 102 : 255;
            }
        }
    }
}

// ---------------------------------------------------------------- score ----
template <int KIND, bool kIdentity>
__global__ __launch_bounds__(kScoreBlock) void k_score(DevProblem p, double T0, double T1, FlagBand fb,
                                                       const RectModel* __restrict__ models,
                                                       const uint8_t* __restrict__ inc, uint32_t nh, ScoreOut out) {
    const uint32_t h = blockIdx.x * kScoreBlock + threadIdx.x;
    if (h >= nh) return;
    if (inc != nullptr && inc[h] > 101) {
        out.n0[h] = 0; out.n1[h] = 0; out.v0[h] = 0.0; out.v1[h] = 0.0; out.tot[h] = 0.0;
        if (out.fl) out.fl[h] = 0;
        return;
    }
    const RectModel m = models[h];
    const DevClass c0 = p.cls[0];
    const ValueConst vc = value_const(m, KIND == 1, KIND == 2);
    uint32_t cnt0 = 0, nfl = 0;
    double acc0 = 0.0;
    for (uint32_t i = 0; i < c0.n; ++i) {
        const double r2 = scale_sq_value<KIND == 1, kIdentity>(c0.x[i], c0.y[i], c0.a[i], m, vc.ac, vc.cut);
        nfl += in_flag_band(r2, fb.mid[0], fb.half[0]) ? 1u : 0u;
        if (r2 <= T0) {
            cnt0 += 1;
            acc0 += -r2;
        }
    }
    uint32_t cnt1 = 0;
    double acc1 = 0.0, tot = acc0;
    if constexpr (KIND == 2) {
        const DevClass c1 = p.cls[1];
        for (uint32_t i = 0; i < c1.n; ++i) {
            const double r2 =
                orient_sq_value<kIdentity>(c1.x[i], c1.y[i], c1.c0[i], c1.c1[i], m, vc.c, vc.s, vc.cphi, vc.cphi2);
            nfl += in_flag_band(r2, fb.mid[1], fb.half[1]) ? 1u : 0u;
            if (r2 <= T1) {
                cnt1 += 1;
                acc1 += -r2;
                tot += -r2;
            }
        }
    }
    out.n0[h] = cnt0;
    out.n1[h] = cnt1;
    out.v0[h] = acc0;
    out.v1[h] = acc1;
    out.tot[h] = tot;
    if (out.fl) out.fl[h] = nfl;
}

// ------------------------------------------------------- split scoring ----
// Exact MSAC with the feature loop split over a 1024-thread workgroup.
//
// A workgroup owns H hypotheses and walks the features in rounds of R.  Waves
// 0..14 (960 threads) evaluate the H x R (hypothesis, feature) pairs of round
// r and leave -r^2 (inlier) or +0.0 (outlier) in LDS tile r % 2; in the same
// interval wave 15 folds tile (r-1) % 2 into H running sums, one lane per
// hypothesis, in feature order.  One barrier per round separates the two.
// Adding +0.0 never changes a sum that starts at +0.0, so every chain is
// bit-identical to the reference's sequential loop (MSAC_scoring_function.hpp:
// 73-85, score.hpp:45-50) for any H and R; the class-1 chain continues the
// class-0 running total exactly as Score::increment_value does.
//
// Compute waves first run a conservative band test on every pair (a few
// fp64 ops: rectified log-scale within exp(+-1.5 thr) * (1 +- 1e-9), or the
// rectified direction within tan(1.5 thr) * (1 + 1e-6) of the phi / phi+pi/2
// line family).  A rejected pair is provably an MSAC outlier under the exact
// arithmetic (margins ~1e6 x the fp64 error of the exact path; NaN/inf, zero or
// negative operands are never rejected).  Surviving pairs are compacted per
// wave (ballot + mbcnt) into an LDS queue and evaluated with the exact
// residual with all 64 lanes busy.
constexpr int kSplitThreads = 1024;
constexpr int kComputeThreads = 960;
constexpr int kComputeWaves = 15;

struct alignas(16) HypConst {   // per-hypothesis constants of the exact and band tests
    union {
        struct {
            // band constants first, in 16-byte pairs (ds_read_b128)
            double h7, h8;      // model
            double lo, hi;      // scale band on s / t^3 (ac-adjusted)
            double cf, sf;      // orientation: twin cos(phi), sin(phi) (band and value; NaN: reference formula)
            double ac, cut;     // scale: alpha^3, the value's cut (rect.h ValueConst)
            double cphi, cphi2; // orientation: clipped phi, clip(clip(phi + pi/2))
        };
        double g[9];            // homography (KIND 3), row-major
    };
};

// branch-free: t is computed exactly as scale_sq_residual computes it, so the
// band and the exact residual see the same t bit for bit
template <int KIND>
__device__ __forceinline__ bool scale_band(double x, double y, double s, const HypConst& q) {
    const double t = (-q.h7 * x - q.h8 * y) + 1.0;
    const double t3 = (t * t) * t;
    const bool odd = !(t > 0.0 && s > 0.0);               // sign / NaN: exact path decides
    return odd | !(s < q.lo * t3 || s > q.hi * t3);
}

// Homography band: the transfer error without its two divisions.  With
// w = h31 x1 + h32 y1 + h33 and e = (h1 . x1 - x2 w, h2 . x1 - y2 w), the
// exact r^2 is |e|^2 / w^2 (in real arithmetic), so a pair can only be an
// inlier if |e|^2 <= Tb w^2, Tb = (sqrt(T)(1 + 1e-7) + 1e-7)^2 (1e-7 px of
// slack against rounding, far above the ~1e-11 px errors at image
// coordinates).  NaN never rejects (the exact residual decides).
__device__ __forceinline__ bool h_band(double x1, double y1, double x2, double y2, const double* h, double Tb) {
    const double w = (h[6] * x1 + h[7] * y1) + h[8];
    const double tu = (h[0] * x1 + h[1] * y1) + h[2];
    const double tv = (h[3] * x1 + h[4] * y1) + h[5];
    const double e1 = tu - x2 * w, e2 = tv - y2 * w;
    return !(e1 * e1 + e2 * e2 > Tb * (w * w));
}

// Fundamental band: the squared Sampson distance without its division.
// With num and den computed exactly as f_sq_sampson (fund.h) computes them,
// r^2 = num^2 / den <= T implies num^2 <= T den up to two roundings, so the
// test num^2 > Tb den with Tb = T (1 + 1e-9) never rejects an inlier.  den is
// a sum of squares (>= 0); den = 0 rejects iff num != 0 (r^2 = inf); NaN never
// rejects (the exact residual decides).
__device__ __forceinline__ bool f_band(double x1, double y1, double x2, double y2, const double* h, double Tb) {
    const double fx0 = (h[0] * x1 + h[1] * y1) + h[2];
    const double fx1 = (h[3] * x1 + h[4] * y1) + h[5];
    const double fx2 = (h[6] * x1 + h[7] * y1) + h[8];
    const double ft0 = (h[0] * x2 + h[3] * y2) + h[6];
    const double ft1 = (h[1] * x2 + h[4] * y2) + h[7];
    const double num = (x2 * fx0 + y2 * fx1) + fx2;
    const double den = ((fx0 * fx0 + fx1 * fx1) + ft0 * ft0) + ft1 * ft1;
    return !(num * num > Tb * den);
}

template <int KIND>
__device__ __forceinline__ bool geo_band(double x1, double y1, double x2, double y2, const double* h, double Tb) {
    if constexpr (KIND == 4) return f_band(x1, y1, x2, y2, h, Tb);
    else return h_band(x1, y1, x2, y2, h, Tb);
}

__device__ __forceinline__ bool orient_band(double x, double y, double ct, double st, const HypConst& q,
                                            double tan_tau) {
    const double numer = (-x * st + y * ct) * q.h7 + st;
    const double denom = (x * st - y * ct) * q.h8 + ct;
    const double u = __builtin_fabs(denom * q.cf + numer * q.sf);
    const double v = __builtin_fabs(numer * q.cf - denom * q.sf);
    const double mx = __builtin_fmax(u, v);
    // a direction of magnitude < 2^-900 (rounding no longer relative) is never rejected
    return !(__builtin_fmin(u, v) > tan_tau * mx) | !(mx >= 0x1p-900);
}

template <int KIND>
__device__ __forceinline__ HypConst make_hyp(const typename ModelOf<KIND>::type& m, double band0) {
    HypConst q;
    if constexpr (KIND >= 3) {
        for (int j = 0; j < 9; ++j) q.g[j] = m.h[j];
    } else {
        const ValueConst vc = value_const(m, KIND == 1, KIND == 2);
        q.h7 = m.h7;
        q.h8 = m.h8;
        q.ac = vc.ac;
        q.cut = vc.cut;
        // s / t^3 must lie in [exp(-tau), exp(tau)] / ac (new) or * ac (original)
        q.lo = (KIND == 1 ? q.ac : 1.0 / q.ac) * (1.0 / band0) * (1.0 - 1e-9);
        q.hi = (KIND == 1 ? q.ac : 1.0 / q.ac) * band0 * (1.0 + 1e-9);
        q.cf = vc.c;
        q.sf = vc.s;
        q.cphi = vc.cphi;
        q.cphi2 = vc.cphi2;
    }
    return q;
}

// in-kernel generation + per-workgroup selection (kGen), see kernels.h
struct GenArgs {
    uint64_t seed, slot0;
    uint8_t* inc;
    RectModel* models;
    WgBest* wg;
    uint32_t m0, m1;
    // correspondence estimators (KIND >= 3): optional compaction map of the
    // live hypotheses (k_compact) -- hypothesis j of the launch is model
    // hmap[j], j < *hcount; results are written at j
    const uint32_t* hmap;
    const uint32_t* hcount;
    // kGen prologue: lanes per slot (a power of two dividing 1024 / H; 0 =
    // 1024 / H, every thread of the workgroup)
    uint32_t glanes;
    // timing probes only (GCR_PROBE, results invalid when set): bit 0 skips
    // the chain fold, bit 1 the exact pass, bit 2 the band test, bit 3 the
    // prologue's attempts (every slot takes attempt 0's default model)
    // k_score_fm: bit 8 no wait for the chain before the exact pass, bit 9
    // no inlier-count atomics; valid A/B: bit 10 the rectification fp64
    // bands instead of the packed fp32 pre-band
    uint32_t probe;
    GenChain chain;                     // k_score_fm<.., true>: batch chaining
    // k_score_fm, KIND >= 3: compact in the prologue instead of k_compact --
    // every workgroup scans scan_inc[0 .. nh) (live: <= 101) and scores live
    // ranks [blockIdx.x H, + H); hmap / hcount are then written, not read
    bool scan;
};

template <int KIND, int H, int R, bool kGen>
__global__ __launch_bounds__(kSplitThreads) void k_score_split(DevProblem p, double T0, double T1, double band0,
                                                               double tan_tau1, FlagBand fband,
                                                               const typename ModelOf<KIND>::type* __restrict__ models,
                                                               const uint8_t* __restrict__ inc, uint32_t nh_in,
                                                               ScoreOut out, GenArgs gen) {
    static_assert((H * R) % kComputeThreads == 0 && kComputeThreads % H == 0, "tile shape");
    uint32_t nh = nh_in;
    if constexpr (KIND >= 3) {
        if (gen.hcount != nullptr) nh = min(nh_in, *gen.hcount);
        if (blockIdx.x * H >= nh) return;            // whole workgroup, before any barrier
    }
    static_assert(H * R <= 65536, "queue entries are 16-bit tile indices");
    constexpr int kPer = H * R / kComputeThreads;    // pairs per compute thread per round
    constexpr int kStride = kComputeThreads / H;     // feature stride between a thread's pairs
    // orientation rounds feed two sequential sums (class sum and total): with
    // H <= 32 they run on two lane groups of the chain wave, else both in-lane
    constexpr bool kSplitTot = KIND == 2 && 2 * H <= 64;
    constexpr bool kDual = KIND == 2 && !kSplitTot;
    // tile: hypothesis-major columns, -r^2 per inlier pair, +0.0 otherwise; the
    // +2 pad keeps 16-byte column alignment and spreads the chain lanes'
    // 16-byte reads over distinct banks
    constexpr int kRP = R + 2;
    // KIND 4: packed in-order inlier segments (sparse chain fold, measured
    // 220 -> 181 us at 4096 slots); KIND 3 goes through the band + queue path
    // with the division-free h_band prefilter
    constexpr bool kPack = KIND == 4;
    __shared__ double tile[2][H * kRP];
    constexpr int kRp = (R + 127) / 128 * 128;       // fbuf row: whole 128-feature DMA strips
    __shared__ double fbuf[2][4][kRp];               // staged features of a round: x, y, s|cos, sin
    __shared__ uint16_t queue[kComputeWaves][kPack ? 1 : kPer * 64];
    __shared__ HypConst hyp[H];
    __shared__ uint32_t cnt_sh[2][H];
    __shared__ uint32_t fl_sh[H];                     // flagged pairs (exact.h), rectification solvers
    // KIND >= 3: per round buffer, compute wave and hypothesis, the number of
    // inlier values the wave packed (in feature order) into its tile segment
    __shared__ uint32_t seg_cnt[2][kPack ? kComputeWaves : 1][kPack ? H : 1];

    const int t = threadIdx.x;
    const int wave = t >> 6;
    const int lane = t & 63;
    const bool chain_wave = t >= kComputeThreads;
    const int h = chain_wave ? (lane % H) : (t % H);
    const int role = (chain_wave && kSplitTot) ? lane / H : 0;   // 0: class sums, 1: total
    const bool chain_lane = chain_wave && lane < (kSplitTot ? 2 * H : H);
    const int fsub = t / H;
    const uint32_t hg = blockIdx.x * H + h;
    // model / inc index of this hypothesis (compacted launches: the map)
    const uint32_t mi = (KIND >= 3 && gen.hmap != nullptr && hg < nh) ? gen.hmap[hg] : hg;

    const uint32_t n0 = p.cls[0].n;
    const uint32_t n1 = (KIND == 2) ? p.cls[1].n : 0;
    const uint32_t r0 = (n0 + R - 1) / R;
    const uint32_t rounds = r0 + (n1 + R - 1) / R;

    // stage the features of round rr into fbuf[buf] (threads tid, tid+nt, ...)
    auto stage = [&](uint32_t rr, int buf, int tid, int nt) {
        const int cls = (rr < r0) ? 0 : 1;
        const DevClass& c = p.cls[cls];
        const uint32_t base = (cls == 0 ? rr : rr - r0) * R;
        for (int e = tid; e < R; e += nt) {
            const uint32_t i = base + e;
            if (i < c.n) {
                fbuf[buf][0][e] = c.x[i];
                fbuf[buf][1][e] = c.y[i];
                if (cls == 0) {
                    fbuf[buf][2][e] = c.a[i];
                    if constexpr (KIND >= 3) fbuf[buf][3][e] = c.c0[i];
                } else {
                    fbuf[buf][2][e] = c.c0[i];
                    fbuf[buf][3][e] = c.c1[i];
                }
            }
        }
    };
    // chain-wave staging by LDS-DMA (global_load_lds, 16 B = 2 features per
    // lane): issued before the fold, retired by the round's barrier, so the
    // global latency hides behind the fold and no registers are spent.
    // Device arrays are padded to even length; strips past the end re-read the
    // last pair (never consumed).
    auto stage_dma = [&](uint32_t rr, int buf) {
        const int cls = (rr < r0) ? 0 : 1;
        const DevClass& c = p.cls[cls];
        const uint32_t base = (cls == 0 ? rr : rr - r0) * R;
        const uint32_t last = ((c.n + 1u) & ~1u) - 2u;
        const double* src[4] = {c.x, c.y, cls == 0 ? c.a : c.c0, cls == 0 ? c.c0 : c.c1};
        const int nf = (cls == 0 && KIND < 3) ? 3 : 4;
        for (int f = 0; f < nf; ++f) {
#pragma unroll
            for (int q = 0; q < kRp / 128; ++q) {
                const uint32_t i = min(base + q * 128 + 2 * lane, last);
                __builtin_amdgcn_global_load_lds((const gvoid*)(src[f] + i), (lvoid*)&fbuf[buf][f][q * 128], 16, 0, 0);
            }
        }
    };

    // kGen: draw this workgroup's H slots, G = 1024 / H lanes per slot trying
    // attempts r*G + g in parallel; the lowest success wins (k_generate's rule)
    __shared__ int gen_a[kGen ? H : 1];
    __shared__ RectModel gen_m[kGen ? H : 1];
    if constexpr (kGen) {
        // G lanes per slot on threads [0, H G): fewer waves contend for the
        // SIMDs, so one round of attempts finishes sooner
        const int G = gen.glanes ? (int)gen.glanes : kSplitThreads / H;
        const bool gact = t < H * G;
        if (t < H) gen_a[t] = 127;
        __syncthreads();
        const int gh = gact ? t / G : 0, g = t % G;
        const uint32_t gs = blockIdx.x * H + gh;
        for (uint32_t rr = 0; rr * G < 101; ++rr) {
            const uint32_t a = rr * G + g;
            RectModel m = default_model();
            bool ok = false;
            if (gact && gs < nh && a < 101 && gen_a[gh] == 127)
                ok = (gen.probe & 8u) ? a == 0 : attempt<KIND>(p, gen.seed, gen.slot0 + gs, a, m);
            if (ok) atomicMin(&gen_a[gh], (int)a);
            __syncthreads();
            if (ok && gen_a[gh] == (int)a) gen_m[gh] = m;
            bool all = true;
            for (int q = 0; q < H; ++q) all = all && (gen_a[q] != 127 || blockIdx.x * H + q >= nh);
            __syncthreads();
            if (all) break;
        }
        if (t < H && hg < nh) {
            const int a = gen_a[t];
            gen.inc[hg] = (uint8_t)(a == 127 ? 102 : a + 1);
            gen.models[hg] = a == 127 ? default_model() : gen_m[t];
        }
    }
    const bool valid_h = hg < nh && (kGen ? gen_a[h] != 127 : (inc == nullptr || inc[mi] <= 101));
    const bool live = !chain_wave && valid_h;

    if (KIND >= 3 && t < H) {
        if constexpr (KIND >= 3) {
            const GeoModel m = valid_h ? models[mi] : default_geo();
            HypConst q;
            for (int j = 0; j < 9; ++j) q.g[j] = m.h[j];
            hyp[h] = q;
        }
    } else if (t < H) {
        const bool v = valid_h;
        RectModel m = default_model();
        if constexpr (KIND < 3) {
            m = v ? (kGen ? gen_m[h] : models[hg]) : default_model();
            hyp[h] = make_hyp<KIND>(m, band0);
        }
    }
    if (t < 2 * H) cnt_sh[t / H][t % H] = 0;
    if (t < H) fl_sh[t] = 0;
    stage(0, 0, t, kSplitThreads);
    __syncthreads();

    // chain-lane state: `run` is the running sum this lane extends; `hold`
    // keeps the finished class-0 sum; `tot2` the in-lane total (kDual)
    double run = 0.0, hold = 0.0, tot2 = 0.0;
    uint32_t geo_count = 0;                           // KIND >= 3: inliers folded so far
    if (chain_wave) __builtin_amdgcn_s_setprio(3);   // latency-bound: issue ahead of the compute waves
    HypConst mine{};
    if (live) mine = hyp[h];

    for (uint32_t r = 0; r <= rounds; ++r) {
        if (!chain_wave) {
            if (r < rounds) {
                const int b = r & 1;
                double* tl = tile[b];
                const double(*fb)[kRp] = fbuf[b];
                const int cls = (r < r0) ? 0 : 1;
                const uint32_t base = (cls == 0 ? r : r - r0) * R;
                const uint32_t nc = cls == 0 ? n0 : n1;
                if constexpr (kPack) {
                    // fundamental matrix: the exact residual is cheap, every
                    // pair is evaluated directly (no band).  Wave w
                    // owns the contiguous feature segment [w kSeg, (w+1) kSeg)
                    // of the round (kPer column steps of G = 64 / H features x
                    // H hypotheses) and packs each hypothesis's inlier values
                    // into the front of that segment IN FEATURE ORDER (ballot +
                    // masked prefix count).  Outliers add +0.0 to the MSAC sum,
                    // an exact no-op, so the chain folds only the packed values.
                    constexpr int G = 64 / H;
                    constexpr int kSeg = kPer * G;
                    constexpr uint64_t kPattern = H == 64 ? 1ull : (H == 16 ? 0x0001000100010001ull
                                                                            : 0x1111111111111111ull);
                    static_assert(kComputeWaves * kSeg == R, "segments tile the round");
                    const int sub = lane / H;
                    const uint64_t hmask = kPattern << h;
                    const uint64_t below = (1ull << lane) - 1ull;
                    double* seg = tl + h * kRP + wave * kSeg;
                    // all residuals first (independent: the divisions interleave),
                    // then the in-order packing
                    double r2[kPer];
#pragma unroll
                    for (int k = 0; k < kPer; ++k) {
                        const uint32_t il = wave * kSeg + k * G + sub;
                        const bool ok = live && base + il < nc;
                        const uint32_t ic = ok ? il : 0u;
                        const double v = geo_sq_residual<KIND>(fb[0][ic], fb[1][ic], fb[2][ic], fb[3][ic], mine.g);
                        r2[k] = ok ? v : __builtin_inf();
                    }
                    uint32_t cnt = 0;
#pragma unroll
                    for (int k = 0; k < kPer; ++k) {
                        const bool inl = r2[k] <= T0;
                        const uint64_t mh = __ballot(inl) & hmask;
                        if (inl) seg[cnt + (uint32_t)__builtin_popcountll(mh & below)] = -r2[k];
                        cnt += (uint32_t)__builtin_popcountll(mh);
                    }
                    if (sub == 0) seg_cnt[b][wave][h] = cnt;
                } else {
                // 1) conservative band test
                uint32_t bits = 0;
#pragma unroll
                for (int k = 0; k < kPer; ++k) {
                    const uint32_t il = fsub + k * kStride;
                    bool cand = false;
                    if (live && base + il < nc && !(gen.probe & 4u)) {
                        if constexpr (KIND == 3) cand = h_band(fb[0][il], fb[1][il], fb[2][il], fb[3][il], mine.g, band0);
                        else if (cls == 0) cand = scale_band<KIND>(fb[0][il], fb[1][il], fb[2][il], mine);
                        else if constexpr (KIND == 2) cand = orient_band(fb[0][il], fb[1][il], fb[2][il], fb[3][il], mine, tan_tau1);
                    }
                    tl[h * kRP + il] = 0.0;
                    bits |= (uint32_t)cand << k;
                }
                // 2) wave-level compaction of the surviving pairs
                uint16_t* qw = queue[wave];
                uint32_t qn = 0;
#pragma unroll
                for (int k = 0; k < kPer; ++k) {
                    const bool cand = (bits >> k) & 1u;
                    const uint64_t mask = __ballot(cand);
                    if (cand) {
                        const uint32_t pos = qn + (uint32_t)__builtin_amdgcn_mbcnt_hi(
                                                      (uint32_t)(mask >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
                        qw[pos] = (uint16_t)((fsub + k * kStride) * H + h);
                    }
                    qn += (uint32_t)__builtin_popcountll(mask);
                }
                // 3) exact residuals of the survivors, all lanes busy
                if (gen.probe & 2u) qn = 0;
                for (uint32_t j = lane; j < qn; j += 64) {
                    const uint32_t idx = qw[j];
                    const int hh = idx % H;
                    const uint32_t il = idx / H;
                    const HypConst& q = hyp[hh];
                    RectModel m = default_model();
                    m.h7 = q.h7;
                    m.h8 = q.h8;
                    double r2;
                    bool inl;
                    if constexpr (KIND == 3) {
                        r2 = h_sq_residual(fb[0][il], fb[1][il], fb[2][il], fb[3][il], q.g);
                        inl = r2 <= T0;
                    } else if (cls == 0) {
                        r2 = scale_sq_value<KIND == 1, true>(fb[0][il], fb[1][il], fb[2][il], m, q.ac, q.cut);
                        inl = r2 <= T0;
                    } else {
                        r2 = orient_sq_value<true>(fb[0][il], fb[1][il], fb[2][il], fb[3][il], m, q.cf, q.sf, q.cphi,
                                                   q.cphi2);
                        inl = r2 <= T1;
                    }
                    if (inl) {
                        tl[hh * kRP + il] = -r2;
                        atomicAdd(&cnt_sh[cls][hh], 1u);
                    }
                    if (KIND <= 2 && in_flag_band(r2, fband.mid[cls], fband.half[cls])) atomicAdd(&fl_sh[hh], 1u);
                }
                }   // band path (KIND <= 3)
            }
        } else {
            // chain wave: stage round r+1's features around the fold of
            // tile r-1, which extends the sums in feature order (outliers
            // hold +0.0: an exact no-op)
            if (r + 1 < rounds) stage_dma(r + 1, (r + 1) & 1);
            if constexpr (kPack) {
                if (r > 0 && chain_lane) {
                    // packed inlier values, segment by segment in feature order
                    constexpr int kSeg = kPer * (64 / H);
                    const int qb = (r - 1) & 1;
                    const double* row = tile[qb] + h * kRP;
                    uint32_t ns[kComputeWaves];
#pragma unroll
                    for (int w = 0; w < kComputeWaves; ++w) ns[w] = seg_cnt[qb][w][h];
#pragma unroll
                    for (int w = 0; w < kComputeWaves; ++w) {
                        const uint32_t n = ns[w];
                        const double* seg = row + w * kSeg;
                        geo_count += n;
                        uint32_t j = 0;
                        for (; j + 4 <= n; j += 4) {
                            const double a0 = seg[j], a1 = seg[j + 1], a2 = seg[j + 2], a3 = seg[j + 3];
                            run += a0;
                            run += a1;
                            run += a2;
                            run += a3;
                        }
                        for (; j < n; ++j) run += seg[j];
                    }
                }
            } else if (r > 0 && chain_lane && !(gen.probe & 1u)) {
                const uint32_t qr = r - 1;
                const bool cls0 = qr < r0;
                if (KIND == 2 && qr == r0 && role == 0) {   // first orientation round
                    hold = run;
                    tot2 = run;
                    run = 0.0;
                }
                const double2* col = reinterpret_cast<const double2*>(tile[qr & 1] + h * kRP);
                const uint32_t len = cls0 ? min((uint32_t)R, n0 - qr * R) : min((uint32_t)R, n1 - (qr - r0) * R);
                // entries in [len, kRP) are +0.0, so the fold may run to an even
                // length; 16-byte reads, one batch ahead of the adds
                const uint32_t np = (len + 1) >> 1;
                const bool dual = kDual && !cls0;
                uint32_t j = 0;
                auto fold2 = [&](const double2& v) {
                    run += v.x;
                    if (dual) tot2 += v.x;
                    run += v.y;
                    if (dual) tot2 += v.y;
                };
                // batches of kB 16-byte reads all in flight, then 2 kB adds:
                // the fold is bound by LDS latency under the compute waves' load
                // (a software-pipelined variant, batch b+1 in flight while
                // batch b is added, measured slower: 0.149 vs 0.135 ms)
                constexpr int kB = KIND == 2 ? 10 : 12;
                for (; j + kB <= np; j += kB) {
                    double2 v[kB];
#pragma unroll
                    for (int u = 0; u < kB; ++u) v[u] = col[j + u];
#pragma unroll
                    for (int u = 0; u < kB; ++u) fold2(v[u]);
                }
                for (; j < np; ++j) fold2(col[j]);
            }
        }
        __syncthreads();
    }
    __shared__ double fin_sh[kGen ? H : 1];
    if (chain_wave) {
        double tot;
        if constexpr (kSplitTot) tot = __shfl(run, (lane + H) & 63);
        else if constexpr (kDual) tot = tot2;
        else tot = run;
        if (lane < H && hg < nh) {
            const double acc0 = KIND == 2 ? hold : run;
            const double acc1 = KIND == 2 ? run : 0.0;
            const uint32_t c0 = valid_h ? (kPack ? geo_count : cnt_sh[0][h]) : 0, c1 = valid_h ? cnt_sh[1][h] : 0;
            out.n0[hg] = c0;
            out.n1[hg] = c1;
            out.v0[hg] = valid_h ? acc0 : 0.0;
            out.v1[hg] = valid_h ? acc1 : 0.0;
            out.tot[hg] = valid_h ? tot : 0.0;
            if (KIND <= 2 && out.fl) out.fl[hg] = valid_h ? fl_sh[h] : 0u;
            if constexpr (kGen) {
                // MSACScoringFunction::getScore finish (MSAC_scoring_function.hpp:108-127)
                double sum = 0.0;
                if (valid_h && c0 >= gen.m0 && (KIND != 2 || c1 >= gen.m1)) {
                    sum = tot;
                    const double ms0 = acc0 / T0 + static_cast<double>(c0);
                    sum -= acc0;
                    sum += ms0;
                    if (KIND == 2) {
                        const double ms1 = acc1 / T1 + static_cast<double>(c1);
                        sum -= acc1;
                        sum += ms1;
                    }
                }
                // candidates of the update rule: score > 0 and a valid model
                const bool cand = valid_h && sum > 0.0 && (KIND != 2 || valid_model_sift22(gen_m[h]));
                fin_sh[h] = cand ? sum : -1.0;
            }
        }
        if constexpr (kGen) {
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) {
                // the workgroup's first strict best, slots in order
                WgBest b{0.0, -1, 0, 0, 0, 0};
                for (int q = 0; q < H; ++q) {
                    const uint32_t gq = blockIdx.x * H + q;
                    if (gq >= nh) break;
                    const int a = gen_a[q];
                    b.iterations += (uint64_t)(a == 127 ? 102 : a + 1);
                    if (a != 127) ++b.models;
                    const double s = fin_sh[q];
                    if (s > 0.0 && b.score < s) {
                        b.score = s;
                        b.slot = (int32_t)gq;
                        b.n0 = cnt_sh[0][q];
                        b.n1 = KIND == 2 ? cnt_sh[1][q] : 0;
                    }
                }
                gen.wg[blockIdx.x] = b;
            }
        }
    }
}


// ------------------------------------------------ diagnostic stamps ----
// Built only into libgcr_stamps.so (make stamps, -DGCR_STAMPS): s_memtime at
// the segment boundaries of k_score_fm for the first kStWG workgroups, read
// back by tools/stamp_probe.py.  The product build executes no stamp.
#ifdef GCR_STAMPS
constexpr int kStWG = 4, kStRounds = 16, kStSlots = 8;
__device__ uint64_t g_stamps[kStWG][16][kStRounds][kStSlots];
__device__ __forceinline__ uint64_t stamp_now() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define GCR_STAMP(slot, rr)                                                                   \
    do {                                                                                      \
        const uint64_t _t = stamp_now();                                                      \
        if (blockIdx.x < kStWG && (rr) < (uint32_t)kStRounds && lane == 0)                    \
            g_stamps[blockIdx.x][wave][rr][slot] = _t;                                        \
    } while (0)
#define GCR_STAMP_VAL(slot, rr, v)                                                            \
    do {                                                                                      \
        if (blockIdx.x < kStWG && (rr) < (uint32_t)kStRounds && lane == 0)                    \
            g_stamps[blockIdx.x][wave][rr][slot] = (v);                                       \
    } while (0)
// every workgroup's start and end on the global 100 MHz clock (s_memrealtime),
// last launch only (tools/wg_spans.py: the spread behind a launch's tail)
constexpr int kSpanWG = 4096;
__device__ uint64_t g_wgspan[kSpanWG][3];    // start, end, exact-pass survivors
__device__ __forceinline__ uint64_t realtime_now() {
    uint64_t t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
#define GCR_WGSPAN(i)                                                                         \
    do {                                                                                      \
        const uint64_t _t = realtime_now();                                                   \
        if (blockIdx.x < (uint32_t)kSpanWG && (threadIdx.x & 63) == 0) g_wgspan[blockIdx.x][i] = _t; \
    } while (0)
#else
#define GCR_WGSPAN(i) do {} while (0)
#define GCR_STAMP(slot, rr) do {} while (0)
#define GCR_STAMP_VAL(slot, rr, v) do {} while (0)
#endif

// ------------------------------------------- feature-major split scoring ----
// Exact MSAC with one feature per compute lane and a sparse, in-order fold.
//
// A workgroup owns H <= 16 hypotheses.  Compute wave w (0..14) owns features
// [64 w, 64 w + 64) of each round of 960 (rounds never straddle the class
// boundary): every lane holds its own feature in registers and tests it
// against the H hypotheses in turn with the conservative band, so the
// survivors of a wave-round are appended hypothesis by hypothesis, each
// hypothesis's entries in feature order.  The exact residuals of the
// survivors are then evaluated with all 64 lanes busy, and the inlier values
// -r^2 are packed by a running ballot prefix: hypothesis q's inlier values of
// the wave-round are a contiguous run of outv[w], in feature order, delimited
// by lohi[.][w][q], lohi[.][w][q + 1].
//
// Wave 15 (the chain wave) folds the runs wave by wave and round by round:
// exactly the inliers in feature order, which is the reference's sequential
// sum (MSAC_scoring_function.hpp:73-85, score.hpp:45-50) because an outlier's
// +0.0 never changes it.  Outliers cost the chain nothing.  Waves hand over
// through LDS flags instead of barriers (ready[w]: rounds published by wave
// w; done[w]: rounds of wave w the chain has folded), so a compute wave only
// waits when the chain still reads its previous run.
// compile-time loop: f(std::integral_constant<int, Q>) for Q in [B, E)
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// lane Q of v takes the (wave-uniform) value c: one v_writelane_b32
template <int Q>
__device__ __forceinline__ uint32_t write_lane(uint32_t v, uint32_t c) {
    asm("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(c), "n"(Q));
    return v;
}

constexpr int kFmWaves = 15;
constexpr int kFmCB = 8;            // chain batch: 16-byte LDS reads (2 values each) per run step
                                    // (16, i.e. 32-value batches: 130.8 vs 127.8 us)

__device__ __forceinline__ void fm_wait_ge(const uint32_t* f, uint32_t v) {
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < v) __builtin_amdgcn_s_sleep(1);
}
__device__ __forceinline__ void fm_publish(uint32_t* f, uint32_t v) {
    __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}


// Correspondence instantiations (KIND >= 3) keep the survivor regions and
// queues in dynamic LDS and are held to 64 VGPRs (8 waves per SIMD's worth):
// with the LDS size unknown at compile time the register cap applies, and a
// scoring workgroup (16 waves x 64 VGPRs) then leaves room on every SIMD for
// one wave of the separately launched generator (k_generate_f, ~240 VGPRs,
// no LDS), which the two-stream batch pipeline of verify_batches overlaps
template <int H, bool kGen>
constexpr size_t fm_dyn_lds_bytes() {
    constexpr int kW = kGen ? kFmWaves - 1 : kFmWaves;
    return (size_t)kW * H * 66 * sizeof(double) + (size_t)kW * 64 * H * sizeof(uint16_t);
}

// Fundamental matrix: a conservative packed-fp32 pre-band on the Sampson
// error, two hypotheses per instruction (v_pk_fma_f32).  With inputs rounded
// to fp32 and every fma rounding counted, each of fx0, fx1, fx2 (F x1) and
// ft0, ft1 (F^T x2) is within e = 1e-6 (|h| . |coords|max) of its real value
// (>= 4 u of slack per term, u = 2^-24), num within sn (the same bound carried
// through num = x2 fx0 + y2 fx1 + fx2), and den <= sum (|f| + e)^2.  A pair is
// rejected only if (|num| - sn)^2 > T (1 + 4e-6) den_up, i.e. only if even the
// smallest num and the largest den the bounds allow give r^2 > T; the margin
// also covers the fp64 rounding of the exact residual.  NaN, overflow or
// unbounded coordinates (amax = inf) never reject.  Survivors get the exact
// f_sq_sampson in the exact pass, so the result is unchanged.
typedef float fpb_f2 __attribute__((ext_vector_type(2)));
struct FPairBand {                 // hypotheses 2 j (.x) and 2 j + 1 (.y)
    fpb_f2 g[9];
    fpb_f2 e[5];                   // error bounds of fx0, fx1, fx2, ft0, ft1
    fpb_f2 sn;                     // error bound of num
    fpb_f2 tq;                     // T (1 + 4e-6), rounded up
};

__device__ __forceinline__ float fpb_up(double v) {
    // a float >= v (v >= 0); +inf past 1e30 or when not finite
    return (v < 1e30) ? (float)(v * (1.0 + 1e-6)) + 1e-30f : __builtin_inff();
}

__device__ __forceinline__ void fpb_setup(FPairBand* fp, int t, const double* h, bool valid, double T,
                                          const DevClass& c) {
    const double X1 = c.amax[0], Y1 = c.amax[1], X2 = c.amax[2], Y2 = c.amax[3];
    double a[9];
    for (int k = 0; k < 9; ++k) a[k] = __builtin_fabs(h[k]);
    const double F0 = (a[0] * X1 + a[1] * Y1) + a[2];
    const double F1 = (a[3] * X1 + a[4] * Y1) + a[5];
    const double F2 = (a[6] * X1 + a[7] * Y1) + a[8];
    const double G0 = (a[0] * X2 + a[3] * Y2) + a[6];
    const double G1 = (a[1] * X2 + a[4] * Y2) + a[7];
    constexpr double gam = 1e-6;
    const double e0 = gam * F0, e1 = gam * F1, e2 = gam * F2, e3 = gam * G0, e4 = gam * G1;
    const double sn = ((X2 * e0 + Y2 * e1) + e2) + gam * ((X2 * (F0 + e0) + Y2 * (F1 + e1)) + (F2 + e2));
    // each thread writes its own 4-byte half of the pair's vectors (no
    // read-modify-write of the 8-byte element its neighbour also writes)
    float* b = reinterpret_cast<float*>(&fp[t >> 1]);
    const int hf = t & 1;
    for (int k = 0; k < 9; ++k) b[2 * k + hf] = valid ? (float)h[k] : 0.0f;
    const double ev[5] = {e0, e1, e2, e3, e4};
    for (int k = 0; k < 5; ++k) b[2 * (9 + k) + hf] = fpb_up(ev[k]);
    // an invalid hypothesis is never scored (vmask); keep its constants inert
    b[2 * 14 + hf] = valid ? fpb_up(sn) : __builtin_inff();
    b[2 * 15 + hf] = fpb_up(T * (1.0 + 4e-6));
}
static_assert(sizeof(FPairBand) == 16 * 8, "FPairBand layout: 16 float pairs");

// reject bits of the pair (.x: hypothesis 2 j, .y: 2 j + 1)
__device__ __forceinline__ fpb_f2 fpb_fma(fpb_f2 a, fpb_f2 b, fpb_f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ void fpb_test(const FPairBand& b, float x1, float y1, float x2, float y2, bool& r0,
                                         bool& r1) {
    const fpb_f2 X1 = {x1, x1}, Y1 = {y1, y1}, X2 = {x2, x2}, Y2 = {y2, y2};
    const fpb_f2 fx0 = fpb_fma(b.g[0], X1, fpb_fma(b.g[1], Y1, b.g[2]));
    const fpb_f2 fx1 = fpb_fma(b.g[3], X1, fpb_fma(b.g[4], Y1, b.g[5]));
    const fpb_f2 fx2 = fpb_fma(b.g[6], X1, fpb_fma(b.g[7], Y1, b.g[8]));
    const fpb_f2 ft0 = fpb_fma(b.g[0], X2, fpb_fma(b.g[3], Y2, b.g[6]));
    const fpb_f2 ft1 = fpb_fma(b.g[1], X2, fpb_fma(b.g[4], Y2, b.g[7]));
    const fpb_f2 num = fpb_fma(X2, fx0, fpb_fma(Y2, fx1, fx2));
    const fpb_f2 d0 = __builtin_elementwise_abs(fx0) + b.e[0];
    const fpb_f2 d1 = __builtin_elementwise_abs(fx1) + b.e[1];
    const fpb_f2 d2 = __builtin_elementwise_abs(ft0) + b.e[3];
    const fpb_f2 d3 = __builtin_elementwise_abs(ft1) + b.e[4];
    const fpb_f2 den = fpb_fma(d3, d3, fpb_fma(d2, d2, fpb_fma(d1, d1, d0 * d0)));
    (void)b.e[2];                  // fx2's bound enters through sn only
    const fpb_f2 a = __builtin_elementwise_abs(num) - b.sn;
    const fpb_f2 lhs = a * a, rhs = b.tq * den;
    r0 = a.x > 0.0f && lhs.x > rhs.x;
    r1 = a.y > 0.0f && lhs.y > rhs.y;
}

// Homography: the same packed-fp32 pre-band on the transfer error.  With
// w = h6 x1 + h7 y1 + h8, tu = h0 x1 + h1 y1 + h2, tv = h3 x1 + h4 y1 + h5 and
// e = (tu - x2 w, tv - y2 w), the fp64 band (h_band) keeps a pair iff
// |e|^2 <= Tb w^2.  In fp32 (inputs rounded, every fma rounding counted) w is
// within ew = 1e-6 W of its real value (W = |h6| X1 + |h7| Y1 + |h8| with the
// problem's largest coordinates; >= 4 u of slack per term, u = 2^-24), and e1,
// e2 within s1 = 1e-6 (U + 3 X2 W), s2 = 1e-6 (V + 3 Y2 W) (U, V the bounds of
// tu, tv).  A pair is rejected only if even the smallest |e| and the largest
// |w| the bounds allow fail the fp64 band with Tb (1 + 4e-6):
// max(|e1| - s1, 0)^2 + max(|e2| - s2, 0)^2 > Tb' (|w| + ew)^2.  The margin
// covers the fp32 rounding of the test itself; h_band's own slack covers the
// exact residual's fp64 rounding.  NaN, overflow or unbounded coordinates
// (amax = inf) never reject.  Survivors get the exact h_sq_residual.
struct HPairBand {                 // hypotheses 2 j (.x) and 2 j + 1 (.y)
    fpb_f2 g[9];
    fpb_f2 ew, s1, s2;             // error bounds of w, e1, e2
    fpb_f2 tq;                     // Tb (1 + 4e-6), rounded up
    fpb_f2 pad[3];
};
static_assert(sizeof(HPairBand) == sizeof(FPairBand), "pair-band records share the LDS slot");

__device__ __forceinline__ void hpb_setup(HPairBand* hp, int t, const double* h, bool valid, double Tb,
                                          const DevClass& c) {
    const double X1 = c.amax[0], Y1 = c.amax[1], X2 = c.amax[2], Y2 = c.amax[3];
    double a[9];
    for (int k = 0; k < 9; ++k) a[k] = __builtin_fabs(h[k]);
    const double W = (a[6] * X1 + a[7] * Y1) + a[8];
    const double U = (a[0] * X1 + a[1] * Y1) + a[2];
    const double V = (a[3] * X1 + a[4] * Y1) + a[5];
    constexpr double gam = 1e-6;
    float* b = reinterpret_cast<float*>(&hp[t >> 1]);
    const int hf = t & 1;
    for (int k = 0; k < 9; ++k) b[2 * k + hf] = valid ? (float)h[k] : 0.0f;
    b[2 * 9 + hf] = fpb_up(gam * W);
    // an invalid hypothesis is never scored (vmask); keep its constants inert
    b[2 * 10 + hf] = valid ? fpb_up(gam * (U + 3.0 * X2 * W)) : __builtin_inff();
    b[2 * 11 + hf] = valid ? fpb_up(gam * (V + 3.0 * Y2 * W)) : __builtin_inff();
    b[2 * 12 + hf] = fpb_up(Tb * (1.0 + 4e-6));
    for (int k = 13; k < 16; ++k) b[2 * k + hf] = 0.0f;
}

__device__ __forceinline__ void hpb_test(const HPairBand& b, float x1, float y1, float x2, float y2, bool& r0,
                                         bool& r1) {
    const fpb_f2 X1 = {x1, x1}, Y1 = {y1, y1}, X2 = {x2, x2}, Y2 = {y2, y2};
    const fpb_f2 w = fpb_fma(b.g[6], X1, fpb_fma(b.g[7], Y1, b.g[8]));
    const fpb_f2 tu = fpb_fma(b.g[0], X1, fpb_fma(b.g[1], Y1, b.g[2]));
    const fpb_f2 tv = fpb_fma(b.g[3], X1, fpb_fma(b.g[4], Y1, b.g[5]));
    const fpb_f2 e1 = fpb_fma(-X2, w, tu), e2 = fpb_fma(-Y2, w, tv);
    const fpb_f2 zero = {0.0f, 0.0f};
    const fpb_f2 a1 = __builtin_elementwise_max(__builtin_elementwise_abs(e1) - b.s1, zero);
    const fpb_f2 a2 = __builtin_elementwise_max(__builtin_elementwise_abs(e2) - b.s2, zero);
    const fpb_f2 d = __builtin_elementwise_abs(w) + b.ew;
    const fpb_f2 lhs = fpb_fma(a2, a2, a1 * a1), rhs = b.tq * (d * d);
    r0 = lhs.x > rhs.x;
    r1 = lhs.y > rhs.y;
}

__device__ __forceinline__ void pb_test(const FPairBand& b, float x1, float y1, float x2, float y2, bool& r0,
                                        bool& r1) {
    fpb_test(b, x1, y1, x2, y2, r0, r1);
}
__device__ __forceinline__ void pb_test(const HPairBand& b, float x1, float y1, float x2, float y2, bool& r0,
                                        bool& r1) {
    hpb_test(b, x1, y1, x2, y2, r0, r1);
}

// Rectification (KIND <= 2): a conservative packed-fp32 pre-band in front of
// the exact pass, two hypotheses per instruction, in place of the fp64 bands
// scale_band / orient_band.  It rejects a pair only when the fp64 band
// would reject it -- with every fp32 rounding bounded -- so the survivors
// are a superset of the fp64 band's, and the exact pass decides them as
// before (results unchanged; GCR_PROBE bit 10 runs the fp64 bands instead).
// u = 2^-24 below; X, Y (and G = X + Y) are the class's largest |x|, |y|
// (DevClass::amax, +inf when any coordinate is not finite: then nothing is
// rejected).
//
// Scale: t = 1 - h7 x - h8 y in fp32 (two fma) is within 4u S of the real t
// (S = |h7| X + |h8| Y + 1, input roundings included); tl = t - B, th = t + B
// with B >= 6u S bracket the fp64 band's t strictly (its own error is
// 3 2^-53 S).  A pair is rejected iff tl > 0 and s < lo'' tl^3 or
// s > hi'' th^3, where lo'' = lo (1 - 2^-19) and hi'' = hi (1 + 2^-19)
// (fp32 products: 4 roundings of s and of the cube, < 2^-20 in all) -- then
// the fp64 band's t > 0, s > 0 and s < lo t^3 (or s > hi t^3) hold too.
// Only scales in [2^-100, 2^100] are tested (others are NaN here: never
// rejected), and only bands with lo, hi in [2^-20, 2^20] (else lo'' = 0,
// hi'' = inf): an overflowing cube then means lo t^3 > 2^107 > s, an
// underflowing one hi t^3 < 2^-105 < s.
//
// Orientation: with g = x st - y ct, numer = st - g h7, denom = ct + g h8,
// U = denom cf + numer sf, V = numer cf - denom sf (the fp64 band's u, v
// before |.|), every fp32 value is within E = 32u (G max(|h7|, |h8|) + 1)
// (+ G 2^-140 for subnormal h, + 2^-90) of the real one.  A pair is rejected
// iff |U| - T |V| > E' and |V| - T |U| > E' with T = tan_tau (1 + 2^-18)
// rounded up and E' = E (1 + T) 1.01: then min(|u|, |v|) > tan_tau max and
// max > 2^-900 hold in fp64 as well (its errors are ~2^-50 (G H + 1)).
struct RPairBand {                 // hypotheses 2 j (.x) and 2 j + 1 (.y)
    fpb_f2 nh7, nh8, tb, lo, hi;   // scale: -h7, -h8, B, lo'', hi''
    fpb_f2 h7, h8, cf, sf, tq, eq; // orientation: h7, h8, cos / sin of phi (twin), T, E'
    fpb_f2 pad[5];
};
static_assert(sizeof(RPairBand) == 16 * 8, "RPairBand layout: 16 float pairs");

static_assert(sizeof(HypConst) == kFmHypBytes && sizeof(RPairBand) == kFmPairBytes, "GenChain constant records");
__device__ __forceinline__ void rpb_setup(RPairBand* rp, int t, const HypConst& q, const DevClass& c0,
                                          const DevClass& c1, double tan_tau1, bool orient, bool valid) {
    constexpr double u = 0x1p-24;
    float* b = reinterpret_cast<float*>(&rp[t >> 1]);
    const int hf = t & 1;                    // this thread's 4-byte half of each pair
    if (!valid) {
        // an invalid hypothesis (no model, or past the launch's count):
        // t = 1, lo'' = inf rejects every scale in range; T = 0, E' = -1
        // every finite direction (its results are discarded anyway; a NaN /
        // out-of-range feature survives and only costs an exact evaluation)
        const float c[11] = {0.0f, 0.0f, 0.0f, __builtin_inff(), __builtin_inff(), 0.0f, 0.0f, 1.0f, 0.0f, 0.0f,
                             -1.0f};
        for (int k = 0; k < 11; ++k) b[2 * k + hf] = c[k];
        return;
    }
    const double a7 = __builtin_fabs(q.h7), a8 = __builtin_fabs(q.h8);
    {
        const double X = c0.amax[0], Y = c0.amax[1];
        const double tb = 6.0 * u * ((a7 * X + a8 * Y) + 1.0) + (X + Y) * 0x1p-140;
        b[2 * 0 + hf] = (float)(-q.h7);
        b[2 * 1 + hf] = (float)(-q.h8);
        b[2 * 2 + hf] = fpb_up(tb);          // +inf when not finite or huge: nothing rejected
        const bool lo_ok = q.lo >= 0x1p-20 && q.lo <= 0x1p20;
        const bool hi_ok = q.hi >= 0x1p-20 && q.hi <= 0x1p20;
        b[2 * 3 + hf] = lo_ok ? (float)(q.lo * (1.0 - 0x1p-19)) : 0.0f;
        b[2 * 4 + hf] = hi_ok ? (float)(q.hi * (1.0 + 0x1p-19)) : __builtin_inff();
    }
    if (orient) {
        const double G = c1.amax[0] + c1.amax[1];
        const double e = 32.0 * u * (G * __builtin_fmax(a7, a8) + 1.0) + G * 0x1p-140 + 0x1p-90;
        const double tq = tan_tau1 * (1.0 + 0x1p-18);
        b[2 * 5 + hf] = (float)q.h7;
        b[2 * 6 + hf] = (float)q.h8;
        b[2 * 7 + hf] = (float)q.cf;
        b[2 * 8 + hf] = (float)q.sf;
        b[2 * 9 + hf] = fpb_up(tq);
        b[2 * 10 + hf] = fpb_up(e * (1.0 + tq) * 1.01);
    }
}

// the fields of one class's test, read from LDS one pair ahead (the queue
// writes in between are LDS stores the compiler cannot move reads across)
struct RScaleC {
    fpb_f2 nh7, nh8, tb, lo, hi;
};
struct ROrientC {
    fpb_f2 h7, h8, cf, sf, tq, eq;
};
__device__ __forceinline__ RScaleC rpb_scale_c(const RPairBand& b) { return RScaleC{b.nh7, b.nh8, b.tb, b.lo, b.hi}; }
__device__ __forceinline__ ROrientC rpb_orient_c(const RPairBand& b) {
    return ROrientC{b.h7, b.h8, b.cf, b.sf, b.tq, b.eq};
}

// reject masks (ballots) of the pair's two hypotheses; sf: the scale in fp32,
// NaN when outside [2^-100, 2^100]
__device__ __forceinline__ void rpb_scale(const RScaleC& b, float x, float y, float sf, uint64_t& r0,
                                          uint64_t& r1) {
    const fpb_f2 X = {x, x}, Y = {y, y}, one = {1.0f, 1.0f};
    const fpb_f2 t = fpb_fma(b.nh7, X, fpb_fma(b.nh8, Y, one));
    const fpb_f2 tl = t - b.tb, th = t + b.tb;
    const fpb_f2 a = ((tl * tl) * tl) * b.lo;
    const fpb_f2 c = ((th * th) * th) * b.hi;
    r0 = __builtin_amdgcn_ballot_w64(tl.x > 0.0f) &
         (__builtin_amdgcn_ballot_w64(sf < a.x) | __builtin_amdgcn_ballot_w64(sf > c.x));
    r1 = __builtin_amdgcn_ballot_w64(tl.y > 0.0f) &
         (__builtin_amdgcn_ballot_w64(sf < a.y) | __builtin_amdgcn_ballot_w64(sf > c.y));
}

__device__ __forceinline__ void rpb_orient(const ROrientC& b, float g, float ct, float st, uint64_t& r0,
                                           uint64_t& r1) {
    const fpb_f2 G = {g, g}, ST = {st, st}, CT = {ct, ct};
    const fpb_f2 N = fpb_fma(-G, b.h7, ST), D = fpb_fma(G, b.h8, CT);
    const fpb_f2 U = __builtin_elementwise_abs(fpb_fma(D, b.cf, N * b.sf));
    const fpb_f2 V = __builtin_elementwise_abs(fpb_fma(N, b.cf, -(D * b.sf)));
    const fpb_f2 P1 = fpb_fma(-b.tq, V, U), P2 = fpb_fma(-b.tq, U, V);
    r0 = __builtin_amdgcn_ballot_w64(P1.x > b.eq.x) & __builtin_amdgcn_ballot_w64(P2.x > b.eq.x);
    r1 = __builtin_amdgcn_ballot_w64(P1.y > b.eq.y) & __builtin_amdgcn_ballot_w64(P2.y > b.eq.y);
}

template <int KIND, int H, bool kGen>
__global__ __launch_bounds__(kSplitThreads) __attribute__((amdgpu_waves_per_eu(KIND >= 3 ? 8 : 1))) void k_score_fm(DevProblem p, double T0, double T1, double band0,
                                                            double tan_tau1, FlagBand fband,
                                                            const typename ModelOf<KIND>::type* __restrict__ models,
                                                            const uint8_t* __restrict__ inc, uint32_t nh,
                                                            ScoreOut out, GenArgs gen) {
    static_assert(H >= 1 && H <= 16 && KIND <= 4, "feature-major scorer: H <= 16");
    static_assert(!kGen || KIND < 3, "in-kernel generation: rectification solvers");
    // compute waves: 15, or 14 plus the look-ahead generator wave (kGen)
    constexpr int kW = kGen ? kFmWaves - 1 : kFmWaves;
    constexpr uint32_t kRound = kW * 64u;
    constexpr int kCap = 64 * H;                        // pairs of one wave-round
    // packed inlier values (-r^2) of hypothesis q in wave w's features, in
    // feature order, zero-padded to whole chain batches
    // region stride 66 doubles: the 16 chain lanes' 16-byte reads (and the
    // exact pass's scattered writes) fall in distinct banks
    constexpr int kReg = 66;
    constexpr bool kDyn = KIND >= 3;                    // regions + queues in dynamic LDS (above)
    static_assert(!kDyn || fm_dyn_lds_bytes<H, kGen>() == (size_t)kW * H * kReg * 8 + (size_t)kW * kCap * 2,
                  "dynamic LDS layout");
    __shared__ double2 outv_st[kDyn ? 1 : kW][H][kReg / 2];
    // survivors: q | lane << 4 | k << 10; the rectification pre-band's
    // branch-free writes put non-survivors in 32 spare entries per wave
    // (lanes l and l + 32 share one: either value may land, neither is read)
    constexpr int kQStride = kDyn ? kCap : kCap + 32;
    __shared__ uint16_t queue_st[kDyn ? 1 : kW][kQStride];
    extern __shared__ double2 fm_dyn_lds[];
    double2 (*const outv)[H][kReg / 2] =
        kDyn ? reinterpret_cast<double2 (*)[H][kReg / 2]>(fm_dyn_lds) : outv_st;
    uint16_t (*const queue)[kQStride] =
        kDyn ? reinterpret_cast<uint16_t (*)[kQStride]>(fm_dyn_lds + (size_t)kW * H * (kReg / 2)) : queue_st;
    __shared__ uint32_t wcnt[2][kW][H];                 // survivors of (wave, q) in the round
    __shared__ uint32_t ready[kW], done[kW];
    __shared__ HypConst hyp[H];
    __shared__ uint32_t hval[H];
    __shared__ uint32_t cnt_sh[2][H];
    __shared__ uint32_t fl_sh[H];                       // flagged pairs (exact.h), rectification solvers
    using PairBand = std::conditional_t<KIND == 3, HPairBand, FPairBand>;
    static_assert(KIND >= 3 || (H & 1) == 0, "rectification pre-band: hypotheses in pairs");
    static_assert(sizeof(PairBand) == sizeof(RPairBand), "pair-band records share one LDS array");
    // the correspondence pre-band records or the rectification ones
    __shared__ RPairBand pb_st[(H + 1) / 2];
    PairBand* const fpb = reinterpret_cast<PairBand*>(pb_st);
    RPairBand* const rpb = pb_st;
    // the value log's table (detmath.h) in LDS: the fused variant has the
    // room (the others read it from L2)
    __shared__ double logtab_sh[kGen ? dm::kLogTabSize : 1];
    __shared__ int gen_a[kGen ? H : 1];
    __shared__ RectModel gen_m[kGen ? H : 1];
    __shared__ double fin_sh[kGen ? H : 1];
    // the look-ahead wave's generated slots (models, attempts)
    __shared__ RectModel nx_m[kGen ? H : 1];
    __shared__ int nx_a[kGen ? H : 1];

    const int t = threadIdx.x;
    const int wave = t >> 6;
    const int lane = t & 63;
    const bool chain_wave = wave == kFmWaves;

    const uint32_t n0 = p.cls[0].n;
    const uint32_t n1 = (KIND == 2) ? p.cls[1].n : 0;
    const uint32_t r0 = (n0 + kRound - 1) / kRound;
    const uint32_t rounds = r0 + (n1 + kRound - 1) / kRound;
    // a compute lane's feature of round rr (x, y, s | x2 | cos, - | y2 | sin)
    // (round 0's requested before the prologue instead of after it: 51.6
    // vs 52.6 x 10^7 hyp/s, the register it holds across the prologue
    // costs the main loop more than the overlap saves)
    auto load = [&](uint32_t rr, double* f, bool& ok) {
        const int cls = rr < r0 ? 0 : 1;
        const DevClass& c = p.cls[cls];
        const uint32_t i = (cls == 0 ? rr : rr - r0) * kRound + wave * 64 + lane;
        ok = i < c.n;
        const uint32_t ic = ok ? i : 0u;
        f[0] = c.x[ic];
        f[1] = c.y[ic];
        if (cls == 0) {
            f[2] = c.a[ic];
            f[3] = (KIND >= 3) ? c.c0[ic] : 0.0;
        } else {
            f[2] = c.c0[ic];
            f[3] = c.c1[ic];
        }
    };

    __shared__ uint32_t smap[KIND >= 3 ? H : 1];
    if constexpr (KIND >= 3) {
        if (gen.scan) {
            // in-order compaction of the launch's live hypotheses (k_compact's
            // result, computed by every workgroup): each thread counts a
            // contiguous chunk, a block scan gives the chunk's first rank,
            // and the chunks holding ranks [blockIdx.x H, + H) fill smap
            __shared__ uint32_t wsum[kSplitThreads / 64];
            __shared__ uint32_t tot_sh;
            const int tid = threadIdx.x, ln = tid & 63, wv = tid >> 6;
            const uint32_t per = (nh + kSplitThreads - 1) / kSplitThreads;
            const uint32_t j0 = min(nh, tid * per), j1 = min(nh, j0 + per);
            uint32_t c = 0;
            for (uint32_t j = j0; j < j1; ++j) c += inc[j] <= 101 ? 1u : 0u;
            uint32_t x = c;                                 // inclusive scan in the wave
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(x, d);
                if (ln >= d) x += o;
            }
            if (ln == 63) wsum[wv] = x;
            __syncthreads();
            if (tid == 0) {
                uint32_t a = 0;
                for (int w = 0; w < kSplitThreads / 64; ++w) {
                    const uint32_t v = wsum[w];
                    wsum[w] = a;
                    a += v;
                }
                tot_sh = a;
            }
            __syncthreads();
            const uint32_t lo = blockIdx.x * H;
            uint32_t r = wsum[wv] + x - c;                  // rank of this chunk's first live entry
            if (r < lo + H && r + c > lo)
                for (uint32_t j = j0; j < j1; ++j)
                    if (inc[j] <= 101) {
                        if (r >= lo && r < lo + H) smap[r - lo] = j;
                        ++r;
                    }
            __syncthreads();
            const uint32_t total = tot_sh;
            if (blockIdx.x == 0 && tid == 0) *const_cast<uint32_t*>(gen.hcount) = total;
            if (tid < H && lo + tid < total) const_cast<uint32_t*>(gen.hmap)[lo + tid] = smap[tid];
            nh = total;
            if (lo >= nh) return;                           // whole workgroup
        } else {
            // compacted launches: hypotheses [0, *hcount) are models hmap[j]
            if (gen.hcount != nullptr) nh = min(nh, *gen.hcount);
            if (blockIdx.x * H >= nh) return;            // whole workgroup, before any barrier
            if (threadIdx.x < H && gen.hmap != nullptr && blockIdx.x * H + threadIdx.x < nh)
                smap[threadIdx.x] = gen.hmap[blockIdx.x * H + threadIdx.x];
        }
    }
    GCR_STAMP(5, 15u);
    if (threadIdx.x == 0) GCR_WGSPAN(0);
#ifdef GCR_STAMPS
    if (threadIdx.x == 0 && blockIdx.x < (uint32_t)kSpanWG) g_wgspan[blockIdx.x][2] = 0;
    __syncthreads();
#endif
    // ---- prologue: this workgroup's H slots (kGen), k_generate's rule, or
    // (chained batches) the previous launch's look-ahead wave's results
    if constexpr (kGen) {
      if (gen.chain.pre_inc != nullptr) {
        // the previous launch's look-ahead results (each thread t < H its
        // own slot: no barrier before the slot's outputs)
        if (t < H) {
            const uint32_t hs = blockIdx.x * H + t;
            const uint8_t iv = hs < nh ? gen.chain.pre_inc[hs] : (uint8_t)102;
            const RectModel m = iv > 101 ? default_model() : gen.chain.pre_models[hs];
            gen_a[t] = iv > 101 ? 127 : (int)iv - 1;
            gen_m[t] = m;
            if (hs < nh) {
                gen.inc[hs] = iv;
                gen.models[hs] = m;
            }
        }
      } else {
        const int G = gen.glanes ? (int)gen.glanes : kSplitThreads / H;
        const bool gact = t < H * G;
        if (t < H) gen_a[t] = 127;
        __syncthreads();
        const int gh = gact ? t / G : 0, g = t % G;
        const uint32_t gs = blockIdx.x * H + gh;
        for (uint32_t rr = 0; rr * G < 101; ++rr) {
            const uint32_t a = rr * G + g;
            RectModel m = default_model();
            bool ok = false;
            if (gact && gs < nh && a < 101 && gen_a[gh] == 127)
                ok = (gen.probe & 8u) ? a == 0 : attempt<KIND>(p, gen.seed, gen.slot0 + gs, a, m);
            if (ok) atomicMin(&gen_a[gh], (int)a);
            __syncthreads();
            if (ok && gen_a[gh] == (int)a) gen_m[gh] = m;
            bool all = true;
            for (int q = 0; q < H; ++q) all = all && (gen_a[q] != 127 || blockIdx.x * H + q >= nh);
            __syncthreads();
            if (all) break;
        }
        if (t < H && blockIdx.x * H + t < nh) {
            const int a = gen_a[t];
            gen.inc[blockIdx.x * H + t] = (uint8_t)(a == 127 ? 102 : a + 1);
            gen.models[blockIdx.x * H + t] = a == 127 ? default_model() : gen_m[t];
        }
      }
    }
    if (t < H) {
        const uint32_t hg = blockIdx.x * H + t;
        const uint32_t mi = (KIND >= 3 && gen.hmap != nullptr && hg < nh) ? smap[t] : hg;
        const bool v = hg < nh && (kGen ? gen_a[t] != 127 : (inc == nullptr || inc[mi] <= 101));
        typename ModelOf<KIND>::type m = ModelOf<KIND>::def();
        if (v) {
            if constexpr (kGen && KIND < 3) m = gen_m[t];
            else m = models[mi];
        }
        bool copied = false;
        if constexpr (kGen && KIND <= 2) {
            // constants the previous launch's look-ahead wave computed for
            // this slot (the same make_hyp / rpb_setup of the same model)
            if (gen.chain.pre_inc != nullptr && gen.chain.pre_hyp != nullptr && hg < nh) {
                hyp[t] = static_cast<const HypConst*>(gen.chain.pre_hyp)[hg];
                const float* src = reinterpret_cast<const float*>(static_cast<const RPairBand*>(gen.chain.pre_pair) +
                                                                  (hg >> 1));
                float* dst = reinterpret_cast<float*>(&rpb[t >> 1]);
#pragma unroll
                for (int k = 0; k < 11; ++k) dst[2 * k + (t & 1)] = src[2 * k + (hg & 1)];
                copied = true;
            }
        }
        if (!copied) {
            hyp[t] = make_hyp<KIND>(m, band0);
            if constexpr (KIND <= 2) rpb_setup(rpb, t, hyp[t], p.cls[0], p.cls[1], tan_tau1, KIND == 2, v);
        }
        if constexpr (KIND == 4) fpb_setup(fpb, t, m.h, v, T0, p.cls[0]);
        if constexpr (KIND == 3) hpb_setup(fpb, t, m.h, v, band0, p.cls[0]);
        hval[t] = v ? 1u : 0u;
        cnt_sh[0][t] = 0;
        cnt_sh[1][t] = 0;
        fl_sh[t] = 0;
    }
    if constexpr (KIND == 4) {
        if ((H & 1) && t == H) fpb_setup(fpb, t, hyp[0].g, false, T0, p.cls[0]);   // odd H: inert pad
    }
    if constexpr (KIND == 3) {
        if ((H & 1) && t == H) hpb_setup(fpb, t, hyp[0].g, false, band0, p.cls[0]);
    }
    GCR_STAMP(6, 15u);
    if constexpr (kGen) {
        for (int i = t; i < dm::kLogTabSize; i += kSplitThreads) logtab_sh[i] = dm::kLogTab[i];
    }
    const double* const logtab = kGen ? logtab_sh : dm::kLogTab;
    if (t < kW) { ready[t] = 0; done[t] = 0; }
    __syncthreads();
    GCR_STAMP(7, 15u);

    if constexpr (kGen) {
        if (wave == kW) {
            // ------------------------------------------ look-ahead generator
            // the next batch's slots of this workgroup (blockIdx.x * H + sl,
            // slot index slot0 + ahead nh + ...), k_generate_fw's widening lane
            // groups: the H slots start with 64 / H lanes each, and after
            // every round the unfinished ones share the whole wave (64 /
            // pow2ceil(k) lanes for k left) from one wave-uniform lowest
            // untried attempt, so each slot's result is still its lowest
            // successful attempt (k_generate's rule).  ~4 attempts per slot at
            // 50 % outliers: fixed groups of 4 lanes needed 3-5 rounds of
            // attempt latency for the slowest of 16 slots, widening ~2-3.
            // Overlaps the rounds below; no barrier follows.
            if (gen.chain.next_inc == nullptr) return;
            const uint32_t hs0 = blockIdx.x * H;
            const uint32_t live = hs0 < nh ? min((uint32_t)H, nh - hs0) : 0u;
            uint64_t pend = live >= 64u ? ~0ull : (1ull << live) - 1ull;
            uint32_t nx = 0;                    // wave-uniform lowest untried attempt
            while (pend) {
                const int k = __builtin_popcountll(pend);
                const int lw = 6 - (k == 1 ? 0 : 32 - __builtin_clz((uint32_t)(k - 1)));
                const int j = lane >> lw;
                const uint32_t a = nx + (uint32_t)(lane & ((1 << lw) - 1));
                int si = -1;                    // this lane's slot: the j-th unfinished one
                {
                    uint64_t m = pend;
                    for (int c = 0; m; ++c) {
                        const int i = __builtin_ctzll(m);
                        m &= m - 1;
                        si = c == j ? i : si;
                    }
                }
                RectModel m = default_model();
                bool ok = false;
                if (si >= 0 && a < 101)
                    ok = (gen.probe & 8u) ? a == 0
                                          : attempt<KIND>(p, gen.seed, gen.slot0 + (uint64_t)gen.chain.ahead * nh + hs0 + (uint32_t)si, a, m);
                const uint64_t mask = __ballot(ok);
                nx += 1u << lw;
                const bool out_of_attempts = nx >= 101;
                uint64_t np = out_of_attempts ? 0ull : pend;
                bool win = false;
                {
                    uint64_t mm = pend;
                    for (int c = 0; mm; ++c) {
                        const int i = __builtin_ctzll(mm);
                        mm &= mm - 1;
                        const uint64_t grp = lw == 6 ? mask : (mask >> (c << lw)) & ((1ull << (1 << lw)) - 1ull);
                        if (grp) {
                            np &= ~(1ull << i);
                            win |= lane == (c << lw) + __builtin_ctzll(grp);
                        }
                    }
                }
                const uint64_t gm = lw == 6 ? ~0ull : ((1ull << (1 << lw)) - 1ull);
                const bool fail = out_of_attempts && si >= 0 && !((mask >> (j << lw)) & gm) &&
                                  (lane & ((1 << lw) - 1)) == 0;
                pend = np;
                const uint32_t hs = hs0 + (uint32_t)si;
                if (win) {
                    gen.chain.next_inc[hs] = (uint8_t)(a + 1);
                    gen.chain.next_models[hs] = m;
                    nx_m[si] = m;
                    nx_a[si] = (int)a;
                } else if (fail) {              // every attempt failed (inc 102, no model)
                    gen.chain.next_inc[hs] = 102;
                    gen.chain.next_models[hs] = default_model();
                    nx_a[si] = 127;
                }
            }
            if (gen.chain.next_hyp == nullptr) return;
            // the slots' constants for the next launch's prologue (make_hyp
            // and rpb_setup as the prologue would run them), one lane a slot
            __builtin_amdgcn_wave_barrier();
            if (lane < (int)live) {
                const bool v = nx_a[lane] != 127;
                const RectModel m = v ? nx_m[lane] : default_model();
                const HypConst q = make_hyp<KIND>(m, band0);
                static_cast<HypConst*>(gen.chain.next_hyp)[hs0 + (uint32_t)lane] = q;
                rpb_setup(static_cast<RPairBand*>(gen.chain.next_pair) + (hs0 >> 1), lane, q, p.cls[0], p.cls[1],
                          tan_tau1, KIND == 2, v);
            }
            return;
        }
    }

    if (!chain_wave) {
        // ---------------------------------------------------- compute waves
        uint64_t vmask = __ballot(lane < H && hval[lane < H ? lane : 0] != 0);
        if (gen.probe & 4u) vmask = 0;
        uint16_t* qw = queue[wave];
        double nxt[4];
        bool nok = false;
        if (rounds > 0) load(0, nxt, nok);
        for (uint32_t r = 0; r < rounds; ++r) {
            GCR_STAMP(0, r);
            const double f0 = nxt[0], f1 = nxt[1], f2 = nxt[2], f3 = nxt[3];
            const bool ok = nok;
            if (r + 1 < rounds) load(r + 1, nxt, nok);
            const int cls = r < r0 ? 0 : 1;
            // 1) band test against each hypothesis.  Each lane holds one
            //    feature, so q's survivors are one ballot: survivor k of q (in
            //    feature order) owns slot k of the region outv[wave][q], and
            //    the queue entry q | lane << 4 | k << 10 carries all of it
            uint32_t qn = 0, my_n = 0;
            uint32_t* wc = wcnt[r & 1][wave];
            // one fully unrolled hypothesis loop per band (the class is
            // uniform over a round): no class branch per q, the band itself
            // branch-free and evaluated on every lane (out-of-range lanes
            // read feature 0 and are masked after), the next hypothesis's
            // constants read from LDS while this one is tested, q's run
            // length written to lane q with one v_writelane
            auto run_band = [&](auto load, auto band) {
                auto cur = load(0);
                static_for<0, H>([&](auto qc) {
                    constexpr int q = decltype(qc)::value;
                    decltype(cur) nxt = cur;
                    if constexpr (q + 1 < H) nxt = load(q + 1);
                    if ((vmask >> q) & 1ull) {
                        const bool cand = ok & band(cur);
                        const uint64_t m = __builtin_amdgcn_ballot_w64(cand);
                        const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                        if (cand) qw[qn + k] = (uint16_t)(q | (lane << 4) | (k << 10));
                        const uint32_t c = (uint32_t)__builtin_popcountll(m);
                        my_n = write_lane<q>(my_n, c);
                        qn += c;
                    }
                    cur = nxt;
                });
            };
            struct C4 { double a, b, c, d; };
            if (__ballot(ok) != 0) {
                if constexpr (KIND >= 3) {
                if (KIND == 4 || !(gen.probe & 128u)) {
                    // correspondences: the packed fp32 pre-band (above), two
                    // hypotheses per pass; survivors go to the exact pass
                    // (GCR_PROBE bit 7: the homography's fp64 band instead)
                    const float x1 = (float)f0, y1 = (float)f1, x2 = (float)f2, y2 = (float)f3;
#pragma unroll 1
                    for (int q = 0; q < H; q += 2) {
                        if (!((vmask >> q) & 3ull)) continue;
                        bool rj[2];
                        pb_test(fpb[q >> 1], x1, y1, x2, y2, rj[0], rj[1]);
#pragma unroll
                        for (int o = 0; o < 2; ++o) {
                            const int qq = q + o;
                            if (qq >= H || !((vmask >> qq) & 1ull)) continue;
                            const bool cand = ok & !rj[o];
                            const uint64_t m = __builtin_amdgcn_ballot_w64(cand);
                            const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                            if (cand) qw[qn + k] = (uint16_t)(qq | (lane << 4) | (k << 10));
                            const uint32_t c = (uint32_t)__builtin_popcountll(m);
                            my_n = lane == qq ? c : my_n;
                            qn += c;
                        }
                    }
                } else {
                    // homography, fp64 band: a rolled loop (the unrolled form holds
                    // ~126 VGPRs; these kernels are held to 64, see above)
#pragma unroll 1
                    for (int q = 0; q < H; ++q) {
                        if (!((vmask >> q) & 1ull)) continue;
                        const bool cand = ok & geo_band<KIND>(f0, f1, f2, f3, hyp[q].g, band0);
                        const uint64_t m = __builtin_amdgcn_ballot_w64(cand);
                        const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                        if (cand) qw[qn + k] = (uint16_t)(q | (lane << 4) | (k << 10));
                        const uint32_t c = (uint32_t)__builtin_popcountll(m);
                        my_n = lane == q ? c : my_n;
                        qn += c;
                    }
                }
                } else if (!(gen.probe & 1024u)) {
                    // rectification: the packed fp32 pre-band (above), two
                    // hypotheses per pass; every mask a direct compare ballot
                    const uint64_t okm = (gen.probe & 4u) ? 0ull : __builtin_amdgcn_ballot_w64(ok);
                    float pa = 0.0f, pb = 0.0f, pc = 0.0f;
                    if (cls == 0) {
                        pa = (float)f0;
                        pb = (float)f1;
                        pc = (f2 >= 0x1p-100 && f2 <= 0x1p100) ? (float)f2 : __builtin_nanf("");
                    } else {
                        const float xf = (float)f0, yf = (float)f1;
                        pb = (float)f2;                     // cos theta
                        pc = (float)f3;                     // sin theta
                        pa = __builtin_fmaf(xf, pc, -(yf * pb));   // g = x st - y ct
                    }
                    // one survivor record per hypothesis, branch-free (one
                    // basic block per class for all H, so the scheduler
                    // overlaps the pairs): a non-survivor lane writes its
                    // entry to a spare slot; invalid hypotheses reject every
                    // feature by their constants (rpb_setup)
                    auto emit = [&](auto qc, uint64_t rej) {
                        constexpr int q = decltype(qc)::value;
                        const uint64_t m = okm & ~rej;
                        const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                        const bool cand = __builtin_amdgcn_inverse_ballot_w64(m);
                        qw[cand ? qn + k : (uint32_t)(kCap + (lane & 31))] = (uint16_t)(q | (lane << 4) | (k << 10));
                        const uint32_t c = (uint32_t)__builtin_popcountll(m);
                        my_n = write_lane<q>(my_n, c);
                        qn += c;
                    };
                    // the next pair's constants are read before this pair's
                    // queue writes (the reads cannot be moved across them)
                    if (cls == 0) {
                        RScaleC cur = rpb_scale_c(rpb[0]);
                        static_for<0, H / 2>([&](auto jc) {
                            constexpr int j = decltype(jc)::value;
                            RScaleC nxt = cur;
                            if constexpr (j + 1 < H / 2) nxt = rpb_scale_c(rpb[j + 1]);
                            uint64_t r0, r1;
                            rpb_scale(cur, pa, pb, pc, r0, r1);
                            emit(std::integral_constant<int, 2 * j>{}, r0);
                            emit(std::integral_constant<int, 2 * j + 1>{}, r1);
                            cur = nxt;
                        });
                    } else {
                        ROrientC cur = rpb_orient_c(rpb[0]);
                        static_for<0, H / 2>([&](auto jc) {
                            constexpr int j = decltype(jc)::value;
                            ROrientC nxt = cur;
                            if constexpr (j + 1 < H / 2) nxt = rpb_orient_c(rpb[j + 1]);
                            uint64_t r0, r1;
                            rpb_orient(cur, pa, pb, pc, r0, r1);
                            emit(std::integral_constant<int, 2 * j>{}, r0);
                            emit(std::integral_constant<int, 2 * j + 1>{}, r1);
                            cur = nxt;
                        });
                    }
                } else if (cls == 0) {
                    run_band([&](int q) { return C4{hyp[q].h7, hyp[q].h8, hyp[q].lo, hyp[q].hi}; },
                             [&](const C4& c) {
                                 HypConst hq;
                                 hq.h7 = c.a; hq.h8 = c.b; hq.lo = c.c; hq.hi = c.d;
                                 return scale_band<KIND>(f0, f1, f2, hq);
                             });
                } else if constexpr (KIND == 2) {
                    run_band([&](int q) { return C4{hyp[q].h7, hyp[q].h8, hyp[q].cf, hyp[q].sf}; },
                             [&](const C4& c) {
                                 HypConst hq;
                                 hq.h7 = c.a; hq.h8 = c.b; hq.cf = c.c; hq.sf = c.d;
                                 return orient_band(f0, f1, f2, f3, hq, tan_tau1);
                             });
                }
            }
            if (gen.probe & 2u) qn = my_n = 0;
            if (lane < H) wc[lane] = my_n;                 // survivors (run length) of (wave, q)
            GCR_STAMP(1, r);
            // 2) + 3) exact residuals of the survivors, all 64 lanes busy: -r^2
            //    for an inlier, +0.0 (an exact no-op of the sum) otherwise.
            //    Each 64-survivor batch's queue entries and features are
            //    requested one batch ahead: the first batch's before waiting
            //    for the chain to release outv (the L2 latency hides behind
            //    the wait), the next batch's before this one is evaluated
            struct Surv {
                double x, y, a2, a3;
                uint32_t e;
#ifdef GCR_FM_HQ_AHEAD
                double h7, h8, c0, c1, c2, c3;    // the entry's hypothesis constants, read with it
#endif
            };
            // the round's class columns, selected once (uniform pointers:
            // no per-batch address arithmetic on a class index)
            const double* const fx = cls == 0 ? p.cls[0].x : p.cls[1].x;
            const double* const fy = cls == 0 ? p.cls[0].y : p.cls[1].y;
            const double* const fa2 = cls == 0 ? p.cls[0].a : p.cls[1].c0;
            const double* const fa3 = KIND >= 3 ? p.cls[0].c0 : p.cls[1].c1;
            const uint32_t fbase = (cls == 0 ? r : r - r0) * kRound + wave * 64;
            const double fl_mid = cls == 0 ? fband.mid[0] : fband.mid[1];
            const double fl_half = cls == 0 ? fband.half[0] : fband.half[1];
            auto fetch = [&](uint32_t j0) {
                Surv sv;
                const uint32_t j = j0 + lane;
                sv.e = j < qn ? qw[j] : 0u;
                const int src = (int)((sv.e >> 4) & 63u);
                sv.a3 = 0.0;
                if (gen.probe & 32u) {
                    // the survivor's feature from its owner lane (LDS permute)
                    sv.x = __shfl(f0, src);
                    sv.y = __shfl(f1, src);
                    sv.a2 = __shfl(f2, src);
                    if (KIND >= 3 || cls == 1) sv.a3 = __shfl(f3, src);
                } else {
                    // ... or re-read from L2 (keeps the LDS pipe to the chain)
                    const uint32_t fi = fbase + (uint32_t)src;
                    sv.x = fx[fi];
                    sv.y = fy[fi];
                    sv.a2 = fa2[fi];
                    if (KIND >= 3 || cls == 1) sv.a3 = fa3[fi];
                }
#ifdef GCR_FM_HQ_AHEAD
                if constexpr (KIND <= 2) {
                    const HypConst& hq = hyp[sv.e & 15u];
                    sv.h7 = hq.h7;
                    sv.h8 = hq.h8;
                    if (cls == 0) {
                        sv.c0 = hq.ac;
                        sv.c1 = hq.cut;
                        sv.c2 = sv.c3 = 0.0;
                    } else {
                        sv.c0 = hq.cf;
                        sv.c1 = hq.sf;
                        sv.c2 = hq.cphi;
                        sv.c3 = hq.cphi2;
                    }
                }
#endif
                return sv;
            };
            // GCR_PROBE bit 6: no look-ahead (each batch fetched when used)
            const bool ahead = KIND < 3 && !(gen.probe & 64u);     // (registers, see above)
            Surv cur{};
            if (ahead && qn > 0) cur = fetch(0);
            // the chain has folded this wave's previous runs (outv reuse)
            if (r > 0 && !(gen.probe & 256u)) fm_wait_ge(&done[wave], r);
            GCR_STAMP(2, r);
            double* ow = reinterpret_cast<double*>(&outv[wave][0][0]);
            for (uint32_t j0 = 0; j0 < qn; j0 += 64) {
                if (!ahead) cur = fetch(j0);
                Surv nxt_s = cur;
                if (ahead && j0 + 64 < qn) nxt_s = fetch(j0 + 64);
                const bool v = j0 + lane < qn;
                const int q = (int)(cur.e & 15u);
                const uint32_t k = cur.e >> 10;
                if (v) {
                    const HypConst& hq = hyp[q];
                    double r2;
                    bool inl;
                    if constexpr (KIND >= 3) {
                        r2 = geo_sq_residual<KIND>(cur.x, cur.y, cur.a2, cur.a3, hq.g);
                        inl = r2 <= T0;
                    } else {
                        RectModel m = default_model();
#ifdef GCR_FM_HQ_AHEAD
                        m.h7 = cur.h7;
                        m.h8 = cur.h8;
                        if (cls == 0) {
                            r2 = scale_sq_value<KIND == 1, true>(cur.x, cur.y, cur.a2, m, cur.c0, cur.c1, logtab);
                            inl = r2 <= T0;
                        } else {
                            r2 = orient_sq_value<true>(cur.x, cur.y, cur.a2, cur.a3, m, cur.c0, cur.c1, cur.c2, cur.c3);
                            inl = r2 <= T1;
                        }
#else
                        m.h7 = hq.h7;
                        m.h8 = hq.h8;
                        if (cls == 0) {
                            r2 = scale_sq_value<KIND == 1, true>(cur.x, cur.y, cur.a2, m, hq.ac, hq.cut, logtab);
                            inl = r2 <= T0;
                        } else {
                            r2 = orient_sq_value<true>(cur.x, cur.y, cur.a2, cur.a3, m, hq.cf, hq.sf, hq.cphi, hq.cphi2);
                            inl = r2 <= T1;
                        }
#endif
                    }
                    ow[q * kReg + k] = inl ? -r2 : 0.0;
                    if (inl && !(gen.probe & 512u)) atomicAdd(&cnt_sh[cls][q], 1u);
                    // a decision the host rechecks with glibc (exact.h); rare
                    if (KIND <= 2 && in_flag_band(r2, fl_mid, fl_half)) atomicAdd(&fl_sh[q], 1u);
                }
                cur = nxt_s;
            }
            GCR_STAMP(3, r);
            GCR_STAMP_VAL(6, r, (uint64_t)qn);
#ifdef GCR_STAMPS
            if (lane == 0 && blockIdx.x < (uint32_t)kSpanWG) atomicAdd((unsigned long long*)&g_wgspan[blockIdx.x][2], (unsigned long long)qn);
#endif
            // 4) zero-pad each run to a whole chain batch
            {
                const int q = lane % H, part = lane / H;
                const uint32_t n = wc[q];
                const uint32_t end = (n + 2 * kFmCB - 1) & ~(uint32_t)(2 * kFmCB - 1);
#pragma unroll
                for (int i = 0; i < 2 * kFmCB * H / 64; ++i) {
                    const uint32_t s = n + part + i * (64 / H);
                    if (s < end) ow[q * kReg + s] = 0.0;
                }
            }
            fm_publish(&ready[wave], r + 1);
            GCR_STAMP(4, r);
        }
    } else {
        // ------------------------------------------------------- chain wave
        __builtin_amdgcn_s_setprio(3);
        // lanes [0, H): class sums; lanes [H, 2H) (KIND 2): the running total
        constexpr bool kTot = KIND == 2;
        const int h = lane % H;
        const int role = kTot ? lane / H : 0;
        const bool chain_lane = lane < (kTot ? 2 * H : H);
        double run = 0.0, hold = 0.0;
        uint32_t c0 = 0, c1 = 0;
        const bool fold_on = !(gen.probe & 1u) && chain_lane;
        for (uint32_t r = 0; r < rounds; ++r) {
            if (KIND == 2 && r == r0 && role == 0) {      // first orientation round
                hold = run;
                run = 0.0;
            }
            GCR_STAMP(0, r);
            // waves that have published round r (bit w), polled all at once
            auto poll = [&]() -> uint64_t {
                const uint32_t f = lane < kW
                                       ? __hip_atomic_load(&ready[lane], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)
                                       : 0u;
                return __ballot(lane < kW && f >= r + 1);
            };
            uint64_t rmask = poll();
            uint32_t n = 0;
            bool have = false;
#pragma unroll 1
            for (int w = 0; w < kW; ++w) {
                while (!((rmask >> w) & 1ull)) {
                    __builtin_amdgcn_s_sleep(1);
                    rmask = poll();
                }
                if (!have) n = wcnt[r & 1][w][h];
                // the next run's length, read ahead if that wave has published
                const bool nhave = w + 1 < kW && ((rmask >> (w + 1)) & 1ull);
                const uint32_t nn = nhave ? wcnt[r & 1][w + 1][h] : 0u;
                if (fold_on) {
                    // whole batches of kFmCB 16-byte reads (zero-padded runs)
                    const double2* reg = outv[w][h];
                    // all of a batch's reads in flight before its adds, one
                    // batch at a time (a ping-pong variant with the next
                    // batch's reads in flight during the adds measured
                    // slower in rounds 1 and 6: MEASUREMENTS.md §2)
                    for (uint32_t j = 0; j < n; j += 2 * kFmCB) {
                        double2 v[kFmCB];
#pragma unroll
                        for (int u = 0; u < kFmCB; ++u) v[u] = reg[j / 2 + u];
#pragma unroll
                        for (int u = 0; u < kFmCB; ++u) {
                            run += v[u].x;
                            run += v[u].y;
                        }
                    }
                }
                // this wave's region is consumed (the adds used every read)
                __hip_atomic_store(&done[w], r + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                n = nn;
                have = nhave;
            }
            GCR_STAMP(4, r);
        }
        const uint32_t hg = blockIdx.x * H + h;
        const bool valid_h = hval[h] != 0;
        // inlier counts: every compute wave's last atomics precede its final
        // publication, which the loop above has acquired
        c0 = cnt_sh[0][h];
        c1 = cnt_sh[1][h];
        double tot = run;
        if constexpr (kTot) tot = __shfl(run, (lane + H) & 63);
        if (lane < H && hg < nh) {
            const double acc0 = KIND == 2 ? hold : run;
            const double acc1 = KIND == 2 ? run : 0.0;
            const uint32_t k0 = valid_h ? c0 : 0, k1 = valid_h ? c1 : 0;
            out.n0[hg] = k0;
            out.n1[hg] = k1;
            out.v0[hg] = valid_h ? acc0 : 0.0;
            out.v1[hg] = valid_h ? acc1 : 0.0;
            out.tot[hg] = valid_h ? tot : 0.0;
            if (KIND <= 2 && out.fl) out.fl[hg] = valid_h ? fl_sh[h] : 0u;
            if constexpr (kGen) {
                // MSACScoringFunction::getScore finish (MSAC_scoring_function.hpp:108-127)
                double sum = 0.0;
                if (valid_h && k0 >= gen.m0 && (KIND != 2 || k1 >= gen.m1)) {
                    sum = tot;
                    const double ms0 = acc0 / T0 + static_cast<double>(k0);
                    sum -= acc0;
                    sum += ms0;
                    if (KIND == 2) {
                        const double ms1 = acc1 / T1 + static_cast<double>(k1);
                        sum -= acc1;
                        sum += ms1;
                    }
                }
                const bool cand = valid_h && sum > 0.0 && (KIND != 2 || valid_model_sift22(gen_m[h]));
                fin_sh[h] = cand ? sum : -1.0;
            }
        }
        if constexpr (kGen) {
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) {
                // the workgroup's first strict best, slots in order
                WgBest b{0.0, -1, 0, 0, 0, 0};
                for (int q = 0; q < H; ++q) {
                    const uint32_t gq = blockIdx.x * H + q;
                    if (gq >= nh) break;
                    const int a = gen_a[q];
                    b.iterations += (uint64_t)(a == 127 ? 102 : a + 1);
                    if (a != 127) ++b.models;
                    const double s = fin_sh[q];
                    if (s > 0.0 && b.score < s) {
                        b.score = s;
                        b.slot = (int32_t)gq;
                        b.n0 = cnt_sh[0][q];
                        b.n1 = KIND == 2 ? cnt_sh[1][q] : 0;
                    }
                }
                gen.wg[blockIdx.x] = b;
            }
        }
        GCR_WGSPAN(1);
    }
}


// ------------------------------------------------- small-batch scoring ----
// model mi's results are written: publish done[mi] = epoch to the host
// (system-scope release first, so the results and the list bits -- coherent
// host memory -- are visible before the flag)
__device__ __forceinline__ void signal_done(const ScoreOut& out, uint32_t mi) {
    if (out.done == nullptr) return;
    __threadfence_system();
    __hip_atomic_store(out.done + mi, out.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// LO trials, refits and reconciliations score a handful of models, so the
// per-workgroup sequential chain of the batch scorers (~90 us at N = 10 000)
// is the whole cost.  Here every (model, feature) pair is evaluated in
// parallel (k_lo_values: -r^2 or +0.0 per pair plus an inlier bitmask, in
// HBM), and one workgroup per model then compacts the inlier values in
// feature order into LDS and one lane adds them (k_lo_chain), so the
// dependent chain holds only the inliers and no compute traffic competes
// with it.  The sums are the reference's sequential
// sums (MSAC_scoring_function.hpp:73-85): inliers in index order, class 0
// then class 1, the running total continuing across classes.
//
// Layout per model: class 0 at [0, pad0), class 1 at [pad0, pad0 + pad1),
// pad_c = n_c rounded up to 64 (unused pairs: value 0, bit 0).
// mask rule of k_mask / launch_mask on a residual: mask_rule, exact.h

// k_lo_chain: one 1024-thread workgroup per model, blocks of kLoBlock
// features.  All 16 waves load the block's values and ballot words at once
// (one memory round trip; a single wave walking 1024-feature spans spent
// 42 us per launch at N = 10 000, mostly waiting on its span loads), compact
// the inlier values in feature order into LDS (chunk popcounts, one wave's
// scan), and wave 0 folds them: lane 0 the class sum, lane 1 (KIND 2) the
// running total.  Blocks alternate between two sets of LDS buffers, so the
// next block's loads are issued while wave 0 still folds.
// DPP helpers of the exact folds below (fp64 moves, wave scan, readlane)
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_f64(double x) {      // DPP move of an fp64 value, 0 where nothing moves in
    const uint64_t u = as_u64(x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, ROWS, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, ROWS, 0xf, true);
    return as_f64(((uint64_t)(uint32_t)hi << 32) | (uint64_t)(uint32_t)lo);
}
__device__ __forceinline__ double wave_incl_scan_f64(double x) {
    x = x + dpp_f64<0x111, 0xf>(x);     // row_shr:1
    x = x + dpp_f64<0x112, 0xf>(x);     // row_shr:2
    x = x + dpp_f64<0x114, 0xf>(x);     // row_shr:4
    x = x + dpp_f64<0x118, 0xf>(x);     // row_shr:8
    x = x + dpp_f64<0x142, 0xa>(x);     // row_bcast:15 into rows 1, 3
    x = x + dpp_f64<0x143, 0xc>(x);     // row_bcast:31 into rows 2, 3
    return x;
}
// the same DPP pattern for 32-bit integers
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xf, true);
}
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t x) {
    x += dpp_u32<0x111, 0xf>(x);
    x += dpp_u32<0x112, 0xf>(x);
    x += dpp_u32<0x114, 0xf>(x);
    x += dpp_u32<0x118, 0xf>(x);
    x += dpp_u32<0x142, 0xa>(x);
    x += dpp_u32<0x143, 0xc>(x);
    return x;
}
// segmented inclusive scan: lanes with equal key (non-decreasing over the
// wave) form the segments; each lane gets the sum over its segment up to it
template <int CTRL, int ROWS>
__device__ __forceinline__ double seg_step(double x, uint32_t key) {
    const double y = dpp_f64<CTRL, ROWS>(x);
    const uint32_t k = dpp_u32<CTRL, ROWS>(key);
    return k == key ? x + y : x;
}
__device__ __forceinline__ double wave_seg_scan_f64(double x, uint32_t key) {
    x = seg_step<0x111, 0xf>(x, key);
    x = seg_step<0x112, 0xf>(x, key);
    x = seg_step<0x114, 0xf>(x, key);
    x = seg_step<0x118, 0xf>(x, key);
    x = seg_step<0x142, 0xa>(x, key);
    x = seg_step<0x143, 0xc>(x, key);
    return x;
}
__device__ __forceinline__ double readlane_f64(double x, int l) {
    const uint64_t u = as_u64(x);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
    return as_f64(((uint64_t)hi << 32) | lo);
}

constexpr uint32_t kLoBlock = 8192;                    // features per block (128 chunks of 64)
constexpr uint32_t kLoChunks = kLoBlock / 64;
constexpr int kLoThreads = 1024;
constexpr int kLoPer = kLoChunks / (kLoThreads / 64); // chunks per wave per block

// The one-lane in-order fold of k_lo_chain: ping-pong batches of 16 LDS
// reads, the next batch in flight during the current batch's dependent adds
// (sched_barrier keeps the scheduler from sinking the reads back next to
// their adds).
__device__ __forceinline__ double fold_seq_lane(const double* __restrict__ cb, uint32_t k, const uint32_t e,
                                                double run, const uint32_t cap = kLoBlock) {
    if (k + 32 <= e) {
        double ta[16], tb[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) ta[u] = cb[k + u];
#pragma unroll 1
        for (; k + 32 <= e; k += 32) {
#pragma unroll
            for (int u = 0; u < 16; ++u) tb[u] = cb[k + 16 + u];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 16; ++u) run += ta[u];
            __builtin_amdgcn_sched_barrier(0);
            // the batch after next (clamped inside the buffer of cap >= e
            // values: a clamped batch lies past e and is never added)
            const uint32_t nx = min(k + 32, cap - 16);
#pragma unroll
            for (int u = 0; u < 16; ++u) ta[u] = cb[nx + u];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 16; ++u) run += tb[u];
            __builtin_amdgcn_sched_barrier(0);
        }
        if (k + 16 <= e) {                         // ta = cb[k, k + 16)
#pragma unroll
            for (int u = 0; u < 16; ++u) run += ta[u];
            k += 16;
        }
    }
    for (; k < e; ++k) run += cb[k];
    return run;
}

// fold_seq_lane with batches of 8 (fewer registers: short ranges)
__device__ __forceinline__ double fold_seq_lane8(const double* __restrict__ cb, uint32_t k, const uint32_t e,
                                                 double run) {
    for (; k + 8 <= e; k += 8) {
        double t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = cb[k + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) run += t[u];
    }
    for (; k < e; ++k) run += cb[k];
    return run;
}

constexpr uint32_t kBlkHead = 128;                    // a chain from a given start (0 when continuing)
constexpr int kBlkSpecials = 63;
constexpr uint32_t kBlkMaxM = 16;                       // values per chunk, held in registers

struct BlkFoldScratch {
    double wsum[kLoThreads / 64];           // wave totals (approximate chunk sums)
    uint32_t wcnt[kLoThreads / 64];         // wave totals of the special counts
    double runA[kBlkSpecials + 1];
    int runEmin[kBlkSpecials + 1], runEmax[kBlkSpecials + 1];
    double specV[kBlkSpecials];
    uint32_t specPos[kBlkSpecials];
    uint32_t bad, nspec;
    double head, hexact, result;         // head: approximate (any order), hexact: in order
};

// One in-order sum of fold_exact_chains: the values cb[k, e) added to a
// start that is either given (from < 0) or the exact result of chain `from`
// (an earlier chain, walked first by the same wave).
struct BlkChain {
    uint32_t k, e;
    double start;
    int from;
};

// the walk of one chain's runs by one wave (wave-uniform): exact running sum
// s at position pos (after the head).  s + U A_r is one exact addition when s
// lies in run r's binade and the result stays in it; then special r by an
// ordinary addition.  The loop has no data-dependent branch: each run's
// checks only clear a sticky `ok` flag, and s / pos stop advancing at the
// first failed check (the serial dependence per run is one fma, one scaling
// and one addition).  A bad chain, too many specials or a failed check fold
// the rest value by value.
__device__ __forceinline__ double blk_walk(const double* __restrict__ cb, uint32_t pos, const uint32_t e, double s,
                                           const BlkFoldScratch& sc, const uint32_t cap, double* dbg = nullptr) {
    const int lane = threadIdx.x & 63;
    const uint32_t nspec = sc.nspec;
    if (sc.bad == 0 && nspec <= (uint32_t)kBlkSpecials) {
        const uint32_t nr = nspec + 1;
        // run r's record in lane r: its sum A_r, binade el (0: the parts
        // disagree), the scalings 2^(1075 - el) / 2^(el - 1075), special r
        const int rl = lane < (int)nr ? lane : 0;
        const double rA = sc.runA[rl];
        const int emin = sc.runEmin[rl], emax = sc.runEmax[rl];
        const uint32_t rE = emin == emax && emin >= 53 && emin < 0x7fe ? (uint32_t)emin : 0u;
        const uint32_t eu = rE != 0u ? rE : 1075u;
        const double up = as_f64((uint64_t)(2098u - eu) << 52), dn = as_f64((uint64_t)(eu - 52u) << 52);
        const double rV = lane < (int)nspec ? sc.specV[lane] : 0.0;
        const uint32_t rP = lane < (int)nspec ? sc.specPos[lane] + 1u : e;
        bool ok = true;
        for (uint32_t r = 0; r < nr; ++r) {
            const uint32_t el = (uint32_t)__builtin_amdgcn_readlane((int)rE, (int)r);
            const bool in_b = el != 0u && (uint32_t)(as_u64(s) >> 52) == (0x800u | el);   // s < 0 in binade el
            const double S = __builtin_fma(s, readlane_f64(up, (int)r), readlane_f64(rA, (int)r));
            const bool fits = (uint32_t)(as_u64(S) >> 52) == 0xc33u;                       // S in (-2^53, -2^52]
            ok = ok && in_b && fits;
            // s * 2^(1075 - el) is exact, so the fma rounds what s*U + A did
            const double sn = S * readlane_f64(dn, (int)r) + readlane_f64(rV, (int)r);
            s = ok ? sn : s;
            pos = ok ? (uint32_t)__builtin_amdgcn_readlane((int)rP, (int)r) : pos;
        }
    }
    if (dbg != nullptr && (threadIdx.x & 63) == 0) {
        dbg[0] = (double)pos;
        dbg[1] = (double)e;
    }
    if (pos < e) s = fold_seq_lane(cb, pos, e, s, cap);
    return s;
}

// a chunk of at most M values: its approximate sum (all reads in flight together)
template <uint32_t M>
__device__ __forceinline__ double blk_chunk_sum(const double* __restrict__ cb, const uint32_t b, const uint32_t ee) {
    double xv[M];
#pragma unroll
    for (uint32_t q = 0; q < M; ++q) xv[q] = b + q < ee ? cb[b + q] : 0.0;
    double a = 0.0;
#pragma unroll
    for (uint32_t q = 0; q < M; ++q)
        if (b + q < ee) a += xv[q];
    return a;
}

// a chunk's integer increments in up to three parts (two specials) from the
// approximate start P (fold_exact_chains, phase 2)
struct BlkParts {
    double acc, a0, a1, v0, v1;
    int e0, e1, el, ns;
    uint32_t q0, q1;
    bool bad;
};

template <uint32_t M>
__device__ __forceinline__ void blk_parts(const double* __restrict__ cb, const uint32_t b, const uint32_t ee, double P,
                                          BlkParts& o) {
    double xv[M];
#pragma unroll
    for (uint32_t q = 0; q < M; ++q) xv[q] = b + q < ee ? cb[b + q] : 0.0;
    bool bd = false;
    int be = (int)((as_u64(P) >> 52) & 0x7ffu);
    double ac = 0.0, a0 = 0.0, a1 = 0.0, v0 = 0.0, v1 = 0.0;
    int e0 = 0, e1 = 0, ns = 0;
    uint32_t q0 = 0, q1 = 0;
    const uint32_t len = ee - b;
#pragma unroll
    for (uint32_t q = 0; q < M; ++q) {
        if (q < len && !bd) {
            const double x = xv[q];
            be = (int)((as_u64(P) >> 52) & 0x7ffu);
            const double tt = x * as_f64((uint64_t)(2098 - be) << 52);
            const double r = __builtin_rint(tt);
            const double Pn = P + x;
            const bool sp = __builtin_fabs(tt - r) == 0.5 || (int)((as_u64(Pn) >> 52) & 0x7ffu) != be;
            bd = !(P < 0.0) || be < 53 || be >= 0x7fe || !(x <= 0.0) || !(__builtin_fabs(tt) < 0x1p53) ||
                 (sp && ns == 2);
            if (sp) {
                if (ns == 0) { a0 = ac; e0 = be; v0 = x; q0 = b + q; }
                else { a1 = ac; e1 = be; v1 = x; q1 = b + q; }
                ac = 0.0;
                ++ns;
            } else {
                ac += r;
            }
            P = Pn;
        }
    }
    o.acc = ac; o.a0 = a0; o.a1 = a1; o.v0 = v0; o.v1 = v1;
    o.e0 = e0; o.e1 = e1; o.ns = ns; o.q0 = q0; o.q1 = q1;
    o.bad = bd;
    o.el = ns > 0 ? (int)((as_u64(P) >> 52) & 0x7ffu) : be;
}

// fold_exact_chains: NC in-order sums by all kLoThreads threads of the
// workgroup at once, sharing the barriers (every thread calls it, in uniform
// control flow).  A chain from a given start adds its first kBlkHead values
// one by one (the sum is still small there and would cross a binade every
// few values; a continuing chain's sum is already large and has no head);
// thread t takes the t-th of the contiguous chunks of 4, 8 or 16 values of
// the rest.  A block scan of approximate chunk sums
// gives every chunk an approximate start (a continuing chain starts at the
// approximate total of the chain it continues); walking its chunk with an
// approximate running sum, a thread adds the integer increments rint(v / U)
// (U the ulp of the binade the running sum is predicted to be in) and marks
// as special every value whose addition is predicted to leave the binade, and
// every tie (v / U ending in exactly .5).  Specials are numbered in sequence
// order (a block scan of the per-thread counts); the parts between
// consecutive specials are runs: run r's increments are summed exactly
// (integers of one sign, below 2^53 whenever the run is valid) by a
// segmented wave scan and one LDS atomic per run and wave, its binade
// recorded.  Then wave c walks chain c (blk_walk) and, right after it, the
// chains continuing it.  A positive / NaN / too large value, a run whose
// parts disagree on the binade, more than two specials in a chunk or more
// than kBlkSpecials in all fold the chain value by value, as do chains too
// short or too long for the chunks.  res[c] = chain c's sum on every thread.
// tests/test_fold.py restates one chain in numpy (fold_exact_block).
template <int NC>
__device__ __forceinline__ void fold_exact_chains(const double* __restrict__ cb, const BlkChain (&ch)[NC],
                                                  BlkFoldScratch (&sc)[NC], const uint32_t cap, double (&res)[NC],
                                                  double* dbg = nullptr) {
    static_assert(NC <= kLoThreads / 64, "one wave per chain");
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    // cycle stamps after each barrier (k_fold3_test only)
    auto stamp = [&](int i) {
        if (dbg != nullptr && t == 0) dbg[i] = (double)__builtin_readcyclecounter();
    };
    stamp(0);
    bool seq[NC];
    uint32_t b[NC], ee[NC], m[NC], hl[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const uint32_t n = ch[c].e - ch[c].k;
        hl[c] = ch[c].from < 0 ? kBlkHead : 0u;
        seq[c] = n < hl[c] + kLoThreads / 4 || n - hl[c] > kBlkMaxM * (uint32_t)kLoThreads;
        const uint32_t rest = seq[c] ? 0u : n - hl[c];
        // values per chunk (uniform: the loops below are unrolled for 4, 8 or 16)
        // chunks of 4, 8 or 16 values (the fewest threads the length needs:
        // the VALU work scales with the busy waves)
        const uint32_t mneed = (uint32_t)__builtin_amdgcn_readfirstlane((int)((rest + kLoThreads - 1) / kLoThreads));
        m[c] = mneed <= 4u ? 4u : (mneed <= 8u ? 8u : kBlkMaxM);
        b[c] = ch[c].k + hl[c] + min(rest, (uint32_t)t * m[c]);
        ee[c] = ch[c].k + hl[c] + min(rest, (uint32_t)t * m[c] + m[c]);
        if (t <= kBlkSpecials) {
            sc[c].runA[t] = 0.0;
            sc[c].runEmin[t] = 0x7fffffff;
            sc[c].runEmax[t] = -1;
        }
        if (t == 0) sc[c].bad = 0;
    }
    // the heads (chains from a given start) on the last waves, which hold no
    // chunk unless the chain fills most of the chunks: here their sum in any
    // order (the chunks' approximate start), in phase 2 their in-order sum
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        if (wave != kLoThreads / 64 - 1 - c) continue;
        double h = 0.0;
        if (!seq[c] && ch[c].from < 0) {
            h = lane == 0 ? ch[c].start : 0.0;
            for (uint32_t q = (uint32_t)lane; q < hl[c]; q += 64) h += cb[ch[c].k + q];
        }
        h = wave_incl_scan_f64(h);
        if (lane == 63) sc[c].head = h;
    }
    // 1. approximate chunk sums, block scans
    double xin[NC], a[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        a[c] = m[c] <= 4 ? blk_chunk_sum<4>(cb, b[c], ee[c])
                         : (m[c] <= 8 ? blk_chunk_sum<8>(cb, b[c], ee[c]) : blk_chunk_sum<kBlkMaxM>(cb, b[c], ee[c]));
        xin[c] = wave_incl_scan_f64(a[c]);
        if (lane == 63) sc[c].wsum[wave] = xin[c];
    }
    __syncthreads();
    stamp(1);
#pragma unroll
    for (int c = 0; c < NC; ++c)
        if (t == kLoThreads - 64 * (c + 1) && !seq[c] && ch[c].from < 0)
            sc[c].hexact = fold_seq_lane8(cb, ch[c].k, ch[c].k + hl[c], ch[c].start);
    // 2. integer increments in up to three parts (two specials) per chunk
    BlkParts pt[NC];
    double total[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        // the earlier waves' totals: one read per lane, a row scan, readlanes
        const double wps = wave_incl_scan_f64(sc[c].wsum[lane & 15]);
        const double wpre = wave > 0 ? readlane_f64(wps, wave - 1) : 0.0;
        total[c] = sc[c].head + readlane_f64(wps, 15);
        double base = sc[c].head;
#pragma unroll
        for (int d = 0; d < c; ++d)
            if (ch[c].from == d) base += total[d];
        const double P = base + (wpre + (xin[c] - a[c]));  // approximate start of the chunk
        if (m[c] <= 4) blk_parts<4>(cb, b[c], ee[c], P, pt[c]);
        else if (m[c] <= 8) blk_parts<8>(cb, b[c], ee[c], P, pt[c]);
        else blk_parts<kBlkMaxM>(cb, b[c], ee[c], P, pt[c]);
    }
    double acc[NC], A0[NC], A1[NC], V0[NC], V1[NC];
    int E0[NC], E1[NC], El[NC], nsp[NC];
    uint32_t p0[NC], p1[NC];
    bool bad[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        acc[c] = pt[c].acc; A0[c] = pt[c].a0; A1[c] = pt[c].a1; V0[c] = pt[c].v0; V1[c] = pt[c].v1;
        E0[c] = pt[c].e0; E1[c] = pt[c].e1; El[c] = pt[c].el; nsp[c] = pt[c].ns; p0[c] = pt[c].q0; p1[c] = pt[c].q1;
        bad[c] = pt[c].bad;
    }
    // 3. number the specials: block scans of the per-thread counts
    uint32_t ci[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        ci[c] = wave_incl_scan_u32((uint32_t)nsp[c]);
        if (lane == 63) sc[c].wcnt[wave] = ci[c];
        if (bad[c]) atomicOr(&sc[c].bad, 1u);
    }
    __syncthreads();
    stamp(2);
    // the runs' increments.  Every thread's last part belongs to run
    // R = base + nsp; those of consecutive lanes with equal R are summed by a
    // segmented wave scan and added by the segment's last lane (one LDS atomic
    // per run and wave, not per thread); the binade is reported by the
    // segment's first and last lanes and by every lane whose binade differs
    // from its left neighbour's (a run whose parts disagree then shows
    // min != max).  The rare parts before a special are added one by one.
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const uint32_t wcs = wave_incl_scan_u32(sc[c].wcnt[lane & 15]);
        const uint32_t base =
            ci[c] - (uint32_t)nsp[c] + (wave > 0 ? (uint32_t)__builtin_amdgcn_readlane((int)wcs, wave - 1) : 0u);
        if (t == kLoThreads - 1) sc[c].nspec = base + (uint32_t)nsp[c];
        const bool fits = base + (uint32_t)nsp[c] <= (uint32_t)kBlkSpecials;
        const uint32_t R = fits ? base + (uint32_t)nsp[c] : 0xffffffffu;
        const double seg = wave_seg_scan_f64(acc[c], R);
        const uint32_t Rl = (uint32_t)__shfl_up((int)R, 1), Rr = (uint32_t)__shfl_down((int)R, 1);
        const int Ell = __shfl_up(El[c], 1);
        const bool first = lane == 0 || Rl != R, last = lane == 63 || Rr != R;
        if (fits && !bad[c]) {
            if (last && seg != 0.0) atomicAdd(&sc[c].runA[R], seg);
            if (first || last || Ell != El[c]) {
                atomicMin(&sc[c].runEmin[R], El[c]);
                atomicMax(&sc[c].runEmax[R], El[c]);
            }
            if (nsp[c] > 0) {
                if (A0[c] != 0.0) atomicAdd(&sc[c].runA[base], A0[c]);
                atomicMin(&sc[c].runEmin[base], E0[c]);
                atomicMax(&sc[c].runEmax[base], E0[c]);
                sc[c].specV[base] = V0[c];
                sc[c].specPos[base] = p0[c];
            }
            if (nsp[c] > 1) {
                if (A1[c] != 0.0) atomicAdd(&sc[c].runA[base + 1], A1[c]);
                atomicMin(&sc[c].runEmin[base + 1], E1[c]);
                atomicMax(&sc[c].runEmax[base + 1], E1[c]);
                sc[c].specV[base + 1] = V1[c];
                sc[c].specPos[base + 1] = p1[c];
            }
        }
    }
    __syncthreads();
    stamp(3);
    // 4. the walks: chain c on wave c, the chains continuing it right after
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        if (ch[c].from >= 0 || wave != c) continue;
        double s = seq[c] ? fold_seq_lane(cb, ch[c].k, ch[c].e, ch[c].start, cap)
                          : blk_walk(cb, ch[c].k + hl[c], ch[c].e, sc[c].hexact, sc[c], cap,
                                     dbg != nullptr && c == 0 ? dbg + 8 : nullptr);
        if (lane == 0) sc[c].result = s;
        if (c == 0) stamp(5);
#pragma unroll
        for (int d = c + 1; d < NC; ++d) {
            if (ch[d].from != c) continue;
            double u;
            if (seq[d]) {
                u = fold_seq_lane(cb, ch[d].k, ch[d].e, s, cap);
            } else {
                if (c == 0) stamp(6);
                u = blk_walk(cb, ch[d].k, ch[d].e, s, sc[d], cap);        // no head: from the exact start
            }
            if (lane == 0) sc[d].result = u;
            if (c == 0) stamp(7);
        }
    }
    __syncthreads();
    stamp(4);
#pragma unroll
    for (int c = 0; c < NC; ++c) res[c] = sc[c].result;
    __syncthreads();                                      // the scratch is reused by the next call
}

// one chain from a given start (k_fold_test)
__device__ __forceinline__ double fold_exact_block(const double* __restrict__ cb, const uint32_t k, const uint32_t e,
                                                   const double run, BlkFoldScratch& sc, const uint32_t cap) {
    const BlkChain ch[1] = {{k, e, run, -1}};
    double res[1];
    fold_exact_chains<1>(cb, ch, *reinterpret_cast<BlkFoldScratch (*)[1]>(&sc), cap, res);
    return res[0];
}

template <int KIND, bool kWide>
__global__ __launch_bounds__(kLoThreads) void k_lo_chain(DevProblem p, const typename ModelOf<KIND>::type* __restrict__ models,
                                                        const uint8_t* __restrict__ inc, double T0, double T1,
                                                        uint32_t pad0, uint32_t ntot, ListBits lb, FlagBand fbm,
                                                        FlagBand fbl, ScoreOut out, uint32_t probe) {
    __shared__ double cbuf[2][kLoBlock];
    __shared__ uint32_t ccnt[2][kLoChunks];                // inliers per chunk
    __shared__ uint32_t coff[2][kLoChunks + 1];            // exclusive prefix; [kLoChunks] = block total
    const uint32_t mi = blockIdx.x;
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    const uint64_t below = (1ull << lane) - 1ull;
    constexpr int kChains = KIND == 2 ? 2 : 1;
    const uint32_t nchunks = ntot / 64;
    const uint32_t cb0 = pad0 / 64;                        // first class-1 chunk (nchunks: none)
    const uint32_t nblk = (nchunks + kLoChunks - 1) / kLoChunks;
    double run = 0.0, hold = 0.0;
    uint32_t cnt0 = 0, cntall = 0;
    double wcc = 0.0, wtt = 0.0, whold = 0.0;             // kWide: the chains, uniform in every thread
    __shared__ BlkFoldScratch bsc[3];
    const auto m = models[mi];
    const bool live = inc == nullptr || inc[mi] <= 101;   // a slot without a model scores zeros
    // flagged decisions (the MSAC test's and the list predicate's, exact.h),
    // counted during the block loop (its barriers order them); the model's
    // value constants (a twin sincos for KIND 2) once per workgroup
    __shared__ uint32_t fcnt[2];
    __shared__ ValueConst vc_sh;
    GCR_STAMP(0, 14u);
    if (t < 2) fcnt[t] = 0;
    if constexpr (KIND <= 2)
        if (t == 0) vc_sh = value_const(m, KIND == 1, KIND == 2);
    __syncthreads();
    GCR_STAMP(1, 14u);
    // kWide with at most 2 kLoBlock pairs (every inlier fits both buffers
    // together): the blocks' inliers are appended to one LDS array and folded
    // once at the end by the whole workgroup
    const bool single = kWide && ntot <= 2u * kLoBlock;
    double* const cball = &cbuf[0][0];
    uint32_t boff = 0;                                     // single: inliers of the previous blocks
    for (uint32_t b = 0; b < nblk; ++b) {
        const uint32_t ch0 = b * kLoChunks;
        const uint32_t nch = min(kLoChunks, nchunks - ch0);
        double* cb = single ? cball + boff : cbuf[b & 1];
        uint32_t* cc = ccnt[b & 1];
        uint32_t* co = coff[b & 1];
        // 1) this wave's chunks j = wave + 16 i: every (model, feature) pair's
        //    residual, -r^2 or +0.0, its MSAC ballot word, the LO list
        //    predicate's ballot (launch_mask's rule) into pinned memory, and
        //    the decisions within the value-glibc bound of their thresholds
        double v[kLoPer];
        uint64_t w[kLoPer];
        uint32_t nfm = 0, nfl = 0;
        // the features of chunk i + 1 are requested before chunk i is
        // evaluated (branch-free loads, index clamped inside the class), so the
        // L2 latency of one chunk hides behind the previous one's arithmetic
        auto fetch = [&](int i, double (&f)[4]) {
            const uint32_t j = (uint32_t)wave + 16u * i;
            const uint32_t jj = (ch0 + (j < nch ? j : 0u)) * 64u + (uint32_t)lane;
            const int cls = jj < pad0 ? 0 : 1;
            const DevClass& c = p.cls[cls];
            const uint32_t fi = cls == 0 ? jj : jj - pad0;
            const uint32_t ic = fi < c.n ? fi : 0u;
            f[0] = c.x[ic];
            f[1] = c.y[ic];
            f[2] = (KIND < 3 && cls == 1) ? c.c0[ic] : c.a[ic];
            f[3] = KIND >= 3 ? c.c0[ic] : (cls == 1 ? c.c1[ic] : 0.0);
        };
        double fc[4], fn[4];
        fetch(0, fc);
#pragma unroll
        for (int i = 0; i < kLoPer; ++i) {
            if (i + 1 < kLoPer) fetch(i + 1, fn);
            const uint32_t j = (uint32_t)wave + 16u * i;
            const uint32_t jj = (ch0 + (j < nch ? j : 0u)) * 64u + (uint32_t)lane;   // pair index
            const int cls = jj < pad0 ? 0 : 1;                // chunk-uniform (pad0 % 64 == 0)
            const uint32_t fi = cls == 0 ? jj : jj - pad0;
            const DevClass& c = p.cls[cls];
            const bool ev = live && j < nch && fi < c.n;
            double r2 = 0.0;
            if (probe & 512u) {
                r2 = ev ? 1e-3 * (double)(fi & 1023u) : 0.0;   // timing probe: no residual evaluation
            } else if (ev) {
                if constexpr (KIND >= 3) {
                    r2 = geo_sq_residual<KIND>(fc[0], fc[1], fc[2], fc[3], m.h);
                } else if (cls == 0) {
                    r2 = scale_sq_value<KIND == 1, true>(fc[0], fc[1], fc[2], m, vc_sh.ac, vc_sh.cut);
                } else {
                    r2 = orient_sq_value<true>(fc[0], fc[1], fc[2], fc[3], m, vc_sh.c, vc_sh.s, vc_sh.cphi,
                                               vc_sh.cphi2);
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) fc[q] = fn[q];
            const bool inl = ev && r2 <= (cls == 0 ? T0 : T1);
            v[i] = inl ? -r2 : 0.0;
            w[i] = __ballot(inl);
            const bool lin = lb.bits != nullptr && ev && mask_rule(r2, lb.rule, cls == 0 ? lb.T[0] : lb.T[1], lb.lambda);
            const uint64_t lbw = __ballot(lin);
            if (j < nch && lane == 0) {
                const size_t wi = (size_t)mi * nchunks + ch0 + j;
                if (lb.bits != nullptr) lb.bits[wi] = lbw;
                if (lb.mbits != nullptr) lb.mbits[wi] = w[i];
            }
            if constexpr (KIND <= 2) {
                nfm += (uint32_t)__builtin_popcountll(__ballot(ev && in_flag_band(r2, fbm.mid[cls], fbm.half[cls])));
                nfl += (uint32_t)__builtin_popcountll(
                    __ballot(ev && lb.bits != nullptr && in_flag_band(r2, fbl.mid[cls], fbl.half[cls])));
            }
        }
        if (KIND <= 2 && lane == 0) {
            if (nfm) atomicAdd(&fcnt[0], nfm);
            if (nfl) atomicAdd(&fcnt[1], nfl);
        }
        GCR_STAMP(0, b);
#pragma unroll
        for (int i = 0; i < kLoPer; ++i) {
            const uint32_t j = (uint32_t)wave + 16u * i;
            if (lane == 0 && j < nch) cc[j] = (uint32_t)__builtin_popcountll(w[i]);
        }
        __syncthreads();
        // 2) exclusive prefix of the chunk counts (wave 0, two chunks a lane)
        if (wave == 0) {
            const uint32_t a = 2u * lane < nch ? cc[2 * lane] : 0u;
            const uint32_t c = 2u * lane + 1u < nch ? cc[2 * lane + 1] : 0u;
            uint32_t inc = a + c;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(inc, d);
                if (lane >= d) inc += o;
            }
            const uint32_t ex = inc - (a + c);
            co[2 * lane] = ex;
            co[2 * lane + 1] = ex + a;
            if (lane == 63) co[kLoChunks] = inc;
        }
        __syncthreads();
        GCR_STAMP(1, b);
        // 3) in-order compaction of the inlier values
#pragma unroll
        for (int i = 0; i < kLoPer; ++i) {
            const uint32_t j = (uint32_t)wave + 16u * i;
            if (j < nch && ((w[i] >> lane) & 1ull)) cb[co[j] + (uint32_t)__builtin_popcountll(w[i] & below)] = v[i];
        }
        __syncthreads();
        // 4) the block's fold.  kWide: every wave takes part in the
        //    block-parallel exact fold (fold_exact_block, barriers inside).
        //    Otherwise wave 0 folds the block one value per step while the
        //    other waves go on to the next block's loads (the other buffer
        //    set: this one is rewritten only after the next block's barriers,
        //    which wave 0 reaches once this fold is done).  KIND 2: the class
        //    chain restarts at the first class-1 value.
        const uint32_t total = co[kLoChunks];
        const bool has_b = cb0 >= ch0 && cb0 < ch0 + nch;
        const uint32_t bpos = cb0 < ch0 ? 0u : (has_b ? co[cb0 - ch0] : total);   // values before class 1
        GCR_STAMP(2, b);
        if (single) {
            cnt0 += bpos;
            cntall += total;
            boff += total;
            continue;
        }
        if (wave != 0) continue;
        cnt0 += bpos;
        cntall += total;
        {
            // one-lane folds: lane 0 the class sum, lane 1 (KIND 2) the total
            auto fold = [&](uint32_t k, uint32_t e) {
                if (lane >= kChains) return;
                if (k + 32 <= e) {
                    // ping-pong batches of 16: the next batch's reads are in
                    // flight during the current batch's dependent adds
                    // (sched_barrier keeps the scheduler from sinking the reads
                    // back next to their adds)
                    double ta[16], tb[16];
    #pragma unroll
                    for (int u = 0; u < 16; ++u) ta[u] = cb[k + u];
    #pragma unroll 1
                    for (; k + 32 <= e; k += 32) {
    #pragma unroll
                        for (int u = 0; u < 16; ++u) tb[u] = cb[k + 16 + u];
                        __builtin_amdgcn_sched_barrier(0);
    #pragma unroll
                        for (int u = 0; u < 16; ++u) run += ta[u];
                        __builtin_amdgcn_sched_barrier(0);
                        // the batch after next (clamped inside the buffer: a
                        // clamped batch lies past e and is never added)
                        const uint32_t nx = min(k + 32, kLoBlock - 16);
    #pragma unroll
                        for (int u = 0; u < 16; ++u) ta[u] = cb[nx + u];
                        __builtin_amdgcn_sched_barrier(0);
    #pragma unroll
                        for (int u = 0; u < 16; ++u) run += tb[u];
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    if (k + 16 <= e) {                         // ta = cb[k, k + 16)
    #pragma unroll
                        for (int u = 0; u < 16; ++u) run += ta[u];
                        k += 16;
                    }
                }
                for (; k < e; ++k) run += cb[k];
            };
            fold(0, bpos);
            if (KIND == 2 && has_b && lane == 0) {
                hold = run;
                run = 0.0;
            }
            fold(bpos, total);
        }
    }
    if (single && !(probe & 256u)) {
        // the class sum and, for KIND 2, the running total: class 0 from +0,
        // class 1 from +0 (the class chain's restart) and from the class-0 sum
        GCR_STAMP(2, 14u);
        if constexpr (KIND == 2) {
            const BlkChain chs[3] = {{0u, cnt0, 0.0, -1}, {cnt0, cntall, 0.0, -1}, {cnt0, cntall, 0.0, 0}};
            double r3[3];
            fold_exact_chains<3>(cball, chs, bsc, 2 * kLoBlock, r3);
            whold = r3[0];
            wcc = r3[1];
            wtt = r3[2];
        } else {
            const BlkChain chs[1] = {{0u, cnt0, 0.0, -1}};
            double r1[1];
            fold_exact_chains<1>(cball, chs, *reinterpret_cast<BlkFoldScratch (*)[1]>(&bsc[0]), 2 * kLoBlock, r1);
            wcc = r1[0];
        }
        GCR_STAMP(3, 14u);
        run = (KIND == 2 && lane == 1) ? wtt : wcc;
        hold = whold;
    }
    if (wave == 0) {
        const double tot = KIND == 2 ? __shfl(run, 1) : run;
        if (lane == 0) {
            out.n0[mi] = cnt0;
            out.n1[mi] = cntall - cnt0;
            out.v0[mi] = KIND == 2 ? hold : run;
            out.v1[mi] = KIND == 2 ? run : 0.0;
            out.tot[mi] = tot;
            if (out.fl) out.fl[mi] = fcnt[0];
            if (out.lfl) out.lfl[mi] = fcnt[1];
            signal_done(out, mi);
        }
    }
}

// ------------------------------------------- split small-batch scorer ----
// The small scorer for a few models (LO trials, refits) in two launches, so
// the per-pair arithmetic spreads over the chip instead of one workgroup per
// model: k_lo_resid evaluates one pair per thread (one 64-pair chunk per
// wave, any number of workgroups per model) and writes its chunk's inlier
// values compacted to the chunk's start in p.lo.vals, the chunk's counts in
// p.lo.meta and the list / MSAC ballots; k_lo_fold (one workgroup per model)
// gathers the chunks in order into LDS and folds them (fold_exact_chains).
// Same results as k_lo_chain<KIND, true> bit for bit.
constexpr int kLrThreads = 256;
static_assert(kSplitMaxPairs == 2 * kLoBlock, "k_lo_fold holds every inlier value in LDS");

// up to kArgModels rectification models passed by value (the kernel-argument
// segment), n = 0: read `models`
struct ArgModels {
    RectModel m[kArgModels];
    uint32_t n;
};

// one (model, feature) pair per lane of chunk j (64 pairs) of model mi:
// the value formula, the MSAC ballot and the chunk's inlier values compacted
// to its start in p.lo.vals, its counts in p.lo.meta, the list / MSAC
// ballots into ListBits (k_lo_resid, k_lo_split)
template <int KIND, bool kWT = false>
__device__ __forceinline__ void lo_resid_chunk(const DevProblem& p, const typename ModelOf<KIND>::type& m,
                                               const ValueConst& vc, const uint8_t* __restrict__ inc, uint32_t mi,
                                               uint32_t j, int lane, double T0, double T1, uint32_t pad0,
                                               uint32_t nchunks, const ListBits& lb, const FlagBand& fbm,
                                               const FlagBand& fbl, double x, double y, double f2, double f3,
                                               int cls, uint32_t fi) {
    const DevClass& c = p.cls[cls];
    const bool live = inc == nullptr || inc[mi] <= 101;
    const bool ev = live && fi < c.n;
    double r2 = 0.0;
    if (ev) {
        if constexpr (KIND >= 3) {
            r2 = geo_sq_residual<KIND>(x, y, f2, f3, m.h);
        } else if (cls == 0) {
            r2 = scale_sq_value<KIND == 1, true>(x, y, f2, m, vc.ac, vc.cut);
        } else {
            r2 = orient_sq_value<true>(x, y, f2, f3, m, vc.c, vc.s, vc.cphi, vc.cphi2);
        }
    }
    const bool inl = ev && r2 <= (cls == 0 ? T0 : T1);
    const uint64_t w = __ballot(inl);
    const size_t wi = (size_t)mi * nchunks + j;
    if (inl) p.lo.vals[wi * 64u + (uint32_t)__builtin_popcountll(w & ((1ull << lane) - 1ull))] = -r2;
    const bool lin = lb.bits != nullptr && ev && mask_rule(r2, lb.rule, cls == 0 ? lb.T[0] : lb.T[1], lb.lambda);
    const uint64_t lbw = __ballot(lin);
    uint32_t nfm = 0, nfl = 0;
    if constexpr (KIND <= 2) {
        nfm = (uint32_t)__builtin_popcountll(__ballot(ev && in_flag_band(r2, fbm.mid[cls], fbm.half[cls])));
        nfl = (uint32_t)__builtin_popcountll(__ballot(ev && lb.bits != nullptr && in_flag_band(r2, fbl.mid[cls], fbl.half[cls])));
    }
    if (p.lo.psum != nullptr) {
        // the chunk's inlier values summed in any order (k_lo_approx)
        double ps = inl ? -r2 : 0.0;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) ps += __shfl_xor(ps, d);
        if (lane == 0) {
            if constexpr (kWT) __hip_atomic_store(p.lo.psum + wi, ps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else p.lo.psum[wi] = ps;
        }
    }
    if (lane == 0) {
        if (lb.bits != nullptr) lb.bits[wi] = lbw;
        if (lb.mbits != nullptr) lb.mbits[wi] = w;
        const uint32_t mt = (uint32_t)__builtin_popcountll(w) | nfm << 8 | nfl << 16;
        if constexpr (kWT) __hip_atomic_store(p.lo.meta + wi, mt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else p.lo.meta[wi] = mt;
    }
}

// the pair's features of chunk j (loaded before the model's constants)
template <int KIND>
__device__ __forceinline__ void lo_pair_features(const DevProblem& p, uint32_t j, int lane, uint32_t pad0, int& cls,
                                                 uint32_t& fi, double& x, double& y, double& f2, double& f3) {
    const uint32_t jj = j * 64u + (uint32_t)lane;             // pair index
    cls = jj < pad0 ? 0 : 1;                                  // chunk-uniform (pad0 % 64 == 0)
    fi = cls == 0 ? jj : jj - pad0;
    const DevClass& c = p.cls[cls];
    const uint32_t ic = fi < c.n ? fi : 0u;                   // a class with chunks has features
    x = c.x[ic];
    y = c.y[ic];
    f2 = (KIND < 3 && cls == 1) ? c.c0[ic] : c.a[ic];
    f3 = KIND >= 3 ? c.c0[ic] : (cls == 1 ? c.c1[ic] : 0.0);
}

template <int KIND>
__device__ __forceinline__ void lo_approx_reduce(const DevProblem& p, uint32_t mi, uint32_t pad0, uint32_t nchunks,
                                                 const ScoreOut& out, bool wt);
// kFuse (approximate LO scoring in one launch): each chunk's psum and meta
// are stored write-through (sc1) and drained, the workgroup counts itself in
// on the model's arrival counter, and the model's last workgroup reduces
// them with sc1 loads (lo_approx_reduce) -- k_lo_approx's work, without the
// second launch; the arrival is an agent-scope release / acquire pair, as in
// k_lo_split (opt-in, GCR_LO_APPROX_FUSE=1: measured slower than two launches)
template <int KIND, bool kFuse = false>
__global__ __launch_bounds__(kLrThreads) void k_lo_resid(DevProblem p, const typename ModelOf<KIND>::type* __restrict__ models,
                                                        const uint8_t* __restrict__ inc, double T0, double T1,
                                                        uint32_t pad0, uint32_t nchunks, ListBits lb, FlagBand fbm,
                                                        FlagBand fbl, ArgModels am, uint32_t mi_base, ScoreOut aout) {
    const uint32_t ml = blockIdx.y;                           // the model in this launch's part
    const uint32_t mi = mi_base + ml;                         // ... and in the whole batch
    const uint32_t j = blockIdx.x * (kLrThreads / 64) + (threadIdx.x >> 6);      // chunk
    const int lane = threadIdx.x & 63;
    const bool jin = j < nchunks;                             // the last workgroup's tail
    // the pair's features first: their latency overlaps the model's read
    // (pinned host memory for small batches) and its value constants
    int cls;
    uint32_t fi;
    double x, y, f2, f3;
    lo_pair_features<KIND>(p, jin ? j : 0u, lane, pad0, cls, fi, x, y, f2, f3);
    __shared__ typename ModelOf<KIND>::type m_sh;
    __shared__ ValueConst vc_sh;
    if (threadIdx.x == 0) {
        if constexpr (KIND <= 2) {
            m_sh = ml < am.n ? am.m[ml] : models[ml];
            vc_sh = value_const(m_sh, KIND == 1, KIND == 2);
        } else {
            m_sh = models[ml];
        }
    }
    __syncthreads();
    if constexpr (!kFuse) {
        if (!jin) return;                                    // wave-uniform, after the barrier
        lo_resid_chunk<KIND>(p, m_sh, vc_sh, inc, mi, j, lane, T0, T1, pad0, nchunks, lb, fbm, fbl, x, y, f2, f3, cls,
                             fi);
    } else {
        __shared__ uint32_t last_sh;
        if (jin)
            lo_resid_chunk<KIND, true>(p, m_sh, vc_sh, inc, mi, j, lane, T0, T1, pad0, nchunks, lb, fbm, fbl, x, y, f2,
                                       f3, cls, fi);
        // every storing wave drains its write-through stores, then one
        // arrival per workgroup
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            // release at agent scope: this workgroup's chunk results before
            // its arrival (the write-through stores alone are not ordered by
            // the memory model)
            const uint32_t prev = __hip_atomic_fetch_add(p.lo.arrive + mi, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            last_sh = prev + 1u == gridDim.x ? 1u : 0u;
            if (last_sh) __hip_atomic_store(p.lo.arrive + mi, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (!last_sh) return;                                // workgroup-uniform
        // acquire at agent scope: every other workgroup's released results
        // are visible to the reduction's loads (k_lo_split's pattern)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        lo_approx_reduce<KIND>(p, mi, pad0, nchunks, aout, true);
    }
}

// The fold of one model's compacted chunks (k_lo_fold, and the last
// workgroup of a model in k_lo_split): scan the chunk counts, gather the
// chunks in feature order into LDS (all of a wave's reads in flight
// together) and fold them (fold_exact_chains).  1024 threads.  Results into
// slot oi of `out`.
template <int KIND>
__device__ __forceinline__ void lo_fold_model(const DevProblem& p, uint32_t mi, uint32_t pad0, uint32_t nchunks,
                                              const ScoreOut& out, uint32_t oi) {
    __shared__ double cball[2 * kLoBlock];
    __shared__ uint32_t coff[2 * kLoChunks + 1];
    __shared__ uint32_t wtot[kLoThreads / 64];
    __shared__ uint32_t fsum[2];
    __shared__ BlkFoldScratch bsc[3];
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    if (t < 2) fsum[t] = 0;
    // the chunk counts (one chunk per thread: nchunks <= 2 kLoChunks), block scan
    const uint32_t mt = (uint32_t)t < nchunks ? p.lo.meta[(size_t)mi * nchunks + t] : 0u;
    const uint32_t cnt = mt & 0xffu;
    const uint32_t ci = wave_incl_scan_u32(cnt);
    if (lane == 63) wtot[wave] = ci;
    uint32_t nfm = mt >> 8 & 0xffu, nfl = mt >> 16 & 0xffu;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        nfm += (uint32_t)__shfl_xor((int)nfm, d);
        nfl += (uint32_t)__shfl_xor((int)nfl, d);
    }
    __syncthreads();
    if (lane == 0 && (nfm | nfl)) {
        atomicAdd(&fsum[0], nfm);
        atomicAdd(&fsum[1], nfl);
    }
    const uint32_t wcs = wave_incl_scan_u32(wtot[lane & 15]);
    const uint32_t excl = ci - cnt + (wave > 0 ? (uint32_t)__builtin_amdgcn_readlane((int)wcs, wave - 1) : 0u);
    if ((uint32_t)t < nchunks) coff[t] = excl;
    if ((uint32_t)t == nchunks - 1) coff[nchunks] = excl + cnt;
    __syncthreads();
    // gather: wave w copies chunks w, w + 16, ... (all reads in flight together)
    {
        constexpr int kPer = 2 * kLoChunks / (kLoThreads / 64);
        const double* src = p.lo.vals + (size_t)mi * nchunks * 64u;
        double g[kPer];
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const uint32_t j = (uint32_t)wave + 16u * i;
            g[i] = (j < nchunks && (uint32_t)lane < coff[j + 1] - coff[j]) ? src[j * 64u + lane] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const uint32_t j = (uint32_t)wave + 16u * i;
            if (j < nchunks && (uint32_t)lane < coff[j + 1] - coff[j]) cball[coff[j] + lane] = g[i];
        }
    }
    __syncthreads();
    const uint32_t cnt0 = coff[min(pad0 / 64u, nchunks)], cntall = coff[nchunks];
    double whold = 0.0, wcc, wtt;
    if constexpr (KIND == 2) {
        const BlkChain chs[3] = {{0u, cnt0, 0.0, -1}, {cnt0, cntall, 0.0, -1}, {cnt0, cntall, 0.0, 0}};
        double r3[3];
        fold_exact_chains<3>(cball, chs, bsc, 2 * kLoBlock, r3);
        whold = r3[0];
        wcc = r3[1];
        wtt = r3[2];
    } else {
        const BlkChain chs[1] = {{0u, cnt0, 0.0, -1}};
        double r1[1];
        fold_exact_chains<1>(cball, chs, *reinterpret_cast<BlkFoldScratch (*)[1]>(&bsc[0]), 2 * kLoBlock, r1);
        wcc = wtt = r1[0];
    }
    if (t == 0) {
        out.n0[oi] = cnt0;
        out.n1[oi] = cntall - cnt0;
        out.v0[oi] = KIND == 2 ? whold : wcc;
        out.v1[oi] = KIND == 2 ? wcc : 0.0;
        out.tot[oi] = wtt;
        if (out.fl) out.fl[oi] = fsum[0];
        if (out.lfl) out.lfl[oi] = fsum[1];
        signal_done(out, oi);
    }
}

// models [src, src + gridDim.x) into slots [slot, slot + gridDim.x); a dead
// slot's chunks hold no inliers
template <int KIND>
__global__ __launch_bounds__(kLoThreads) void k_lo_fold(DevProblem p, uint32_t pad0, uint32_t nchunks, ScoreOut out,
                                                       uint32_t src, uint32_t slot) {
    lo_fold_model<KIND>(p, src + blockIdx.x, pad0, nchunks, out, slot + blockIdx.x);
}

// The approximate scores of k_lo_resid's models (blockIdx.x) from its chunk
// partial sums (p.lo.psum): exact counts and flag counts, class sums in a
// fixed tree order instead of the reference's sequential one.  The host
// bounds the difference (both orders sum the same non-positive values, so
// each is within (n - 1) u sum|a| of the real sum) and decides a comparison
// with them only when the bounds cannot change it; the winner's exact sums
// follow from k_lo_fold.
constexpr int kLaThreads = 256;
static_assert(kLaThreads == kLrThreads, "k_lo_resid<kFuse> reduces in its own workgroup");
// the reduction of model mi's chunks (wt: loads write-through, sc1, for
// chunks stored write-through by other workgroups of the same launch)
template <int KIND>
__device__ __forceinline__ void lo_approx_reduce(const DevProblem& p, uint32_t mi, uint32_t pad0, uint32_t nchunks,
                                                 const ScoreOut& out, bool wt) {
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    const uint32_t c1 = pad0 / 64u;                           // the first class-1 chunk
    uint32_t n0 = 0, n1 = 0, fm = 0, fl = 0;
    double s0 = 0.0, s1 = 0.0;
    for (uint32_t j = (uint32_t)t; j < nchunks; j += kLaThreads) {
        const size_t wi = (size_t)mi * nchunks + j;
        const uint32_t mt = wt ? __hip_atomic_load(p.lo.meta + wi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                               : p.lo.meta[wi];
        const double ps = wt ? __hip_atomic_load(p.lo.psum + wi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                             : p.lo.psum[wi];
        if (j < c1) {
            n0 += mt & 0xffu;
            s0 += ps;
        } else {
            n1 += mt & 0xffu;
            s1 += ps;
        }
        fm += mt >> 8 & 0xffu;
        fl += mt >> 16 & 0xffu;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        n0 += (uint32_t)__shfl_xor((int)n0, d);
        n1 += (uint32_t)__shfl_xor((int)n1, d);
        fm += (uint32_t)__shfl_xor((int)fm, d);
        fl += (uint32_t)__shfl_xor((int)fl, d);
        s0 += __shfl_xor(s0, d);
        s1 += __shfl_xor(s1, d);
    }
    __shared__ uint32_t cn[4][kLaThreads / 64];
    __shared__ double cs[2][kLaThreads / 64];
    if (lane == 0) {
        cn[0][wave] = n0;
        cn[1][wave] = n1;
        cn[2][wave] = fm;
        cn[3][wave] = fl;
        cs[0][wave] = s0;
        cs[1][wave] = s1;
    }
    __syncthreads();
    if (t == 0) {
        uint32_t a0 = 0, a1 = 0, af = 0, al = 0;
        double v0 = 0.0, v1 = 0.0;
#pragma unroll
        for (int w = 0; w < kLaThreads / 64; ++w) {
            a0 += cn[0][w];
            a1 += cn[1][w];
            af += cn[2][w];
            al += cn[3][w];
            v0 += cs[0][w];
            v1 += cs[1][w];
        }
        out.n0[mi] = a0;
        out.n1[mi] = a1;
        out.v0[mi] = v0;
        out.v1[mi] = KIND == 2 ? v1 : 0.0;
        out.tot[mi] = KIND == 2 ? v0 + v1 : v0;
        if (out.fl) out.fl[mi] = af;
        if (out.lfl) out.lfl[mi] = al;
        signal_done(out, mi);
    }
}
template <int KIND>
__global__ __launch_bounds__(kLaThreads) void k_lo_approx(DevProblem p, uint32_t pad0, uint32_t nchunks, ScoreOut out) {
    lo_approx_reduce<KIND>(p, blockIdx.x, pad0, nchunks, out, false);
}

// The split scorer in ONE launch (GCR_LO_FUSED=1; measured slower than the
// two launches on MI355X, see launch_score_small): 1024-thread
// workgroups, blockIdx.y the model, each workgroup evaluating per wave
// `cpw` chunks of the model (k_lo_resid's work), then counting itself done on
// the model's arrival counter; the model's last workgroup to arrive folds
// the model's chunks (k_lo_fold's work) and resets the counter for the next
// launch.  No second launch, and no kernel boundary between the last
// residual of a model and its fold: the fold of one model overlaps the
// residuals of the next.
template <int KIND>
__global__ __launch_bounds__(kLoThreads) void k_lo_split(DevProblem p, const typename ModelOf<KIND>::type* __restrict__ models,
                                                        const uint8_t* __restrict__ inc, double T0, double T1,
                                                        uint32_t pad0, uint32_t nchunks, uint32_t cpw, ListBits lb,
                                                        FlagBand fbm, FlagBand fbl, ArgModels am, ScoreOut out) {
    const uint32_t mi = blockIdx.y;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t j0 = (blockIdx.x * (kLoThreads / 64) + (uint32_t)wave) * cpw;    // this wave's first chunk
    __shared__ typename ModelOf<KIND>::type m_sh;
    __shared__ ValueConst vc_sh;
    __shared__ uint32_t last_sh;
    // the first chunk's features ahead of the model's constants
    int cls;
    uint32_t fi;
    double x, y, f2, f3;
    lo_pair_features<KIND>(p, j0 < nchunks ? j0 : 0u, lane, pad0, cls, fi, x, y, f2, f3);
    if (threadIdx.x == 0) {
        if constexpr (KIND <= 2) {
            m_sh = mi < am.n ? am.m[mi] : models[mi];
            vc_sh = value_const(m_sh, KIND == 1, KIND == 2);
        } else {
            m_sh = models[mi];
        }
    }
    __syncthreads();
    for (uint32_t q = 0; q < cpw; ++q) {
        const uint32_t j = j0 + q;
        if (j >= nchunks) break;                             // wave-uniform
        if (q > 0) lo_pair_features<KIND>(p, j, lane, pad0, cls, fi, x, y, f2, f3);
        lo_resid_chunk<KIND>(p, m_sh, vc_sh, inc, mi, j, lane, T0, T1, pad0, nchunks, lb, fbm, fbl, x, y, f2, f3,
                             cls, fi);
    }
    // arrival: this workgroup's chunk values and counts are visible device-
    // wide before its count (one agent-scope release after the barrier: the
    // release is an L2 writeback on gfx950, whose XCDs have their own L2s --
    // once per workgroup, not per thread); the last arrival acquires them
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        const uint32_t prev = atomicAdd(&p.lo.arrive[mi], 1u);
        last_sh = prev + 1u == gridDim.x ? 1u : 0u;
        if (last_sh) p.lo.arrive[mi] = 0u;                  // reset for the next launch (no other arrival left)
    }
    __syncthreads();
    if (!last_sh) return;                                    // workgroup-uniform
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    lo_fold_model<KIND>(p, mi, pad0, nchunks, out, mi);
}

// -------------------------------------------------------------- compact ----
// Order-preserving list of the live hypotheses (inc <= 101) of a launch: one
// workgroup, contiguous chunks per thread, exclusive scan in LDS.  Used by the
// fundamental matrix, whose slots carry up to three hypotheses of which on
// average ~1.1 exist.
constexpr int kCompactThreads = 1024;

__global__ __launch_bounds__(kCompactThreads) void k_compact(const uint8_t* __restrict__ inc, uint32_t n,
                                                            uint32_t* __restrict__ map, uint32_t* __restrict__ count) {
    // tiles of 16 x kCompactThreads entries: thread t tests entries
    // [16 t, 16 t + 16) of the tile (16 byte loads in flight), a wave scan and
    // the waves' totals give its first output index, and the map is written
    // in entry order.  (Round 4's form -- one contiguous n / 1024 chunk per
    // thread, strided byte loads, a 20-barrier Hillis-Steele scan -- took
    // 36 us at 44 544 entries.)
    constexpr uint32_t kPer = 16, kWaves = kCompactThreads / 64;
    __shared__ uint32_t wsum[kWaves];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t base = 0;
    for (uint32_t t0 = 0; t0 < n; t0 += kPer * kCompactThreads) {
        const uint32_t i0 = t0 + kPer * t;
        uint32_t live = 0;
#pragma unroll
        for (uint32_t k = 0; k < kPer; ++k)
            if (i0 + k < n && inc[i0 + k] <= 101) live |= 1u << k;
        const uint32_t c = (uint32_t)__builtin_popcount(live);
        uint32_t x = c;                                  // inclusive scan in the wave
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(x, d);
            if (lane >= (uint32_t)d) x += o;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        uint32_t wb = 0, tot = 0;
#pragma unroll
        for (uint32_t v = 0; v < kWaves; ++v) {
            const uint32_t sv = wsum[v];
            wb += v < w ? sv : 0u;
            tot += sv;
        }
        uint32_t o = base + wb + x - c;
        while (live) {
            const uint32_t k = (uint32_t)__builtin_ctz(live);
            live &= live - 1;
            map[o++] = i0 + k;
        }
        base += tot;
        __syncthreads();                                 // wsum is rewritten by the next tile
    }
    if (t == 0) *count = base;
}

// --------------------------------------------------------------- select ----
constexpr int kSelectThreads = 1024;

// `per` hypotheses per slot (3 for the fundamental matrix: inc 0 = extra
// model of the slot, 255 = absent, neither adds iterations).
template <class M>
__global__ __launch_bounds__(kSelectThreads) void k_select(int solver, ScoreOut sc, const uint8_t* __restrict__ inc,
                                                           const M* __restrict__ models, uint32_t n,
                                                           uint64_t slot0, uint32_t m0, uint32_t m1, double Tm0,
                                                           double Tm1, BatchRecord* out, uint32_t per = 1,
                                                           const uint32_t* __restrict__ hmap = nullptr,
                                                           const uint32_t* __restrict__ hcount = nullptr,
                                                           uint32_t stride = 0) {
    // deferred selection of consecutive batches: workgroup b reduces the
    // batch whose arrays start `stride` hypotheses after batch b - 1's
    if (stride != 0) {
        const size_t o = (size_t)blockIdx.x * stride;
        sc.n0 += o; sc.n1 += o; sc.v0 += o; sc.v1 += o; sc.tot += o;
        inc += o;
        if (hmap != nullptr) { hmap += o; hcount += blockIdx.x; }
        slot0 += (uint64_t)blockIdx.x * (n / per);
        out += blockIdx.x;
    }
    __shared__ double s_val[kSelectThreads];
    __shared__ uint32_t s_idx[kSelectThreads];
    __shared__ unsigned long long s_models[kSelectThreads], s_its[kSelectThreads];
    const int t = threadIdx.x;
    const int K = solver == 2 ? 2 : 1;
    double best = 0.0;
    uint32_t bi = 0xffffffffu;
    unsigned long long nm = 0, its = 0;
    // score index j: hypothesis j, or hmap[j] of a compacted launch (the map
    // is increasing, so the lowest j is still the first hypothesis)
    auto consider = [&](uint32_t j, uint32_t hyp) {
        ++nm;
        double sum = sc.tot[j];
        bool zero = false;
        for (int c = 0; c < K; ++c) {
            const uint32_t nc = c == 0 ? sc.n0[j] : sc.n1[j];
            if (nc < (c == 0 ? m0 : m1)) { zero = true; break; }
            const double v = c == 0 ? sc.v0[j] : sc.v1[j];
            const double msac = v / (c == 0 ? Tm0 : Tm1) + static_cast<double>(nc);
            sum -= v;
            sum += msac;
        }
        if (zero) sum = 0.0;
        bool valid = true;
        if constexpr (std::is_same<M, RectModel>::value) valid = solver != 2 || valid_model_sift22(models[hyp]);
        if (best < sum && valid) {
            best = sum;
            bi = j;
        }
    };
    for (uint32_t j = t; j < n; j += kSelectThreads) {
        const uint32_t in = inc[j];
        its += in <= 102 ? in : 0;
        if (hmap == nullptr && in <= 101) consider(j, j);
    }
    if (hmap != nullptr) {
        const uint32_t nc = min(n, *hcount);
        for (uint32_t j = t; j < nc; j += kSelectThreads) consider(j, hmap[j]);
    }
    s_val[t] = best;
    s_idx[t] = bi;
    s_models[t] = nm;
    s_its[t] = its;
    __syncthreads();
    for (int w = kSelectThreads / 2; w > 0; w >>= 1) {
        if (t < w) {
            const uint32_t ia = s_idx[t], ib = s_idx[t + w];
            const double va = s_val[t], vb = s_val[t + w];
            if (ib != 0xffffffffu && (ia == 0xffffffffu || vb > va || (vb == va && ib < ia))) {
                s_idx[t] = ib;
                s_val[t] = vb;
            }
            s_models[t] += s_models[t + w];
            s_its[t] += s_its[t + w];
        }
        __syncthreads();
    }
    if (t == 0) {
        BatchRecord r;
        r.models = s_models[0];
        r.iterations = s_its[0];
        r.best_slot = -1;
        r.best_score = 0.0;
        r.best_inliers[0] = r.best_inliers[1] = 0;
        r.best_model = default_model();
        const uint32_t j = s_idx[0];
        if (j != 0xffffffffu) {
            r.best_slot = static_cast<int64_t>(slot0 + (hmap != nullptr ? hmap[j] : j) / per);
            r.best_score = s_val[0];
            r.best_inliers[0] = sc.n0[j];
            r.best_inliers[1] = K == 2 ? sc.n1[j] : 0;
            if constexpr (std::is_same<M, RectModel>::value) r.best_model = models[j];
        }
        *out = r;
    }
}

// ---------------------------------------------------------------- refit ----
constexpr int kRowBlock = 256;

// thread per row; pair p = r - ns maps to (i, j), i < j, row-major over i:
// off(i) = i * (2 no - i - 1) / 2 pairs precede row i
__device__ __forceinline__ void sift_row_at(const DevClass& sc, const DevClass& oc, const uint32_t* __restrict__ si,
                                            uint32_t ns, const uint32_t* __restrict__ oi, uint32_t no, uint64_t r,
                                            double out[4]) {
    if (r < ns) {
        const uint32_t j = si[r];
        const double w = 1.0;
        out[0] = w * sc.x[j];
        out[1] = w * sc.y[j];
        out[2] = w * sc.c0[j];
        out[3] = w;
        return;
    }
    const uint64_t p = r - ns;
    const uint64_t n = no;
    auto off = [n](uint64_t i) { return i * (2 * n - i - 1) / 2; };
    const double q = (double)(2 * n - 1);
    int64_t i = (int64_t)((q - sqrt(q * q - 8.0 * (double)p)) * 0.5);
    if (i < 0) i = 0;
    if (i > (int64_t)n - 2) i = (int64_t)n - 2;
    while (i > 0 && off((uint64_t)i) > p) --i;
    while ((uint64_t)i + 2 < n && off((uint64_t)i + 1) <= p) ++i;
    const uint64_t j = p - off((uint64_t)i) + (uint64_t)i + 1;
    const uint32_t a = oi[i], c = oi[j];
    sift_pair_row(oc.x[a], oc.y[a], oc.c0[a], oc.c1[a], oc.x[c], oc.y[c], oc.c0[c], oc.c1[c], out);
}

// The hybrid system's double-double Gram matrix (gram.h): k_gram_prep copies
// the index lists in and computes every orientation inlier's line once;
// k_sift_gram, one workgroup per tile of kGramTile rows, lane l accumulating
// rows tile + l + 256 u.  Rows go in batches of kGramBatch per lane: the
// batch's (i, j) first (each lane's pair index advances by 256 pairs per row,
// a carry into the next first index when it runs past the end of a row),
// then every line load of the batch, then the arithmetic -- one round trip
// per batch instead of two dependent ones per row (measured: the kernel was
// memory-latency bound, 55 % of its wave cycles waiting).  The 256 lane sums are
// combined by gram.h's halving tree in LDS into the tile's sums
// (k_gram_final combines the tiles: a last-arrival combination inside this
// kernel needs an agent-scope release per workgroup -- an L2 writeback on
// gfx950 -- and measured ~40 us slower).
constexpr int kGramBlock = kGramLanes;
constexpr int kGramPer = (int)(kGramTile / kGramLanes);

// a double-double shuffled down by h lanes (wave-wide)
__device__ __forceinline__ DD dd_shfl_down(DD x, int h) { return DD{__shfl_down(x.hi, h), __shfl_down(x.lo, h)}; }

// gram.h's halving tree x[l] += x[l + h], h = 128 .. 1, over the 256 lane
// sums red[k][0 .. 256) of every product k, the work spread over the four
// waves: levels 128 and 64 as (product, lane) items over all threads, then
// wave w takes products w, w + 4, ... through levels 32 .. 1 with shuffles
// (the same additions in the same order); product k's sum to out[k]
__device__ __forceinline__ void gram_tree_out(DD (*red)[kGramBlock], int t, DD* __restrict__ out) {
    static_assert(kGramBlock == 256, "gram tree");
    for (int i = t; i < kGramN * 128; i += kGramBlock) {
        const int k = i >> 7, l = i & 127;
        red[k][l] = dd_add(red[k][l], red[k][l + 128]);
    }
    __syncthreads();
    for (int i = t; i < kGramN * 64; i += kGramBlock) {
        const int k = i >> 6, l = i & 63;
        red[k][l] = dd_add(red[k][l], red[k][l + 64]);
    }
    __syncthreads();
    const int wave = t >> 6, lane = t & 63;
    for (int k = wave; k < kGramN; k += kGramBlock / 64) {
        DD x = red[k][lane];
#pragma unroll
        for (int h = 32; h >= 1; h >>= 1) x = dd_add(x, dd_shfl_down(x, h));
        if (lane == 0) out[k] = x;
    }
}

// the tile sums combined in gram.h's order (one workgroup, after
// k_sift_gram on the stream): wave k takes product k, lane l adds tiles
// l, l + 64, ... in order (their loads in flight eight at a time), then the
// halving tree with shuffles; the matrix to fin.out, then fin.epoch to fin.done
constexpr int kGramFinalLanes = 64;
__global__ __launch_bounds__(64 * kGramN) void k_gram_final(const DD* __restrict__ tiles, uint32_t ntiles, GramFinal fin) {
    const int k = threadIdx.x >> 6, lane = threadIdx.x & 63;
    DD acc{0.0, 0.0};
#pragma unroll 1
    for (uint32_t t0 = (uint32_t)lane; t0 < ntiles; t0 += 8 * kGramFinalLanes) {
        DD v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint32_t t = t0 + (uint32_t)q * kGramFinalLanes;
            v[q] = t < ntiles ? tiles[(size_t)t * kGramN + k] : DD{0.0, 0.0};
        }
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (t0 + (uint32_t)q * kGramFinalLanes < ntiles) acc = dd_add(acc, v[q]);
    }
#pragma unroll
    for (int h = 32; h >= 1; h >>= 1) acc = dd_add(acc, dd_shfl_down(acc, h));
    if (lane == 0) fin.out[k] = acc;
    __syncthreads();
    if (threadIdx.x == 0 && fin.done != nullptr) {
        __threadfence_system();
        __hip_atomic_store(fin.done, fin.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// the index lists from pinned host memory (hidx: si then oi) into idx, and
// the line (line_from) of every orientation inlier, SoA, into lines[3][no]
__global__ __launch_bounds__(kGramBlock) void k_gram_prep(DevClass oc, const uint32_t* __restrict__ hidx, uint32_t ns,
                                                          uint32_t no, uint32_t* __restrict__ idx,
                                                          double* __restrict__ lines) {
    const uint32_t t = blockIdx.x * kGramBlock + threadIdx.x;
    if (t >= ns + no) return;
    const uint32_t v = hidx[t];
    idx[t] = v;
    if (t < ns) return;
    double l[3];
    line_from(oc.x[v], oc.y[v], oc.c0[v], oc.c1[v], l);
    const uint32_t i = t - ns;
    lines[i] = l[0];
    lines[no + i] = l[1];
    lines[2 * (size_t)no + i] = l[2];
}

template <int kGramBatch>
__global__ __launch_bounds__(kGramBlock) void k_sift_gram(DevClass sc, const uint32_t* __restrict__ si, uint32_t ns,
                                                          const double* __restrict__ lines, uint32_t no, uint64_t rows,
                                                          DD* __restrict__ tiles) {
    static_assert(kGramPer % kGramBatch == 0, "gram batches");
    __shared__ DD red[kGramN][kGramBlock];
    const int l = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * kGramTile;
    const double* L0 = lines;
    const double* L1 = lines + no;
    const double* L2 = lines + 2 * (size_t)no;
    DD acc[kGramN];
#pragma unroll
    for (int k = 0; k < kGramN; ++k) acc[k] = DD{0.0, 0.0};
    bool have = false;
    uint64_t pi = 0, pj = 0;
    for (int g = 0; g < kGramPer; g += kGramBatch) {
        if (base + (uint64_t)l + (uint64_t)kGramLanes * (uint64_t)g >= rows) break;
        // 1) the batch's rows: a scale row's feature index, a pair row's (i, j)
        uint32_t ja[kGramBatch], jb[kGramBatch];
        int kind[kGramBatch];                                 // 0 none, 1 scale row, 2 pair row
#pragma unroll
        for (int b = 0; b < kGramBatch; ++b) {
            const uint64_t r = base + (uint64_t)l + (uint64_t)kGramLanes * (uint64_t)(g + b);
            kind[b] = 0;
            ja[b] = jb[b] = 0;
            if (r >= rows) continue;
            if (r < ns) {
                kind[b] = 1;
                ja[b] = (uint32_t)r;
                continue;
            }
            if (!have) {
                pair_of(r - ns, no, pi, pj);
                have = true;
            } else {
                pj += kGramLanes;
                while (pj >= no) {
                    pj = pj - no + pi + 2;
                    ++pi;
                }
            }
            kind[b] = 2;
            ja[b] = (uint32_t)pi;
            jb[b] = (uint32_t)pj;
        }
        // 2) every load of the batch (one round trip; a scale row's feature
        //    index is a second)
        double fa[kGramBatch][3], fb[kGramBatch][3];
#pragma unroll
        for (int b = 0; b < kGramBatch; ++b) {
            if (kind[b] == 1) {
                const uint32_t j = si[ja[b]];
                fa[b][0] = sc.x[j];
                fa[b][1] = sc.y[j];
                fa[b][2] = sc.c0[j];
                fb[b][0] = fb[b][1] = fb[b][2] = 0.0;
            } else if (kind[b] == 2) {
                fa[b][0] = L0[ja[b]];
                fa[b][1] = L1[ja[b]];
                fa[b][2] = L2[ja[b]];
                fb[b][0] = L0[jb[b]];
                fb[b][1] = L1[jb[b]];
                fb[b][2] = L2[jb[b]];
            } else {
                fa[b][0] = fa[b][1] = fa[b][2] = fb[b][0] = fb[b][1] = fb[b][2] = 0.0;
            }
        }
        // 3) the rows, in order
#pragma unroll
        for (int b = 0; b < kGramBatch; ++b) {
            if (kind[b] == 0) continue;
            double row[4];
            if (kind[b] == 1) {
                const double w = 1.0;
                row[0] = w * fa[b][0];
                row[1] = w * fa[b][1];
                row[2] = w * fa[b][2];
                row[3] = w;
            } else {
                sift_pair_row_lines(fa[b], fb[b], row);
                // row[2] == 0: the same sums as gram_add_row while the row and
                // the four accumulators its zeros would touch are finite (an
                // infinite accumulator plus a zero double-double is NaN)
                if (__builtin_isfinite(row[0]) && __builtin_isfinite(row[1]) && __builtin_isfinite(row[3]) &&
                    __builtin_isfinite(acc[2].hi) && __builtin_isfinite(acc[5].hi) && __builtin_isfinite(acc[7].hi) &&
                    __builtin_isfinite(acc[8].hi)) {
                    gram_add_pair_row(acc, row);
                    continue;
                }
            }
            gram_add_row(acc, row);
        }
    }
#pragma unroll
    for (int k = 0; k < kGramN; ++k) red[k][l] = acc[k];
    __syncthreads();
    gram_tree_out(red, l, tiles + (size_t)blockIdx.x * kGramN);
}

__global__ __launch_bounds__(kRowBlock) void k_sift_rows(DevClass sc, DevClass oc, const uint32_t* __restrict__ si,
                                                         uint32_t ns, const uint32_t* __restrict__ oi, uint32_t no,
                                                         uint64_t rows, double* A0, double* A1, double* A2,
                                                         double* b) {
    const uint64_t r = (uint64_t)blockIdx.x * kRowBlock + threadIdx.x;
    if (r >= rows) return;
    double row[4];
    sift_row_at(sc, oc, si, ns, oi, no, r, row);
    A0[r] = row[0];
    A1[r] = row[1];
    A2[r] = row[2];
    b[r] = row[3];
}

// blocked_sum's block partial (qr3.h) of one 256-thread workgroup: thread t
// holds the sequential sum of its rows base + t + 256 q; the halving tree's
// levels 128 and 64 go through LDS, the rest is a butterfly in wave 0, whose
// lane 0 then holds x[0] of the halving tree.  `acc` / `lds` hold nred
// reductions (lds: nred x 256 doubles); the results are valid in thread 0.
__device__ __forceinline__ double qr_butterfly(double a) {
#pragma unroll
    for (int sft = 32; sft >= 1; sft >>= 1) a += __shfl_xor(a, sft, 64);
    return a;
}
template <int NR>
__device__ __forceinline__ void qr_block_tree(double (&acc)[NR], int nred, double* lds) {
    const int t = threadIdx.x;
#pragma unroll
    for (int r = 0; r < NR; ++r)
        if (r < nred) lds[r * 256 + t] = acc[r];
    __syncthreads();
    if (t < 128) {
#pragma unroll
        for (int r = 0; r < NR; ++r)
            if (r < nred) lds[r * 256 + t] = lds[r * 256 + t] + lds[r * 256 + t + 128];
    }
    __syncthreads();
    if (t < 64) {
#pragma unroll
        for (int r = 0; r < NR; ++r)
            if (r < nred) acc[r] = qr_butterfly(lds[r * 256 + t] + lds[r * 256 + t + 64]);
    }
}

// one 256-thread workgroup per aligned block of kSumBlock rows: thread t sums
// rows base + t + 256 q of [lo, hi) sequentially (coalesced loads, all in
// flight), then the block tree -- blocked_sum's block partial
constexpr int kPartWaves = 4;
__device__ __forceinline__ void qr_partials_body(const double* __restrict__ a, const double* __restrict__ c,
                                                 uint64_t lo, uint64_t hi, uint64_t blk0, uint64_t nblk,
                                                 double* __restrict__ partials) {
    __shared__ double lds[256];
    const int t = threadIdx.x;
    const uint64_t blk = blockIdx.x;
    if (blk >= nblk) return;
    const uint64_t base = (blk0 + blk) * kSumBlock;
    constexpr int kPer = (int)(kSumBlock / 256);
    double av[kPer], cv[kPer];
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        const uint64_t i = base + t + 256 * q;
        const bool in = i >= lo && i < hi;
        av[q] = in ? a[i] : 0.0;
        cv[q] = in ? c[i] : 0.0;
    }
    double acc[1] = {0.0};
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        const uint64_t i = base + t + 256 * q;
        if (i >= lo && i < hi) acc[0] += av[q] * cv[q];
    }
    qr_block_tree<1>(acc, 1, lds);
    if (t == 0) partials[blk] = acc[0];
}

__global__ __launch_bounds__(64 * kPartWaves) void k_qr_partials(const double* __restrict__ a,
                                                                 const double* __restrict__ c, uint64_t lo,
                                                                 uint64_t hi, uint64_t blk0, uint64_t nblk,
                                                                 double* __restrict__ partials) {
    qr_partials_body(a, c, lo, hi, blk0, nblk, partials);
}

// ---- device-resident QR driver (qr3.h qr_solve<3> with its decisions on
// the GPU): a fixed launch sequence of reductions (k_qrd_partials),
// control steps (k_qrd_ctl, one thread: the driver's scalar logic, the
// same fp64 operations in the same order as qr3.h) and element-wise steps
// (k_qrd_ew), whose parameters live in a QRDevState in device memory.  The
// host enqueues the whole sequence and synchronises once for x.
__global__ __launch_bounds__(64 * kPartWaves) void k_qrd_partials(QRCols cols, const QRDevState* __restrict__ st,
                                                                  double* __restrict__ partials) {
    if (!st->red_on) return;
    const uint64_t lo = st->red_lo, hi = st->red_hi;
    const uint64_t blk0 = lo / kSumBlock, nblk = (hi - 1) / kSumBlock - blk0 + 1;
    qr_partials_body(cols.col[st->red_a], cols.col[st->red_c], lo, hi, blk0, nblk, partials);
}

__global__ __launch_bounds__(256) void k_qrd_ew(QRCols cols, const QRDevState* __restrict__ st) {
    const int op = st->ew_op;
    if (op == 0) return;
    const uint64_t i = st->ew_lo + (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= st->ew_hi) return;
    double* c = cols.col[st->ew_c];
    if (op == 1) c[i] = c[i] / st->ew_p0;                                   // scale
    else if (op == 2) c[i] = 0.0;                                          // zero
    else c[i] -= (st->ew_p0 * cols.col[st->ew_e][i]) * st->ew_p1;          // update
}

constexpr int kQrdSup = 256;            // super-blocks a control step can sum (16.7 M rows)

__global__ __launch_bounds__(64) void k_qrd_ctl(QRCols cols, QRDevState* st, const double* __restrict__ partials,
                                                uint64_t m_rows, int step, int k, int j) {
    __shared__ double sup[kQrdSup];
    __shared__ double total_sh;
    const int t = threadIdx.x;
    const bool had = st->red_on != 0;
    if (had) {
        // the previous reduction's block partials in blocked_sum's order:
        // sequentially inside each aligned super-block, then the super-block
        // partials sequentially
        const uint64_t lo = st->red_lo, hi = st->red_hi;
        const uint64_t blk0 = lo / kSumBlock, nblk = (hi - 1) / kSumBlock - blk0 + 1;
        constexpr uint64_t per = kSumSuper / kSumBlock;
        const uint64_t s0 = blk0 / per, nsup = (blk0 + nblk - 1) / per - s0 + 1;
        for (uint64_t u = t; u < nsup; u += 64) {
            const uint64_t b_lo = max(blk0, (s0 + u) * per), b_hi = min(blk0 + nblk, (s0 + u + 1) * per);
            // the super-block's (<= 64) partials all in flight, then summed in order
            double v[per];
#pragma unroll
            for (uint64_t q = 0; q < per; ++q) v[q] = b_lo + q < b_hi ? partials[b_lo + q - blk0] : 0.0;
            double sp = 0.0;
#pragma unroll
            for (uint64_t q = 0; q < per; ++q)
                if (b_lo + q < b_hi) sp += v[q];
            sup[u] = sp;
        }
        __syncthreads();
        if (t == 0) {
            double tot = 0.0;
            for (uint64_t u = 0; u < nsup; ++u) tot += sup[u];
            total_sh = tot;
        }
    }
    __syncthreads();
    if (t != 0) return;
    const double total = had ? total_sh : 0.0;
    st->red_on = 0;
    st->ew_op = 0;
    if (st->done) return;
    const uint64_t m = m_rows;
    const double eps = 2.220446049250313e-16;           // numeric_limits<double>::epsilon()
    double* const* col = cols.col;
    auto set_red = [&](int a, int c, uint64_t lo, uint64_t hi) {
        st->red_a = a;
        st->red_c = c;
        st->red_lo = lo;
        st->red_hi = hi;
        st->red_on = hi > lo ? 1 : 0;
    };
    auto set_ew = [&](int op, int c, int e, uint64_t lo, uint64_t hi, double p0, double p1) {
        st->ew_op = hi > lo ? op : 0;
        st->ew_c = c;
        st->ew_e = e;
        st->ew_lo = lo;
        st->ew_hi = hi;
        st->ew_p0 = p0;
        st->ew_p1 = p1;
    };
    auto pivot = [&](int kk) {                           // qr3.h: pivot choice of step kk
        int big = kk;
        double bign = st->nu[kk];
        for (int jj = kk + 1; jj < 3; ++jj)
            if (bign < st->nu[jj]) { bign = st->nu[jj]; big = jj; }
        if (st->nonzero == 3 && bign * bign < st->thr_helper * (double)(m - kk)) st->nonzero = kk;
        st->transp[kk] = big;
        if (kk != big) {
            int tp = st->pc[kk]; st->pc[kk] = st->pc[big]; st->pc[big] = tp;
            double tv = st->nu[kk]; st->nu[kk] = st->nu[big]; st->nu[big] = tv;
            tv = st->nd[kk]; st->nd[kk] = st->nd[big]; st->nd[big] = tv;
        }
        st->ck = st->pc[kk];
    };
    switch (step) {
        case kQsInit:
            for (int q = 0; q < 3; ++q) { st->pc[q] = q; st->tau_k[q] = 0.0; st->transp[q] = q; }
            st->m = m_rows;
            st->nonzero = 3;
            set_red(0, 0, 0, m);
            break;
        case kQsNorm:
            st->nd[k] = sqrt(total);
            st->nu[k] = st->nd[k];
            if (k < 2) {
                set_red(k + 1, k + 1, 0, m);
            } else {
                double maxn = st->nu[0];
                for (int q = 1; q < 3; ++q)
                    if (maxn < st->nu[q]) maxn = st->nu[q];
                const double me = maxn * eps;
                st->thr_helper = (me * me) / (double)m;
                pivot(0);
                set_red(st->ck, st->ck, 1, m);
            }
            break;
        case kQsTail: {
            const int ck = st->ck;
            const double tail = total;
            const double c0 = col[ck][k];
            double tau, beta;
            if (tail <= 2.2250738585072014e-308) {       // numeric_limits<double>::min()
                tau = 0.0;
                beta = c0;
                set_ew(2, ck, 0, k + 1, m, 0.0, 0.0);
            } else {
                beta = sqrt(c0 * c0 + tail);
                if (c0 >= 0.0) beta = -beta;
                set_ew(1, ck, 0, k + 1, m, c0 - beta, 0.0);
                tau = (beta - c0) / beta;
            }
            st->tau_k[k] = tau;
            col[ck][k] = beta;
            if (k + 1 < 3 && tau != 0.0) set_red(ck, st->pc[k + 1], k + 1, m);
            break;
        }
        case kQsRefl: {                                  // apply_reflector(ck, k, tau, pc[j])
            const int ck = st->ck, c = st->pc[j];
            const double tau = st->tau_k[k];
            if (tau != 0.0) {
                double tt = total;
                const double ckv = col[c][k];
                tt += ckv;
                col[c][k] = ckv - tau * tt;
                set_ew(3, c, ck, k + 1, m, tau, tt);
                if (j + 1 < 3) set_red(ck, st->pc[j + 1], k + 1, m);
            }
            break;
        }
        case kQsDd: {                                    // norm downdates of step k
            const double downdate_thr = sqrt(eps);
            for (int jj = k + 1; jj < 3; ++jj) {
                st->ddflag[jj] = 0;
                if (st->nu[jj] != 0.0) {
                    double temp = fabs(col[st->pc[jj]][k]) / st->nu[jj];
                    temp = (1.0 + temp) * (1.0 - temp);
                    temp = temp < 0.0 ? 0.0 : temp;
                    const double r = st->nu[jj] / st->nd[jj];
                    const double temp2 = temp * (r * r);
                    if (temp2 <= downdate_thr) st->ddflag[jj] = 1;
                    else st->nu[jj] *= sqrt(temp);
                }
            }
            if (st->ddflag[k + 1]) set_red(st->pc[k + 1], st->pc[k + 1], k + 1, m);
            break;
        }
        case kQsDd2:
            if (st->ddflag[j]) {
                st->nd[j] = sqrt(total);
                st->nu[j] = st->nd[j];
            }
            if (j + 1 < 3) {
                if (st->ddflag[j + 1]) set_red(st->pc[j + 1], st->pc[j + 1], k + 1, m);
            } else {
                pivot(k + 1);
                set_red(st->ck, st->ck, k + 2, m);
            }
            break;
        case kQsBStart:
            if (st->nonzero == 0) {
                st->x[0] = st->x[1] = st->x[2] = 0.0;
                st->done = 1;
                break;
            }
            if (st->tau_k[0] != 0.0) set_red(st->pc[0], 3, 1, m);
            break;
        case kQsBRefl: {                                 // apply_reflector(pc[k], k, tau_k[k], b)
            if (k < st->nonzero && st->tau_k[k] != 0.0) {
                double tt = total;
                const double bk = col[3][k];
                tt += bk;
                col[3][k] = bk - st->tau_k[k] * tt;
                set_ew(3, 3, st->pc[k], k + 1, m, st->tau_k[k], tt);
            }
            if (k + 1 < 3 && k + 1 < st->nonzero && st->tau_k[k + 1] != 0.0) set_red(st->pc[k + 1], 3, k + 2, m);
            break;
        }
        default: {                                       // kQsFinal: back substitution
            int perm[3] = {0, 1, 2};
            for (int q = 0; q < 3; ++q) {
                const int tq = st->transp[q];
                const int tv = perm[q]; perm[q] = perm[tq]; perm[tq] = tv;
            }
            const int nz = st->nonzero;
            double c[3];
            for (int q = 0; q < 3; ++q) c[q] = col[3][q];
            for (int jj = nz; jj-- > 0;) {
                c[jj] = c[jj] / col[st->pc[jj]][jj];
                for (int i = 0; i < jj; ++i) c[i] -= c[jj] * col[st->pc[jj]][i];
            }
            for (int i = 0; i < nz; ++i) st->x[perm[i]] = c[i];
            for (int i = nz; i < 3; ++i) st->x[perm[i]] = 0.0;
            st->done = 1;
            break;
        }
    }
}

// ---- fused device QR (QRFState, kernels.h) ------------------------------
// One pass: a 256-thread workgroup per aligned block of kSumBlock rows; thread
// t walks rows base + t + 256 q (q = 0..3, coalesced, all loads in flight),
// applies the pass's element-wise step to rows >= lo, stores the changed
// columns, and accumulates every reduction's products of its range
// sequentially; the block tree then gives blocked_sum's block partial, stored
// at partials[r * nblk + blk].  Columns are addressed through slots (slot 0 =
// the Householder column in modes 2 / 3).
__global__ __launch_bounds__(256) void k_qrf_pass(QRCols cols, const QRFState* __restrict__ st, uint64_t m,
                                                  uint64_t nblk, double* __restrict__ partials) {
    __shared__ double lds[kQrfMaxRed * 256];
    const int mode = st->mode;
    if (mode == 0) return;
    const int t = threadIdx.x;
    const uint64_t blk = blockIdx.x;
    if (blk >= nblk) return;
    const uint64_t base = blk * kSumBlock;
    const uint64_t lo = st->lo;
    const int nslot = st->nslot, nred = st->nred, nt = st->nt;
    const double* src[4];
    double* dst[4];
    for (int k = 0; k < 4; ++k) {
        src[k] = k < nslot ? cols.col[st->scol[k]] : nullptr;
        dst[k] = k < nslot ? cols.col[st->scol[k]] : nullptr;
    }
    const bool zero = st->zero != 0, wr0 = st->write_ck != 0;
    const double den = st->den, tau = st->tau;
    const double tt[4] = {0.0, st->tt[0], st->tt[1], st->tt[2]};
    int ra[kQrfMaxRed], rb[kQrfMaxRed];
    uint64_t rlo[kQrfMaxRed];
    double acc[kQrfMaxRed];
#pragma unroll
    for (int r = 0; r < kQrfMaxRed; ++r) {
        ra[r] = r < nred ? st->ra[r] : 0;
        rb[r] = r < nred ? st->rc[r] : 0;
        rlo[r] = r < nred ? st->rlo[r] : m;
        acc[r] = 0.0;
    }
    constexpr int kU = (int)(kSumBlock / 256);
    double v[kU][4];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const uint64_t i = base + t + 256 * u;
#pragma unroll
        for (int k = 0; k < 4; ++k) v[u][k] = (k < nslot && i < m) ? src[k][i] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const uint64_t i = base + t + 256 * u;
        if (i >= m) continue;
        if (i >= lo) {
            if (mode == 2) {                    // Householder column: scale (or zero)
                v[u][0] = zero ? 0.0 : v[u][0] / den;
                if (wr0) dst[0][i] = v[u][0];
            } else if (mode == 3) {             // reflector on the targets (slots 1 .. nt)
#pragma unroll
                for (int k = 1; k < 4; ++k)
                    if (k <= nt) {
                        v[u][k] -= (tau * v[u][0]) * tt[k];
                        dst[k][i] = v[u][k];
                    }
            }
        }
#pragma unroll
        for (int r = 0; r < kQrfMaxRed; ++r) {
            if (r >= nred || i < rlo[r]) continue;
            double pa = 0.0, pb = 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (ra[r] == k) pa = v[u][k];
                if (rb[r] == k) pb = v[u][k];
            }
            acc[r] += pa * pb;
        }
    }
    qr_block_tree<kQrfMaxRed>(acc, nred, lds);
    if (t == 0)
        for (int r = 0; r < nred; ++r) partials[(uint64_t)r * nblk + blk] = acc[r];
}

// P0 of the hybrid refit: builds the rows (sift_row_at, as k_sift_rows) of a
// block and takes the six reductions the first step needs from them:
// r = c: sumsq(col c, 0, m), r = 3 + c: sumsq(col c, 1, m), c = 0..2
__global__ __launch_bounds__(256) void k_qrf_p0(DevClass sc, DevClass oc, const uint32_t* __restrict__ si,
                                                uint32_t ns, const uint32_t* __restrict__ oi, uint32_t no,
                                                QRCols cols, uint64_t m, uint64_t nblk,
                                                double* __restrict__ partials) {
    __shared__ double lds[6 * 256];
    const int t = threadIdx.x;
    const uint64_t blk = blockIdx.x;
    if (blk >= nblk) return;
    const uint64_t base = blk * kSumBlock;
    double acc[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < (int)(kSumBlock / 256); ++q) {
        const uint64_t i = base + t + 256 * q;
        if (i >= m) break;
        double row[4];
        sift_row_at(sc, oc, si, ns, oi, no, i, row);
#pragma unroll
        for (int c = 0; c < 4; ++c) cols.col[c][i] = row[c];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double pr = row[c] * row[c];
            acc[c] += pr;
            if (i >= 1) acc[3 + c] += pr;
        }
    }
    qr_block_tree<6>(acc, 6, lds);
    if (t == 0)
        for (int r = 0; r < 6; ++r) partials[(uint64_t)r * nblk + blk] = acc[r];
}

constexpr int kQrfCtlThreads = 512;     // >= kQrfMaxRed x 64 super-blocks (4 M rows) in one sweep
__global__ __launch_bounds__(kQrfCtlThreads) void k_qrf_ctl(QRCols cols, QRFState* st,
                                                            const double* __restrict__ partials, uint64_t m,
                                                            uint64_t nblk, int step, int k) {
    constexpr uint64_t per = kSumSuper / kSumBlock;
    __shared__ double sup[kQrfMaxRed * kQrdSup];
    // totals of the previous pass's reductions (all ranges start in block 0):
    // the block partials sequentially inside each aligned super-block (one
    // lane per (reduction, super-block), its <= 64 loads in flight), then the
    // super-block partials sequentially -- blocked_sum's order
    // STEP(0) follows P0 (six reductions, state not yet initialised)
    const bool first = step == kQfStep && k == 0;
    const int nred = first ? 6 : (st->mode == 0 ? 0 : st->nred);
    const uint64_t nsup = (nblk - 1) / per + 1;
    for (uint64_t idx = threadIdx.x; idx < (uint64_t)nred * nsup; idx += kQrfCtlThreads) {
        const uint64_t r = idx / nsup, u = idx % nsup;
        const double* part = partials + r * nblk;
        const uint64_t b_lo = u * per, b_hi = min(nblk, (u + 1) * per);
        double w[per];
#pragma unroll
        for (uint64_t q = 0; q < per; ++q) w[q] = b_lo + q < b_hi ? part[b_lo + q] : 0.0;
        double sp = 0.0;
#pragma unroll
        for (uint64_t q = 0; q < per; ++q)
            if (b_lo + q < b_hi) sp += w[q];
        sup[idx] = sp;
    }
    __syncthreads();
    // lane r: the super-block partials of reduction r, sequentially
    __shared__ double tot_sh[kQrfMaxRed];
    if (threadIdx.x < (unsigned)nred) {
        const double* sr = sup + (uint64_t)threadIdx.x * nsup;
        double tv = 0.0;
        uint64_t u = 0;
        for (; u + 8 <= nsup; u += 8) {
            double w[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) w[q] = sr[u + q];
#pragma unroll
            for (int q = 0; q < 8; ++q) tv += w[q];
        }
        for (; u < nsup; ++u) tv += sr[u];
        tot_sh[threadIdx.x] = tv;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    double tot[kQrfMaxRed];
    for (int r = 0; r < kQrfMaxRed; ++r) tot[r] = r < nred ? tot_sh[r] : 0.0;
    if (first) {
        for (int q = 0; q < 3; ++q) { st->pc[q] = q; st->tau_k[q] = 0.0; st->transp[q] = q; }
        st->nonzero = 3;
        st->done = 0;
    }
    double* const* col = cols.col;
    const double eps = 2.220446049250313e-16;           // numeric_limits<double>::epsilon()
    st->mode = 0;
    st->nred = 0;
    st->nt = 0;
    if (st->done) return;
    if (step == kQfStep) {
        double tail_of[3] = {0.0, 0.0, 0.0};
        if (k == 0) {
            for (int c = 0; c < 3; ++c) {
                st->nd[c] = sqrt(tot[c]);               // pc[c] == c before the first pivot
                st->nu[c] = st->nd[c];
                tail_of[c] = tot[3 + c];
            }
            double maxn = st->nu[0];
            for (int q = 1; q < 3; ++q)
                if (maxn < st->nu[q]) maxn = st->nu[q];
            const double me = maxn * eps;
            st->thr_helper = (me * me) / (double)m;
        } else {
            // the norm downdates of step k - 1 (qr3.h): remaining columns
            // pc[j], j >= k; U(k-1) summed sumsq(pc[j], k, m) at 2 (j - k) and
            // sumsq(pc[j], k + 1, m) at 2 (j - k) + 1
            const double downdate_thr = sqrt(eps);
            for (int j = k; j < 3; ++j) {
                const int cj = st->pc[j];
                tail_of[cj] = tot[2 * (j - k) + 1];
                if (st->nu[j] != 0.0) {
                    double temp = fabs(col[cj][k - 1]) / st->nu[j];
                    temp = (1.0 + temp) * (1.0 - temp);
                    temp = temp < 0.0 ? 0.0 : temp;
                    const double r = st->nu[j] / st->nd[j];
                    const double temp2 = temp * (r * r);
                    if (temp2 <= downdate_thr) {
                        st->nd[j] = sqrt(tot[2 * (j - k)]);
                        st->nu[j] = st->nd[j];
                    } else {
                        st->nu[j] *= sqrt(temp);
                    }
                }
            }
        }
        // pivot of step k
        int big = k;
        double bign = st->nu[k];
        for (int jj = k + 1; jj < 3; ++jj)
            if (bign < st->nu[jj]) { bign = st->nu[jj]; big = jj; }
        if (st->nonzero == 3 && bign * bign < st->thr_helper * (double)(m - k)) st->nonzero = k;
        st->transp[k] = big;
        if (k != big) {
            int tp = st->pc[k]; st->pc[k] = st->pc[big]; st->pc[big] = tp;
            double tv = st->nu[k]; st->nu[k] = st->nu[big]; st->nu[big] = tv;
            tv = st->nd[k]; st->nd[k] = st->nd[big]; st->nd[big] = tv;
        }
        const int ck = st->pc[k];
        const double tail = tail_of[ck];
        const double c0 = col[ck][k];
        double tau, beta;
        st->ck = ck;
        st->lo = (uint64_t)k + 1;
        if (tail <= 2.2250738585072014e-308) {       // numeric_limits<double>::min()
            tau = 0.0;
            beta = c0;
            st->zero = 1;
            st->den = 0.0;
        } else {
            beta = sqrt(c0 * c0 + tail);
            if (c0 >= 0.0) beta = -beta;
            st->zero = 0;
            st->den = c0 - beta;
            tau = (beta - c0) / beta;
        }
        st->tau_k[k] = tau;
        st->tau = tau;
        col[ck][k] = beta;
        // A(k): the reflector's dots with the remaining columns and with b
        // (b's reflector k runs iff k < nonzero, decided by this pivot)
        st->dob = (k < st->nonzero && tau != 0.0) ? 1 : 0;
        st->scol[0] = ck;
        int n = 0;
        if (tau != 0.0)
            for (int j = k + 1; j < 3; ++j) {
                st->scol[1 + n] = st->pc[j];
                st->ra[n] = 0;
                st->rc[n] = 1 + n;
                st->rlo[n] = (uint64_t)k + 1;
                ++n;
            }
        if (st->dob) {
            st->scol[1 + n] = 3;
            st->ra[n] = 0;
            st->rc[n] = 1 + n;
            st->rlo[n] = (uint64_t)k + 1;
            ++n;
        }
        st->nslot = 1 + n;
        st->nred = n;
        st->nt = 0;
        st->write_ck = k < 2 ? 1 : 0;     // v_2 is only needed for b's dot, taken in this pass
        st->mode = 2;
        return;
    }
    if (step == kQfApply) {
        // reflector k applied to the tops of its targets (apply_reflector)
        const int ck = st->ck;
        const double tau = st->tau_k[k];
        int n = 0, nt = 0;
        st->scol[0] = ck;
        if (tau != 0.0)
            for (int j = k + 1; j < 3; ++j) {
                const int c = st->pc[j];
                double tt = tot[n++];
                const double ckv = col[c][k];
                tt += ckv;
                col[c][k] = ckv - tau * tt;
                st->scol[1 + nt] = c;
                st->tt[nt] = tt;
                ++nt;
            }
        if (st->dob) {
            double tt = tot[n++];
            const double bk = col[3][k];
            tt += bk;
            col[3][k] = bk - tau * tt;
            st->scol[1 + nt] = 3;
            st->tt[nt] = tt;
            ++nt;
        }
        // U(k): the updates (slots 1 .. nt), then the downdate sums
        // sumsq(pc[j], k+1, m) and the next tails sumsq(pc[j], k+2, m) of the
        // remaining columns (read-only slots when tau = 0)
        int ns = 1 + nt;
        st->nt = nt;
        st->ck = ck;
        st->tau = tau;
        st->lo = (uint64_t)k + 1;
        int r = 0;
        for (int j = k + 1; j < 3; ++j) {
            int slot = -1;
            for (int q = 1; q < ns; ++q)
                if (st->scol[q] == st->pc[j]) slot = q;
            if (slot < 0) {
                slot = ns++;
                st->scol[slot] = st->pc[j];
            }
            st->ra[r] = st->rc[r] = slot;
            st->rlo[r] = (uint64_t)k + 1;
            ++r;
            st->ra[r] = st->rc[r] = slot;
            st->rlo[r] = (uint64_t)k + 2;
            ++r;
        }
        st->nslot = ns;
        st->nred = r;
        st->mode = 3;
        return;
    }
    // kQfFinal (after A(2)): b's reflector 2 on the top row, back substitution
    {
        const double tau = st->tau_k[2];
        if (st->dob) {
            double tt = tot[0];
            const double bk = col[3][2];
            tt += bk;
            col[3][2] = bk - tau * tt;
        }
        if (st->nonzero == 0) {
            st->x[0] = st->x[1] = st->x[2] = 0.0;
            st->done = 1;
            return;
        }
        int perm[3] = {0, 1, 2};
        for (int q = 0; q < 3; ++q) {
            const int tq = st->transp[q];
            const int tv = perm[q]; perm[q] = perm[tq]; perm[tq] = tv;
        }
        const int nz = st->nonzero;
        double c[3];
        for (int q = 0; q < 3; ++q) c[q] = col[3][q];
        for (int jj = nz; jj-- > 0;) {
            c[jj] = c[jj] / col[st->pc[jj]][jj];
            for (int i = 0; i < jj; ++i) c[i] -= c[jj] * col[st->pc[jj]][i];
        }
        for (int i = 0; i < nz; ++i) st->x[perm[i]] = c[i];
        for (int i = nz; i < 3; ++i) st->x[perm[i]] = 0.0;
        st->done = 1;
    }
}

// rows 0..2 of the four columns (the only rows the QR driver reads on the
// host) into out[c * 3 + i]
__global__ void k_qr_top(const double* c0, const double* c1, const double* c2, const double* c3, uint64_t m,
                         double* out) {
    const int t = threadIdx.x;
    if (t >= 12) return;
    const int c = t / 3, i = t % 3;
    const double* col = c == 0 ? c0 : c == 1 ? c1 : c == 2 ? c2 : c3;
    out[t] = (uint64_t)i < m ? col[i] : 0.0;
}

__global__ void k_qr_scale(double* c, uint64_t lo, uint64_t hi, double den) {
    const uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < hi) c[i] = c[i] / den;
}
__global__ void k_qr_zero(double* c, uint64_t lo, uint64_t hi) {
    const uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < hi) c[i] = 0.0;
}
__global__ void k_qr_update(double* c, const double* e, uint64_t lo, uint64_t hi, double tau, double t) {
    const uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < hi) c[i] -= (tau * e[i]) * t;
}

// workgroup records -> one BatchRecord: first strict best over workgroups in
// order (= slots in order), ties to the lower slot
// Workgroup b of the launch reduces batch b (deferred selection: records at
// wg + b * wg_stride, models at models + b * nslots, slots from
// slot0 + b * nslots, record out[b]); a per-launch selection is one workgroup.
__global__ __launch_bounds__(kSelectThreads) void k_select_wg(const WgBest* __restrict__ wg, uint32_t nwg,
                                                              const RectModel* __restrict__ models, uint64_t slot0,
                                                              BatchRecord* out, uint32_t wg_stride = 0,
                                                              uint32_t nslots = 0) {
    wg += (size_t)blockIdx.x * wg_stride;
    models += (size_t)blockIdx.x * nslots;
    slot0 += (uint64_t)blockIdx.x * nslots;
    out += blockIdx.x;
    __shared__ double s_val[kSelectThreads];
    __shared__ int32_t s_slot[kSelectThreads];
    __shared__ uint32_t s_n0[kSelectThreads], s_n1[kSelectThreads];
    __shared__ unsigned long long s_models[kSelectThreads], s_its[kSelectThreads];
    const int t = threadIdx.x;
    double best = 0.0;
    int32_t bs = -1;
    uint32_t b0 = 0, b1 = 0;
    unsigned long long nm = 0, its = 0;
    for (uint32_t j = t; j < nwg; j += kSelectThreads) {
        const WgBest w = wg[j];
        nm += w.models;
        its += w.iterations;
        if (w.slot >= 0 && best < w.score) { best = w.score; bs = w.slot; b0 = w.n0; b1 = w.n1; }
    }
    s_val[t] = best; s_slot[t] = bs; s_n0[t] = b0; s_n1[t] = b1; s_models[t] = nm; s_its[t] = its;
    __syncthreads();
    for (int w = kSelectThreads / 2; w > 0; w >>= 1) {
        if (t < w) {
            const int32_t ia = s_slot[t], ib = s_slot[t + w];
            const double va = s_val[t], vb = s_val[t + w];
            if (ib >= 0 && (ia < 0 || vb > va || (vb == va && ib < ia))) {
                s_slot[t] = ib; s_val[t] = vb; s_n0[t] = s_n0[t + w]; s_n1[t] = s_n1[t + w];
            }
            s_models[t] += s_models[t + w];
            s_its[t] += s_its[t + w];
        }
        __syncthreads();
    }
    if (t == 0) {
        BatchRecord r;
        r.models = s_models[0];
        r.iterations = s_its[0];
        r.best_slot = -1;
        r.best_score = 0.0;
        r.best_inliers[0] = r.best_inliers[1] = 0;
        r.best_model = default_model();
        if (s_slot[0] >= 0) {
            r.best_slot = (int64_t)(slot0 + (uint64_t)s_slot[0]);
            r.best_score = s_val[0];
            r.best_inliers[0] = s_n0[0];
            r.best_inliers[1] = s_n1[0];
            r.best_model = models[s_slot[0]];
        }
        *out = r;
    }
}

// ----------------------------------------------------------------- mask ----
template <int KIND>
__global__ __launch_bounds__(kMaskBlock) void k_mask(DevClass c, int cls, typename ModelOf<KIND>::type m, int rule,
                                                     double T, double lambda, double fmid, double fhalf,
                                                     uint8_t* __restrict__ mask) {
    const uint32_t i = blockIdx.x * kMaskBlock + threadIdx.x;
    if (i >= c.n) return;
    double r2;
    if constexpr (KIND >= 3) r2 = geo_sq_residual<KIND>(c.x[i], c.y[i], c.a[i], c.c0[i], m.h);
    else {
        const ValueConst vc = value_const(m, KIND == 1, cls == 1);
        if (cls == 0) r2 = scale_sq_value<KIND == 1, false>(c.x[i], c.y[i], c.a[i], m, vc.ac, vc.cut);
        else r2 = orient_sq_value<false>(c.x[i], c.y[i], c.c0[i], c.c1[i], m, vc.c, vc.s, vc.cphi, vc.cphi2);
    }
    // rule 2: labeling(), BK max-flow with no pairwise edges (empty grid
    // graph, gcransac_python.cpp:63-68) -> SINK iff terminal capacity < 0;
    // bit 1: a decision within the twin-glibc bound (exact.h), rechecked by
    // the host
    const bool flag = KIND <= 2 && in_flag_band(r2, fmid, fhalf);
    mask[i] = (uint8_t)((mask_rule(r2, rule, T, lambda) ? 1 : 0) | (flag ? 2 : 0));
}

// ----------------------------------------------------------------- math ----
__global__ void k_math(int op, const double* __restrict__ a, const double* __restrict__ b, size_t n,
                       double* __restrict__ out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    double r;
    switch (op) {
        case 0: r = dm::dm_log(a[i]); break;
        case 1: r = dm::dm_pow_m3(a[i]); break;
        case 2: r = dm::dm_atan2(a[i], b[i]); break;
        case 3: r = a[i] / b[i]; break;
        case 5: r = dm::clip_angle_small(a[i]); break;
        case 6: r = dm::clip_angle(a[i]); break;
        case 8: r = dm::dm_log_fd(a[i]); break;
        case 9: { double sn, cs; dm::dm_sincos(a[i], sn, cs); r = sn; } break;
        case 10: { double sn, cs; dm::dm_sincos(a[i], sn, cs); r = cs; } break;
        case 11: r = dm::atan_ratio(a[i], b[i]); break;
        default: r = sqrt(a[i]); break;
    }
    out[i] = r;
}

inline unsigned blocks_for(size_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

template <int G>
void launch_generate_g(const DevProblem& p, uint64_t seed, uint64_t slot0, uint32_t nslots, uint8_t* inc,
                       RectModel* models, hipStream_t stream) {
    const dim3 grid(blocks_for((size_t)nslots * G, kGenBlock)), block(kGenBlock);
    switch (p.solver) {
        case 0: hipLaunchKernelGGL((k_generate<0, G>), grid, block, 0, stream, p, seed, slot0, nslots, inc, models); break;
        case 1: hipLaunchKernelGGL((k_generate<1, G>), grid, block, 0, stream, p, seed, slot0, nslots, inc, models); break;
        default: hipLaunchKernelGGL((k_generate<2, G>), grid, block, 0, stream, p, seed, slot0, nslots, inc, models); break;
    }
}

hipError_t launch_generate(const DevProblem& p, uint64_t seed, uint64_t slot0, uint32_t nslots, uint8_t* inc,
                           RectModel* models, hipStream_t stream) {
    if (nslots == 0) return hipSuccess;
    // lanes per slot: enough lanes in flight to cover the chip (~128k), at
    // most 16 parallel attempts per slot
    if (nslots <= 8192) launch_generate_g<16>(p, seed, slot0, nslots, inc, models, stream);
    else if (nslots <= 16384) launch_generate_g<8>(p, seed, slot0, nslots, inc, models, stream);
    else if (nslots <= 32768) launch_generate_g<4>(p, seed, slot0, nslots, inc, models, stream);
    else if (nslots <= 65536) launch_generate_g<2>(p, seed, slot0, nslots, inc, models, stream);
    else launch_generate_g<1>(p, seed, slot0, nslots, inc, models, stream);
    return hipGetLastError();
}

template <bool kIdentity>
void launch_score_t(const DevProblem& p, const double T[2], const RectModel* models, const uint8_t* inc, uint32_t nh,
                    const ScoreOut& out, hipStream_t stream) {
    const dim3 grid(blocks_for(nh, kScoreBlock)), block(kScoreBlock);
    switch (p.solver) {
        case 0: hipLaunchKernelGGL((k_score<0, kIdentity>), grid, block, 0, stream, p, T[0], T[1], flag_band(T), models, inc, nh, out); break;
        case 1: hipLaunchKernelGGL((k_score<1, kIdentity>), grid, block, 0, stream, p, T[0], T[1], flag_band(T), models, inc, nh, out); break;
        default: hipLaunchKernelGGL((k_score<2, kIdentity>), grid, block, 0, stream, p, T[0], T[1], flag_band(T), models, inc, nh, out); break;
    }
}

// band constants of the conservative prefilters: exp(1.5 thr) bounds the
// rectified log-scale residual, tan(1.5 thr) the rectified angular one (host
// libm; the in-kernel tests widen them further)
void band_consts(const double T[2], double& band0, double& tan_tau1) {
    band0 = exp(sqrt(T[0] / 2.25) * 1.5) * (1.0 + 1e-9);
    const double tau1 = sqrt(T[1]);
    // + 1e-12: the flag band of exact.h reaches kDevOrient = 4e-14 past sqrt(T)
    tan_tau1 = (tau1 < 0.7) ? tan(tau1) * (1.0 + 1e-6) + 1e-12 : HUGE_VAL;
}

template <int H, int R>
void launch_split_t(const DevProblem& p, const double T[2], const RectModel* models, const uint8_t* inc, uint32_t nh,
                    const ScoreOut& out, hipStream_t stream) {
    const dim3 grid((nh + H - 1) / H), block(kSplitThreads);
    double band0, tan_tau1;
    band_consts(T, band0, tan_tau1);
    switch (p.solver) {
        case 0: hipLaunchKernelGGL((k_score_split<0, H, R, false>), grid, block, 0, stream, p, T[0], T[1], band0, tan_tau1, flag_band(T), models, inc, nh, out, GenArgs{}); break;
        case 1: hipLaunchKernelGGL((k_score_split<1, H, R, false>), grid, block, 0, stream, p, T[0], T[1], band0, tan_tau1, flag_band(T), models, inc, nh, out, GenArgs{}); break;
        default: hipLaunchKernelGGL((k_score_split<2, H, R, false>), grid, block, 0, stream, p, T[0], T[1], band0, tan_tau1, flag_band(T), models, inc, nh, out, GenArgs{}); break;
    }
}

// GCR_SCORER=split selects the round-synchronous split scorer (k_score_split)
// instead of the feature-major one (k_score_fm) for the band estimators
bool use_fm() {
    static const bool fm = [] {
        const char* e = getenv("GCR_SCORER");
        return !(e && e[0] == 's');
    }();
    return fm;
}

// the correspondence scorer compacts a launch of nh hypotheses itself, in
// the feature-major scorer's prologue (launch_score_geo with compact = true
// at H = 16); the engine's verify pipeline compacts behind the generator
// otherwise.  One cached source (use_fm) for both sides.
bool geo_scorer_scans(uint32_t nh) { return use_fm() && split_h(nh) == 16; }

template <int H, bool kGen>
void launch_fm_t(const DevProblem& p, const double T[2], uint32_t nh, const ScoreOut& out, const GenArgs& g,
                 hipStream_t stream, const RectModel* models = nullptr, const uint8_t* inc = nullptr) {
    const dim3 grid((nh + H - 1) / H), block(kSplitThreads);
    double band0, tan_tau1;
    band_consts(T, band0, tan_tau1);
    switch (p.solver) {
        case 0: hipLaunchKernelGGL((k_score_fm<0, H, kGen>), grid, block, 0, stream, p, T[0], T[1], band0, tan_tau1, flag_band(T), models, inc, nh, out, g); break;
        case 1: hipLaunchKernelGGL((k_score_fm<1, H, kGen>), grid, block, 0, stream, p, T[0], T[1], band0, tan_tau1, flag_band(T), models, inc, nh, out, g); break;
        default: hipLaunchKernelGGL((k_score_fm<2, H, kGen>), grid, block, 0, stream, p, T[0], T[1], band0, tan_tau1, flag_band(T), models, inc, nh, out, g); break;
    }
}

int score_mode() {
    static const int mode = [] {          // thread-safe one-time init (gcr_solve_batch threads)
        const char* e = getenv("GCR_SCORE_KERNEL");
        return (e && e[0] == 'n') ? 1 : 0;   // "naive" -> lane-per-hypothesis kernel
    }();
    return mode;
}

// GCR_SPLIT_H=64|16|4 pins the split-scorer variant (tuning sweeps); default:
// by batch size, so that the grid still covers the 256 CUs.
int split_h(uint32_t nh) {
    static const int forced = [] {
        const char* e = getenv("GCR_SPLIT_H");
        const int v = e ? atoi(e) : 0;
        return (v == 64 || v == 16 || v == 4) ? v : 0;
    }();
    if (forced) return forced;
    return nh >= 16384 ? 64 : nh >= 2048 ? 16 : 4;
}

hipError_t launch_select(int solver, const ScoreOut& sc, const uint8_t* inc, const RectModel* models,
                         uint32_t nslots, uint64_t slot0, const uint32_t m[2], const double Tm[2], BatchRecord* out,
                         hipStream_t stream) {
    hipLaunchKernelGGL(k_select<RectModel>, dim3(1), dim3(kSelectThreads), 0, stream, solver, sc, inc, models,
                       nslots, slot0, m[0], m[1], Tm[0], Tm[1], out);
    return hipGetLastError();
}

hipError_t launch_score(const DevProblem& p, const double T[2], const RectModel* models, const uint8_t* inc,
                        uint32_t nh, bool identity, const ScoreOut& out, hipStream_t stream) {
    if (nh == 0) return hipSuccess;
    if (!identity) launch_score_t<false>(p, T, models, inc, nh, out, stream);
    else if (score_mode() == 1) launch_score_t<true>(p, T, models, inc, nh, out, stream);
    else {
        const int h = split_h(nh);
        if (h == 64) launch_split_t<64, 120>(p, T, models, inc, nh, out, stream);
        else if (h == 16 && use_fm()) launch_fm_t<16, false>(p, T, nh, out, GenArgs{}, stream, models, inc);
        else if (h == 16) launch_split_t<16, 420>(p, T, models, inc, nh, out, stream);
        else launch_split_t<4, 960>(p, T, models, inc, nh, out, stream);
    }
    return hipGetLastError();
}

// A prefetched chunk's budget cut (the replay's `while (cnt < B && itp < L)`):
// slot j stays iff budget - sum_{k < j} inc[k] > 0; later slots are marked
// absent (inc = 255: no model), so the scorer skips them.  One workgroup,
// each thread a contiguous run of slots.
constexpr int kTruncThreads = 1024;
__global__ __launch_bounds__(kTruncThreads) void k_truncate(uint8_t* __restrict__ inc, uint32_t n, uint64_t budget) {
    __shared__ uint64_t part[kTruncThreads];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (n + kTruncThreads - 1) / kTruncThreads;
    const uint32_t b = t * per, e = min(n, b + per);
    uint64_t sum = 0;
    for (uint32_t j = b; j < e; ++j) sum += inc[j];
    part[t] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < kTruncThreads; off <<= 1) {     // inclusive scan
        const uint64_t v = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t before = t == 0 ? 0 : part[t - 1];
    for (uint32_t j = b; j < e; ++j) {
        const uint64_t cur = inc[j];
        if (before >= budget) inc[j] = 255;
        before += cur;
    }
}

hipError_t launch_truncate(uint8_t* inc, uint32_t n, uint64_t budget, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_truncate, dim3(1), dim3(kTruncThreads), 0, stream, inc, n, budget);
    return hipGetLastError();
}

hipError_t launch_sift_rows(const DevClass& sc, const DevClass& oc, const uint32_t* si, uint32_t ns,
                            const uint32_t* oi, uint32_t no, size_t rows, double* A0, double* A1, double* A2,
                            double* b, hipStream_t stream) {
    if (rows == 0) return hipSuccess;
    hipLaunchKernelGGL(k_sift_rows, dim3((unsigned)((rows + kRowBlock - 1) / kRowBlock)), dim3(kRowBlock), 0, stream,
                       sc, oc, si, ns, oi, no, (uint64_t)rows, A0, A1, A2, b);
    return hipGetLastError();
}

hipError_t launch_sift_gram(const DevClass& sc, const DevClass& oc, const uint32_t* hidx, uint32_t ns, uint32_t no,
                            size_t rows, uint32_t* idx, double* lines, DD* tiles, const GramFinal& fin,
                            hipStream_t stream) {
    if (rows == 0) return hipSuccess;
    if (ns + no > 0)
        hipLaunchKernelGGL(k_gram_prep, dim3((ns + no + kGramBlock - 1) / kGramBlock), dim3(kGramBlock), 0, stream, oc,
                           hidx, ns, no, idx, lines);
    const dim3 grid((unsigned)((rows + kGramTile - 1) / kGramTile));
    const char* e = getenv("GCR_GRAM_BATCH");                 // read per call (measurements)
    const int batch = e ? atoi(e) : 1;
    if (batch == 1)
        hipLaunchKernelGGL(k_sift_gram<1>, grid, dim3(kGramBlock), 0, stream, sc, idx, ns, lines, no, (uint64_t)rows, tiles);
    else if (batch == 2)
        hipLaunchKernelGGL(k_sift_gram<2>, grid, dim3(kGramBlock), 0, stream, sc, idx, ns, lines, no, (uint64_t)rows, tiles);
    else
        hipLaunchKernelGGL(k_sift_gram<4>, grid, dim3(kGramBlock), 0, stream, sc, idx, ns, lines, no, (uint64_t)rows, tiles);
    if (fin.out != nullptr)
        hipLaunchKernelGGL(k_gram_final, dim3(1), dim3(64 * kGramN), 0, stream, tiles, grid.x, fin);
    return hipGetLastError();
}

hipError_t launch_qr_partials(const double* a, const double* c, size_t lo, size_t hi, double* partials,
                              size_t* nblocks, hipStream_t stream) {
    *nblocks = 0;
    if (hi <= lo) return hipSuccess;
    const uint64_t blk0 = lo / kSumBlock, nblk = (hi - 1) / kSumBlock - blk0 + 1;
    *nblocks = nblk;
    hipLaunchKernelGGL(k_qr_partials, dim3((unsigned)nblk), dim3(256), 0, stream, a, c, (uint64_t)lo, (uint64_t)hi,
                       blk0, nblk, partials);
    return hipGetLastError();
}

hipError_t launch_qr_device(double* const cols[4], size_t m, QRDevState* st, double* partials, double x_out[3],
                            hipStream_t stream) {
    if (m < 4 || m > (size_t)kQrdSup * kSumSuper) return hipErrorInvalidValue;
    QRCols qc{{cols[0], cols[1], cols[2], cols[3]}};
    const uint64_t nblk = (m - 1) / kSumBlock + 1;
    const dim3 gr((unsigned)nblk), br(256);
    const dim3 ge((unsigned)((m + 255) / 256)), be(256);
    hipError_t e = hipMemsetAsync(st, 0, sizeof(QRDevState), stream);   // no reduction pending, not done
    if (e != hipSuccess) return e;
    auto C = [&](int step, int k, int j) {
        hipLaunchKernelGGL(k_qrd_ctl, dim3(1), dim3(64), 0, stream, qc, st, partials, (uint64_t)m, step, k, j);
    };
    auto R = [&]() { hipLaunchKernelGGL(k_qrd_partials, gr, br, 0, stream, qc, st, partials); };
    auto E = [&]() { hipLaunchKernelGGL(k_qrd_ew, ge, be, 0, stream, qc, st); };
    // qr3.h qr_solve<3>, step for step
    C(kQsInit, 0, 0);
    for (int k = 0; k < 3; ++k) { R(); C(kQsNorm, k, 0); }
    for (int k = 0; k < 3; ++k) {
        R(); C(kQsTail, k, 0); E();
        for (int j = k + 1; j < 3; ++j) { R(); C(kQsRefl, k, j); E(); }
        if (k < 2) {
            C(kQsDd, k, 0);
            for (int j = k + 1; j < 3; ++j) { R(); C(kQsDd2, k, j); }
        }
    }
    C(kQsBStart, 0, 0);
    for (int k = 0; k < 3; ++k) { R(); C(kQsBRefl, k, 0); E(); }
    C(kQsFinal, 0, 0);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    const double* dx = reinterpret_cast<const double*>(reinterpret_cast<const char*>(st) + offsetof(QRDevState, x));
    e = hipMemcpyAsync(x_out, dx, 3 * sizeof(double), hipMemcpyDeviceToHost, stream);
    if (e != hipSuccess) return e;
    return hipStreamSynchronize(stream);
}

hipError_t launch_sift_refit_fused(const DevClass& sc, const DevClass& oc, const uint32_t* si, uint32_t ns,
                                   const uint32_t* oi, uint32_t no, size_t m, double* const cols[4], QRFState* st,
                                   double* partials, double x_out[3], hipStream_t stream) {
    if (m < 4 || m > (size_t)kQrdSup * kSumSuper) return hipErrorInvalidValue;
    QRCols qc{{cols[0], cols[1], cols[2], cols[3]}};
    const uint64_t nblk = (m - 1) / kSumBlock + 1;
    const dim3 gp((unsigned)nblk), bp(256);
    auto C = [&](int step, int k) {
        hipLaunchKernelGGL(k_qrf_ctl, dim3(1), dim3(kQrfCtlThreads), 0, stream, qc, st, partials, (uint64_t)m, nblk,
                           step, k);
    };
    auto P = [&]() { hipLaunchKernelGGL(k_qrf_pass, gp, bp, 0, stream, qc, st, (uint64_t)m, nblk, partials); };
    hipLaunchKernelGGL(k_qrf_p0, gp, bp, 0, stream, sc, oc, si, ns, oi, no, qc, (uint64_t)m, nblk, partials);
    for (int k = 0; k < 3; ++k) {
        C(kQfStep, k);
        P();                                // A(k)
        if (k < 2) {
            C(kQfApply, k);
            P();                            // U(k)
        }
    }
    C(kQfFinal, 2);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const double* dx = reinterpret_cast<const double*>(reinterpret_cast<const char*>(st) + offsetof(QRFState, x));
    e = hipMemcpyAsync(x_out, dx, 3 * sizeof(double), hipMemcpyDeviceToHost, stream);
    if (e != hipSuccess) return e;
    return hipStreamSynchronize(stream);
}

hipError_t launch_qr_top(const double* c0, const double* c1, const double* c2, const double* c3, size_t m,
                         double* out, hipStream_t stream) {
    hipLaunchKernelGGL(k_qr_top, dim3(1), dim3(64), 0, stream, c0, c1, c2, c3, (uint64_t)m, out);
    return hipGetLastError();
}

hipError_t launch_qr_scale(double* c, size_t lo, size_t hi, double den, hipStream_t stream) {
    if (hi <= lo) return hipSuccess;
    hipLaunchKernelGGL(k_qr_scale, dim3((unsigned)((hi - lo + 255) / 256)), dim3(256), 0, stream, c, (uint64_t)lo,
                       (uint64_t)hi, den);
    return hipGetLastError();
}

hipError_t launch_qr_zero(double* c, size_t lo, size_t hi, hipStream_t stream) {
    if (hi <= lo) return hipSuccess;
    hipLaunchKernelGGL(k_qr_zero, dim3((unsigned)((hi - lo + 255) / 256)), dim3(256), 0, stream, c, (uint64_t)lo,
                       (uint64_t)hi);
    return hipGetLastError();
}

hipError_t launch_qr_update(double* c, const double* e, size_t lo, size_t hi, double tau, double t,
                            hipStream_t stream) {
    if (hi <= lo) return hipSuccess;
    hipLaunchKernelGGL(k_qr_update, dim3((unsigned)((hi - lo + 255) / 256)), dim3(256), 0, stream, c, e,
                       (uint64_t)lo, (uint64_t)hi, tau, t);
    return hipGetLastError();
}

template <int H, int R>
void launch_fused_t(const DevProblem& p, const double T[2], uint32_t nh, const ScoreOut& out, const GenArgs& g,
                    hipStream_t stream) {
    const dim3 grid((nh + H - 1) / H), block(kSplitThreads);
    double band0, tan_tau1;
    band_consts(T, band0, tan_tau1);
    switch (p.solver) {
        case 0: hipLaunchKernelGGL((k_score_split<0, H, R, true>), grid, block, 0, stream, p, T[0], T[1], band0, tan_tau1, flag_band(T), nullptr, nullptr, nh, out, g); break;
        case 1: hipLaunchKernelGGL((k_score_split<1, H, R, true>), grid, block, 0, stream, p, T[0], T[1], band0, tan_tau1, flag_band(T), nullptr, nullptr, nh, out, g); break;
        default: hipLaunchKernelGGL((k_score_split<2, H, R, true>), grid, block, 0, stream, p, T[0], T[1], band0, tan_tau1, flag_band(T), nullptr, nullptr, nh, out, g); break;
    }
}

bool verify_chains(uint32_t nslots) { return split_h(nslots) == 16 && use_fm(); }

// GCR_PROBE: timing-probe bits of the batch scorers (GenArgs::probe)
uint32_t probe_bits() {
    static const uint32_t v = [] {
        const char* e = getenv("GCR_PROBE");
        return e ? (uint32_t)atoi(e) : 0u;
    }();
    return v;
}

hipError_t launch_verify_fused(const DevProblem& p, const double T[2], uint64_t seed, uint64_t slot0,
                               uint32_t nslots, const uint32_t m[2], uint8_t* inc, RectModel* models,
                               const ScoreOut& out, WgBest* wg, size_t wg_cap, BatchRecord* rec,
                               hipEvent_t ev0, hipEvent_t ev1, hipStream_t stream, const GenChain& chain) {
    if (nslots == 0) return hipErrorInvalidValue;
    const int h = split_h(nslots);
    if ((chain.pre_inc != nullptr || chain.next_inc != nullptr) && !verify_chains(nslots))
        return hipErrorInvalidValue;
    const uint32_t nwg = (nslots + h - 1) / h;
    if (nwg > wg_cap) return hipErrorInvalidValue;
    GenArgs g{seed, slot0, inc, models, wg, m[0], m[1]};
    // GCR_GEN_LANES pins the prologue's lanes per slot (sweeps); must be a
    // power of two dividing 1024 / H
    static const uint32_t glanes = [] {
        const char* e = getenv("GCR_GEN_LANES");
        return e ? (uint32_t)atoi(e) : 0u;
    }();
    g.probe = probe_bits();
    // default 16 lanes per slot (one wave per SIMD at H = 16): 16 parallel
    // attempts resolve nearly every slot in one round, and fewer contending
    // waves finish it sooner (sweep at 4096 slots: 64 -> 16 lanes, 142 ->
    // 134.5 us per fused launch)
    const uint32_t gl = glanes ? glanes : 16u;
    g.glanes = ((1024u / h) % gl == 0 && (gl & (gl - 1)) == 0) ? gl : 0u;
    g.chain = chain;
    if (ev0) (void)hipEventRecord(ev0, stream);
    if (h == 16 && use_fm()) launch_fm_t<16, true>(p, T, nslots, out, g, stream);
    else if (h == 64) launch_fused_t<64, 120>(p, T, nslots, out, g, stream);
    else if (h == 16) launch_fused_t<16, 420>(p, T, nslots, out, g, stream);
    else launch_fused_t<4, 960>(p, T, nslots, out, g, stream);
    if (ev1) (void)hipEventRecord(ev1, stream);
    if (rec != nullptr)
        hipLaunchKernelGGL(k_select_wg, dim3(1), dim3(kSelectThreads), 0, stream, wg, nwg, models, slot0, rec, 0u,
                           0u);
    return hipGetLastError();
}

hipError_t launch_select_batches(const WgBest* wg, size_t wg_stride, const RectModel* models, uint64_t slot0,
                                 uint32_t nslots, uint32_t count, BatchRecord* rec, hipStream_t stream) {
    if (count == 0) return hipSuccess;
    if (nslots == 0 || wg_stride < (size_t)(nslots + split_h(nslots) - 1) / split_h(nslots))
        return hipErrorInvalidValue;
    const uint32_t nwg = (nslots + split_h(nslots) - 1) / split_h(nslots);
    hipLaunchKernelGGL(k_select_wg, dim3(count), dim3(kSelectThreads), 0, stream, wg, nwg, models, slot0, rec,
                       (uint32_t)wg_stride, nslots);
    return hipGetLastError();
}


// k_lo_chain's fold: the block-parallel exact fold (default, round 4:
// M2 latency 0.865 -> 0.836 ms on one box, profiles/r4_s7_lat.log) or, with
// GCR_LO_FOLD=seq, one lane per chain (read per launch)
bool lo_fold_wide() {
    const char* e = getenv("GCR_LO_FOLD");
    return !(e && e[0] == 's');
}

// launch_score_small: the split scorer (k_lo_resid + k_lo_fold) when the
// problem has its scratch and the launch fits it; GCR_LO_SPLIT=0 keeps one
// k_lo_chain workgroup per model (read per launch)
bool lo_split() {
    const char* e = getenv("GCR_LO_SPLIT");
    return !(e && e[0] == '0');
}

// GCR_LO_ARGMODELS=0: the split scorer reads its models from `models` even
// when they fit the kernel arguments (read per launch)
bool lo_argmodels() {
    const char* e = getenv("GCR_LO_ARGMODELS");
    return !(e && e[0] == '0');
}

// GCR_LO_FUSED=1: the split scorer as ONE launch (k_lo_split) instead of
// k_lo_resid + k_lo_fold -- measured slower on MI355X (M2 LO trial scoring
// 0.16 -> 0.23 ms per call, gpurun_out session r5_s6: the fold's 138 KB of
// LDS makes every residual workgroup a whole-CU 1024-thread workgroup, and
// each one's arrival needs an L2 writeback), kept as an A/B (read per launch)
bool lo_fused() {
    const char* e = getenv("GCR_LO_FUSED");
    return e && e[0] == '1';
}
// GCR_LO_APPROX_FUSE=1: the approximate LO scores by k_lo_resid's last
// workgroups instead of a second launch (k_lo_approx) -- measured slower on
// MI355X (session r5_s24: the fused residual launch 30 us against 12 + 5;
// every wave drains its list-bit stores to host memory before its arrival),
// so off (read per call)
bool lo_approx_fuse() {
    const char* e = getenv("GCR_LO_APPROX_FUSE");
    return e && e[0] == '1';
}

// k_lo_split's chunks per wave: every workgroup takes a whole CU (the fold's
// LDS), so the launch is sized to about one workgroup per CU -- the fewest
// chunks per wave with nm x workgroups <= 256 (GCR_LO_CPW=n pins it)
uint32_t lo_cpw(uint32_t nm, uint32_t nchunks) {
    if (const char* e = getenv("GCR_LO_CPW")) {
        const long v = atol(e);
        if (v >= 1 && v <= 64) return (uint32_t)v;
    }
    const uint32_t wpw = kLoThreads / 64;
    for (uint32_t c = 1; c < 64; ++c) {
        const uint32_t nwg = (nchunks + wpw * c - 1) / (wpw * c);
        if ((size_t)nwg * nm <= 256) return c;
    }
    return 64;
}

size_t small_score_pairs(const DevProblem& p) {
    const uint32_t pad0 = (p.cls[0].n + 63u) & ~63u;
    const uint32_t pad1 = (p.solver == 2) ? ((p.cls[1].n + 63u) & ~63u) : 0u;
    return (size_t)pad0 + pad1;
}

hipError_t launch_score_small(const DevProblem& p, const double T[2], const void* models, const uint8_t* inc,
                              uint32_t nm, const ScoreOut& out, hipStream_t stream, const ListBits* lists,
                              const void* hmodels) {
    const ListBits lb = lists ? *lists : ListBits{{0.0, 0.0}, 0, 0.0, nullptr, nullptr};
    if (nm == 0) return hipSuccess;
    const uint32_t pad0 = (p.cls[0].n + 63u) & ~63u;
    const uint32_t ntot = (uint32_t)small_score_pairs(p);
    if (ntot == 0) return hipErrorInvalidValue;
    auto go = [&](auto ktag) {
        constexpr int KIND = decltype(ktag)::value;
        using M = typename ModelOf<KIND>::type;
        const M* mp = static_cast<const M*>(models);
        const uint32_t probe = probe_bits();               // GCR_PROBE bits 8 / 9: timing probes (results invalid)
        const uint32_t nchunks = ntot / 64;
        // the split pays where the per-pair arithmetic is heavy (the value
        // formulas); the correspondence estimators' residuals are cheap and
        // their one-kernel launch was faster (F latency A/B, round 4)
        if (KIND <= 2 && lo_split() && lo_fold_wide() && probe == 0 && ntot <= 2 * kLoBlock && nm <= p.lo.cap_models &&
            p.lo.vals != nullptr && p.lo.meta != nullptr) {
            const dim3 grid((nchunks + kLrThreads / 64 - 1) / (kLrThreads / 64), nm);
            ArgModels am;
            am.n = 0;
            if (KIND <= 2 && hmodels != nullptr && nm <= kArgModels && lo_argmodels()) {
                std::memcpy(am.m, hmodels, (size_t)nm * sizeof(RectModel));
                am.n = nm;
            }
            DevProblem q = p;
            q.lo.psum = nullptr;
            if (lo_fused() && p.lo.arrive != nullptr) {
                const uint32_t cpw = lo_cpw(nm, nchunks);
                const uint32_t per = (kLoThreads / 64) * cpw;
                const dim3 g2((nchunks + per - 1) / per, nm);
                hipLaunchKernelGGL((k_lo_split<KIND>), g2, dim3(kLoThreads), 0, stream, q, mp, inc, T[0], T[1], pad0,
                                   nchunks, cpw, lb, flag_band(T), flag_band(lb.T), am, out);
            } else {
                hipLaunchKernelGGL((k_lo_resid<KIND>), grid, dim3(kLrThreads), 0, stream, q, mp, inc, T[0], T[1],
                                   pad0, nchunks, lb, flag_band(T), flag_band(lb.T), am, 0u, out);
                hipLaunchKernelGGL((k_lo_fold<KIND>), dim3(nm), dim3(kLoThreads), 0, stream, q, pad0, nchunks, out,
                                   0u, 0u);
            }
        } else if (lo_fold_wide())
            hipLaunchKernelGGL((k_lo_chain<KIND, true>), dim3(nm), dim3(kLoThreads), 0, stream, p, mp, inc, T[0], T[1],
                               pad0, ntot, lb, flag_band(T), flag_band(lb.T), out, probe);
        else
            hipLaunchKernelGGL((k_lo_chain<KIND, false>), dim3(nm), dim3(kLoThreads), 0, stream, p, mp, inc, T[0],
                               T[1], pad0, ntot, lb, flag_band(T), flag_band(lb.T), out, probe);
    };
    switch (p.solver) {
        case 0: go(std::integral_constant<int, 0>{}); break;
        case 1: go(std::integral_constant<int, 1>{}); break;
        case 2: go(std::integral_constant<int, 2>{}); break;
        case 3: go(std::integral_constant<int, 3>{}); break;
        default: go(std::integral_constant<int, 4>{}); break;
    }
    return hipGetLastError();
}

bool score_small_splits(const DevProblem& p, uint32_t nm_total) {
    const uint32_t ntot = (uint32_t)small_score_pairs(p);
    return p.solver <= 2 && lo_split() && lo_fold_wide() && !lo_fused() && probe_bits() == 0 && ntot > 0 &&
           ntot <= 2 * kLoBlock && nm_total <= p.lo.cap_models && p.lo.vals != nullptr && p.lo.meta != nullptr;
}

hipError_t launch_score_small_part(const DevProblem& p, const double T[2], const void* models, uint32_t mi_base,
                                   uint32_t nm, int stage, uint32_t nm_fold, const ScoreOut& out, hipStream_t stream,
                                   const ListBits* lists, const void* hmodels) {
    if (!score_small_splits(p, std::max(mi_base + nm, nm_fold))) return hipErrorInvalidValue;
    const ListBits lb = lists ? *lists : ListBits{{0.0, 0.0}, 0, 0.0, nullptr, nullptr};
    const uint32_t pad0 = (p.cls[0].n + 63u) & ~63u;
    const uint32_t nchunks = (uint32_t)small_score_pairs(p) / 64;
    if ((stage & 4) && (stage & 2)) return hipErrorInvalidValue;
    if ((stage & 4) && p.lo.psum == nullptr) return hipErrorInvalidValue;
    DevProblem q = p;
    if (!(stage & 4)) q.lo.psum = nullptr;                   // chunk partial sums only for k_lo_approx
    auto go = [&](auto ktag) {
        constexpr int KIND = decltype(ktag)::value;
        using M = typename ModelOf<KIND>::type;
        if ((stage & 1) && nm > 0) {
            const dim3 grid((nchunks + kLrThreads / 64 - 1) / (kLrThreads / 64), nm);
            ArgModels am;
            am.n = 0;
            if (hmodels != nullptr && nm <= kArgModels && lo_argmodels()) {
                std::memcpy(am.m, hmodels, (size_t)nm * sizeof(RectModel));
                am.n = nm;
            }
            // stage 4 with the whole batch in this launch: the approximate
            // scores by its last workgroups (GCR_LO_APPROX_FUSE=0: k_lo_approx)
            if ((stage & 4) && mi_base == 0 && nm == nm_fold && p.lo.arrive != nullptr && lo_approx_fuse()) {
                hipLaunchKernelGGL((k_lo_resid<KIND, true>), grid, dim3(kLrThreads), 0, stream, q,
                                   static_cast<const M*>(models), nullptr, T[0], T[1], pad0, nchunks, lb, flag_band(T),
                                   flag_band(lb.T), am, mi_base, out);
                stage &= ~4;
            } else {
                hipLaunchKernelGGL((k_lo_resid<KIND>), grid, dim3(kLrThreads), 0, stream, q,
                                   static_cast<const M*>(models), nullptr, T[0], T[1], pad0, nchunks, lb, flag_band(T),
                                   flag_band(lb.T), am, mi_base, out);
            }
        }
        if ((stage & 2) && nm_fold > 0)
            hipLaunchKernelGGL((k_lo_fold<KIND>), dim3(nm_fold), dim3(kLoThreads), 0, stream, q, pad0, nchunks, out,
                               0u, 0u);
        if ((stage & 4) && nm_fold > 0)
            hipLaunchKernelGGL((k_lo_approx<KIND>), dim3(nm_fold), dim3(kLaThreads), 0, stream, q, pad0, nchunks,
                               out);
    };
    switch (p.solver) {
        case 0: go(std::integral_constant<int, 0>{}); break;
        case 1: go(std::integral_constant<int, 1>{}); break;
        default: go(std::integral_constant<int, 2>{}); break;
    }
    return hipGetLastError();
}

hipError_t launch_lo_fold_slots(const DevProblem& p, uint32_t src, uint32_t nm, uint32_t slot, const ScoreOut& out,
                                hipStream_t stream) {
    if (nm == 0) return hipSuccess;
    if (!score_small_splits(p, src + nm)) return hipErrorInvalidValue;
    DevProblem q = p;
    q.lo.psum = nullptr;
    const uint32_t pad0 = (p.cls[0].n + 63u) & ~63u;
    const uint32_t nchunks = (uint32_t)small_score_pairs(p) / 64;
    switch (p.solver) {
        case 0: hipLaunchKernelGGL((k_lo_fold<0>), dim3(nm), dim3(kLoThreads), 0, stream, q, pad0, nchunks, out, src, slot); break;
        case 1: hipLaunchKernelGGL((k_lo_fold<1>), dim3(nm), dim3(kLoThreads), 0, stream, q, pad0, nchunks, out, src, slot); break;
        default: hipLaunchKernelGGL((k_lo_fold<2>), dim3(nm), dim3(kLoThreads), 0, stream, q, pad0, nchunks, out, src, slot); break;
    }
    return hipGetLastError();
}

hipError_t launch_mask(const DevProblem& p, int cls, const RectModel& model, int rule, double T, double lambda,
                       uint8_t* mask, hipStream_t stream) {
    const DevClass& c = p.cls[cls];
    if (c.n == 0) return hipSuccess;
    const dim3 grid(blocks_for(c.n, kMaskBlock)), block(kMaskBlock);
    double fmid, fhalf;
    flag_band_1(T, cls, fmid, fhalf);
    switch (p.solver) {
        case 0: hipLaunchKernelGGL(k_mask<0>, grid, block, 0, stream, c, cls, model, rule, T, lambda, fmid, fhalf, mask); break;
        case 1: hipLaunchKernelGGL(k_mask<1>, grid, block, 0, stream, c, cls, model, rule, T, lambda, fmid, fhalf, mask); break;
        default: hipLaunchKernelGGL(k_mask<2>, grid, block, 0, stream, c, cls, model, rule, T, lambda, fmid, fhalf, mask); break;
    }
    return hipGetLastError();
}

// op 7 of gcr_debug_math: out[0] = fold_exact_block over a[0, n) from +0.0
// (one kLoThreads workgroup), out[1] = the same sum by one lane's sequential
// loop.  For n <= kLoBlock both run over an LDS copy (as in k_lo_chain) and
// out[2..5] = cycles of the block fold, cycles of the one-lane fold, the
// number of special values, whether any fallback occurred (n >= 6).
__global__ __launch_bounds__(kLoThreads) void k_fold_test(const double* __restrict__ a, uint32_t n, double* out) {
    __shared__ double buf[kLoBlock];
    __shared__ BlkFoldScratch bsc;
    const int t = threadIdx.x;
    const bool lds = n <= kLoBlock;
    if (lds)
        for (uint32_t i = t; i < n; i += kLoThreads) buf[i] = a[i];
    __syncthreads();
    const double* v = lds ? buf : a;
    const uint64_t t0 = __builtin_readcyclecounter();
    const double w = fold_exact_block(v, 0, n, 0.0, bsc, lds ? kLoBlock : n);
    const uint64_t t1 = __builtin_readcyclecounter();
    double s = 0.0;
    if (t == 0) {
        if (lds) s = fold_seq_lane(buf, 0, n, 0.0);
        else
            for (uint32_t k = 0; k < n; ++k) s = s + v[k];
    }
    const uint64_t t2 = __builtin_readcyclecounter();
    if (t == 0) {
        out[0] = w;
        out[1] = s;
        if (lds && n >= 6) {                  // out holds n doubles
            out[2] = (double)(t1 - t0);
            out[3] = (double)(t2 - t1);
            out[4] = (double)bsc.nspec;
            out[5] = (double)bsc.bad;
        }
    }
}

// op 12 of gcr_debug_math: the three chains of k_lo_chain's KIND-2 fold over
// an LDS copy of a[0, n), split at h = b[0]: out[0] = a[0, h) from +0,
// out[1] = a[h, n) from +0, out[2] = a[h, n) from out[0] (fold_exact_chains);
// out[3..5] = the same sums by one lane's sequential loop, out[6] = cycles of
// the chains (n >= 7); out[8..15] = cycle stamps: after the fold's four
// barriers, then wave 0's walks (chain 0 done, chain 2's head, chain 2 done)
// (n >= 16).
__global__ __launch_bounds__(kLoThreads) void k_fold3_test(const double* __restrict__ a, uint32_t n,
                                                          const double* __restrict__ hb, double* out) {
    __shared__ double buf[kLoBlock];
    __shared__ BlkFoldScratch bsc[3];
    const int t = threadIdx.x;
    const double hd = hb[0];
    const uint32_t h = hd >= 0.0 && hd <= (double)n ? (uint32_t)hd : 0u;
    for (uint32_t i = t; i < n; i += kLoThreads) buf[i] = a[i];
    __syncthreads();
    const BlkChain ch[3] = {{0u, h, 0.0, -1}, {h, n, 0.0, -1}, {h, n, 0.0, 0}};
    double r[3];
    const uint64_t t0 = __builtin_readcyclecounter();
    fold_exact_chains<3>(buf, ch, bsc, kLoBlock, r, n >= 18 ? out + 8 : nullptr);
    const uint64_t t1 = __builtin_readcyclecounter();
    if (t == 0) {
        double s0 = 0.0, s1 = 0.0;
        for (uint32_t k = 0; k < h; ++k) s0 = s0 + buf[k];
        for (uint32_t k = h; k < n; ++k) s1 = s1 + buf[k];
        double s2 = s0;
        for (uint32_t k = h; k < n; ++k) s2 = s2 + buf[k];
        out[0] = r[0];
        out[1] = r[1];
        out[2] = r[2];
        out[3] = s0;
        out[4] = s1;
        out[5] = s2;
        out[6] = (double)(t1 - t0);
    }
}

hipError_t launch_math(int op, const double* a, const double* b, size_t n, double* out, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (op == 12) {
        if (n < 7 || n > kLoBlock) return hipErrorInvalidValue;
        hipLaunchKernelGGL(k_fold3_test, dim3(1), dim3(kLoThreads), 0, stream, a, (uint32_t)n, b, out);
        return hipGetLastError();
    }
    if (op == 7) {
        if (n < 2 || n > 0xffffffffull) return hipErrorInvalidValue;
        hipLaunchKernelGGL(k_fold_test, dim3(1), dim3(kLoThreads), 0, stream, a, (uint32_t)n, out);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_math, dim3(blocks_for(n, 256)), dim3(256), 0, stream, op, a, b, n, out);
    return hipGetLastError();
}

// ------------------------------------ homography (3) / fundamental (4) ----
hipError_t launch_generate_geo(const DevProblem& p, uint64_t seed, uint64_t slot0, uint32_t nslots, uint8_t* inc,
                               GeoModel* models, hipStream_t stream) {
    if (nslots == 0) return hipSuccess;
    // GCR_GEN_WIDEN=0: the fundamental-matrix generator keeps fixed groups of
    // G lanes per slot (k_generate_f) instead of widening them (k_generate_fw).
    // Both knobs are read per launch (tests switch them in-process).
    const char* ew = getenv("GCR_GEN_WIDEN");
    const bool widen = !(ew && ew[0] == '0');
    // GCR_GEN_HWIDEN=1: the homography generator widens its groups too (A/B)
    const char* eh = getenv("GCR_GEN_HWIDEN");
    const bool hwiden = eh && eh[0] == '1';
    auto go = [&](auto gtag) {
        constexpr int G = decltype(gtag)::value;
        const dim3 grid(blocks_for((size_t)nslots * G, kGenBlock)), block(kGenBlock);
        if (p.solver == 4) {
            if (widen)
                hipLaunchKernelGGL((k_generate_fw<4, G>), grid, block, 0, stream, p, seed, slot0, nslots, inc, models);
            else
                hipLaunchKernelGGL((k_generate_f<G>), grid, block, 0, stream, p, seed, slot0, nslots, inc, models);
        } else if (hwiden) {
            hipLaunchKernelGGL((k_generate_fw<3, G>), grid, block, 0, stream, p, seed, slot0, nslots, inc, models);
        } else {
            hipLaunchKernelGGL((k_generate<3, G>), grid, block, 0, stream, p, seed, slot0, nslots, inc, models);
        }
    };
    // GCR_GEN_G overrides the lanes per slot (1 .. 64)
    const char* eg = getenv("GCR_GEN_G");
    const int env_g = eg ? atoi(eg) : 0;
    // 7-point solver: ~7.7 attempts per slot at 80 % outliers (p99 35), latency-
    // bound per attempt.  Fixed groups (round 1): G = 8 / 16 / 32 / 64 -> 0.46 /
    // 0.37 / 0.34 / 0.36 ms per 4096-slot step.  Widening groups (F bench line,
    // 3712 slots, two-stream pipeline, profiles/r2_v8_fwiden.txt): G = 4 / 8 /
    // 16 / 32 / 64 -> 0.173 / 0.143 / 0.126 / 0.139 / 0.159 ms per step, fixed
    // G = 32 0.138 ms.  The replay path's large chunks (F wall time to 0.99,
    // every launch forced, profiles/r2_v13_bconc.txt): G = 2 / 4 / 8 / 16 ->
    // 8.08 / 7.77 / 7.38 / 7.43 ms
    int g = p.solver == 4 ? (nslots <= 8192 ? 16 : 8)
                          : (nslots <= 8192 ? 16 : nslots <= 32768 ? 4 : 1);
    if (env_g == 1 || env_g == 2 || env_g == 4 || env_g == 8 || env_g == 16 || env_g == 32 || env_g == 64) g = env_g;
    switch (g) {
        case 64: go(std::integral_constant<int, 64>{}); break;
        case 32: go(std::integral_constant<int, 32>{}); break;
        case 16: go(std::integral_constant<int, 16>{}); break;
        case 8: go(std::integral_constant<int, 8>{}); break;
        case 4: go(std::integral_constant<int, 4>{}); break;
        case 2: go(std::integral_constant<int, 2>{}); break;
        default: go(std::integral_constant<int, 1>{}); break;
    }
    return hipGetLastError();
}

hipError_t launch_score_geo(const DevProblem& p, double T, const GeoModel* models, const uint8_t* inc, uint32_t nh,
                            const ScoreOut& out, hipStream_t stream, const uint32_t* hmap, const uint32_t* hcount,
                            bool compact) {
    if (nh == 0) return hipSuccess;
    GenArgs ga{};
    ga.hmap = hmap;
    ga.hcount = hcount;
    ga.probe = probe_bits();
    // the feature-major scorer also for launches of >= 16384 hypotheses (the
    // replay's large chunks), instead of k_score_split<KIND, 64, 120>;
    // GCR_GEO_FM_LARGE=0 (read per launch) restores the split scorer there
    const char* el = getenv("GCR_GEO_FM_LARGE");
    const bool fm_large = !(el && el[0] == '0');
    const int sh = split_h(nh);
    const bool fm = use_fm() && (sh == 16 || (sh == 64 && fm_large));
    if (compact) {
        if (hmap == nullptr || hcount == nullptr) return hipErrorInvalidValue;
        if (fm && sh == 16) {
            ga.scan = true;                     // the feature-major scorer compacts in its prologue
        } else {
            const hipError_t e = launch_compact(inc, nh, const_cast<uint32_t*>(hmap), const_cast<uint32_t*>(hcount),
                                                stream);
            if (e != hipSuccess) return e;
        }
    }
    auto go = [&](auto ktag, auto htag, auto rtag) {
        constexpr int KIND = decltype(ktag)::value, H = decltype(htag)::value, R = decltype(rtag)::value;
        const double sb = sqrt(T) * (1.0 + 1e-7) + 1e-7;     // h_band slack
        hipLaunchKernelGGL((k_score_split<KIND, H, R, false>), dim3((nh + H - 1) / H), dim3(kSplitThreads), 0,
                           stream, p, T, 0.0, sb * sb, 0.0, FlagBand{}, models, inc, nh, out, ga);
    };
    auto by_h = [&](auto ktag) {
        const int h = split_h(nh);
        if (h == 64) go(ktag, std::integral_constant<int, 64>{}, std::integral_constant<int, 120>{});
        else if (h == 16) go(ktag, std::integral_constant<int, 16>{}, std::integral_constant<int, 420>{});
        else go(ktag, std::integral_constant<int, 4>{}, std::integral_constant<int, 960>{});
    };
    if (fm) {
        // the feature-major scorer with the division-free band prefilter:
        // h_band (transfer error) or f_band (Sampson distance)
        constexpr size_t dyn = fm_dyn_lds_bytes<16, false>();
        static const bool attr = [] {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_score_fm<3, 16, false>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_score_fm<4, 16, false>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
            return true;
        }();
        (void)attr;
        if (p.solver == 4) {
            hipLaunchKernelGGL((k_score_fm<4, 16, false>), dim3((nh + 15) / 16), dim3(kSplitThreads), dyn, stream, p,
                               T, 0.0, T * (1.0 + 1e-9), 0.0, FlagBand{}, models, inc, nh, out, ga);
        } else {
            const double sb = sqrt(T) * (1.0 + 1e-7) + 1e-7;
            hipLaunchKernelGGL((k_score_fm<3, 16, false>), dim3((nh + 15) / 16), dim3(kSplitThreads), dyn, stream, p,
                               T, 0.0, sb * sb, 0.0, FlagBand{}, models, inc, nh, out, ga);
        }
    } else if (p.solver == 4) {
        by_h(std::integral_constant<int, 4>{});
    } else {
        by_h(std::integral_constant<int, 3>{});
    }
    return hipGetLastError();
}

hipError_t launch_mask_geo(const DevProblem& p, const GeoModel& model, int rule, double T, double lambda,
                           uint8_t* mask, hipStream_t stream) {
    const DevClass& c = p.cls[0];
    if (c.n == 0) return hipSuccess;
    const dim3 grid(blocks_for(c.n, kMaskBlock)), block(kMaskBlock);
    if (p.solver == 4)
        hipLaunchKernelGGL(k_mask<4>, grid, block, 0, stream, c, 0, model, rule, T, lambda, 0.0, -1.0, mask);
    else
        hipLaunchKernelGGL(k_mask<3>, grid, block, 0, stream, c, 0, model, rule, T, lambda, 0.0, -1.0, mask);
    return hipGetLastError();
}

// squared residuals of one model against every correspondence (graph-cut
// labeling with pairwise terms, GCRANSAC.h:789-811)
template <int KIND>
__global__ __launch_bounds__(kMaskBlock) void k_sqres(DevClass c, GeoModel m, double* __restrict__ r2) {
    const uint32_t i = blockIdx.x * kMaskBlock + threadIdx.x;
    if (i >= c.n) return;
    r2[i] = geo_sq_residual<KIND>(c.x[i], c.y[i], c.a[i], c.c0[i], m.h);
}

hipError_t launch_sqres_geo(const DevProblem& p, const GeoModel& model, double* r2, hipStream_t stream) {
    const DevClass& c = p.cls[0];
    if (c.n == 0) return hipSuccess;
    const dim3 grid(blocks_for(c.n, kMaskBlock)), block(kMaskBlock);
    if (p.solver == 4) hipLaunchKernelGGL(k_sqres<4>, grid, block, 0, stream, c, model, r2);
    else hipLaunchKernelGGL(k_sqres<3>, grid, block, 0, stream, c, model, r2);
    return hipGetLastError();
}

hipError_t launch_select_geo(int solver, const ScoreOut& sc, const uint8_t* inc, uint32_t nh, uint64_t slot0,
                             uint32_t m, double Tm, BatchRecord* out, hipStream_t stream, const uint32_t* hmap,
                             const uint32_t* hcount) {
    hipLaunchKernelGGL(k_select<GeoModel>, dim3(1), dim3(kSelectThreads), 0, stream, solver, sc, inc,
                       (const GeoModel*)nullptr, nh, slot0, m, 0u, Tm, 0.0, out, solver == 4 ? kFModels : 1u, hmap,
                       hcount);
    return hipGetLastError();
}

hipError_t launch_select_geo_batches(int solver, const ScoreOut& sc, const uint8_t* inc, uint32_t nh, uint32_t stride,
                                     uint64_t slot0, uint32_t m, double Tm, uint32_t count, BatchRecord* out,
                                     hipStream_t stream, const uint32_t* hmap, const uint32_t* hcount) {
    if (count == 0) return hipSuccess;
    if (stride < nh || stride == 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_select<GeoModel>, dim3(count), dim3(kSelectThreads), 0, stream, solver, sc, inc,
                       (const GeoModel*)nullptr, nh, slot0, m, 0u, Tm, 0.0, out, solver == 4 ? kFModels : 1u, hmap,
                       hcount, stride);
    return hipGetLastError();
}

hipError_t launch_compact(const uint8_t* inc, uint32_t n, uint32_t* map, uint32_t* count, hipStream_t stream) {
    hipLaunchKernelGGL(k_compact, dim3(1), dim3(kCompactThreads), 0, stream, inc, n, map, count);
    return hipGetLastError();
}

}  // namespace gcr

#ifdef GCR_STAMPS
extern "C" int gcr_debug_stamps(uint64_t* host, size_t bytes) {
    const size_t n = bytes < sizeof(gcr::g_stamps) ? bytes : sizeof(gcr::g_stamps);
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(gcr::g_stamps), n, 0, hipMemcpyDeviceToHost) == hipSuccess ? (int)n : -1;
}
extern "C" int gcr_debug_wgspans(uint64_t* host, size_t bytes) {
    const size_t n = bytes < sizeof(gcr::g_wgspan) ? bytes : sizeof(gcr::g_wgspan);
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(gcr::g_wgspan), n, 0, hipMemcpyDeviceToHost) == hipSuccess ? (int)n : -1;
}
#endif

namespace gcr {

// --------------------------------------------------------- HBM peak probe ----
// Streaming copy used by bench.py to measure the box's achievable HBM
// bandwidth (the roofline's measured peak beside the 8 TB/s spec).  One 16-byte
// load and store per lane and one 4 KB tile per workgroup, a grid of n / 256
// workgroups (no grid-stride loop): the hardware keeps every CU's queue full.
// Measured on MI355X (tools/micro/hbm_copy.hip, 2 GiB, read + write bytes):
// this shape 6.24 TB/s; grid-stride loops with 2-8 strips in flight per lane
// 4.6-5.5 TB/s; tiles of 2-8 strips per lane 5.4-5.9 TB/s.  NT = nontemporal
// hints (the probe reports the better of the two).
typedef double hbm_v2d __attribute__((ext_vector_type(2)));
template <bool NT>
__global__ __launch_bounds__(256) void k_hbm_copy(const hbm_v2d* __restrict__ src, hbm_v2d* __restrict__ dst,
                                                  size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    if (NT) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
    else dst[i] = src[i];
}

hipError_t launch_hbm_copy(const void* src, void* dst, size_t bytes, int nontemporal, hipStream_t stream) {
    const size_t n = bytes / sizeof(hbm_v2d);
    if (n == 0) return hipSuccess;
    if ((n + 255) / 256 > 0x7fffffffull) return hipErrorInvalidValue;
    const dim3 grid((unsigned)((n + 255) / 256)), block(256);
    if (nontemporal)
        hipLaunchKernelGGL(k_hbm_copy<true>, grid, block, 0, stream, static_cast<const hbm_v2d*>(src),
                           static_cast<hbm_v2d*>(dst), n);
    else
        hipLaunchKernelGGL(k_hbm_copy<false>, grid, block, 0, stream, static_cast<const hbm_v2d*>(src),
                           static_cast<hbm_v2d*>(dst), n);
    return hipGetLastError();
}

// ------------------------------------------------------ perspective warp ----
// examples/utils.py:92-123 (perspective_warp -> cv2.warpPerspective, INTER_LINEAR):
// every output pixel (x, y) samples the source at M (x, y, 1)^T / w, M the
// dst -> src map, with bilinear weights over the 4 neighbours; neighbours
// outside the source take the border (constant value, or the nearest edge
// pixel for `replicate`).  One lane per output pixel and channel loop inside:
// consecutive lanes read neighbouring source pixels, so the gathers coalesce
// along rows; the output row is written contiguously.
template <typename T>
__device__ __forceinline__ float warp_texel(const T* __restrict__ src, int h, int w, int ch, int x, int y, int c,
                                            int border_mode, float bval) {
    if (x < 0 || y < 0 || x >= w || y >= h) {
        if (border_mode == 0) return bval;
        x = x < 0 ? 0 : (x >= w ? w - 1 : x);
        y = y < 0 ? 0 : (y >= h ? h - 1 : y);
    }
    return (float)src[((size_t)y * w + x) * ch + c];
}

template <typename T>
__global__ __launch_bounds__(256) void k_warp(const T* __restrict__ src, int sh, int sw, int ch,
                                              WarpMap M, T* __restrict__ dst, int dh, int dw, int border_mode) {
    const int x = blockIdx.x * 256 + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= dw || y >= dh) return;
    const double X = (double)x, Y = (double)y;
    const double wz = M.m[6] * X + M.m[7] * Y + M.m[8];
    const double iw = wz != 0.0 ? 1.0 / wz : 0.0;
    const double sx = (M.m[0] * X + M.m[1] * Y + M.m[2]) * iw;
    const double sy = (M.m[3] * X + M.m[4] * Y + M.m[5]) * iw;
    T* out = dst + ((size_t)y * dw + x) * ch;
    // far outside (or a point at infinity): the border alone
    if (!(fabs(sx) < 1e9 && fabs(sy) < 1e9)) {
        for (int c = 0; c < ch; ++c) {
            const float v = border_mode == 0 ? M.border[c] : 0.f;
            out[c] = (T)v;
        }
        return;
    }
    const double fx0 = floor(sx), fy0 = floor(sy);
    const int x0 = (int)fx0, y0 = (int)fy0;
    const float ax = (float)(sx - fx0), ay = (float)(sy - fy0);
    for (int c = 0; c < ch; ++c) {
        const float b = M.border[c];
        const float p00 = warp_texel(src, sh, sw, ch, x0, y0, c, border_mode, b);
        const float p01 = warp_texel(src, sh, sw, ch, x0 + 1, y0, c, border_mode, b);
        const float p10 = warp_texel(src, sh, sw, ch, x0, y0 + 1, c, border_mode, b);
        const float p11 = warp_texel(src, sh, sw, ch, x0 + 1, y0 + 1, c, border_mode, b);
        const float top = p00 + ax * (p01 - p00);
        const float bot = p10 + ax * (p11 - p10);
        float v = top + ay * (bot - top);
        if constexpr (sizeof(T) == 1) {
            v = rintf(v);
            v = v < 0.f ? 0.f : (v > 255.f ? 255.f : v);
        }
        out[c] = (T)v;
    }
}

hipError_t launch_warp(const void* src, int sh, int sw, int ch, int dtype, const WarpMap& M, void* dst, int dh,
                       int dw, int border_mode, hipStream_t stream) {
    if (dh <= 0 || dw <= 0) return hipSuccess;
    const dim3 grid((unsigned)((dw + 255) / 256), (unsigned)dh), block(256);
    if (dtype == 0)
        hipLaunchKernelGGL(k_warp<uint8_t>, grid, block, 0, stream, static_cast<const uint8_t*>(src), sh, sw, ch, M,
                           static_cast<uint8_t*>(dst), dh, dw, border_mode);
    else
        hipLaunchKernelGGL(k_warp<float>, grid, block, 0, stream, static_cast<const float*>(src), sh, sw, ch, M,
                           static_cast<float*>(dst), dh, dw, border_mode);
    return hipGetLastError();
}

}  // namespace gcr
