// kernels.hip -- gfx950 kernels of the hypothesize-and-verify hot path.
//
//   k_generate   one lane per outer-iteration slot: up to 101 attempts of
//                Philox sample -> sample validity -> 3x4 Gauss minimal solve,
//                all in fp64 registers (GCRANSAC.h:296-339, solvers' minimal fits)
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

#include <cmath>
#include <cstdlib>

namespace gcr {

namespace {

constexpr int kGenBlock = 256;
constexpr int kScoreBlock = 256;
constexpr int kMaskBlock = 256;

// ------------------------------------------------------------- generate ----
template <int KIND>
__global__ __launch_bounds__(kGenBlock) void k_generate(DevProblem p, uint64_t seed, uint64_t slot0,
                                                        uint32_t nslots, uint8_t* __restrict__ inc,
                                                        RectModel* __restrict__ models) {
    const uint32_t s = blockIdx.x * kGenBlock + threadIdx.x;
    if (s >= nslots) return;
    const uint64_t slot = slot0 + s;
    RectModel m = default_model();
    for (uint32_t a = 0; a < 101; ++a) {
        if constexpr (KIND != 2) {
            const DevClass& c = p.cls[0];
            uint32_t idx[3];
            WordStream ws(seed, slot, a, kStreamMain, 0);
            if (!sample_distinct<3>(ws, c.n, 3, idx)) continue;
            double x[3], y[3], pw[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                x[j] = c.x[idx[j]];
                y[j] = c.y[idx[j]];
                pw[j] = c.c0[idx[j]];
            }
            // areAllPointsCollinear on the single consecutive triplet
            if (are_collinear(x[0], y[0], x[1], y[1], x[2], y[2], 1.0)) continue;
            const bool ok = (KIND == 1) ? solve_scale3<true>(x, y, pw, m) : solve_scale3<false>(x, y, pw, m);
            if (ok) {
                models[s] = m;
                inc[s] = (uint8_t)(a + 1);
                return;
            }
        } else {
            const DevClass& sc = p.cls[0];
            const DevClass& oc = p.cls[1];
            uint32_t si[2], oi[2];
            WordStream ws0(seed, slot, a, kStreamMain, 0);
            if (!sample_distinct<2>(ws0, sc.n, 2, si)) continue;
            WordStream ws1(seed, slot, a, kStreamMain, 1);
            if (!sample_distinct<2>(ws1, oc.n, 2, oi)) continue;
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
            if (!valid_sample_sift22(sx, sy, ox, oy, oco, osi)) continue;
            if (solve_sift22(sx, sy, sp, ox, oy, oco, osi, m)) {
                models[s] = m;
                inc[s] = (uint8_t)(a + 1);
                return;
            }
        }
    }
    models[s] = default_model();
    inc[s] = 102;
}

// ---------------------------------------------------------------- score ----
template <int KIND, bool kIdentity>
__global__ __launch_bounds__(kScoreBlock) void k_score(DevProblem p, double T0, double T1,
                                                       const RectModel* __restrict__ models,
                                                       const uint8_t* __restrict__ inc, uint32_t nh, ScoreOut out) {
    const uint32_t h = blockIdx.x * kScoreBlock + threadIdx.x;
    if (h >= nh) return;
    if (inc != nullptr && inc[h] > 101) {
        out.n0[h] = 0; out.n1[h] = 0; out.v0[h] = 0.0; out.v1[h] = 0.0; out.tot[h] = 0.0;
        return;
    }
    const RectModel m = models[h];
    const DevClass c0 = p.cls[0];
    const double ac = alpha_cube(m);
    uint32_t cnt0 = 0;
    double acc0 = 0.0;
    for (uint32_t i = 0; i < c0.n; ++i) {
        const double r2 = scale_sq_residual<KIND == 1, kIdentity>(c0.x[i], c0.y[i], c0.a[i], m, ac);
        if (r2 <= T0) {
            cnt0 += 1;
            acc0 += -r2;
        }
    }
    uint32_t cnt1 = 0;
    double acc1 = 0.0, tot = acc0;
    if constexpr (KIND == 2) {
        const DevClass c1 = p.cls[1];
        const OrientConst oc = orient_const(m);
        for (uint32_t i = 0; i < c1.n; ++i) {
            const double r2 = orient_sq_residual<kIdentity>(c1.x[i], c1.y[i], c1.c0[i], c1.c1[i], m, oc);
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

struct HypConst {       // per-hypothesis constants of the exact and band tests
    double h7, h8, ac;  // scale: model, alpha^3
    double lo, hi;      // scale band on s / t^3 (ac-adjusted)
    double cphi, cphi2; // orientation: clipped phi, clip(clip(phi + pi/2))
    double cf, sf;      // orientation: cos(phi), sin(phi) (band test only)
};

template <int KIND>
__device__ __forceinline__ bool scale_band(double x, double y, double s, const HypConst& q) {
    const double t = (-q.h7 * x - q.h8 * y) + 1.0;
    if (!(t > 0.0 && s > 0.0)) return true;               // sign / NaN: exact path decides
    const double t3 = (t * t) * t;
    return !(s < q.lo * t3 || s > q.hi * t3);
}

__device__ __forceinline__ bool orient_band(double x, double y, double ct, double st, const HypConst& q,
                                            double tan_tau) {
    const double numer = (-x * st + y * ct) * q.h7 + st;
    const double denom = (x * st - y * ct) * q.h8 + ct;
    const double u = __builtin_fabs(denom * q.cf + numer * q.sf);
    const double v = __builtin_fabs(numer * q.cf - denom * q.sf);
    return !(__builtin_fmin(u, v) > tan_tau * __builtin_fmax(u, v));
}

template <int KIND, int H, int R>
__global__ __launch_bounds__(kSplitThreads) void k_score_split(DevProblem p, double T0, double T1, double band0,
                                                               double tan_tau1, const RectModel* __restrict__ models,
                                                               const uint8_t* __restrict__ inc, uint32_t nh,
                                                               ScoreOut out) {
    static_assert((H * R) % kComputeThreads == 0 && kComputeThreads % H == 0, "tile shape");
    static_assert(H * R <= 65536, "queue entries are 16-bit tile indices");
    constexpr int kPer = H * R / kComputeThreads;    // pairs per compute thread per round
    constexpr int kStride = kComputeThreads / H;     // feature stride between a thread's pairs
    __shared__ double tile[2][H * R];                // -r^2 / +0.0 per (feature, hypothesis)
    __shared__ double fbuf[2][4][R];                 // staged features of a round: x, y, s|cos, sin
    __shared__ uint16_t queue[kComputeWaves][kPer * 64];
    __shared__ HypConst hyp[H];
    __shared__ uint32_t cnt_sh[2][H];

    const int t = threadIdx.x;
    const int wave = t >> 6;
    const int lane = t & 63;
    const bool chain_wave = t >= kComputeThreads;
    const int h = chain_wave ? (t - kComputeThreads) : (t % H);
    const int fsub = t / H;
    const uint32_t hg = blockIdx.x * H + h;
    const bool valid_h = h < H && hg < nh && (inc == nullptr || inc[hg] <= 101);
    const bool live = !chain_wave && valid_h;

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
                } else {
                    fbuf[buf][2][e] = c.c0[i];
                    fbuf[buf][3][e] = c.c1[i];
                }
            }
        }
    };

    if (t < H) {
        const bool v = hg < nh && (inc == nullptr || inc[hg] <= 101);
        const RectModel m = v ? models[hg] : default_model();
        HypConst q;
        q.h7 = m.h7;
        q.h8 = m.h8;
        q.ac = alpha_cube(m);
        // s / t^3 must lie in [exp(-tau), exp(tau)] / ac (new) or * ac (original)
        q.lo = (KIND == 1 ? q.ac : 1.0 / q.ac) * (1.0 / band0) * (1.0 - 1e-9);
        q.hi = (KIND == 1 ? q.ac : 1.0 / q.ac) * band0 * (1.0 + 1e-9);
        q.cphi = 0.0; q.cphi2 = 0.0; q.cf = 1.0; q.sf = 0.0;
        if constexpr (KIND == 2) {
            const OrientConst oc = orient_const(m);
            q.cphi = oc.cphi;
            q.cphi2 = oc.cphi2;
            sincos(m.phi, &q.sf, &q.cf);
        }
        hyp[h] = q;
    }
    if (t < 2 * H) cnt_sh[t / H][t % H] = 0;
    stage(0, 0, t, kSplitThreads);
    __syncthreads();

    double acc0 = 0.0, acc1 = 0.0, tot = 0.0;
    HypConst mine{};
    if (live) mine = hyp[h];

    for (uint32_t r = 0; r <= rounds; ++r) {
        if (!chain_wave) {
            if (r < rounds) {
                double* tl = tile[r & 1];
                const double(*fb)[R] = fbuf[r & 1];
                const int cls = (r < r0) ? 0 : 1;
                const uint32_t base = (cls == 0 ? r : r - r0) * R;
                const uint32_t nc = cls == 0 ? n0 : n1;
                // 1) band test + default +0.0
                uint32_t bits = 0;
#pragma unroll
                for (int k = 0; k < kPer; ++k) {
                    const uint32_t il = fsub + k * kStride;
                    bool cand = false;
                    if (live && base + il < nc) {
                        if (cls == 0) cand = scale_band<KIND>(fb[0][il], fb[1][il], fb[2][il], mine);
                        else if constexpr (KIND == 2) cand = orient_band(fb[0][il], fb[1][il], fb[2][il], fb[3][il], mine, tan_tau1);
                    }
                    tl[il * H + h] = 0.0;
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
                    if (cls == 0) {
                        r2 = scale_sq_residual<KIND == 1, true>(fb[0][il], fb[1][il], fb[2][il], m, q.ac);
                        inl = r2 <= T0;
                    } else {
                        const OrientConst oc{q.cphi, q.cphi2};
                        r2 = orient_sq_residual<true>(fb[0][il], fb[1][il], fb[2][il], fb[3][il], m, oc);
                        inl = r2 <= T1;
                    }
                    if (inl) {
                        tl[idx] = -r2;
                        atomicAdd(&cnt_sh[cls][hh], 1u);
                    }
                }
            }
        } else {
            // chain wave: stage round r+1's features, then fold tile r-1
            if (r + 1 < rounds) stage(r + 1, (r + 1) & 1, lane, 64);
            if (r > 0 && h < H) {
                // sequential fold of one tile column; LDS reads issued 8 ahead so
                // only the dependent fp64 adds remain on the critical path
                const uint32_t qr = r - 1;
                const double* col = tile[qr & 1] + h;
                if (qr < r0) {
                    const uint32_t len = min((uint32_t)R, n0 - qr * R);
                    uint32_t il = 0;
                    for (; il + 8 <= len; il += 8) {
                        double v[8];
#pragma unroll
                        for (int u = 0; u < 8; ++u) v[u] = col[(il + u) * H];
#pragma unroll
                        for (int u = 0; u < 8; ++u) acc0 += v[u];
                    }
                    for (; il < len; ++il) acc0 += col[il * H];
                    tot = acc0;
                } else {
                    const uint32_t len = min((uint32_t)R, n1 - (qr - r0) * R);
                    uint32_t il = 0;
                    for (; il + 8 <= len; il += 8) {
                        double v[8];
#pragma unroll
                        for (int u = 0; u < 8; ++u) v[u] = col[(il + u) * H];
#pragma unroll
                        for (int u = 0; u < 8; ++u) { acc1 += v[u]; tot += v[u]; }
                    }
                    for (; il < len; ++il) {
                        const double v = col[il * H];
                        acc1 += v;
                        tot += v;
                    }
                }
            }
        }
        __syncthreads();
    }
    if (chain_wave && h < H && hg < nh) {
        out.n0[hg] = valid_h ? cnt_sh[0][h] : 0;
        out.n1[hg] = valid_h ? cnt_sh[1][h] : 0;
        out.v0[hg] = valid_h ? acc0 : 0.0;
        out.v1[hg] = valid_h ? acc1 : 0.0;
        out.tot[hg] = valid_h ? tot : 0.0;
    }
}

// ----------------------------------------------------------------- mask ----
template <int KIND>
__global__ __launch_bounds__(kMaskBlock) void k_mask(DevClass c, int cls, RectModel m, int rule, double T,
                                                     double lambda, uint8_t* __restrict__ mask) {
    const uint32_t i = blockIdx.x * kMaskBlock + threadIdx.x;
    if (i >= c.n) return;
    double r2;
    if (cls == 0) r2 = scale_sq_residual<KIND == 1, false>(c.x[i], c.y[i], c.a[i], m, alpha_cube(m));
    else r2 = orient_sq_residual<false>(c.x[i], c.y[i], c.c0[i], c.c1[i], m, orient_const(m));
    bool inl;
    if (rule == 2) {
        // labeling(): BK max-flow with no pairwise edges (empty grid graph,
        // gcransac_python.cpp:63-68) -> SINK iff terminal capacity < 0.
        const double oml = 1.0 - lambda;
        double q = r2 / T;
        q = (q < 0.0) ? 0.0 : ((1.0 < q) ? 1.0 : q);      // std::clamp
        const double energy = 1.0 - q;
        const double tr = (r2 <= T) ? (0.0 - oml * energy) : (oml * (1.0 - energy) - 0.0);
        inl = tr < 0.0;
    } else {
        inl = r2 <= T;
    }
    mask[i] = inl ? 1 : 0;
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
        default: r = sqrt(a[i]); break;
    }
    out[i] = r;
}

inline unsigned blocks_for(size_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

hipError_t launch_generate(const DevProblem& p, uint64_t seed, uint64_t slot0, uint32_t nslots, uint8_t* inc,
                           RectModel* models, hipStream_t stream) {
    if (nslots == 0) return hipSuccess;
    const dim3 grid(blocks_for(nslots, kGenBlock)), block(kGenBlock);
    switch (p.solver) {
        case 0: hipLaunchKernelGGL(k_generate<0>, grid, block, 0, stream, p, seed, slot0, nslots, inc, models); break;
        case 1: hipLaunchKernelGGL(k_generate<1>, grid, block, 0, stream, p, seed, slot0, nslots, inc, models); break;
        default: hipLaunchKernelGGL(k_generate<2>, grid, block, 0, stream, p, seed, slot0, nslots, inc, models); break;
    }
    return hipGetLastError();
}

template <bool kIdentity>
void launch_score_t(const DevProblem& p, const double T[2], const RectModel* models, const uint8_t* inc, uint32_t nh,
                    const ScoreOut& out, hipStream_t stream) {
    const dim3 grid(blocks_for(nh, kScoreBlock)), block(kScoreBlock);
    switch (p.solver) {
        case 0: hipLaunchKernelGGL((k_score<0, kIdentity>), grid, block, 0, stream, p, T[0], T[1], models, inc, nh, out); break;
        case 1: hipLaunchKernelGGL((k_score<1, kIdentity>), grid, block, 0, stream, p, T[0], T[1], models, inc, nh, out); break;
        default: hipLaunchKernelGGL((k_score<2, kIdentity>), grid, block, 0, stream, p, T[0], T[1], models, inc, nh, out); break;
    }
}

template <int H, int R>
void launch_split_t(const DevProblem& p, const double T[2], const RectModel* models, const uint8_t* inc, uint32_t nh,
                    const ScoreOut& out, hipStream_t stream) {
    const dim3 grid((nh + H - 1) / H), block(kSplitThreads);
    // band constants: exp(1.5 thr) bounds the rectified log-scale residual,
    // tan(1.5 thr) the rectified angular one (host libm; margins in-kernel)
    const double band0 = exp(sqrt(T[0] / 2.25) * 1.5) * (1.0 + 1e-9);
    const double tau1 = sqrt(T[1]);
    const double tan_tau1 = (tau1 < 0.7) ? tan(tau1) * (1.0 + 1e-6) + 1e-300 : HUGE_VAL;
    switch (p.solver) {
        case 0: hipLaunchKernelGGL((k_score_split<0, H, R>), grid, block, 0, stream, p, T[0], T[1], band0, tan_tau1, models, inc, nh, out); break;
        case 1: hipLaunchKernelGGL((k_score_split<1, H, R>), grid, block, 0, stream, p, T[0], T[1], band0, tan_tau1, models, inc, nh, out); break;
        default: hipLaunchKernelGGL((k_score_split<2, H, R>), grid, block, 0, stream, p, T[0], T[1], band0, tan_tau1, models, inc, nh, out); break;
    }
}

int score_mode() {
    static int mode = -1;
    if (mode < 0) {
        const char* e = getenv("GCR_SCORE_KERNEL");
        mode = (e && e[0] == 'n') ? 1 : 0;   // "naive" -> lane-per-hypothesis kernel
    }
    return mode;
}

hipError_t launch_score(const DevProblem& p, const double T[2], const RectModel* models, const uint8_t* inc,
                        uint32_t nh, bool identity, const ScoreOut& out, hipStream_t stream) {
    if (nh == 0) return hipSuccess;
    if (!identity) launch_score_t<false>(p, T, models, inc, nh, out, stream);
    else if (score_mode() == 1) launch_score_t<true>(p, T, models, inc, nh, out, stream);
    else if (nh >= 16384) launch_split_t<64, 120>(p, T, models, inc, nh, out, stream);
    else if (nh >= 2048) launch_split_t<16, 360>(p, T, models, inc, nh, out, stream);
    else launch_split_t<4, 960>(p, T, models, inc, nh, out, stream);
    return hipGetLastError();
}

hipError_t launch_mask(const DevProblem& p, int cls, const RectModel& model, int rule, double T, double lambda,
                       uint8_t* mask, hipStream_t stream) {
    const DevClass& c = p.cls[cls];
    if (c.n == 0) return hipSuccess;
    const dim3 grid(blocks_for(c.n, kMaskBlock)), block(kMaskBlock);
    switch (p.solver) {
        case 0: hipLaunchKernelGGL(k_mask<0>, grid, block, 0, stream, c, cls, model, rule, T, lambda, mask); break;
        case 1: hipLaunchKernelGGL(k_mask<1>, grid, block, 0, stream, c, cls, model, rule, T, lambda, mask); break;
        default: hipLaunchKernelGGL(k_mask<2>, grid, block, 0, stream, c, cls, model, rule, T, lambda, mask); break;
    }
    return hipGetLastError();
}

hipError_t launch_math(int op, const double* a, const double* b, size_t n, double* out, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_math, dim3(blocks_for(n, 256)), dim3(256), 0, stream, op, a, b, n, out);
    return hipGetLastError();
}

}  // namespace gcr
